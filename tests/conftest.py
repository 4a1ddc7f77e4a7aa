import json
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

GOLDEN_DIR = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); run with -m gpu")


@pytest.fixture(scope="session", autouse=True)
def _native_provenance(request):
    """A GPU session must run the library built from this tree (hfg_version carries the
    sha256 of csrc/ + include/ that build.py compiled in)."""
    if not any(item.get_closest_marker("gpu") for item in request.session.items):
        return
    import __graft_entry__ as ge
    p = ge.load_package()
    print(f"\n[provenance] {p.load_library().hfg_version().decode()}")
    p.check_provenance()


@pytest.fixture(scope="session")
def pkg():
    import __graft_entry__ as ge
    return ge.load_package()


@pytest.fixture(scope="session")
def golden_index():
    with open(os.path.join(GOLDEN_DIR, "golden_index.json")) as f:
        return json.load(f)


def load_golden(name):
    d = np.load(os.path.join(GOLDEN_DIR, name + ".npz"))
    return {k: d[k] for k in d.files}


def golden_case_state(case):
    """(GenConfig, numpy state dict, mel) reconstructed from a golden index entry."""
    from oracle import config as C
    cfg = C.GenConfig(**case["config"])
    if case["weight_norm"]:
        sd = C.make_weight_norm_state_dict(cfg, case["seed"])
    else:
        sd = C.make_state_dict(cfg, case["seed"], case["weight_scale"])
    return cfg, sd
