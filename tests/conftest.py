import json
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

GOLDEN_DIR = os.path.join(ROOT, "tests", "golden")


_EVIDENCE = []


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); run with -m gpu")


def pytest_terminal_summary(terminalreporter):
    """The measured numbers parity tests recorded through the `evidence` fixture (max |err|
    against the oracle, ...), printed at the end of every run, -q included: a passing test's
    print() output is captured and dropped, these lines are not."""
    if _EVIDENCE:
        terminalreporter.section("parity evidence (measured)")
        for line in _EVIDENCE:
            terminalreporter.write_line(line)


@pytest.fixture
def evidence(request):
    """evidence(text): record one measured figure of this test for the end-of-run summary."""
    def add(text):
        _EVIDENCE.append(f"{request.node.nodeid}: {text}")
        print(text)
    return add


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


@pytest.fixture
def sched(pkg):
    """sched(knob, value): force one schedule choice for the handles this test creates
    (hfg_debug_schedule_set; the library reads no HFG_* environment knob); every override
    is dropped when the test ends."""
    def set_(knob, value):
        pkg.schedule_override(knob, int(value))
    yield set_
    pkg.schedule_clear()


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
