"""Product-side synthetic workload (tts-sambert_hifigan_amd/synth.py) used by bench.py:
same architecture / state_dict layout as the reference (checked against the oracle's
restatement of models/hifigan.py's parameter list), default-init bounds, and the
SURVEY.md §8(d) canonical byte model."""
import importlib
import os

import numpy as np
import pytest

from oracle import config as OC


@pytest.fixture(scope="module")
def S(pkg):
    import __graft_entry__ as ge
    return importlib.import_module(ge.PKG_NAME + ".synth")


@pytest.mark.parametrize("preset", ["v1", "v2star", "nonexact"])
def test_param_specs_match_reference_layout(S, preset):
    assert S.param_specs(S.PRESETS[preset]) == OC.param_specs(OC.PRESETS[preset])
    assert S.PRESETS[preset].kwargs() == OC.PRESETS[preset].kwargs()


def test_random_state_dict_bounds_and_determinism(S):
    cfg = S.V2STAR
    a = S.random_state_dict(cfg, seed=3)
    b = S.random_state_dict(cfg, seed=3)
    c = S.random_state_dict(cfg, seed=4)
    specs = {k: (shape, fan_in) for k, shape, fan_in in S.param_specs(cfg)}
    assert list(a) == list(specs)
    for k, v in a.items():
        shape, fan_in = specs[k]
        assert v.dtype == np.float32 and v.shape == shape
        assert np.abs(v).max() <= 1.0 / np.sqrt(fan_in)
        assert np.array_equal(v, b[k])
    assert not np.array_equal(a["conv_pre.weight"], c["conv_pre.weight"])


def test_canonical_byte_model(S):
    # V1 5,436,736 B per frame (21,237 B/sample), V2* 960,832 B per frame
    assert S.layer_streaming_bytes_per_frame(S.V1) == 5436736
    assert S.layer_streaming_bytes_per_frame(S.V2STAR) == 960832
    assert S.param_bytes(S.V1) == 4 * 13926017  # 13,926,017 params


def test_bench_pmc_key_maps_profile_labels_to_kernel_names():
    """bench.py joins the library's per-kernel profile labels with the rocprofv3 PMC rows by
    kernel name: the whole-ResBlock labels ('persist' / no flag) map to the template's bool."""
    import importlib.util
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(root, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    pmc = {"resblock_bf16x3<11,2,4,1,3,1,true>": {}, "resblock_bf16x3<3,4,2,1,3,1,false>": {},
           "conv1d_bf16x3<11,2,2,2,2,4,2,false,3,true,1>": {}, "absmax_kernel": {}}
    assert bench._pmc_key("resblock_bf16x3<11, 2, 4, 1, 3, 1, persist>", pmc) == \
        "resblock_bf16x3<11,2,4,1,3,1,true>"
    assert bench._pmc_key("resblock_bf16x3<3, 4, 2, 1, 3, 1>", pmc) == \
        "resblock_bf16x3<3,4,2,1,3,1,false>"
    assert bench._pmc_key("conv1d_bf16x3<11, 2, 2, 2, 2, 4, 2, false, 3, true, 1>", pmc) == \
        "conv1d_bf16x3<11,2,2,2,2,4,2,false,3,true,1>"
    assert bench._pmc_key("absmax", pmc) == "absmax_kernel"
    assert bench._pmc_key("ups_bf16x3<1, 4, 1, 2, 3, 1>", pmc) is None
