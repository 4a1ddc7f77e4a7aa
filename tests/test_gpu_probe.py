"""hfg_probe_mfma_rate (csrc/probe.hip): the live sustained-MFMA figure bench.py reports
beside the datasheet peak.  Plausibility only: below the datasheet dense rate, above a
floor no working MI355X falls under, and a shader clock in the part's range."""
import ctypes

import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("kind,lo,hi", [(0, 300.0, 2500.0 * 1.02), (1, 40.0, 157.3 * 1.02),
                                         (2, 100.0, 2500.0 * 1.02), (3, 10.0, 157.3 * 1.02),
                                         (4, 300.0, 2500.0 * 1.02), (5, 100.0, 2500.0 * 1.02)])
def test_probe_mfma_rate_plausible(pkg, kind, lo, hi):
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    lib = pkg.load_library()
    tf, mhz = ctypes.c_double(0.0), ctypes.c_double(0.0)
    assert lib.hfg_probe_mfma_rate(0, kind, 20000, ctypes.byref(tf), ctypes.byref(mhz)) == 0
    print(f"\nkind {kind}: {tf.value:.1f} TFLOP/s dense at {mhz.value:.0f} MHz")
    assert lo < tf.value < hi
    assert 500.0 < mhz.value < 2600.0
    assert lib.hfg_probe_mfma_rate(0, 6, 10, ctypes.byref(tf), ctypes.byref(mhz)) == -22
