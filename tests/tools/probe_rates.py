"""Sustained MFMA rate of this GPU per instruction kind (hfg_probe_mfma_rate): bf16 vs f16
on random operands — the f16x3 kernels' instruction against bf16x3's.  GPU box only.

    python tests/tools/probe_rates.py
"""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import __graft_entry__ as ge  # noqa: E402

pkg = ge.load_package()
lib = pkg.load_library()
out = {}
for rep in range(2):
    for kind, name in ((0, "bf16_4chains"), (4, "f16_4chains"), (2, "bf16_1chain"),
                       (5, "f16_1chain"), (1, "fp32_4chains")):
        tf, mhz = ctypes.c_double(), ctypes.c_double()
        iters = 50000 if kind != 1 else 40000
        rc = lib.hfg_probe_mfma_rate(0, kind, iters, ctypes.byref(tf), ctypes.byref(mhz))
        out.setdefault(name, []).append({"rc": rc, "TFLOPs": round(tf.value, 1),
                                         "MHz": round(mhz.value, 1)})
print(json.dumps(out, indent=1))
