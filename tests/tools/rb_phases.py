"""Phase times inside the whole-ResBlock kernels from the diagnostic build's clock stamps
(resblock_bf16x3.hip, -DHFG_RB_TIMING=1; built as ab/rbts.so by profiles/r04/ab_build.sh).

GPU box:  python tests/tools/rb_phases.py LIB.so [--precision f16x3]
Runs 3 V1 [8, 80, 1024] forwards with that library, reads the stamps of the last one and
prints per kernel instance and launch half: blocks, rounds (distinct start waves), the median
shader-clock cycles of each phase (prologue, each conv's MFMA loop, each transition, the MRF
epilogue) and the clock (s_memtime vs the 100 MHz s_memrealtime)."""
import ctypes
import importlib
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
SLOTS, BLOCKS, REGIONS = 24, 8192, 20
NAMES = {}
for kt_i, kt in enumerate((3, 7, 11)):
    for wm_i, wm in enumerate(("C32", "C64", "C128")):
        for half in (0, 1):
            NAMES[(kt_i * 3 + wm_i) * 2 + half] = f"k{kt} {wm} half{half}"
NAMES[18] = "k3 C64 narrow half0"
NAMES[19] = "k3 C64 narrow half1"


def main():
    lib_path = sys.argv[1]
    prec = sys.argv[3] if len(sys.argv) > 3 and sys.argv[2] == "--precision" else "f16x3"
    sys.path.insert(0, ROOT)
    import torch
    import __graft_entry__ as ge
    pkg = ge.load_package()
    lib = pkg.load_library()
    dl = ctypes.CDLL(lib_path)
    S = importlib.import_module(ge.PKG_NAME + ".synth")
    cfg = S.PRESETS["v1"]
    sd = {k: torch.from_numpy(v) for k, v in S.random_state_dict(cfg, seed=0).items()}
    dev = torch.device("cuda:0")
    gen = pkg.HiFiGANGenerator(**cfg.kwargs(), precision=prec).eval()
    gen.load_state_dict(sd)
    h = gen.hip_handle(dev)
    B, T = 8, 1024
    mel = torch.randn(B, cfg.n_mels, T, generator=torch.Generator().manual_seed(1)).to(dev)
    out_len = h.out_len(T)
    wav = torch.empty((B, 1, out_len), dtype=torch.float32, device=dev)
    h.set_streams(1)
    ws_bytes = h.workspace_bytes(B, T)
    ws = torch.empty(ws_bytes, dtype=torch.uint8, device=dev)
    st = torch.cuda.current_stream(dev).cuda_stream
    for _ in range(2):
        h.forward_ws(mel.data_ptr(), B, T, wav.data_ptr(), out_len, ws.data_ptr(), ws_bytes, st)
    torch.cuda.synchronize(dev)
    assert dl.hfg_debug_rb_ts_clear() == 0
    h.forward_ws(mel.data_ptr(), B, T, wav.data_ptr(), out_len, ws.data_ptr(), ws_bytes, st)
    torch.cuda.synchronize(dev)
    buf = np.zeros(REGIONS * BLOCKS * SLOTS, dtype=np.uint64)
    assert dl.hfg_debug_rb_ts(buf.ctypes.data_as(ctypes.c_void_p), ctypes.c_size_t(buf.nbytes)) == 0
    buf = buf.reshape(REGIONS, BLOCKS, SLOTS).astype(np.int64)
    out = {}
    for r in range(REGIONS):
        blk = buf[r]
        used = blk[:, 1] != 0
        if not used.any():
            continue
        blk = blk[used]
        # last filled slot = realtime end (4 + 2 n_conv)
        nz = (blk[:, :20] != 0).sum(axis=1)
        last = int(np.median(nz)) - 1
        n_conv = (last - 4) // 2
        t = blk[:, 1:last].astype(np.float64)  # memtime stamps 1 .. 3 + 2n
        d = np.diff(t, axis=1)
        rt = (blk[:, last] - blk[:, 0]).astype(np.float64)  # 100 MHz ticks
        mhz = np.median((t[:, -1] - t[:, 0]) / np.maximum(rt, 1) * 100.0)
        names = ["prologue"]
        for cv in range(n_conv):
            names += [f"conv{cv}", f"trans{cv}"]
        names += ["epilogue"]
        med = np.median(d, axis=1 - 1)
        starts = np.sort(blk[:, 0])
        # rounds: gaps in the start times larger than half a block time
        blk_ticks = np.median(rt)
        rounds = 1 + int((np.diff(starts) > 0.5 * blk_ticks).sum())
        tot = float(np.median(t[:, -1] - t[:, 0]))
        row = {"blocks": int(used.sum()), "rounds": rounds, "MHz": round(float(mhz)),
               "block_us": round(float(blk_ticks) / 100.0, 1),
               "span_us": round(float(starts[-1] - starts[0] + blk_ticks) / 100.0, 1),
               "cycles": {n: int(v) for n, v in zip(names, med)},
               "frac": {n: round(float(v) / tot, 3) for n, v in zip(names, med)}}
        sub = {}
        if (blk[:, 22] != 0).all():
            sub = {"setup": blk[:, 20] - blk[:, 1], "x_wait": blk[:, 21] - blk[:, 20],
                   "amax_bar": blk[:, 22] - blk[:, 21], "op_write": blk[:, 2] - blk[:, 22]}
        if (blk[:, 23] != 0).all():
            sub["mrf_wait"] = blk[:, 23] - blk[:, 2 + 2 * n_conv]
            sub["mrf_store"] = blk[:, 3 + 2 * n_conv] - blk[:, 23]
        row["sub"] = {k: int(np.median(v)) for k, v in sub.items()}
        out[NAMES.get(r, str(r))] = row
        print(NAMES.get(r, str(r)), json.dumps(row))
    os.makedirs(os.path.join(ROOT, "gpurun_out", "r04"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", "r04", f"rb_phases_{prec}.json"), "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
