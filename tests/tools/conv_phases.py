"""Phase times inside the tile-5 layer-conv kernel from the diagnostic build's clock stamps
(conv_bf16x3.hip, -DHFG_CONV_TIMING=1; built as ab/cvts.so by profiles/r04/ab_build.sh).

GPU box:  python tests/tools/conv_phases.py LIB.so   (LIB.so = the package's library path,
holding the diagnostic build).  Per KT (the last launch of that KT in a V1 [8, 80, 1024]
forward): blocks, the clock, median cycles of prologue / group loop / epilogue, the loop's
summed barrier waits, and the block start-time spread.  A stamp is a global store, and
vmcnt counts loads and stores in one in-order queue: a load waited for after a stamp also
waits for the stamp's write, so the stamps add latency to the phases they split."""
import ctypes
import importlib
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
SLOTS, BLOCKS, REGIONS = 16, 8192, 12


def main():
    lib_path = sys.argv[1]
    sys.path.insert(0, ROOT)
    import torch
    import __graft_entry__ as ge
    pkg = ge.load_package()
    pkg.load_library()
    dl = ctypes.CDLL(lib_path)
    S = importlib.import_module(ge.PKG_NAME + ".synth")
    cfg = S.PRESETS["v1"]
    sd = {k: torch.from_numpy(v) for k, v in S.random_state_dict(cfg, seed=0).items()}
    dev = torch.device("cuda:0")
    gen = pkg.HiFiGANGenerator(**cfg.kwargs(), precision="f16x3").eval()
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
    assert dl.hfg_debug_cv_ts_clear() == 0
    h.forward_ws(mel.data_ptr(), B, T, wav.data_ptr(), out_len, ws.data_ptr(), ws_bytes, st)
    torch.cuda.synchronize(dev)
    buf = np.zeros(REGIONS * BLOCKS * SLOTS, dtype=np.uint64)
    assert dl.hfg_debug_cv_ts(buf.ctypes.data_as(ctypes.c_void_p), ctypes.c_size_t(buf.nbytes)) == 0
    buf = buf.reshape(REGIONS, BLOCKS, SLOTS).astype(np.int64)
    odir = os.path.join(ROOT, "gpurun_out", "r05")
    os.makedirs(odir, exist_ok=True)
    tag = os.environ.get("CVP_TAG", "default")
    # raw stamps (slot 12: HW_ID | XCC_ID << 32 of the block's wave 0) for offline analysis
    np.save(os.path.join(odir, f"cvp_raw_{tag}.npy"), buf[:9])
    out = {}
    for r, (kt, epi) in enumerate((k, e) for k in (3, 7, 11, 0) for e in ("plain", "res", "res+mrf")):
        blk = buf[r]
        blk = blk[(blk[:, 1] != 0) & (blk[:, 4] != 0)]
        if not len(blk):
            continue
        tot = blk[:, 4] - blk[:, 1]
        rt = np.maximum(blk[:, 6] - blk[:, 0], 1)
        starts = np.sort(blk[:, 0])
        row = {"blocks": int(len(blk)), "MHz": round(float(np.median(tot / rt * 100.0))),
               "block_us": round(float(np.median(rt)) / 100.0, 1),
               "span_us": round(float(blk[:, 6].max() - starts[0]) / 100.0, 1),
               "prologue": int(np.median(blk[:, 2] - blk[:, 1])),
               "loop": int(np.median(blk[:, 3] - blk[:, 2])),
               "barrier_wait": int(np.median(blk[:, 5])),
               "epilogue": int(np.median(blk[:, 4] - blk[:, 3])),
               "epi_wait_barrier": int(np.median(blk[:, 7] - blk[:, 3])),
               "epi_stage0": int(np.median(blk[:, 8] - blk[:, 7])),
               "epi_tile0": int(np.median(blk[:, 9] - blk[:, 8])),
               "epi_stage1": int(np.median(blk[:, 10] - blk[:, 9])),
               "epi_tile1": int(np.median(blk[:, 11] - blk[:, 10])),
               "epi_commit": int(np.median(blk[:, 4] - blk[:, 11])),
               "start_spread_us": [round(float(np.percentile(starts - starts[0], q)) / 100.0, 1)
                                   for q in (25, 50, 75, 100)]}
        out[f"k{kt} {epi}"] = row
        print(f"k{kt} {epi}", json.dumps(row))
    with open(os.path.join(odir, f"conv_phases_{tag}.json"), "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
