"""Experiment: one [8,80,1024] forward vs two [4,80,1024] forwards on two HIP streams
(each with its own workspace), to see whether overlapping the halves' launch tails
pays.  Prints one JSON line.  Not part of the product path.

    python tests/tools/exp_two_streams.py
"""
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import __graft_entry__ as ge  # noqa: E402
from oracle import config as C  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    pkg = ge.load_package()
    cfg = C.V1
    sd = {k: torch.from_numpy(v) for k, v in C.make_state_dict(cfg, seed=0).items()}
    gen = pkg.HiFiGANGenerator(**cfg.kwargs(), precision="bf16x3").eval()
    gen.load_state_dict(sd)
    h = gen.hip_handle(dev)
    B, T = 8, 1024
    mel = torch.randn(B, cfg.n_mels, T, generator=torch.Generator().manual_seed(1)).to(dev)
    out_len = h.out_len(T)
    wav = torch.empty((B, 1, out_len), device=dev)
    s0 = torch.cuda.current_stream(dev)
    streams = [torch.cuda.Stream(dev) for _ in range(4)]
    esz = 4

    def make(nsplit):
        hb = B // nsplit
        wsb = h.workspace_bytes(hb, T)
        wss = [torch.empty(wsb, dtype=torch.uint8, device=dev) for _ in range(nsplit)]

        def fn():
            if nsplit == 1:
                h.forward_ws(mel.data_ptr(), B, T, wav.data_ptr(), out_len, wss[0].data_ptr(), wsb,
                             s0.cuda_stream)
                return
            e = torch.cuda.Event()
            e.record(s0)
            for i in range(nsplit):
                streams[i].wait_event(e)
                h.forward_ws(mel.data_ptr() + i * hb * cfg.n_mels * T * esz, hb, T,
                             wav.data_ptr() + i * hb * out_len * esz, out_len, wss[i].data_ptr(),
                             wsb, streams[i].cuda_stream)
            for i in range(nsplit):
                s0.wait_stream(streams[i])
        return fn

    one, two, four = make(1), make(2), make(4)
    res = {}
    ref = None
    for name, fn in (("one", one), ("two", two), ("four", four), ("one_again", one),
                     ("two_again", two), ("four_again", four)):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(10):
            fn()
        torch.cuda.synchronize()
        res[name + "_ms"] = (time.perf_counter() - t0) * 100.0
        if ref is None:
            ref = wav.clone()
        else:
            res[name + "_maxdiff"] = float((wav - ref).abs().max())
    print(json.dumps(res))


if __name__ == "__main__":
    main()
