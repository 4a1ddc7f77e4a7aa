"""Experiment (GPU): C2 step time of the 2-stream production forward launched eagerly vs
replayed from a captured hipGraph (same launches, same workspace).  Prints one JSON line."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import __graft_entry__ as ge  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    pkg = ge.load_package()
    pkg.load_library()
    import importlib
    S = importlib.import_module(ge.PKG_NAME + ".synth")
    cfg = S.PRESETS["v1"]
    sd = {k: torch.from_numpy(v) for k, v in S.random_state_dict(cfg, seed=0).items()}
    B, T, K = 8, 1024, 20
    mel = torch.randn(B, 80, T, generator=torch.Generator().manual_seed(1234)).to(dev)
    gen = pkg.HiFiGANGenerator(**cfg.kwargs(), precision="bf16x3").eval()
    gen.load_state_dict(sd)
    h = gen.hip_handle(dev)
    out_len = h.out_len(T)
    wav = torch.empty((B, 1, out_len), device=dev)
    h.set_streams(2)
    ws_bytes = h.workspace_bytes(B, T)
    ws = torch.empty(ws_bytes, dtype=torch.uint8, device=dev)
    res = {}
    s = torch.cuda.Stream(dev)
    with torch.cuda.stream(s):
        def step():
            h.forward_ws(mel.data_ptr(), B, T, wav.data_ptr(), out_len, ws.data_ptr(), ws_bytes,
                         s.cuda_stream)
        for _ in range(3):
            step()
        torch.cuda.synchronize()
        for rep in range(2):
            t0 = time.perf_counter()
            for _ in range(K):
                step()
            torch.cuda.synchronize()
            res[f"eager_ms_{rep}"] = (time.perf_counter() - t0) / K * 1e3
        ref = wav.clone()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            step()
        g.replay()
        torch.cuda.synchronize()
        res["graph_equals_eager"] = bool(torch.equal(wav, ref))
        for rep in range(2):
            t0 = time.perf_counter()
            for _ in range(K):
                g.replay()
            torch.cuda.synchronize()
            res[f"graph_ms_{rep}"] = (time.perf_counter() - t0) / K * 1e3
    print(json.dumps(res))


if __name__ == "__main__":
    main()
