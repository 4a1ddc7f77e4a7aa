"""Diagnostic (GPU): 1-stream vs 2-stream and run-to-run bitwise equality of the
Generator, per precision, with and without ragged lengths.
usage: python tests/tools/diag_split.py"""
import os, sys
import numpy as np
import torch
ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..")
sys.path.insert(0, ROOT)
import __graft_entry__ as ge
from oracle import config as C, prng

pkg = ge.load_package()
dev = torch.device("cuda:0")
cfg = C.V1
sd = C.make_state_dict(cfg, seed=17)
B, T = 5, 1000
mel = torch.as_tensor(prng.mel_input(23, (B, cfg.n_mels, T))).to(dev)
lens = torch.tensor([1000, 731, 1000, 2, 517], dtype=torch.int32, device=dev)
for prec in sys.argv[1:] or ["bf16x3", "fp32"]:
    gen = pkg.HiFiGANGenerator(**cfg.kwargs(), precision=prec).eval()
    gen.load_state_dict({k: torch.from_numpy(np.ascontiguousarray(v)) for k, v in sd.items()})
    gen = gen.to(dev)
    h = gen.hip_handle(dev)
    runs = {}
    for tag, n in (("s1a", 1), ("s2a", 2), ("s1b", 1), ("s2b", 2)):
        h.set_streams(n)
        with torch.no_grad():
            a = gen(mel).cpu().numpy()
            b = gen(mel, lengths=lens).cpu().numpy()
        torch.cuda.synchronize()
        runs[tag] = (a, b)
    for x, y in (("s1a", "s1b"), ("s2a", "s2b"), ("s1a", "s2a"), ("s1b", "s2b")):
        for k, name in ((0, "full"), (1, "ragged")):
            d = np.abs(runs[x][k] - runs[y][k])
            per = d.reshape(B, -1).max(axis=1)
            if d.max() > 0:
                idx = np.argwhere(d.reshape(B, -1) > 0)
                first = idx[:, 1].min(); last = idx[:, 1].max()
                print(f"{prec} {x} vs {y} {name}: max {d.max():.3e} per-utt {per} nz {len(idx)} "
                      f"cols [{first},{last}]", flush=True)
            else:
                print(f"{prec} {x} vs {y} {name}: equal", flush=True)
