"""Experiment (GPU): the C5 workload (32 ragged utterances of 60-63 frames, [B,T,80] glue
layout) and a mid-size batch, per 2-stream split threshold (HFG_SPLIT_MIN) and concurrent
ResBlocks (HFG_RB_CONC).  Prints one JSON line per setting."""
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
    glue = importlib.import_module(ge.PKG_NAME + ".glue")
    cfg = S.PRESETS["v1"]
    sd = {k: torch.from_numpy(v) for k, v in S.random_state_dict(cfg, seed=0).items()}
    g = torch.Generator().manual_seed(5)
    lens = [int(x) for x in torch.randint(60, 64, (32,), generator=g)]
    mel_pred = torch.randn(32, max(lens), 80, generator=g).to(dev)
    mel16 = torch.randn(16, 80, 256, generator=g).to(dev)
    for env in ({}, {"HFG_SPLIT_MIN": "1024"}, {"HFG_SPLIT_MIN": "1024", "HFG_RB_CONC": "0"},
                {"HFG_RB_CONC": "0"}):
        old = {k: os.environ.get(k) for k in env}
        os.environ.update(env)
        gen = pkg.HiFiGANGenerator(**cfg.kwargs(), precision="bf16x3").eval()
        gen.load_state_dict(sd)
        gen = gen.to(dev)
        gen.hip_handle(dev)
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
        res = {"env": env}
        for name, fn in (("C5", lambda: glue.vocode_acoustic(gen, mel_pred, lens)),
                         ("B16_T256", lambda: gen(mel16))):
            with torch.no_grad():
                for _ in range(3):
                    fn()
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for _ in range(20):
                    fn()
                torch.cuda.synchronize()
            res[name + "_ms"] = (time.perf_counter() - t0) / 20 * 1e3
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
