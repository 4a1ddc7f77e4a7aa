"""Diagnostic (GPU): a ragged batch of the non-exact config under each execution toggle,
every item against the oracle run on that item alone.  usage: python tests/tools/diag_ragged.py"""
import importlib.util
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from oracle import config as C  # noqa: E402
from oracle import hifigan_torch as H  # noqa: E402

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
from test_gpu_latency_paths import _gen  # noqa: E402


def main():
    spec = importlib.util.spec_from_file_location("pkg", "tts-sambert_hifigan_amd/__init__.py",
                                                  submodule_search_locations=["tts-sambert_hifigan_amd"])
    pkg = importlib.util.module_from_spec(spec)
    sys.modules["pkg"] = pkg
    spec.loader.exec_module(pkg)
    dev = torch.device("cuda:0")
    preset = sys.argv[1] if len(sys.argv) > 1 else "nonexact"
    cfg = C.PRESETS[preset]
    sd = C.make_state_dict(cfg, seed=37)
    mel = torch.randn(3, 80, 77, generator=torch.Generator().manual_seed(13))
    lens = [77, 60, 33]
    refs = [H.generator_forward(H.to_torch_state(sd), cfg, mel[b:b + 1, :, :n]).numpy()[0]
            for b, n in enumerate(lens)]
    cases = [("f16x3", {}), ("bf16x3", {}), ("fp32", {}), ("f16x3", {"RB_CONC": "0"}),
             ("f16x3", {"FUSED_RB": "0"}), ("f16x3", {"SMALL_TILE": "0"}),
             ("f16x3", {"SMALL_TILE": "1"}), ("f16x3", {"UPS_FRAMES": "2"}),
             ("fp32", {"RB_CONC": "0"})]
    for prec, env in cases:
        gen = _gen(pkg, cfg, sd, dev, prec, env)
        with torch.no_grad():
            out = gen(mel.to(dev), lengths=lens).cpu().numpy()
            solo = [gen(mel[b:b + 1, :, :n].to(dev)).cpu().numpy()[0] for b, n in enumerate(lens)]
        torch.cuda.synchronize()
        errs = []
        for b, r in enumerate(refs):
            n = r.shape[-1]
            errs.append((float(np.abs(out[b, :, :n] - r).max()), float(np.abs(solo[b] - r).max()),
                         int(np.argmax(np.abs(out[b, 0, :n] - r[0]) > 1e-4)) if
                         np.abs(out[b, :, :n] - r).max() > 1e-4 else -1))
        print(prec, env, " ".join(f"[item{b}: batch {e:.1e} solo {s:.1e} first>1e-4 @{i}]"
                                  for b, (e, s, i) in enumerate(errs)), flush=True)


if __name__ == "__main__":
    main()
