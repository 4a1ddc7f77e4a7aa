"""Where does the device log-mel differ from the float64-spectrum restatement?  (GPU box)
Prints, per signal, the largest |device - log_mel64| with its (band, frame), the oracle value
there, and the error profile over frames.  Test infrastructure only."""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def main():
    import importlib
    import __graft_entry__ as ge
    ge.load_package()
    melmod = importlib.import_module(ge.PKG_NAME + ".mel")
    from oracle import mel_torch as M
    n = 22050 + 77
    g = torch.Generator().manual_seed(0)
    t = torch.arange(n) / 22050.0
    tone = 0.3 * torch.sin(2 * np.pi * 220.0 * t) + 0.2 * torch.sin(2 * np.pi * 3100.0 * t)
    noise = 0.1 * torch.randn(n, generator=g)
    chirp = 0.5 * torch.sin(2 * np.pi * (100 + 2000 * t) * t)
    wav = torch.stack([tone + noise, chirp])
    dev = torch.device("cuda:0")
    got = melmod.MelSpectrogram(device=dev)(wav.to(dev)).cpu().double()
    ref = M.log_mel64(wav)
    e = (got - ref).abs()
    out = {}
    for b in range(2):
        eb = e[b]
        m, f = np.unravel_index(int(eb.argmax()), eb.shape)
        out[b] = {"max": float(eb.max()), "band": int(m), "frame": int(f),
                  "ref": float(ref[b, m, f]), "got": float(got[b, m, f]),
                  "per_frame_max": [round(float(v), 8) for v in eb.max(0).values[:12]],
                  "frames_over_1e-5": int((eb.max(0).values > 1e-5).sum()),
                  "bands_over_1e-5": int((eb.max(1).values > 1e-5).sum())}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
