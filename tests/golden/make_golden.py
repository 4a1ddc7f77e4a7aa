"""Generate the golden fixtures under tests/golden/ from the REFERENCE implementation.

Run in the build container only (needs /root/reference, read-only):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py

For each case: PRNG weights (oracle/prng.py, keyed by (seed, state_dict key))
are loaded into the reference ``models.hifigan.HiFiGANGenerator`` (optionally
after its own ``apply_weight_norm``), the reference forward runs on a PRNG mel,
and we store: the mel input, the final wav, per-stage tensors captured with
forward hooks on the reference modules (conv_pre, ups.i, mrfs.i), and stats
(sha256 of the f32 bytes, mean, std, L2, max|.|) for every stage.  Full
per-stage tensors are stored only when <= 64 KiB.  Nothing of the reference's
source is copied; only its outputs are written.
"""
from __future__ import annotations

import hashlib
import json
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
REF = "/root/reference"

from oracle import config as C  # noqa: E402
from oracle import prng  # noqa: E402
from oracle import hifigan_torch, hifigan_np64  # noqa: E402

CASES = [
    # name, preset, (B, T), seed, weight-scale, weight-norm
    ("g1_v1_b1_t32", "v1", (1, 32), 1, 1.0, False),
    ("g2_v1_b2_t17", "v1", (2, 17), 2, 1.0, False),
    ("g3_v2star_b2_t32", "v2star", (2, 32), 3, 1.0, False),
    ("g4_nonexact_b1_t20", "nonexact", (1, 20), 4, 1.0, False),
    ("g5_v1_weightnorm_b1_t16", "v1", (1, 16), 5, 1.0, True),
    ("g6_v1_loud2x_b1_t24", "v1", (1, 24), 6, 2.0, False),
    ("g7_v1_b3_t1", "v1", (3, 1), 7, 1.0, False),
    ("g8_v2star_b1_t3", "v2star", (1, 3), 8, 1.0, False),
    # SURVEY.md §8(c) G6 "loud" at the specified x4 weight scale (tanh far from linear)
    ("g9_v1_loud4x_b1_t24", "v1", (1, 24), 9, 4.0, False),
    ("g10_v2star_loud4x_b1_t40", "v2star", (1, 40), 10, 4.0, False),
]

FULL_LIMIT = 64 * 1024


def stats(a: np.ndarray):
    a = np.ascontiguousarray(a, dtype=np.float32)
    return {
        "shape": list(a.shape),
        "sha256": hashlib.sha256(a.tobytes()).hexdigest(),
        "mean": float(a.astype(np.float64).mean()),
        "std": float(a.astype(np.float64).std()),
        "l2": float(np.sqrt((a.astype(np.float64) ** 2).sum())),
        "maxabs": float(np.abs(a).max()),
    }


def sd_sha(sd) -> str:
    h = hashlib.sha256()
    for k, v in sd.items():
        h.update(k.encode())
        h.update(np.ascontiguousarray(v, dtype=np.float32).tobytes())
    return h.hexdigest()


def main():
    sys.path.insert(0, REF)
    os.environ.setdefault("PYTHONDONTWRITEBYTECODE", "1")
    from models.hifigan import HiFiGANGenerator  # the reference

    torch.set_num_threads(8)
    index = {}
    for name, preset, (bsz, t), seed, scale, wn in CASES:
        cfg = C.PRESETS[preset]
        ref = HiFiGANGenerator(**cfg.kwargs()).eval()
        if wn:
            ref.apply_weight_norm()
            sd = C.make_weight_norm_state_dict(cfg, seed)
        else:
            sd = C.make_state_dict(cfg, seed, scale)
        ref.load_state_dict({k: torch.from_numpy(v.copy()) for k, v in sd.items()}, strict=True)
        mel = prng.mel_input(seed, (bsz, cfg.n_mels, t))

        taps = {}

        def hook(nm):
            def f(_m, _i, out):
                taps[nm] = out.detach().clone().numpy()
            return f

        ref.conv_pre.register_forward_hook(hook("conv_pre"))
        for i in range(len(cfg.upsample_rates)):
            ref.ups[i].register_forward_hook(hook(f"ups.{i}"))
            ref.mrfs[i].register_forward_hook(hook(f"mrfs.{i}"))
        with torch.no_grad():
            wav = ref(torch.from_numpy(mel)).numpy()
        taps["wav"] = wav

        # cross-checks of the restatements against the reference (recorded, not asserted)
        tsd = hifigan_torch.to_torch_state(sd)
        wav_t = hifigan_torch.generator_forward(tsd, cfg, torch.from_numpy(mel)).numpy()
        wav_64 = hifigan_np64.generator_forward(sd, cfg, mel)

        arrays = {"mel": mel, "wav": wav}
        for k, v in taps.items():
            if k != "wav" and v.nbytes <= FULL_LIMIT:
                arrays["stage__" + k] = v
        np.savez(os.path.join(HERE, name + ".npz"), **arrays)
        index[name] = {
            "preset": preset,
            "config": cfg.kwargs(),
            "batch": bsz,
            "frames": t,
            "seed": seed,
            "weight_scale": scale,
            "weight_norm": wn,
            "state_dict_sha256": sd_sha(sd),
            "n_params_tensors": len(sd),
            "out_len": int(wav.shape[-1]),
            "stages": {k: stats(v) for k, v in taps.items()},
            "torch_restatement_bitwise_equal": bool(np.array_equal(wav_t, wav)),
            "torch_restatement_maxabs_diff": float(np.abs(wav_t - wav).max()),
            "np64_maxabs_diff": float(np.abs(wav_64 - wav).max()),
        }
        print(name, wav.shape, "torch==", index[name]["torch_restatement_bitwise_equal"],
              "np64 diff", index[name]["np64_maxabs_diff"], "maxabs", index[name]["stages"]["wav"]["maxabs"])
    with open(os.path.join(HERE, "golden_index.json"), "w") as f:
        json.dump({"generator": "tests/golden/make_golden.py",
                   "reference": "models/hifigan.py (terrense/TTS-sambert_hifiGAN), imported read-only",
                   "torch": torch.__version__, "threads": 8, "cases": index}, f, indent=1)


if __name__ == "__main__":
    main()
