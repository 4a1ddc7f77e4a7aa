"""Generate the config-5 fixture (SAM-BERT acoustic model -> mel -> vocoder) from the
REFERENCE implementation.

BASELINE.json config 5: "Full SAM-BERT acoustic_model.py (CPU) -> mel -> MI355X
HiFi-GAN end-to-end, batch 32 variable-length utterances".  The acoustic model is
out of scope as a build target, so its output is pinned here
as data and the GPU test vocodes it:

* 32 random ASCII texts of 10-60 characters (python ``random.Random(0)``), turned
  into linguistic features by the reference ``FrontEnd.batch_forward``
  (models/frontend.py:211-265, pads to the longest with PAD_ID 0);
* the reference ``SAMBERTAcousticModel`` (models/acoustic_model.py:24), random
  init after ``torch.manual_seed(0)``, ``inference`` (:267-297) -> mel_pred
  [32, Tfrm, 80] in the acoustic layout, plus ``predictions['dur']``: the
  per-utterance frame count is ``dur[b].sum()`` (LengthRegulator,
  models/variance_adaptor.py:223-264; every phoneme incl. padding gets >= 1
  frame, :746-748);
* the reference ``HiFiGANGenerator`` (models/hifigan.py) with the PRNG V1 weights
  of ``oracle.config.make_state_dict(V1, seed=C5_SEED)`` run on each utterance
  ALONE (``mel_pred[b, :len_b].T``): the glue contract ``mel_pred.transpose(1,2)
  -> HiFiGAN(mel)`` of .kiro/specs/tts-sam-bert-hifigan/design.md:905-906.

Stored (tests/golden/c5_sambert_b32.npz): ``mel_pred`` [32, T, 80] f32,
``lengths`` [32] i32, ``wav_{b}`` for the utterances in ``FULL_WAV`` (full
tensors), and in golden_c5.json the sha256 / L2 / max|.| of every utterance's wav.

Run in the build container only (needs /root/reference, read-only):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_c5_golden.py
"""
from __future__ import annotations

import contextlib
import hashlib
import io
import json
import os
import random
import string
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
REF = "/root/reference"

from oracle import config as C  # noqa: E402

N_UTT = 32
C5_SEED = 55
FULL_WAV = [0, 7, 13, 31]  # utterances whose whole wav is committed


def texts(n=N_UTT, seed=0):
    rng = random.Random(seed)
    alphabet = string.ascii_letters + string.digits + "     ,.!?"
    return ["".join(rng.choice(alphabet) for _ in range(rng.randint(10, 60))) for _ in range(n)]


def stats(a):
    a = np.ascontiguousarray(a, dtype=np.float32)
    return {"shape": list(a.shape), "sha256": hashlib.sha256(a.tobytes()).hexdigest(),
            "l2": float(np.sqrt((a.astype(np.float64) ** 2).sum())),
            "maxabs": float(np.abs(a).max())}


def main():
    sys.path.insert(0, REF)
    os.environ.setdefault("PYTHONDONTWRITEBYTECODE", "1")
    os.environ["DEBUG_SHAPES"] = "0"
    torch.set_num_threads(8)
    sink = io.StringIO()  # the acoustic stack prints unconditionally
    with contextlib.redirect_stdout(sink):
        from models.frontend import FrontEnd
        from models.acoustic_model import SAMBERTAcousticModel
        from models.hifigan import HiFiGANGenerator
        torch.manual_seed(0)
        fe = FrontEnd()
        am = SAMBERTAcousticModel().eval()
        txt = texts()
        feats = fe.batch_forward(txt)
        mel_pred, preds = am.inference(feats.ph_ids, feats.tone_ids, feats.boundary_ids)
    mel_pred = mel_pred.detach().float().contiguous()
    lengths = preds["dur"].sum(dim=1).to(torch.int32)
    assert int(lengths.max()) == mel_pred.shape[1], (lengths, mel_pred.shape)

    cfg = C.V1
    sd = C.make_state_dict(cfg, seed=C5_SEED)
    gen = HiFiGANGenerator(**cfg.kwargs()).eval()
    gen.load_state_dict({k: torch.from_numpy(v.copy()) for k, v in sd.items()}, strict=True)
    arrays = {"mel_pred": mel_pred.numpy(), "lengths": lengths.numpy()}
    wav_stats = {}
    with torch.no_grad():
        for b in range(N_UTT):
            n = int(lengths[b])
            wav = gen(mel_pred[b:b + 1, :n].transpose(1, 2).contiguous())[0, 0].numpy()
            wav_stats[str(b)] = stats(wav)
            if b in FULL_WAV:
                arrays[f"wav_{b}"] = wav
    np.savez(os.path.join(HERE, "c5_sambert_b32.npz"), **arrays)
    meta = {
        "generator": "tests/golden/make_c5_golden.py",
        "reference": "models/frontend.py, models/acoustic_model.py, models/hifigan.py "
                     "(terrense/TTS-sambert_hifiGAN), imported read-only",
        "torch": torch.__version__,
        "texts": txt,
        "acoustic_seed": 0,
        "vocoder_preset": "v1",
        "vocoder_seed": C5_SEED,
        "mel_pred_shape": list(mel_pred.shape),
        "mel_pred_stats": {"mean": float(mel_pred.mean()), "std": float(mel_pred.std())},
        "lengths": [int(x) for x in lengths],
        "full_wav": FULL_WAV,
        "wav": wav_stats,
    }
    with open(os.path.join(HERE, "golden_c5.json"), "w") as f:
        json.dump(meta, f, indent=1)
    print("mel_pred", tuple(mel_pred.shape), "lengths", meta["lengths"])


if __name__ == "__main__":
    main()
