"""CPU restatement of the reference's resampling step.

TEST INFRASTRUCTURE ONLY (see ``oracle/__init__.py``).

Reference: ``data/audio_processing.py:81-88`` calls
``torchaudio.transforms.Resample(orig_freq=sample_rate, new_freq=target_sr)`` with
torchaudio's defaults (``resampling_method="sinc_interp_hann"``,
``lowpass_filter_width=6``, ``rolloff=0.99``, kernel dtype float64 → float32).
torchaudio (``>=2.0.0``, requirements.txt:3) is absent from this image, so this module
restates its published algorithm (``torchaudio.functional.functional.
_get_sinc_resample_kernel`` / ``_apply_sinc_resample_kernel``) in numpy:

* ``g = gcd(orig, new)``; ``orig, new = orig // g, new // g``;
  ``base = min(orig, new) * rolloff``; ``width = ceil(lpw * orig / base)``;
* ``idx = arange(-width, width + orig) / orig`` (float64);
  ``t = (arange(0, -new, -1) / new)[:, None] + idx`` — the first term is a float32
  division there (an int64 tensor divided by an int), then promoted;
* ``t = clamp(t * base, -lpw, lpw)``; ``window = cos(t * pi / lpw / 2) ** 2``;
  ``t *= pi``; ``kernel = where(t == 0, 1, sin(t) / t) * (window * base / orig)``
  → float32;
* ``y = conv1d(pad(x, (width, width + orig)), kernel[:, None], stride=orig)``, phases
  interleaved, truncated to ``ceil(new * n / orig)``.

PARITY UNPINNED: no reference output of this path exists (torchaudio absent; the
reference's tests never resample).
"""
from __future__ import annotations

import math

import numpy as np


def sinc_kernel(orig_freq: int, new_freq: int, lowpass_filter_width: int = 6,
                rolloff: float = 0.99):
    """(kernel float32 [new/g, 2*width + orig/g], width)"""
    g = math.gcd(int(orig_freq), int(new_freq))
    orig, new = int(orig_freq) // g, int(new_freq) // g
    base = min(orig, new) * rolloff
    width = math.ceil(lowpass_filter_width * orig / base)
    idx = np.arange(-width, width + orig, dtype=np.float64) / orig
    off = (np.arange(0, -new, -1).astype(np.float32) / np.float32(new)).astype(np.float64)
    t = off[:, None] + idx[None, :]
    t = t * base
    t = np.clip(t, -lowpass_filter_width, lowpass_filter_width)
    window = np.cos(t * math.pi / lowpass_filter_width / 2) ** 2
    t = t * math.pi
    scale = base / orig
    with np.errstate(invalid="ignore", divide="ignore"):
        k = np.where(t == 0, 1.0, np.sin(t) / t)
    k = k * (window * scale)
    return k.astype(np.float32), width


def resample(x: np.ndarray, orig_freq: int, new_freq: int, lowpass_filter_width: int = 6,
             rolloff: float = 0.99) -> np.ndarray:
    """x [..., n] → [..., ceil(n * new / orig)], accumulated in float64."""
    if orig_freq == new_freq:
        return np.array(x, dtype=np.float32)
    g = math.gcd(int(orig_freq), int(new_freq))
    orig, new = int(orig_freq) // g, int(new_freq) // g
    kern, width = sinc_kernel(orig_freq, new_freq, lowpass_filter_width, rolloff)
    shape = x.shape
    x2 = np.asarray(x, np.float64).reshape(-1, shape[-1])
    n = x2.shape[1]
    xp = np.pad(x2, ((0, 0), (width, width + orig)))
    n_frames = (xp.shape[1] - kern.shape[1]) // orig + 1
    frames = np.lib.stride_tricks.sliding_window_view(xp, kern.shape[1], axis=1)[:, ::orig][:, :n_frames]
    y = np.einsum("bfk,jk->bfj", frames, kern.astype(np.float64)).reshape(x2.shape[0], -1)
    target = math.ceil(new * n / orig)
    return y[:, :target].reshape(shape[:-1] + (target,)).astype(np.float32)
