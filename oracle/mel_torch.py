"""CPU restatement of the reference's log-mel framing.

TEST INFRASTRUCTURE ONLY (see ``oracle/__init__.py``).

Reference: ``data/audio_processing.py:31-139`` (``extract_mel``) builds
``torchaudio.transforms.MelSpectrogram(sample_rate=22050, n_fft=1024,
hop_length=256, win_length=1024, n_mels=80, f_min=0, f_max=8000,
mel_scale="slaney", norm="slaney", power=2.0)`` (:99-110) and takes
``log10(mel + 1e-10)`` (:123-127).  torchaudio (pinned ``>=2.0.0`` in
requirements.txt) is NOT installed in this image, so the reference cannot run
here: this module restates torchaudio's published algorithm with torch ops in
the same dtype (float32) —

* ``Spectrogram``: ``torch.stft(center=True, pad_mode="reflect",
  window=hann_window(win_length) (periodic), normalized=False, onesided=True)``,
  ``.abs().pow(2)``;
* ``MelScale``: ``melscale_fbanks`` (slaney/htk ``_hz_to_mel``/``_mel_to_hz``,
  ``_create_triangular_filterbank``, slaney area norm ``2/(f[m+2]-f[m])``),
  ``(spec^T @ fb)^T``.

PARITY UNPINNED: no reference output of this path exists (torchaudio absent;
the reference's own tests check only shapes, tests/test_audio_processing.py:16-104).
"""
from __future__ import annotations

import math

import torch

CONFIG = dict(sample_rate=22050, n_fft=1024, hop_length=256, win_length=1024, n_mels=80,
              f_min=0.0, f_max=8000.0, mel_scale="slaney", norm="slaney", eps=1e-10)


def _hz_to_mel(freq: float, mel_scale: str) -> float:
    if mel_scale == "htk":
        return 2595.0 * math.log10(1.0 + freq / 700.0)
    f_min, f_sp = 0.0, 200.0 / 3
    mels = (freq - f_min) / f_sp
    min_log_hz = 1000.0
    min_log_mel = (min_log_hz - f_min) / f_sp
    logstep = math.log(6.4) / 27.0
    if freq >= min_log_hz:
        mels = min_log_mel + math.log(freq / min_log_hz) / logstep
    return mels


def _mel_to_hz(mels: torch.Tensor, mel_scale: str) -> torch.Tensor:
    if mel_scale == "htk":
        return 700.0 * (10.0 ** (mels / 2595.0) - 1.0)
    f_min, f_sp = 0.0, 200.0 / 3
    freqs = f_min + f_sp * mels
    min_log_hz = 1000.0
    min_log_mel = (min_log_hz - f_min) / f_sp
    logstep = math.log(6.4) / 27.0
    log_t = mels >= min_log_mel
    freqs[log_t] = min_log_hz * torch.exp(logstep * (mels[log_t] - min_log_mel))
    return freqs


def melscale_fbanks(n_freqs, f_min, f_max, n_mels, sample_rate, norm, mel_scale):
    all_freqs = torch.linspace(0, sample_rate // 2, n_freqs)
    m_min = _hz_to_mel(f_min, mel_scale)
    m_max = _hz_to_mel(f_max, mel_scale)
    m_pts = torch.linspace(m_min, m_max, n_mels + 2)
    f_pts = _mel_to_hz(m_pts, mel_scale)
    f_diff = f_pts[1:] - f_pts[:-1]
    slopes = f_pts.unsqueeze(0) - all_freqs.unsqueeze(1)
    zero = torch.zeros(1)
    down_slopes = (-1.0 * slopes[:, :-2]) / f_diff[:-1]
    up_slopes = slopes[:, 2:] / f_diff[1:]
    fb = torch.max(zero, torch.min(down_slopes, up_slopes))
    if norm == "slaney":
        enorm = 2.0 / (f_pts[2:n_mels + 2] - f_pts[:n_mels])
        fb *= enorm.unsqueeze(0)
    return fb  # [n_freqs, n_mels]


@torch.no_grad()
def log_mel(wav: torch.Tensor, cfg=CONFIG) -> torch.Tensor:
    """wav [B, N] or [N] float32 → log10 mel [B, n_mels, N // hop + 1] (or [n_mels, T])."""
    squeeze = wav.dim() == 1
    if squeeze:
        wav = wav[None]
    window = torch.hann_window(cfg["win_length"])
    spec = torch.stft(wav, cfg["n_fft"], hop_length=cfg["hop_length"],
                      win_length=cfg["win_length"], window=window, center=True,
                      pad_mode="reflect", normalized=False, onesided=True,
                      return_complex=True).abs().pow(2.0)
    fb = melscale_fbanks(cfg["n_fft"] // 2 + 1, cfg["f_min"], cfg["f_max"], cfg["n_mels"],
                         cfg["sample_rate"], cfg["norm"], cfg["mel_scale"])
    mel = torch.matmul(spec.transpose(-1, -2), fb).transpose(-1, -2)
    out = torch.log10(mel + cfg["eps"])
    return out[0] if squeeze else out


@torch.no_grad()
def log_mel64(wav: torch.Tensor, cfg=CONFIG, log_base=10.0) -> torch.Tensor:
    """The same log-mel with the spectrum in float64 (numpy rfft): the window product in
    float32 as torch.stft forms it, then FFT, power, mel projection (torchaudio's float32
    filterbank) and log in float64.  The fp32 torch.stft above carries an absolute error of
    ~1e-7 of the frame energy per bin, i.e. up to ~1e-2 in log10 on bins 60 dB under the
    peak; this restatement has none, so it pins quiet bands (the on-device FFT computes in
    float64 too).  Returns float64."""
    import numpy as np
    squeeze = wav.dim() == 1
    if squeeze:
        wav = wav[None]
    n_fft, hop, win = cfg["n_fft"], cfg["hop_length"], cfg["win_length"]
    window = torch.hann_window(win)
    w = torch.zeros(n_fft)
    left = (n_fft - win) // 2
    w[left:left + win] = window
    x = torch.nn.functional.pad(wav[:, None], (n_fft // 2, n_fft // 2), mode="reflect")[:, 0]
    n_frames = wav.shape[-1] // hop + 1
    idx = torch.arange(n_frames)[:, None] * hop + torch.arange(n_fft)[None]
    frames = (x[:, idx] * w).numpy().astype(np.float64)  # fp32 product, as torch.stft
    spec = np.abs(np.fft.rfft(frames, axis=-1)) ** 2     # [B, frames, bins]
    fb = melscale_fbanks(n_fft // 2 + 1, cfg["f_min"], cfg["f_max"], cfg["n_mels"],
                         cfg["sample_rate"], cfg["norm"], cfg["mel_scale"]).numpy().astype(np.float64)
    mel = np.einsum("bfk,km->bmf", spec, fb) + cfg["eps"]
    out = np.log(mel) / np.log(float(log_base)) if log_base != 10.0 else np.log10(mel)
    out = torch.from_numpy(out)
    return out[0] if squeeze else out
