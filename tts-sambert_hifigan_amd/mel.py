"""On-device log-mel framing, the vocoder's input.

Mirrors ``data/audio_processing.py``: :func:`extract_mel` has the reference's
signature and shape contract (``[time]`` or ``[channels, time]`` → ``[n_mels,
time // hop + 1]``, mono by channel mean, ``log10(mel + 1e-10)``), computed by
the HIP kernels of ``libhifigan_hip.so`` (windowed DFT on the fp32 matrix
cores + mel projection + log).  :class:`MelSpectrogram` is the batched form
``[B, N] → [B, n_mels, N // hop + 1]`` that feeds ``HiFiGANGenerator`` directly.
Resampling (``audio_processing.py:81-88``, torchaudio ``Resample``) is not part
of this path: a waveform at another rate raises.
"""
from __future__ import annotations

import ctypes
from typing import Optional

import torch

from . import _lib


class MelSpectrogram:
    """torchaudio.transforms.MelSpectrogram(power=2) + log on the HIP device."""

    def __init__(self, sample_rate: int = 22050, n_fft: int = 1024, hop_length: int = 256,
                 win_length: int = 1024, n_mels: int = 80, f_min: float = 0.0,
                 f_max: float = 8000.0, mel_scale: str = "slaney", norm: Optional[str] = "slaney",
                 log_eps: float = 1e-10, log_base: float = 10.0, device=None):
        self.lib = _lib.load_library()
        c = _lib.HfgMelConfig()
        c.sample_rate, c.n_fft, c.hop_length, c.win_length, c.n_mels = (
            sample_rate, n_fft, hop_length, win_length, n_mels)
        c.f_min, c.f_max = f_min, f_max
        c.mel_scale = {"slaney": 0, "htk": 1}[mel_scale]
        c.norm = 1 if norm == "slaney" else 0
        c.log_eps = log_eps
        if log_base in (10.0, "10"):
            c.log_base = 10
        elif log_base in ("e", 2.718281828459045):
            c.log_base = 0
        else:
            raise NotImplementedError("log_base must be 10 or e")
        self.cfg = c
        self.hop = hop_length
        self.n_mels = n_mels
        self.sample_rate = sample_rate
        if device is None:
            device = torch.device("cuda", torch.cuda.current_device())
        self.device = torch.device(device)
        h = ctypes.c_void_p()
        rc = self.lib.hfg_mel_create(ctypes.byref(c), self.device.index or 0, ctypes.byref(h))
        if rc != 0:
            raise _lib.HfgError(rc, self.lib.hfg_mel_last_error().decode())
        self.ptr = h

    def __del__(self):
        try:
            if getattr(self, "ptr", None):
                self.lib.hfg_mel_destroy(self.ptr)
                self.ptr = None
        except Exception:
            pass

    def filterbank(self) -> torch.Tensor:
        fb = torch.zeros(self.cfg.n_fft // 2 + 1, self.n_mels)
        self.lib.hfg_mel_filterbank(ctypes.byref(self.cfg),
                                    ctypes.cast(fb.data_ptr(), ctypes.POINTER(ctypes.c_float)))
        return fb

    def frames(self, n_samples: int) -> int:
        return n_samples // self.hop + 1

    def __call__(self, wav: torch.Tensor) -> torch.Tensor:
        """wav [B, N] float32 on the HIP device → log-mel [B, n_mels, N//hop + 1]."""
        if not wav.is_cuda:
            raise RuntimeError("MelSpectrogram (MI355X) needs a HIP tensor; no CPU fallback")
        if wav.dim() != 2:
            raise RuntimeError("expected wav [B, N]")
        wav = wav.detach().to(torch.float32).contiguous()
        B, N = wav.shape
        T = self.frames(N)
        mel = torch.empty(B, self.n_mels, T, device=wav.device, dtype=torch.float32)
        ws_bytes = int(self.lib.hfg_mel_workspace_bytes(self.ptr, B, N))
        ws = torch.empty(max(ws_bytes, 1), dtype=torch.uint8, device=wav.device)
        rc = self.lib.hfg_mel_forward(self.ptr, ctypes.c_void_p(wav.data_ptr()), B, N,
                                      ctypes.c_void_p(mel.data_ptr()),
                                      ctypes.c_void_p(ws.data_ptr()), ws_bytes,
                                      ctypes.c_void_p(torch.cuda.current_stream(wav.device).cuda_stream))
        if rc != 0:
            raise _lib.HfgError(rc, self.lib.hfg_mel_last_error().decode())
        return mel


_EXTRACTORS = {}


def extract_mel(waveform: torch.Tensor, sample_rate: Optional[int] = None,
                config: Optional[dict] = None, config_path: str = "configs/config.yaml"
                ) -> torch.Tensor:
    """data/audio_processing.py:31-139 on the HIP device: [time] or [channels, time]
    → log-mel [n_mels, time // hop + 1]."""
    if config is None:
        import yaml
        with open(config_path) as f:
            config = yaml.safe_load(f)
    a = config["audio"]
    if sample_rate is not None and sample_rate != a["sample_rate"]:
        raise NotImplementedError("resampling is not part of the MI355X mel path")
    if waveform.dim() == 1:
        waveform = waveform.unsqueeze(0)
    if waveform.size(0) > 1:
        waveform = torch.mean(waveform, dim=0, keepdim=True)
    key = (a["sample_rate"], a["n_fft"], a["hop_length"], a["win_length"], a["n_mels"],
           a["fmin"], a["fmax"], a.get("mel_scale", "slaney"), a.get("norm", "slaney"),
           a.get("log_base", 10.0), waveform.device)
    ex = _EXTRACTORS.get(key)
    if ex is None:
        ex = MelSpectrogram(a["sample_rate"], a["n_fft"], a["hop_length"], a["win_length"],
                            a["n_mels"], float(a["fmin"]), float(a["fmax"]),
                            a.get("mel_scale", "slaney"), a.get("norm", "slaney"),
                            1e-10, a.get("log_base", 10.0), device=waveform.device)
        _EXTRACTORS[key] = ex
    return ex(waveform)[0]
