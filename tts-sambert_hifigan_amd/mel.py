"""On-device log-mel framing, the vocoder's input.

Mirrors ``data/audio_processing.py``:

* :func:`extract_mel` (:31-139) — same signature, shape contract (``[time]`` or
  ``[channels, time]`` → ``[n_mels, time // hop + 1]``), resampling when
  ``sample_rate`` differs from the config's (:81-88), mono by channel mean (:93-94),
  ``log(mel + 1e-10)`` in base 10, e or a custom base (:121-133), and the
  ``debug.print_shapes`` lines (:58-59, 77-78, 89-90, 95-96, 118-119, 135-137).
* :func:`extract_mel_from_file` (:142-164), :func:`save_mel` / :func:`load_mel`
  (:167-200), :func:`load_config` (:16-28).

The arithmetic runs in the HIP kernels of ``libhifigan_hip.so``: one launch of an
FFT with a float64 spectrum + mel projection + log (:class:`MelSpectrogram`, the batched
``[B, N] → [B, n_mels, N // hop + 1]`` form that feeds ``HiFiGANGenerator``), and the
polyphase sinc resampler (:class:`Resample`, torchaudio ``Resample`` defaults).
There is no CPU fallback: a CPU waveform raises.
"""
from __future__ import annotations

import ctypes
import os
import struct
from pathlib import Path
from typing import Optional, Tuple, Union

import numpy as np
import torch

from . import _lib


def _check_mel(lib, rc):
    if rc != 0:
        raise _lib.HfgError(rc, lib.hfg_mel_last_error().decode())


def _log_base_code(log_base):
    """audio_processing.py:125-133: 10 / "10" → log10, "e" / math.e → ln, else custom."""
    if log_base == 10.0 or log_base == "10":
        return 10, 10.0
    if log_base == "e" or log_base == 2.718281828459045:
        return 0, 0.0
    return 1, float(log_base)


# torchaudio.functional.melscale_fbanks / _hz_to_mel / _mel_to_hz, evaluated with the same
# float32 torch ops (the reference's MelSpectrogram builds its filterbank this way,
# audio_processing.py:99-110), so the device tables are bitwise the reference's
def _hz_to_mel(freq: float, mel_scale: str) -> float:
    import math
    if mel_scale == "htk":
        return 2595.0 * math.log10(1.0 + freq / 700.0)
    f_sp, min_log_hz = 200.0 / 3, 1000.0
    mels = freq / f_sp
    if freq >= min_log_hz:
        mels = min_log_hz / f_sp + math.log(freq / min_log_hz) / (math.log(6.4) / 27.0)
    return mels


def _mel_to_hz(mels: torch.Tensor, mel_scale: str) -> torch.Tensor:
    import math
    if mel_scale == "htk":
        return 700.0 * (10.0 ** (mels / 2595.0) - 1.0)
    f_sp, min_log_hz = 200.0 / 3, 1000.0
    freqs = f_sp * mels
    min_log_mel = min_log_hz / f_sp
    logstep = math.log(6.4) / 27.0
    log_t = mels >= min_log_mel
    freqs[log_t] = min_log_hz * torch.exp(logstep * (mels[log_t] - min_log_mel))
    return freqs


def melscale_fbanks(n_freqs: int, f_min: float, f_max: float, n_mels: int, sample_rate: int,
                    norm: Optional[str], mel_scale: str) -> torch.Tensor:
    """[n_freqs, n_mels] float32 triangular filterbank (torchaudio's algorithm)."""
    all_freqs = torch.linspace(0, sample_rate // 2, n_freqs)
    m_pts = torch.linspace(_hz_to_mel(f_min, mel_scale), _hz_to_mel(f_max, mel_scale), n_mels + 2)
    f_pts = _mel_to_hz(m_pts, mel_scale)
    f_diff = f_pts[1:] - f_pts[:-1]
    slopes = f_pts.unsqueeze(0) - all_freqs.unsqueeze(1)
    down = (-1.0 * slopes[:, :-2]) / f_diff[:-1]
    up = slopes[:, 2:] / f_diff[1:]
    fb = torch.max(torch.zeros(1), torch.min(down, up))
    if norm == "slaney":
        fb *= (2.0 / (f_pts[2:n_mels + 2] - f_pts[:n_mels])).unsqueeze(0)
    return fb


def stft_window(n_fft: int, win_length: int) -> torch.Tensor:
    """torch.stft's effective window: torch.hann_window(win_length) (periodic, float32)
    zero-padded to n_fft, centred."""
    w = torch.zeros(n_fft)
    left = (n_fft - win_length) // 2
    w[left:left + win_length] = torch.hann_window(win_length)
    return w


class MelSpectrogram:
    """torchaudio.transforms.MelSpectrogram(power=2) + log on the HIP device."""

    def __init__(self, sample_rate: int = 22050, n_fft: int = 1024, hop_length: int = 256,
                 win_length: int = 1024, n_mels: int = 80, f_min: float = 0.0,
                 f_max: float = 8000.0, mel_scale: str = "slaney", norm: Optional[str] = "slaney",
                 log_eps: float = 1e-10, log_base=10.0, device=None):
        self.lib = _lib.load_library()
        c = _lib.HfgMelConfig()
        c.sample_rate, c.n_fft, c.hop_length, c.win_length, c.n_mels = (
            sample_rate, n_fft, hop_length, win_length, n_mels)
        c.f_min, c.f_max = f_min, f_max
        c.mel_scale = {"slaney": 0, "htk": 1}[mel_scale]
        c.norm = 1 if norm == "slaney" else 0
        c.log_eps = log_eps
        c.log_base, c.log_base_value = _log_base_code(log_base)
        self.cfg = c
        self.hop = hop_length
        self.n_mels = n_mels
        self.sample_rate = sample_rate
        if device is None:
            device = torch.device("cuda", torch.cuda.current_device())
        self.device = torch.device(device)
        h = ctypes.c_void_p()
        _check_mel(self.lib, self.lib.hfg_mel_create(ctypes.byref(c), self.device.index or 0,
                                                     ctypes.byref(h)))
        self.ptr = h
        # the reference's float32 window and filterbank (bitwise torch.stft / torchaudio)
        self._window = stft_window(n_fft, win_length).contiguous()
        self._fb = melscale_fbanks(n_fft // 2 + 1, float(f_min), float(f_max), n_mels,
                                   sample_rate, norm, mel_scale).contiguous()
        fp = ctypes.POINTER(ctypes.c_float)
        if not hasattr(self.lib, "hfg_mel_set_tables"):
            # only an A/B against an older library (HFG_ALLOW_OLD_LIB=1) gets here: its
            # device tables are double-evaluated, not torchaudio's float32 ones
            import warnings
            warnings.warn("libhifigan_hip.so lacks hfg_mel_set_tables: mel tables are "
                          "double-evaluated, not the reference's float32 window / filterbank")
            return
        _check_mel(self.lib, self.lib.hfg_mel_set_tables(
            self.ptr, ctypes.cast(self._window.data_ptr(), fp), ctypes.cast(self._fb.data_ptr(), fp)))

    def __del__(self):
        try:
            if getattr(self, "ptr", None):
                self.lib.hfg_mel_destroy(self.ptr)
                self.ptr = None
        except Exception:
            pass

    def filterbank(self) -> torch.Tensor:
        """The [n_fft/2+1, n_mels] filterbank the device uses (torchaudio's, float32)."""
        return self._fb.clone()

    def window(self) -> torch.Tensor:
        """The [n_fft] window the device uses (torch.hann_window(win_length), centred)."""
        return self._window.clone()

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
        _check_mel(self.lib, self.lib.hfg_mel_forward(
            self.ptr, ctypes.c_void_p(wav.data_ptr()), B, N, ctypes.c_void_p(mel.data_ptr()),
            ctypes.c_void_p(ws.data_ptr()), ws_bytes,
            ctypes.c_void_p(torch.cuda.current_stream(wav.device).cuda_stream)))
        return mel


class Resample:
    """torchaudio.transforms.Resample(orig_freq, new_freq) with its defaults
    (resampling_method="sinc_interp_hann", lowpass_filter_width=6, rolloff=0.99) on the
    HIP device: ``[..., time]`` → ``[..., ceil(time * new / orig)]``.  The kernel table
    is torchaudio's ``_get_sinc_resample_kernel`` (float64, stored fp32), built by
    ``hfg_resample_kernel``; the polyphase convolution runs in ``resample_sinc``."""

    def __init__(self, orig_freq: int = 16000, new_freq: int = 16000,
                 resampling_method: str = "sinc_interp_hann", lowpass_filter_width: int = 6,
                 rolloff: float = 0.99, beta: Optional[float] = None, *, device=None):
        if resampling_method != "sinc_interp_hann":
            raise NotImplementedError("only sinc_interp_hann (torchaudio's default, the one "
                                      "audio_processing.py:84-87 uses) is implemented")
        self.lib = _lib.load_library()
        self.orig_freq, self.new_freq = int(orig_freq), int(new_freq)
        self.lowpass_filter_width, self.rolloff = int(lowpass_filter_width), float(rolloff)
        if device is None:
            device = torch.device("cuda", torch.cuda.current_device())
        self.device = torch.device(device)
        h = ctypes.c_void_p()
        _check_mel(self.lib, self.lib.hfg_resample_create(
            self.orig_freq, self.new_freq, self.lowpass_filter_width, self.rolloff,
            self.device.index or 0, ctypes.byref(h)))
        self.ptr = h

    def __del__(self):
        try:
            if getattr(self, "ptr", None):
                self.lib.hfg_resample_destroy(self.ptr)
                self.ptr = None
        except Exception:
            pass

    def kernel(self) -> Tuple[torch.Tensor, int]:
        """(kernel [new/g, 2*width + orig/g], width) — torchaudio's (kernel, width)."""
        w, n, k = ctypes.c_int32(), ctypes.c_int32(), ctypes.c_int32()
        _check_mel(self.lib, self.lib.hfg_resample_kernel(
            self.orig_freq, self.new_freq, self.lowpass_filter_width, self.rolloff, None,
            ctypes.byref(w), ctypes.byref(n), ctypes.byref(k)))
        out = torch.zeros(n.value, k.value)
        _check_mel(self.lib, self.lib.hfg_resample_kernel(
            self.orig_freq, self.new_freq, self.lowpass_filter_width, self.rolloff,
            ctypes.cast(out.data_ptr(), ctypes.POINTER(ctypes.c_float)), None, None, None))
        return out, w.value

    def out_len(self, n: int) -> int:
        return int(self.lib.hfg_resample_out_len(self.ptr, int(n)))

    def __call__(self, waveform: torch.Tensor) -> torch.Tensor:
        if not waveform.is_cuda:
            raise RuntimeError("Resample (MI355X) needs a HIP tensor; no CPU fallback")
        if self.orig_freq == self.new_freq:
            return waveform
        shape = waveform.shape
        x = waveform.detach().to(torch.float32).reshape(-1, shape[-1]).contiguous()
        B, n = x.shape
        y = torch.empty(B, self.out_len(n), device=x.device, dtype=torch.float32)
        _check_mel(self.lib, self.lib.hfg_resample_forward(
            self.ptr, ctypes.c_void_p(x.data_ptr()), B, n, ctypes.c_void_p(y.data_ptr()),
            ctypes.c_void_p(torch.cuda.current_stream(x.device).cuda_stream)))
        return y.reshape(shape[:-1] + (y.shape[-1],))


def load_config(config_path: str = "configs/config.yaml") -> dict:
    """data/audio_processing.py:16-28"""
    import yaml
    with open(config_path, "r", encoding="utf-8") as f:
        return yaml.safe_load(f)


_EXTRACTORS = {}
_RESAMPLERS = {}


def extract_mel(waveform: torch.Tensor, sample_rate: Optional[int] = None,
                config: Optional[dict] = None, config_path: str = "configs/config.yaml"
                ) -> torch.Tensor:
    """data/audio_processing.py:31-139 on the HIP device: [time] or [channels, time]
    → log-mel [n_mels, time // hop + 1] (after resampling to the config's rate)."""
    if config is None:
        config = load_config(config_path)
    a = config["audio"]
    print_shapes = config.get("debug", {}).get("print_shapes", False)
    target_sr = a["sample_rate"]
    log_base = a.get("log_base", 10.0)
    if waveform.dim() == 1:
        waveform = waveform.unsqueeze(0)
    if print_shapes:
        print(f"[extract_mel] Input waveform shape: {waveform.shape}")
    if sample_rate is not None and sample_rate != target_sr:
        if print_shapes:
            print(f"[extract_mel] Resampling from {sample_rate}Hz to {target_sr}Hz")
        key = (int(sample_rate), int(target_sr), waveform.device)
        rs = _RESAMPLERS.get(key)
        if rs is None:
            rs = _RESAMPLERS[key] = Resample(sample_rate, target_sr, device=waveform.device)
        waveform = rs(waveform)
        if print_shapes:
            print(f"[extract_mel] Resampled waveform shape: {waveform.shape}")
    if waveform.size(0) > 1:
        waveform = torch.mean(waveform, dim=0, keepdim=True)
        if print_shapes:
            print(f"[extract_mel] Converted to mono, shape: {waveform.shape}")
    key = (target_sr, a["n_fft"], a["hop_length"], a["win_length"], a["n_mels"],
           a["fmin"], a["fmax"], a.get("mel_scale", "slaney"), a.get("norm", "slaney"),
           str(log_base), waveform.device)
    ex = _EXTRACTORS.get(key)
    if ex is None:
        ex = MelSpectrogram(target_sr, a["n_fft"], a["hop_length"], a["win_length"],
                            a["n_mels"], float(a["fmin"]), float(a["fmax"]),
                            a.get("mel_scale", "slaney"), a.get("norm", "slaney"),
                            1e-10, log_base, device=waveform.device)
        _EXTRACTORS[key] = ex
    log_mel = ex(waveform)[0]
    if print_shapes:
        # the reference prints the shape before the log; the fused kernel has the same shape
        print(f"[extract_mel] Mel spectrogram shape (before log): {log_mel.shape}")
        print(f"[extract_mel] Log-mel spectrogram shape: {log_mel.shape}")
        print(f"[extract_mel] Log-mel range: [{log_mel.min().item():.2f}, "
              f"{log_mel.max().item():.2f}]")
    return log_mel


def read_wav(path: Union[str, Path]) -> Tuple[torch.Tensor, int]:
    """(waveform [channels, time] float32, sample_rate) from a RIFF/WAVE file, normalised
    as torchaudio.load does: integer PCM divided by 2^(bits-1) (8-bit: (v - 128) / 128),
    IEEE float as stored.  Host-side file parsing (torchaudio is absent in this image)."""
    data = Path(path).read_bytes()
    if len(data) < 12 or data[:4] != b"RIFF" or data[8:12] != b"WAVE":
        raise RuntimeError(f"{path}: not a RIFF/WAVE file")
    pos, fmt, pcm = 12, None, None
    while pos + 8 <= len(data):
        cid, size = data[pos:pos + 4], struct.unpack("<I", data[pos + 4:pos + 8])[0]
        body = data[pos + 8:pos + 8 + size]
        if cid == b"fmt ":
            tag, ch, sr, _, _, bits = struct.unpack("<HHIIHH", body[:16])
            if tag == 0xFFFE and len(body) >= 26:  # WAVE_FORMAT_EXTENSIBLE: subformat tag
                tag = struct.unpack("<H", body[24:26])[0]
            fmt = (tag, ch, sr, bits)
        elif cid == b"data":
            pcm = body
        pos += 8 + size + (size & 1)
    if fmt is None or pcm is None:
        raise RuntimeError(f"{path}: missing fmt or data chunk")
    tag, ch, sr, bits = fmt
    width = bits // 8
    n = len(pcm) // (width * ch)
    pcm = pcm[:n * width * ch]
    if tag == 3 and bits == 32:
        x = np.frombuffer(pcm, "<f4").astype(np.float32)
    elif tag == 3 and bits == 64:
        x = np.frombuffer(pcm, "<f8").astype(np.float32)
    elif tag == 1 and bits == 8:
        x = (np.frombuffer(pcm, np.uint8).astype(np.float32) - 128.0) / 128.0
    elif tag == 1 and bits == 16:
        x = np.frombuffer(pcm, "<i2").astype(np.float32) / 32768.0
    elif tag == 1 and bits == 24:
        b = np.frombuffer(pcm, np.uint8).reshape(-1, 3).astype(np.int32)
        v = b[:, 0] | (b[:, 1] << 8) | (b[:, 2] << 16)
        v = np.where(v >= 1 << 23, v - (1 << 24), v)
        x = v.astype(np.float32) / float(1 << 23)
    elif tag == 1 and bits == 32:
        x = (np.frombuffer(pcm, "<i4").astype(np.float64) / 2147483648.0).astype(np.float32)
    else:
        raise RuntimeError(f"{path}: unsupported WAV encoding (format {tag}, {bits} bits)")
    return torch.from_numpy(x.reshape(n, ch).T.copy()), sr


def extract_mel_from_file(audio_path: Union[str, Path], config: Optional[dict] = None,
                          config_path: str = "configs/config.yaml", device=None
                          ) -> Tuple[torch.Tensor, int]:
    """data/audio_processing.py:142-164: (log-mel [n_mels, T], sample_rate).  The file is
    parsed on the host (read_wav) and the waveform moved to the HIP device."""
    waveform, sample_rate = read_wav(audio_path)
    if device is None:
        device = torch.device("cuda", torch.cuda.current_device())
    log_mel = extract_mel(waveform.to(device), sample_rate, config, config_path)
    return log_mel, sample_rate


def save_mel(mel: torch.Tensor, output_path: Union[str, Path]) -> None:
    """data/audio_processing.py:167-184 (numpy .npy)."""
    output_path = Path(output_path)
    output_path.parent.mkdir(parents=True, exist_ok=True)
    np.save(output_path, mel.cpu().numpy())


def load_mel(mel_path: Union[str, Path]) -> torch.Tensor:
    """data/audio_processing.py:187-200."""
    return torch.from_numpy(np.load(mel_path)).float()
