"""Log-mel framing on the CPU: the library's filterbank (C++, float64) against
the torchaudio restatement (oracle/mel_torch.py), and the oracle's own shape
contract (reference tests/test_audio_processing.py:16-104).  Parity of this
row is UNPINNED: torchaudio is absent, no reference output exists."""
import ctypes

import numpy as np
import torch

from oracle import mel_torch as M


def _cfg(pkg):
    c = pkg._lib.HfgMelConfig()
    c.sample_rate, c.n_fft, c.hop_length, c.win_length, c.n_mels = 22050, 1024, 256, 1024, 80
    c.f_min, c.f_max, c.mel_scale, c.norm, c.log_eps, c.log_base = 0.0, 8000.0, 0, 1, 1e-10, 10
    return c


def test_filterbank_matches_restatement(pkg):
    lib = pkg.load_library()
    for scale, norm in [(0, 1), (1, 0), (1, 1), (0, 0)]:
        c = _cfg(pkg)
        c.mel_scale, c.norm = scale, norm
        fb = np.zeros((513, 80), np.float32)
        assert lib.hfg_mel_filterbank(ctypes.byref(c),
                                      fb.ctypes.data_as(ctypes.POINTER(ctypes.c_float))) == 0
        ref = M.melscale_fbanks(513, 0.0, 8000.0, 80, 22050, "slaney" if norm else None,
                                "slaney" if scale == 0 else "htk").numpy()
        # torchaudio builds it in float32 (cancellation in f_pts - freqs); ours in float64
        assert np.abs(fb - ref).max() <= 2e-5 * np.abs(ref).max()


def test_mel_handle_host_only(pkg):
    lib = pkg.load_library()
    h = ctypes.c_void_p()
    c = _cfg(pkg)
    assert lib.hfg_mel_create(ctypes.byref(c), -1, ctypes.byref(h)) == 0
    assert lib.hfg_mel_frames(h, 22050) == 22050 // 256 + 1
    assert lib.hfg_mel_workspace_bytes(h, 2, 22050) == 4 * 2 * 87 * 513
    assert lib.hfg_mel_forward(h, None, 1, 22050, None, None, 0, None) == -22
    lib.hfg_mel_destroy(h)
    c.win_length = 2048
    assert lib.hfg_mel_create(ctypes.byref(c), -1, ctypes.byref(h)) == -22


def test_oracle_shape_contract_and_tone():
    sr = 22050
    t = torch.arange(sr) / sr
    wav = 0.5 * torch.sin(2 * np.pi * 440.0 * t)
    mel = M.log_mel(wav)
    assert mel.dim() == 2 and mel.shape == (80, sr // 256 + 1)
    assert mel.max() <= 10
    # energy peaks in the mel band containing 440 Hz
    fb = M.melscale_fbanks(513, 0.0, 8000.0, 80, sr, "slaney", "slaney")
    band = int(torch.argmax(fb[round(440 / (sr / 1024))]))
    assert abs(int(torch.argmax(mel[:, 40])) - band) <= 1
