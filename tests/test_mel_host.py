"""Log-mel framing on the CPU: the library's filterbank (C++, float64) against
the torchaudio restatement (oracle/mel_torch.py), and the oracle's own shape
contract (reference tests/test_audio_processing.py:16-104).  Parity of this
row is UNPINNED: torchaudio is absent, no reference output exists."""
import ctypes
import math

import numpy as np
import pytest
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
    # n_fft 1024 (a power of two): the one-launch FFT path, spectra in LDS, a token
    # workspace (the DFT path's B x frames x bins buffer is not allocated)
    assert lib.hfg_mel_workspace_bytes(h, 2, 22050) == 256
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


def test_custom_log_base_validated(pkg):
    """audio_processing.py:131-133 custom base: log_base 1 + log_base_value; bad bases are
    refused at creation."""
    lib = pkg.load_library()
    h = ctypes.c_void_p()
    c = _cfg(pkg)
    c.log_base, c.log_base_value = 1, 2.0
    assert lib.hfg_mel_create(ctypes.byref(c), -1, ctypes.byref(h)) == 0
    lib.hfg_mel_destroy(h)
    for bad in (1.0, 0.0, -3.0):
        c.log_base_value = bad
        assert lib.hfg_mel_create(ctypes.byref(c), -1, ctypes.byref(h)) == -22
    c.log_base = 7
    assert lib.hfg_mel_create(ctypes.byref(c), -1, ctypes.byref(h)) == -22


@pytest.mark.parametrize("orig,new", [(16000, 22050), (44100, 22050), (48000, 22050),
                                      (8000, 22050), (22050, 16000), (24000, 22050)])
def test_resample_kernel_matches_restatement(pkg, orig, new):
    """hfg_resample_kernel (C++, float64) = torchaudio's _get_sinc_resample_kernel as
    restated in oracle/resample_np.py (parity unpinned: torchaudio absent)."""
    from oracle import resample_np as R
    lib = pkg.load_library()
    w, n, k = ctypes.c_int32(), ctypes.c_int32(), ctypes.c_int32()
    assert lib.hfg_resample_kernel(orig, new, 6, 0.99, None, ctypes.byref(w), ctypes.byref(n),
                                   ctypes.byref(k)) == 0
    ref, width = R.sinc_kernel(orig, new)
    assert (w.value, n.value, k.value) == (width, ref.shape[0], ref.shape[1])
    got = np.zeros(ref.shape, np.float32)
    assert lib.hfg_resample_kernel(orig, new, 6, 0.99,
                                   got.ctypes.data_as(ctypes.POINTER(ctypes.c_float)),
                                   None, None, None) == 0
    assert np.abs(got - ref).max() <= 1e-7
    # unit DC gain: each phase's taps sum to ~ new/orig... of the reduced rates x orig/new
    g = math.gcd(orig, new)
    assert np.allclose(ref.sum(1), 1.0, atol=2e-2), ref.sum(1)[:4]


def test_resample_handle_host_only(pkg):
    lib = pkg.load_library()
    h = ctypes.c_void_p()
    assert lib.hfg_resample_create(16000, 22050, 6, 0.99, -1, ctypes.byref(h)) == 0
    assert lib.hfg_resample_out_len(h, 16000) == 22050
    assert lib.hfg_resample_out_len(h, 1001) == math.ceil(441 * 1001 / 320)
    assert lib.hfg_resample_forward(h, None, 1, 100, None, None) == -22
    lib.hfg_resample_destroy(h)
    assert lib.hfg_resample_create(0, 22050, 6, 0.99, -1, ctypes.byref(h)) == -22
    assert lib.hfg_resample_create(16000, 22050, 6, 1.5, -1, ctypes.byref(h)) == -22


def test_oracle_resample_tone():
    """The restatement itself: a 440 Hz tone resampled 16 kHz -> 22.05 kHz is the same
    tone at the new rate (away from the zero-padded edges)."""
    from oracle import resample_np as R
    n = 16000
    x = np.sin(2 * np.pi * 440.0 * np.arange(n) / 16000.0).astype(np.float32)
    y = R.resample(x, 16000, 22050)
    assert y.shape == (math.ceil(22050 * n / 16000),)
    ref = np.sin(2 * np.pi * 440.0 * np.arange(y.shape[0]) / 22050.0)
    assert np.abs(y[200:-200] - ref[200:-200]).max() < 2e-3


def test_read_wav_pcm16_and_float(tmp_path):
    """extract_mel_from_file's host WAV parser: torchaudio.load's normalisation
    (int16 / 32768, float32 as stored), [channels, time]."""
    import importlib
    import struct
    import wave
    mel = importlib.import_module("tts_sambert_hifigan_amd.mel")
    rng = np.random.default_rng(0)
    pcm = rng.integers(-32768, 32767, size=(500, 2), dtype=np.int16)
    p16 = tmp_path / "a.wav"
    with wave.open(str(p16), "wb") as w:
        w.setnchannels(2)
        w.setsampwidth(2)
        w.setframerate(16000)
        w.writeframes(pcm.tobytes())
    x, sr = mel.read_wav(p16)
    assert sr == 16000 and tuple(x.shape) == (2, 500)
    assert np.array_equal(x.numpy(), (pcm.T / 32768.0).astype(np.float32))
    f = rng.standard_normal(300).astype(np.float32)
    data = f.tobytes()
    fmt = struct.pack("<HHIIHH", 3, 1, 22050, 22050 * 4, 4, 32)
    riff = (b"RIFF" + struct.pack("<I", 4 + 8 + len(fmt) + 8 + len(data)) + b"WAVE" +
            b"fmt " + struct.pack("<I", len(fmt)) + fmt + b"data" + struct.pack("<I", len(data)) +
            data)
    pf = tmp_path / "f.wav"
    pf.write_bytes(riff)
    y, sr2 = mel.read_wav(pf)
    assert sr2 == 22050 and np.array_equal(y.numpy()[0], f)


def test_save_load_mel_roundtrip(tmp_path):
    import importlib
    mel = importlib.import_module("tts_sambert_hifigan_amd.mel")
    m = torch.randn(80, 33)
    mel.save_mel(m, tmp_path / "sub" / "m.npy")
    assert torch.equal(mel.load_mel(tmp_path / "sub" / "m.npy"), m)


def test_product_tables_bitwise_torch(pkg):
    """The tables mel.MelSpectrogram hands the device (hfg_mel_set_tables) are bitwise the
    float32 ones the reference's torchaudio builds: torch.hann_window (centred in n_fft)
    and the melscale_fbanks restatement, for both scales and norms."""
    import importlib
    melmod = importlib.import_module("tts_sambert_hifigan_amd.mel")
    for scale in ("slaney", "htk"):
        for norm in ("slaney", None):
            a = melmod.melscale_fbanks(513, 0.0, 8000.0, 80, 22050, norm, scale)
            b = M.melscale_fbanks(513, 0.0, 8000.0, 80, 22050, norm, scale)
            assert torch.equal(a, b), (scale, norm)
    w = melmod.stft_window(1024, 800)
    assert torch.equal(w[112:912], torch.hann_window(800)) and not w[:112].any()
    assert not w[912:].any()


def test_mel_set_tables_host_handle(pkg):
    lib = pkg.load_library()
    h = ctypes.c_void_p()
    c = _cfg(pkg)
    assert lib.hfg_mel_create(ctypes.byref(c), -1, ctypes.byref(h)) == 0
    w = torch.hann_window(1024)
    fb = M.melscale_fbanks(513, 0.0, 8000.0, 80, 22050, "slaney", "slaney").contiguous()
    fp = ctypes.POINTER(ctypes.c_float)
    assert lib.hfg_mel_set_tables(h, ctypes.cast(w.data_ptr(), fp), ctypes.cast(fb.data_ptr(), fp)) == 0
    assert lib.hfg_mel_set_tables(h, None, None) == -22
    lib.hfg_mel_destroy(h)
