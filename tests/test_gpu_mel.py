"""On-device log-mel framing against the torchaudio
restatement (oracle/mel_torch.py).  PARITY UNPINNED: torchaudio, which the
reference calls, is absent from this image, so the oracle is a restatement of
its published algorithm (same torch.stft call, same float32 filterbank code).
Tolerance: |log10 mel - oracle| <= 2e-3 where the oracle mel >= 1e-6 x its max
(fp32 DFT by direct summation vs pocketfft), and <= 5e-2 everywhere else."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    return torch.device("cuda:0")


def _signals(n):
    g = torch.Generator().manual_seed(0)
    t = torch.arange(n) / 22050.0
    tone = 0.3 * torch.sin(2 * np.pi * 220.0 * t) + 0.2 * torch.sin(2 * np.pi * 3100.0 * t)
    noise = 0.1 * torch.randn(n, generator=g)
    chirp = 0.5 * torch.sin(2 * np.pi * (100 + 2000 * t) * t)
    return torch.stack([tone + noise, chirp])


def _check(got, ref):
    big = ref >= np.log10(1e-6) + ref.max()
    err = (got - ref).abs()
    assert err[big].max().item() <= 2e-3, err[big].max().item()
    assert err.max().item() <= 5e-2, err.max().item()


@pytest.mark.parametrize("n", [22050 + 77, 513, 4096])
def test_mel_vs_restatement(pkg, dev, n):
    import importlib
    melmod = importlib.import_module("tts_sambert_hifigan_amd.mel")
    from oracle import mel_torch as M
    wav = _signals(n)
    ext = melmod.MelSpectrogram(device=dev)
    got = ext(wav.to(dev)).cpu()
    ref = M.log_mel(wav)
    assert got.shape == ref.shape == (2, 80, n // 256 + 1)
    _check(got, ref)


def test_extract_mel_contract(pkg, dev):
    """data/audio_processing.py:31-139 contract: [ch, time] -> mono -> [80, T]."""
    import importlib
    melmod = importlib.import_module("tts_sambert_hifigan_amd.mel")
    from oracle import mel_torch as M
    cfg = {"audio": {"sample_rate": 22050, "n_fft": 1024, "hop_length": 256, "win_length": 1024,
                     "n_mels": 80, "fmin": 0, "fmax": 8000, "mel_scale": "slaney",
                     "norm": "slaney", "log_base": 10.0}}
    stereo = _signals(30000)
    mel = melmod.extract_mel(stereo.to(dev), config=cfg)
    assert mel.dim() == 2 and mel.size(0) == 80 and mel.shape[1] == 30000 // 256 + 1
    assert mel.max() <= 10
    _check(mel.cpu(), M.log_mel(stereo.mean(0)))
    with pytest.raises(NotImplementedError):
        melmod.extract_mel(stereo.to(dev), sample_rate=16000, config=cfg)


def test_mel_feeds_vocoder(pkg, dev):
    """wav -> on-device mel -> vocoder, no host round trip; equals the vocoder on
    the oracle mel within the mel tolerance propagated (loose: 1e-3)."""
    import importlib
    melmod = importlib.import_module("tts_sambert_hifigan_amd.mel")
    from oracle import config as C, mel_torch as M
    gen = pkg.HiFiGANGenerator(**C.V1.kwargs()).eval()
    gen.load_state_dict({k: torch.from_numpy(v) for k, v in C.make_state_dict(C.V1, 2).items()})
    gen = gen.to(dev)
    wav = _signals(8192)
    mel_dev = melmod.MelSpectrogram(device=dev)(wav.to(dev))
    with torch.no_grad():
        out = gen(mel_dev)
        ref = gen(M.log_mel(wav).to(dev))
    torch.cuda.synchronize()
    assert out.shape == (2, 1, (8192 // 256 + 1) * 256)
    assert (out - ref).abs().max().item() < 1e-3
