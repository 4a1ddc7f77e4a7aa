"""SURVEY.md §8(f) rows 2-3 on the GPU: acoustic-model glue ([B, T, 80] input,
ragged batches) and streaming vocoding, both against the one-shot Generator
(bitwise) and the CPU oracle (atol 1e-4)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
ATOL = 1e-4


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    return torch.device("cuda:0")


@pytest.fixture(scope="module", params=["fp32", "f16x3"])
def gen_sd(pkg, dev, request):
    from oracle import config as C
    sd = C.make_state_dict(C.V1, seed=4)
    gen = pkg.HiFiGANGenerator(**C.V1.kwargs(), precision=request.param).eval()
    gen.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()})
    return gen.to(dev), sd


def run(gen, mel, **kw):
    with torch.no_grad():
        out = gen(mel, **kw)
    torch.cuda.synchronize()
    return out


def test_btc_layout_equals_bct(gen_sd, dev):
    gen, _ = gen_sd
    mel = torch.randn(3, 80, 57, device=dev)
    a = run(gen, mel)
    b = run(gen, mel.transpose(1, 2).contiguous(), mel_layout="btc")
    assert torch.equal(a, b)


def test_ragged_batch_equals_per_utterance(pkg, gen_sd, dev):
    import importlib
    glue = importlib.import_module("tts_sambert_hifigan_amd.glue")
    from oracle import config as C, hifigan_torch as H
    gen, sd = gen_sd
    lens = [61, 40, 7, 1]
    T = max(lens)
    g = torch.Generator().manual_seed(3)
    mel_pred = torch.randn(len(lens), T, 80, generator=g)  # acoustic-model layout
    for b, n in enumerate(lens):
        mel_pred[b, n:] = 123.0  # garbage in the padding must not leak
    wavs = glue.vocode_acoustic(gen, mel_pred.to(dev), lens)
    full = run(gen, mel_pred.to(dev), lengths=lens, mel_layout="btc")
    for b, n in enumerate(lens):
        alone = run(gen, mel_pred[b:b + 1, :n].transpose(1, 2).contiguous().to(dev))
        assert wavs[b].shape[0] == n * 256
        assert torch.equal(wavs[b], alone[0, 0]), b
        assert torch.count_nonzero(full[b, 0, n * 256:]) == 0
        ref = H.generator_forward(H.to_torch_state(sd), C.V1, mel_pred[b:b + 1, :n].transpose(1, 2))
        assert (wavs[b].cpu() - ref[0, 0]).abs().max().item() < ATOL


def test_vocode_list(pkg, gen_sd, dev):
    import importlib
    glue = importlib.import_module("tts_sambert_hifigan_amd.glue")
    gen, _ = gen_sd
    mels = [torch.randn(80, n, device=dev) for n in (33, 5, 48)]
    wavs = glue.vocode_list(gen, mels)
    for m, w in zip(mels, wavs):
        assert torch.equal(w, run(gen, m[None])[0, 0])


def test_streaming_equals_one_shot(pkg, gen_sd, dev):
    import importlib
    glue = importlib.import_module("tts_sambert_hifigan_amd.glue")
    gen, _ = gen_sd
    assert gen.receptive_field_frames() == 15
    T = 230
    mel = torch.randn(80, T, device=dev)
    ref = run(gen, mel[None])[0, 0]
    sv = glue.StreamingVocoder(gen, chunk_frames=40)
    pieces, pos = [], 0
    rng = np.random.default_rng(0)
    while pos < T:
        n = int(rng.integers(1, 37))
        pieces.append(sv.push(mel[:, pos:pos + n]))
        pos += n
    pieces.append(sv.flush())
    out = torch.cat(pieces)
    torch.cuda.synchronize()
    assert out.shape == ref.shape
    assert torch.equal(out, ref)


@pytest.mark.parametrize("precision", ["fp32", "f16x3", "bf16x3", "bf16w"])
@pytest.mark.parametrize("preset", ["v1", "v2star", "nonexact"])
def test_ragged_sweep_equals_solo(pkg, dev, preset, precision):
    """Ragged batches of random lengths (1, odd, even; garbage in the padding) in both mel
    layouts, for every config family and precision: each item bitwise equal to the
    utterance run alone, zero past its length, and (fp32 / f16x3 / bf16x3) within 1e-4 of the
    oracle.  Covers every execution schedule a length mix selects (small-grid tile,
    concurrent ResBlocks + mrf_combine, thin stages, 2-stream split)."""
    from oracle import config as C, hifigan_torch as H
    cfg = C.PRESETS[preset]
    sd = C.make_state_dict(cfg, seed=41)
    gen = pkg.HiFiGANGenerator(**cfg.kwargs(), precision=precision).eval()
    gen.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()})
    gen = gen.to(dev)
    rng = np.random.default_rng({"v1": 1, "v2star": 2, "nonexact": 3}[preset])
    for lens in ([int(n) for n in rng.integers(1, 70, size=5)], [1, 2, 3], [66, 65]):
        T = max(lens)
        mel = torch.randn(len(lens), 80, T, generator=torch.Generator().manual_seed(T))
        for b, n in enumerate(lens):
            mel[b, :, n:] = -77.0  # garbage in the padding must not leak
        bct = run(gen, mel.to(dev), lengths=lens)
        btc = run(gen, mel.transpose(1, 2).contiguous().to(dev), lengths=lens, mel_layout="btc")
        assert torch.equal(bct, btc), lens
        for b, n in enumerate(lens):
            solo = run(gen, mel[b:b + 1, :, :n].contiguous().to(dev))
            m = solo.shape[-1]
            assert torch.equal(bct[b:b + 1, :, :m], solo), (lens, b)
            assert torch.count_nonzero(bct[b, :, m:]) == 0, (lens, b)
            if precision != "bf16w" and b < 2:
                ref = H.generator_forward(H.to_torch_state(sd), cfg, mel[b:b + 1, :, :n])
                err = (solo.cpu() - ref).abs().max().item()
                assert err < ATOL, (lens, b, err)


def test_multi_stream_batched_equals_one_shot(pkg, gen_sd, dev):
    """Several streams share each forward (one ragged batch per step, glue.StreamingVocoder
    .step): every stream's audio is bitwise its one-shot run, whatever the push pattern."""
    import importlib
    glue = importlib.import_module("tts_sambert_hifigan_amd.glue")
    gen, _ = gen_sd
    lens = [230, 41, 1, 97, 64]
    g = torch.Generator().manual_seed(12)
    mels = [torch.randn(80, n, generator=g).to(dev) for n in lens]
    refs = [run(gen, m[None])[0, 0] for m in mels]
    S = len(mels)
    sv = glue.StreamingVocoder(gen, chunk_frames=32, n_streams=S)
    outs = {s: [] for s in range(S)}
    pos = [0] * S
    rng = np.random.default_rng(5)
    batched = 0
    while True:
        for s in range(S):
            if pos[s] < lens[s]:
                n = int(rng.integers(1, 40))
                sv.feed(mels[s][:, pos[s]:pos[s] + n], s)
                pos[s] += n
                if pos[s] >= lens[s]:
                    sv.finish(s)
        r = sv.step()
        batched = max(batched, len(r))
        for s, a in r.items():
            outs[s].append(a)
        if not r and all(p >= n for p, n in zip(pos, lens)):
            break
    torch.cuda.synchronize()
    assert batched > 1
    for s in range(S):
        assert torch.equal(torch.cat(outs[s]), refs[s]), s


def test_ten_minute_stream_constant_memory(pkg, dev):
    """A 10-minute stream (51,680 frames at 22.05 kHz / hop 256) in 64-frame pushes: the
    buffer is allocated once, device memory does not grow after the first chunks, and the
    streamed audio equals the one-shot forward of the whole utterance — bitwise in bf16x3
    / fp32; in f16x3 to ~1e-9: a chunk's operands are scaled by the max over the chunk, the
    one-shot run's by the max over 10 minutes, and only values whose f16 lo half falls
    below the normal range (< 2^-17 of that max) can round differently."""
    import importlib
    glue = importlib.import_module("tts_sambert_hifigan_amd.glue")
    from oracle import config as C
    sd = C.make_state_dict(C.V1, seed=4)
    gen = pkg.HiFiGANGenerator(**C.V1.kwargs(), precision="f16x3").eval()
    gen.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()})
    gen = gen.to(dev)
    T = 22050 * 600 // 256
    mel = torch.randn(80, T, generator=torch.Generator().manual_seed(2)).to(dev)
    sv = glue.StreamingVocoder(gen, chunk_frames=64)
    out = torch.empty(T * 256, device=dev)
    pos, w, caps, mem = 0, 0, set(), []
    while pos < T:
        a = sv.push(mel[:, pos:pos + 64])
        out[w:w + a.numel()] = a
        w += a.numel()
        pos += 64
        caps.add(sv.capacity())
        if pos // 64 in (50, 400, 800):
            torch.cuda.synchronize()
            mem.append(torch.cuda.memory_allocated(dev))
    a = sv.flush()
    out[w:w + a.numel()] = a
    w += a.numel()
    torch.cuda.synchronize()
    assert w == T * 256
    assert len(caps) == 1 and sv.buffered_frames() <= 64 + 2 * sv.ctx
    assert mem[-1] <= mem[0], mem
    ref = run(gen, mel[None])[0, 0]
    d = (out - ref).abs().max().item()
    print(f"\n10-minute stream vs one-shot [f16x3]: max diff {d:.2e}")
    assert d <= 1e-7
