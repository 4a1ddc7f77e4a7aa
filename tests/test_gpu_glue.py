"""SURVEY.md §8(f) rows 2-3 on the GPU: acoustic-model glue ([B, T, 80] input,
ragged batches) and streaming vocoding, against the one-shot Generator and the CPU
oracle (atol 1e-4).

Contracts: a ragged item is bitwise its solo run in every mode; a
streamed chunk is bitwise the crop of the Generator run on its context window in every
mode; a whole stream is bitwise the one-shot run in fp32 / bf16x3 and within 1e-7 of it
in f16x3, whose per-launch power-of-two operand scales come from the max over what the
launch sees (the window, or the whole utterance).  Every device input is seeded."""
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


STREAM_F16X3_TOL = 1e-7  # f16x3 stream vs one-shot at default scale (measured 0-1.5e-8)
# Away from default scale the f16x3 stream and the one-shot run are two evaluations with
# different power-of-two operand scales (a window's max vs the utterance's), each within the
# mode's accuracy of the exact result, and their difference grows with that accuracy (2x
# weights: 4.8e-7, round 6).  The contract there: the stream is as accurate as the one-shot run
# — max|stream - oracle| <= 2 x max|one-shot - oracle| + 1e-7
# (test_streaming_accuracy_away_from_default_scale); the exact modes stay bitwise at every scale.
STREAM_F16X3_ACC = 2.0


def randn(*shape, seed, dev):
    return torch.randn(*shape, generator=torch.Generator().manual_seed(seed)).to(dev)


@pytest.fixture(scope="module", params=["fp32", "f16x3", "bf16x3"])
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
    mel = randn(3, 80, 57, seed=101, dev=dev)
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
    mels = [randn(80, n, seed=102 + n, dev=dev) for n in (33, 5, 48)]
    wavs = glue.vocode_list(gen, mels)
    for m, w in zip(mels, wavs):
        assert torch.equal(w, run(gen, m[None])[0, 0])


def _stage_exponents(sd, mel):
    """floor(log2(max |stage|)) of every oracle stage: the f16x3 scale exponents a launch
    over `mel` derives (up to the per-block ResBlock windows)."""
    from oracle import config as C, hifigan_torch as H
    ex = {}
    H.generator_forward(H.to_torch_state(sd), C.V1, mel.cpu()[None],
                        tap=lambda n, t: ex.__setitem__(n, int(np.floor(np.log2(
                            t.abs().max().item() + 1e-30)))))
    return ex


def _check_stream(gen, sd, mel, out, windows, label, cfg=None, evidence=print, strict=True):
    """The streaming contract for one stream: every chunk bitwise the crop of gen(window);
    the stream bitwise (fp32, bf16x3) the one-shot run, and in f16x3 within 1e-7 of it at
    default scale (strict) / as accurate as it against the oracle (any scale), with the
    evidence printed (max |diff|, differing samples, first one, the chunk's and the one-shot
    run's stage exponents); within 1e-4 of the oracle."""
    from oracle import config as C, hifigan_torch as H
    cfg = cfg or C.V1
    hop = gen.output_length(2) - gen.output_length(1)
    ref = run(gen, mel[None])[0, 0]
    assert out.shape == ref.shape, label
    worst = (0.0, None)
    for (a, b, lo, hi) in windows:
        win = run(gen, mel[None, :, lo:hi])[0, 0, (a - lo) * hop:(b - lo) * hop]
        assert torch.equal(out[a * hop:b * hop], win), (label, "chunk != gen(window)", a, b)
        d = (win - ref[a * hop:b * hop]).abs().max().item()
        if d > worst[0]:
            worst = (d, (a, b, lo, hi))
    diff = (out - ref).abs()
    dmax = diff.max().item()
    n_diff = int(torch.count_nonzero(diff).item())
    first = int(torch.nonzero(diff)[0, 0].item()) if n_diff else -1
    msg = (f"{label}: stream vs one-shot max|diff| {dmax:.3e}, {n_diff} of {out.numel()} samples "
           f"differ (first at {first})")
    if worst[1] is not None and n_diff:
        a, b, lo, hi = worst[1]
        msg += (f"; worst chunk frames [{a}, {b}) window [{lo}, {hi}): stage exponents window "
                f"{_stage_exponents(sd, mel[:, lo:hi])} vs one-shot {_stage_exponents(sd, mel)}")
    o = H.generator_forward(H.to_torch_state(sd), cfg, mel.cpu()[None])[0, 0]
    err = (out.cpu() - o).abs().max().item()
    err_one = (ref.cpu() - o).abs().max().item()
    msg += f"; vs oracle: stream {err:.3e}, one-shot {err_one:.3e}"
    evidence(msg)
    if gen.precision == "f16x3":
        if strict:
            assert dmax <= STREAM_F16X3_TOL, msg
        assert err <= STREAM_F16X3_ACC * err_one + STREAM_F16X3_TOL, msg
    else:
        assert n_diff == 0, msg
    assert err < ATOL, (label, err)


def _stream_once(glue, gen, mel, chunk, seed):
    sv = glue.StreamingVocoder(gen, chunk_frames=chunk)
    pieces, windows, pos, T = [], [], 0, mel.shape[1]
    rng = np.random.default_rng(seed)
    while pos < T:
        n = int(rng.integers(1, 37))
        sv.feed(mel[:, pos:pos + n])
        while sv._window(0) is not None:
            pieces.append(sv.step([0])[0])
            windows.append(sv.last_windows[0])
        pos += n
    sv.finish()
    while sv._window(0) is not None:
        pieces.append(sv.step([0])[0])
        windows.append(sv.last_windows[0])
    return torch.cat(pieces), windows


def test_streaming_equals_one_shot(pkg, gen_sd, dev, evidence):
    import importlib
    glue = importlib.import_module("tts_sambert_hifigan_amd.glue")
    gen, sd = gen_sd
    assert gen.receptive_field_frames() == 15
    T = 230
    for seed in (0, 1, 2):
        mel = randn(80, T, seed=200 + seed, dev=dev)
        out, windows = _stream_once(glue, gen, mel, 40, seed)
        assert len(windows) >= 5
        _check_stream(gen, sd, mel, out, windows, f"[{gen.precision}] seed {seed}",
                      evidence=evidence)
    # push / flush give the same audio as feed / step
    sv = glue.StreamingVocoder(gen, chunk_frames=40)
    rng, pieces, pos = np.random.default_rng(2), [], 0
    while pos < T:
        n = int(rng.integers(1, 37))
        pieces.append(sv.push(mel[:, pos:pos + n]))
        pos += n
    pieces.append(sv.flush())
    assert torch.equal(torch.cat(pieces), out)


@pytest.mark.parametrize("wscale,mscale", [(2.0, 1.0), (4.0, 3.0)])
def test_streaming_accuracy_away_from_default_scale(pkg, dev, evidence, wscale, mscale):
    """The f16x3 streaming contract away from default scale: 2x weights (tanh not
    saturated: the g6 fixture's regime; the stream differs from the one-shot run by up to ~5e-7
    there, round 6) and 4x weights with a 3x mel (stage maxima ~2e6, tanh saturated), chunks of
    40 frames pushed in random pieces.  Every chunk is still bitwise its window's crop; the stream
    is as accurate as the one-shot run (max |stream - oracle| <= 2 x max |one-shot - oracle| +
    1e-7) and within 1e-4 of the oracle; fp32 and bf16x3 stay bitwise."""
    import importlib
    glue = importlib.import_module("tts_sambert_hifigan_amd.glue")
    from oracle import config as C
    sd = {k: v * wscale for k, v in C.make_state_dict(C.V1, seed=9).items()}
    mel = mscale * randn(80, 150, seed=230, dev=dev)
    for precision in ("f16x3", "fp32", "bf16x3"):
        gen = pkg.HiFiGANGenerator(**C.V1.kwargs(), precision=precision).eval()
        gen.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()})
        gen = gen.to(dev)
        out, windows = _stream_once(glue, gen, mel, 40, 11)
        _check_stream(gen, sd, mel, out, windows,
                      f"weights x{wscale:g} mel x{mscale:g} [{precision}]", evidence=evidence,
                      strict=False)


def test_streaming_is_deterministic_across_unrelated_forwards(pkg, gen_sd, dev):
    """State independence: a stream repeated after forwards of
    other configurations and sizes — which leave other values in LDS, in the per-item scale
    slots and in the workspace — is bitwise the first run, in every mode.  So the f16x3
    stream-vs-one-shot difference is the data-dependent scale (window max vs utterance
    max), not state left behind by earlier launches."""
    import importlib
    glue = importlib.import_module("tts_sambert_hifigan_amd.glue")
    from oracle import config as C
    gen, _ = gen_sd
    mel = randn(80, 230, seed=210, dev=dev)
    first, w1 = _stream_once(glue, gen, mel, 40, 7)
    for preset, seed in (("v2star", 211), ("nonexact", 212)):
        cfg = C.PRESETS[preset]
        other = pkg.HiFiGANGenerator(**cfg.kwargs(), precision=gen.precision).eval()
        other.load_state_dict({k: torch.from_numpy(v * 4.0)
                               for k, v in C.make_state_dict(cfg, seed=seed).items()})
        other = other.to(dev)
        run(other, 30.0 * randn(3, 80, 301, seed=seed, dev=dev))
        again, w2 = _stream_once(glue, gen, mel, 40, 7)
        assert w1 == w2
        assert torch.equal(first, again), (preset, (first - again).abs().max().item())


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
    .step): every stream's audio is, whatever the push pattern, chunk by chunk bitwise the
    crop of gen(window) (a ragged item equals its solo run), and bitwise (fp32, bf16x3) /
    within 1e-7 (f16x3) its one-shot run."""
    import importlib
    glue = importlib.import_module("tts_sambert_hifigan_amd.glue")
    gen, sd = gen_sd
    lens = [230, 41, 1, 97, 64]
    g = torch.Generator().manual_seed(12)
    mels = [torch.randn(80, n, generator=g).to(dev) for n in lens]
    S = len(mels)
    sv = glue.StreamingVocoder(gen, chunk_frames=32, n_streams=S)
    outs = {s: [] for s in range(S)}
    wins = {s: [] for s in range(S)}
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
            wins[s].append(sv.last_windows[s])
        if not r and all(p >= n for p, n in zip(pos, lens)):
            break
    torch.cuda.synchronize()
    assert batched > 1
    for s in range(S):
        _check_stream(gen, sd, mels[s], torch.cat(outs[s]), wins[s],
                      f"[{gen.precision}] stream {s} of {S}")


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
