"""GPU behaviour tests: the reference's own vocoder contract
(tests/test_hifigan_generator.py, tests/test_hifigan_integration.py of the
reference, restated against the MI355X module), full-size (BASELINE config 2)
size-independent properties, and the C ABI called directly.

Run on an MI355X:  python -m pytest tests -m gpu -x -q
"""
import ctypes
import io
import sys

import numpy as np
import pytest
import torch



def _randn(*shape, seed, dev):
    """Seeded device input (every GPU test input is reproducible from the record)."""
    return torch.randn(*shape, generator=torch.Generator().manual_seed(seed)).to(dev)

pytestmark = pytest.mark.gpu
ATOL = 1e-4


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    return torch.device("cuda:0")


@pytest.fixture(scope="module")
def v1(pkg, dev):
    from oracle import config as C
    sd = C.make_state_dict(C.V1, seed=0)
    gen = pkg.HiFiGANGenerator(**C.V1.kwargs()).eval()
    gen.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()})
    return gen.to(dev), sd


def run(gen, mel):
    with torch.no_grad():
        out = gen(mel)
    torch.cuda.synchronize()
    return out


# ---- reference contract (tests/test_hifigan_generator.py) -------------------------
def test_forward_shape_and_range(v1, dev):
    gen, _ = v1
    mel = _randn(2, 80, 100, seed=301, dev=dev)
    wav = run(gen, mel)
    assert wav.shape == (2, 1, 100 * 256)
    assert wav.dtype == torch.float32
    assert wav.min() >= -1.0 and wav.max() <= 1.0


@pytest.mark.parametrize("T", [50, 100, 200])
def test_different_lengths(v1, dev, T):
    wav = run(v1[0], _randn(1, 80, T, seed=302, dev=dev))
    assert wav.shape == (1, 1, T * 256)


@pytest.mark.parametrize("B", [1, 4, 8])
def test_batch_sizes(v1, dev, B):
    wav = run(v1[0], _randn(B, 80, 100, seed=303, dev=dev))
    assert wav.shape == (B, 1, 100 * 256)


def test_nonexact_upsampling_shape(pkg, dev):
    # reference test_hifigan_integration.py:147-164; oracle gives [1, 1, 10048] for T=50
    gen = pkg.HiFiGAN(n_mels=80, upsample_rates=[5, 5, 4, 2],
                      upsample_kernel_sizes=[10, 10, 8, 4]).to(dev).eval()
    wav = run(gen, _randn(1, 80, 50, seed=304, dev=dev))
    assert wav.shape == (1, 1, 10048)


def test_generate_alias_and_logging(pkg, dev):
    model = pkg.HiFiGAN(n_mels=80, debug_shapes=True).to(dev).eval()
    mel = _randn(1, 80, 10, seed=305, dev=dev)
    buf = io.StringIO()
    old, sys.stdout = sys.stdout, buf
    try:
        w1 = run(model, mel)
        w2 = model.generate(mel)
        torch.cuda.synchronize()
    finally:
        sys.stdout = old
    assert torch.equal(w1, w2)
    out = buf.getvalue()
    assert "[HiFiGAN]" in out and "[HiFiGANGenerator]" in out and "shape" in out.lower()


def test_inputs_rejected(v1, dev):
    gen, _ = v1
    with pytest.raises(RuntimeError):
        gen(torch.randn(1, 80, 8))  # CPU tensor: no CPU fallback
    with pytest.raises(RuntimeError):
        gen(_randn(1, 81, 8, seed=306, dev=dev))
    mel = torch.randn(1, 80, 8, device=dev, requires_grad=True)
    with pytest.raises(NotImplementedError):
        gen(mel)


def test_weights_follow_load_state_dict(pkg, dev):
    from oracle import config as C, hifigan_torch as H, prng
    cfg = C.V2STAR
    gen = pkg.HiFiGANGenerator(**cfg.kwargs()).eval().to(dev)
    mel = prng.mel_input(5, (1, 80, 12))
    for seed in (1, 2):
        sd = C.make_state_dict(cfg, seed=seed)
        gen.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()})
        wav = run(gen, torch.from_numpy(mel).to(dev)).cpu()
        ref = H.generator_forward(H.to_torch_state(sd), cfg, torch.from_numpy(mel))
        assert (wav - ref).abs().max().item() < ATOL


# ---- full size (BASELINE config 2) ----------------------------------------------
@pytest.fixture(scope="module")
def full(v1, dev):
    gen, sd = v1
    g = torch.Generator().manual_seed(1234)
    mel = torch.randn(8, 80, 1024, generator=g)
    wav = run(gen, mel.to(dev))
    return gen, sd, mel, wav


def test_full_size_deterministic(full, dev):
    gen, _, mel, wav = full
    again = run(gen, mel.to(dev))
    assert torch.equal(wav, again)


def test_full_size_batch_split_invariance(full, dev):
    gen, _, mel, wav = full
    for b in (0, 5):
        one = run(gen, mel[b:b + 1].to(dev))
        assert torch.equal(one[0], wav[b])
    pair = run(gen, mel[2:4].to(dev))
    assert torch.equal(pair, wav[2:4])


@pytest.mark.parametrize("item,start", [(0, 0), (3, 500), (7, 1024 - 48)])
def test_full_size_windowed_oracle(full, item, start):
    """Receptive field is ±13 frames; the oracle on the window
    plus a 16-frame margin reproduces the full-size output in that window."""
    from oracle import config as C, hifigan_torch as H
    gen, sd, mel, wav = full
    W, M = 48, 16
    a, b = max(0, start - M), min(1024, start + W + M)
    ref = H.generator_forward(H.to_torch_state(sd), C.V1, mel[item:item + 1, :, a:b])
    ref = ref[0, 0, (start - a) * 256:(start - a + W) * 256].numpy()
    got = wav[item, 0, start * 256:(start + W) * 256].cpu().numpy()
    assert np.abs(got - ref).max() < ATOL


# ---- C ABI directly ---------------------------------------------------------------
def test_c_abi_forward_internal_workspace(pkg, full, dev):
    gen, _, mel, wav = full
    h = gen.hip_handle(dev)
    lib = pkg.load_library()
    m = mel[:2].contiguous().to(dev)
    L = lib.hfg_out_len(h.ptr, 1024)
    out = torch.empty(2, 1, L, device=dev)
    assert lib.hfg_reserve(h.ptr, 2, 1024) == 0
    rc = lib.hfg_forward(h.ptr, ctypes.c_void_p(m.data_ptr()), 2, 1024,
                         ctypes.c_void_p(out.data_ptr()), L,
                         ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
    assert rc == 0, lib.hfg_last_error()
    torch.cuda.synchronize()
    assert torch.equal(out, wav[:2])
    # error paths: wrong out_len, too-small workspace
    assert lib.hfg_forward(h.ptr, ctypes.c_void_p(m.data_ptr()), 2, 1024,
                           ctypes.c_void_p(out.data_ptr()), L + 1, None) == -22
    assert lib.hfg_forward_ws(h.ptr, ctypes.c_void_p(m.data_ptr()), 2, 1024,
                              ctypes.c_void_p(out.data_ptr()), L, ctypes.c_void_p(out.data_ptr()),
                              16, None) == -22


def test_profiling_summary(pkg, v1, dev):
    gen, _ = v1
    h = gen.hip_handle(dev)
    h.profile_reset()
    h.set_profiling(True)
    run(gen, _randn(1, 80, 64, seed=307, dev=dev))
    h.set_profiling(False)
    prof = h.profile_summary()
    # the default (f16x3) schedule: conv_pre, 4 upsamplers, conv_post, the stage-0 and stage-1
    # k = 7 / 11 ResBlocks layer by layer (6 launches each), the other ResBlocks one whole-
    # ResBlock launch each (two for the split k = 11 ones at C = 32 / 64); a small forward
    # runs its MRFs' ResBlocks on concurrent streams and adds one mrf_combine launch per such
    # stage (hifigan_capi.cpp run_mrf); the mel's scale slot comes from one absmax launch
    assert gen.precision == "f16x3"
    combine = prof.get("mrf_combine", {"launches": 0})["launches"]
    assert prof.get("absmax", {"launches": 0})["launches"] == 1, sorted(prof)
    n_conv = sum(v["launches"] for k, v in prof.items() if k not in ("mrf_combine", "absmax"))
    # 6 (pre, ups x4, post) + stage 0: 3 x 6 + stage 1: 2 x 6 + 1 + stages 2, 3: 1 + 1 + 2 each
    assert n_conv == 6 + 3 * 6 + 2 * 6 + 1 + 4 + 4, sorted(prof.items())
    assert combine <= 4
    assert all(v["ms"] > 0 for k, v in prof.items() if k != "mrf_combine")
    from oracle import config as C
    total_flop = sum(v["flop"] for v in prof.values())
    assert abs(total_flop - 2398848 * 64 * 256) / total_flop < 1e-5  # summary prints 7 digits


def test_hipgraph_capture_replay(v1, dev):
    """The 78 launches of one forward can be captured into a hipGraph (torch.cuda.graph
    on the capture stream) and replayed; the replay equals the eager result."""
    gen, _ = v1
    mel = _randn(2, 80, 40, seed=308, dev=dev)
    with torch.no_grad():
        ref = gen(mel)
        s = torch.cuda.Stream(dev)
        s.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(s):
            gen(mel)
        torch.cuda.current_stream(dev).wait_stream(s)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            out = gen(mel)
        mel.copy_(_randn(2, 80, 40, seed=309, dev=dev))
        g.replay()
        ref2 = gen(mel)
    torch.cuda.synchronize()
    assert torch.equal(out, ref2)
    assert not torch.equal(out, ref)


# ---- full size, headline precision (f16x3, 2 streams: what bench.py times) -------
@pytest.fixture(scope="module")
def full_split(pkg, full, dev):
    from oracle import config as C
    _, sd, mel, wav32 = full
    gen = pkg.HiFiGANGenerator(**C.V1.kwargs(), precision="f16x3").eval()
    gen.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()})
    gen = gen.to(dev)
    return gen, sd, mel, run(gen, mel.to(dev)), wav32


def test_full_size_split_vs_fp32_path(full_split):
    """At the bench size ([8,80,1024]) the split-precision path stays within the
    north_star tolerance of the exact-fp32 path on every sample of every utterance."""
    _, _, _, wav, wav32 = full_split
    assert (wav - wav32).abs().max().item() < ATOL


@pytest.mark.parametrize("item,start", [(1, 0), (6, 700), (4, 1024 - 48)])
def test_full_size_split_windowed_oracle(full_split, item, start):
    """f16x3 full-size output against the oracle on a receptive-field window."""
    from oracle import config as C, hifigan_torch as H
    _, sd, mel, wav, _ = full_split
    W, M = 48, 16
    a, b = max(0, start - M), min(1024, start + W + M)
    ref = H.generator_forward(H.to_torch_state(sd), C.V1, mel[item:item + 1, :, a:b])
    ref = ref[0, 0, (start - a) * 256:(start - a + W) * 256].numpy()
    got = wav[item, 0, start * 256:(start + W) * 256].cpu().numpy()
    assert np.abs(got - ref).max() < ATOL


def test_full_size_split_batch_split_invariance(full_split, dev):
    """Utterances are independent on the headline path too (bitwise), whatever the
    batch composition and stream split."""
    gen, _, mel, wav, _ = full_split
    one = run(gen, mel[3:4].to(dev))
    assert torch.equal(one[0], wav[3])
    five = run(gen, mel[1:6].to(dev))
    assert torch.equal(five, wav[1:6])


# ---- maximum size ------------------------------------------------------------------
T_MAX = 131071  # V1: 8192 * T fp32 per item < 2^30 elements, the kernels' 32-bit byte offsets


@pytest.mark.parametrize("precision", ["f16x3", "bf16x3", "fp32"])
def test_max_length_utterance_windowed_oracle(pkg, dev, precision):
    """One utterance at the longest T the C ABI accepts (2^30 - 8192 activation elements per
    item, ~25 min of audio): the output at the head, the middle and the very end matches
    the oracle on a receptive-field window, so no byte offset wraps."""
    from oracle import config as C, hifigan_torch as H
    sd = C.make_state_dict(C.V1, seed=0)
    gen = pkg.HiFiGANGenerator(**C.V1.kwargs(), precision=precision).eval()
    gen.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()})
    gen = gen.to(dev)
    g = torch.Generator().manual_seed(77)
    mel = torch.randn(1, 80, T_MAX, generator=g)
    wav = run(gen, mel.to(dev))
    assert wav.shape == (1, 1, T_MAX * 256)
    W, M = 32, 16
    tsd = H.to_torch_state(sd)
    for start in (0, T_MAX // 2 + 5, T_MAX - W):
        a, b = max(0, start - M), min(T_MAX, start + W + M)
        ref = H.generator_forward(tsd, C.V1, mel[:, :, a:b])
        ref = ref[0, 0, (start - a) * 256:(start - a + W) * 256].numpy()
        got = wav[0, 0, start * 256:(start + W) * 256].cpu().numpy()
        assert np.abs(got - ref).max() < ATOL, (precision, start)
    del wav
    torch.cuda.empty_cache()


def test_over_max_length_rejected(pkg, v1, dev):
    """One frame past the limit is refused with EINVAL before any launch."""
    gen, _ = v1
    h = gen.hip_handle(dev)
    lib = pkg.load_library()
    T = T_MAX + 1
    L = lib.hfg_out_len(h.ptr, T)
    dummy = torch.empty(64, device=dev)
    rc = lib.hfg_forward_ws(h.ptr, ctypes.c_void_p(dummy.data_ptr()), 1, T,
                            ctypes.c_void_p(dummy.data_ptr()), L, ctypes.c_void_p(dummy.data_ptr()),
                            256, None)
    assert rc == -22
    assert b"reaches 2^30" in lib.hfg_last_error()


# ---- weight tracking and 2-stream capture -------------------------------------------
def test_weight_edit_through_data_is_picked_up(pkg, dev):
    """An in-place edit through ``param.data`` leaves autograd's version counter alone;
    with ``verify_weights`` on (opt-in since round 3: it costs a host sync per forward) the
    module's content hash (hfg_checksum32) still notices it, so the next forward runs on
    the new weights.  Same for a ResBlock on its own.  By default the
    version / data_ptr fingerprint is the only check and ``refresh_weights()`` is the
    route for ``.data`` edits."""
    from oracle import config as C, hifigan_torch as H, prng
    cfg = C.V2STAR
    sd = C.make_state_dict(cfg, seed=8)
    gen = pkg.HiFiGANGenerator(**cfg.kwargs()).eval()
    gen.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()})
    gen = gen.to(dev)
    assert gen.verify_weights is False  # default: no per-forward hash / host sync
    gen.verify_weights = True
    gen.mrfs[0].resblocks[1].verify_weights = True
    mel = torch.from_numpy(prng.mel_input(8, (1, 80, 20))).to(dev)
    w0 = run(gen, mel).clone()
    v0 = gen.ups[1].weight._version
    gen.ups[1].weight.data.mul_(1.5)
    gen.mrfs[2].resblocks[0].convs2[1].bias.data.add_(0.01)
    assert gen.ups[1].weight._version == v0
    w1 = run(gen, mel)
    assert not torch.equal(w0, w1)
    sd2 = {k: v.detach().cpu() for k, v in gen.state_dict().items()}
    ref = H.generator_forward(sd2, cfg, mel.cpu())
    assert (w1.cpu() - ref).abs().max().item() < ATOL
    rb = gen.mrfs[0].resblocks[1]
    x = _randn(2, rb.channels, 50, seed=310, dev=dev)
    y0 = run(rb, x).clone()
    rb.convs1[0].weight.data.neg_()
    assert not torch.equal(y0, run(rb, x))
    # with verification off, refresh_weights() is the explicit route
    gen.verify_weights = False
    gen.ups[1].weight.data.mul_(1 / 1.5)
    assert torch.equal(run(gen, mel), w1)
    gen.refresh_weights()
    assert not torch.equal(run(gen, mel), w1)


def test_hipgraph_capture_two_stream_forward(v1, dev):
    """A forward big enough for the two-stream batch split (B x T >= 4096 frames: the
    caller's stream forks to the handle's internal stream and joins back) is captured
    into a hipGraph and replays to the eager result."""
    gen, _ = v1
    h = gen.hip_handle(dev)
    h.set_streams(2)
    mel = _randn(4, 80, 1100, seed=311, dev=dev)
    with torch.no_grad():
        s = torch.cuda.Stream(dev)
        s.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(s):
            gen(mel)
        torch.cuda.current_stream(dev).wait_stream(s)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            out = gen(mel)
        mel.copy_(_randn(4, 80, 1100, seed=312, dev=dev))
        g.replay()
        torch.cuda.synchronize()
        ref = gen(mel)
    torch.cuda.synchronize()
    assert torch.equal(out, ref)
