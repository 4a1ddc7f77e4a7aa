"""GPU parity of the HIP Generator against the reference (golden fixtures) and
the CPU oracle.  Tolerance: fp32 atol 1e-4 on the wav (BASELINE.json north_star).

Run on an MI355X:  python -m pytest tests -m gpu -x -q
"""
import numpy as np
import pytest
import torch

from conftest import golden_case_state, load_golden

pytestmark = pytest.mark.gpu

ATOL = 1e-4  # north_star: fp32 output within 1e-4 of the reference


def _dev():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    return torch.device("cuda:0")


def _gen(pkg, cfg, sd, dev, precision="fp32"):
    gen = pkg.HiFiGANGenerator(**cfg.kwargs(), precision=precision).eval()
    if any(k.endswith("weight_g") for k in sd):
        gen.apply_weight_norm()
    gen.load_state_dict({k: torch.from_numpy(np.ascontiguousarray(v)) for k, v in sd.items()})
    return gen.to(dev)


def _oracle(cfg, sd, mel):
    from oracle import hifigan_torch as H
    return H.generator_forward(H.to_torch_state(sd), cfg, torch.as_tensor(mel)).numpy()


def _run(gen, mel, dev):
    with torch.no_grad():
        out = gen(torch.as_tensor(mel).to(dev))
    torch.cuda.synchronize()
    return out.cpu().numpy()


GOLDEN = ["g1_v1_b1_t32", "g2_v1_b2_t17", "g3_v2star_b2_t32", "g4_nonexact_b1_t20",
          "g5_v1_weightnorm_b1_t16", "g6_v1_loud2x_b1_t24", "g7_v1_b3_t1", "g8_v2star_b1_t3"]


@pytest.mark.parametrize("name", GOLDEN)
def test_golden_fixture(pkg, golden_index, name, evidence):
    dev = _dev()
    case = golden_index["cases"][name]
    cfg, sd = golden_case_state(case)
    g = load_golden(name)
    gen = _gen(pkg, cfg, sd, dev)
    wav = _run(gen, g["mel"], dev)
    assert wav.shape == g["wav"].shape
    err = np.abs(wav - g["wav"]).max()
    scale = np.abs(g["wav"]).max()
    evidence(f"{name}: max|hip-ref| = {err:.3e} (max|ref| {scale:.3e})")
    assert err < ATOL
    # relative check too: a near-constant output could hide a bug
    rel = np.linalg.norm(wav - g["wav"]) / np.linalg.norm(g["wav"])
    assert rel < 1e-3, rel


@pytest.mark.parametrize("preset,B,T", [("v1", 2, 64), ("v2star", 3, 96), ("nonexact", 2, 33)])
def test_random_vs_oracle(pkg, preset, B, T, evidence):
    from oracle import config as C, prng
    dev = _dev()
    cfg = C.PRESETS[preset]
    sd = C.make_state_dict(cfg, seed=100 + B + T)
    mel = prng.mel_input(100 + T, (B, cfg.n_mels, T))
    gen = _gen(pkg, cfg, sd, dev)
    wav = _run(gen, mel, dev)
    ref = _oracle(cfg, sd, mel)
    assert wav.shape == ref.shape
    err = np.abs(wav - ref).max()
    evidence(f"{preset} B={B} T={T}: max err {err:.3e}")
    assert err < ATOL


@pytest.mark.parametrize("precision", ["f16x3", "bf16x3"])
@pytest.mark.parametrize("name", GOLDEN)
def test_golden_fixture_split(pkg, golden_index, name, precision, evidence):
    """Split-precision modes (scaled f16 / bf16 hi-lo operands, fp32 accumulate) meet the
    same 1e-4 bar against the reference outputs."""
    dev = _dev()
    case = golden_index["cases"][name]
    cfg, sd = golden_case_state(case)
    g = load_golden(name)
    gen = _gen(pkg, cfg, sd, dev, precision=precision)
    wav = _run(gen, g["mel"], dev)
    err = np.abs(wav - g["wav"]).max()
    evidence(f"{name} [{precision}]: max|hip-ref| = {err:.3e}")
    assert err < ATOL
    rel = np.linalg.norm(wav - g["wav"]) / np.linalg.norm(g["wav"])
    assert rel < 1e-3, rel


@pytest.mark.parametrize("precision,fused", [("f16x3", "1"), ("f16x3", "0"), ("bf16x3", "1"),
                                             ("bf16x3", "0")])
@pytest.mark.parametrize("preset,B,T", [("v1", 2, 300), ("v2star", 2, 200)])
def test_split_vs_oracle_longer(pkg, preset, B, T, precision, fused, sched):
    """Random weights/mel vs the oracle with the whole-ResBlock kernel for C in {32, 64, 128}
    on (schedule knob FUSED_RB=1, default) or off (layer per launch), in both split formats."""
    from oracle import config as C, prng
    sched("FUSED_RB", fused)
    dev = _dev()
    cfg = C.PRESETS[preset]
    sd = C.make_state_dict(cfg, seed=7)
    mel = prng.mel_input(70 + T, (B, cfg.n_mels, T))
    wav = _run(_gen(pkg, cfg, sd, dev, precision=precision), mel, dev)
    ref = _oracle(cfg, sd, mel)
    err = np.abs(wav - ref).max()
    print(f"{preset} B={B} T={T} [{precision} fused={fused}]: max err {err:.3e}")
    assert err < ATOL


@pytest.mark.parametrize("precision", ["f16x3", "bf16x3"])
def test_fused_resblock_matches_layer_path(pkg, precision, sched):
    """Whole-ResBlock kernel vs the layer-per-launch schedule on a ragged batch long enough
    for many windows per utterance (window seams, lengths that end inside a window, an
    utterance shorter than one window)."""
    from oracle import config as C, prng
    dev = _dev()
    cfg = C.V1
    sd = C.make_state_dict(cfg, seed=21)
    B, T = 4, 160
    mel = torch.as_tensor(prng.mel_input(21, (B, cfg.n_mels, T))).to(dev)
    lens = torch.tensor([160, 97, 3, 131], dtype=torch.int32, device=dev)
    outs = []
    for fused in ("0", "1"):
        sched("FUSED_RB", fused)
        gen = _gen(pkg, cfg, sd, dev, precision=precision)
        with torch.no_grad():
            outs.append(gen(mel, lengths=lens).cpu().numpy())
        torch.cuda.synchronize()
    err = np.abs(outs[0] - outs[1]).max()
    print(f"fused vs layer path [{precision}]: max diff {err:.3e}")
    assert err < (2e-5 if precision == "bf16x3" else 2e-6)


@pytest.mark.gpu
@pytest.mark.parametrize("precision", ["f16x3", "bf16x3", "fp32"])
def test_two_stream_split_is_bitwise_equal(pkg, precision):
    """hfg_set_streams(2) runs the batch halves on the caller's stream and an internal
    one; every wav equals the 1-stream run bit for bit (odd batch, ragged lengths,
    a batch large enough to be split: B x T >= 4096 frames)."""
    from oracle import config as C, prng
    dev = _dev()
    cfg = C.V1
    sd = C.make_state_dict(cfg, seed=17)
    B, T = 5, 1000
    mel = torch.as_tensor(prng.mel_input(23, (B, cfg.n_mels, T))).to(dev)
    lens = torch.tensor([1000, 731, 1000, 2, 517], dtype=torch.int32, device=dev)
    gen = _gen(pkg, cfg, sd, dev, precision=precision)
    h = gen.hip_handle(dev)
    outs = []
    for n in (1, 2, 1):
        h.set_streams(n)
        with torch.no_grad():
            outs.append((gen(mel).cpu().numpy(), gen(mel, lengths=lens).cpu().numpy()))
        torch.cuda.synchronize()
    h.set_streams(2)
    for a, b in zip(outs[0], outs[1]):
        assert np.array_equal(a, b)
    for a, b in zip(outs[0], outs[2]):
        assert np.array_equal(a, b)


@pytest.mark.gpu
@pytest.mark.parametrize("precision", ["f16x3", "bf16x3", "fp32"])
def test_ragged_forward_ignores_workspace_contents(pkg, precision):
    """A ragged batch never reads workspace frames past an item's length (the
    output-frame upsampler masked them by a multiply, and 0 * NaN is NaN).  The same forward
    on a workspace pre-filled with NaN, with +inf and with zeros gives bitwise the same wavs,
    and every valid sample is finite."""
    from oracle import config as C, prng
    dev = _dev()
    cfg = C.V1
    sd = C.make_state_dict(cfg, seed=19)
    B, T = 4, 300
    mel = torch.as_tensor(prng.mel_input(29, (B, cfg.n_mels, T))).to(dev)
    lens = torch.tensor([300, 157, 3, 242], dtype=torch.int32, device=dev)
    gen = _gen(pkg, cfg, sd, dev, precision=precision)
    h = gen.hip_handle(dev)
    out_len = h.out_len(T)
    ws_bytes = h.workspace_bytes(B, T)
    stream = torch.cuda.current_stream(dev).cuda_stream
    outs = []
    for fill in (float("nan"), float("inf"), 0.0):
        ws = torch.full((ws_bytes // 4 + 1,), fill, dtype=torch.float32, device=dev)
        wav = torch.full((B, 1, out_len), 7.0, dtype=torch.float32, device=dev)
        h.forward_ex(mel.data_ptr(), B, T, wav.data_ptr(), out_len, ws.data_ptr(), ws_bytes,
                     stream, lengths_ptr=lens.data_ptr())
        torch.cuda.synchronize()
        outs.append(wav.cpu().numpy())
    for i, n in enumerate(lens.tolist()):
        valid = outs[2][i, 0, :n * 256]
        assert np.isfinite(valid).all(), f"item {i}: non-finite valid samples"
    assert np.array_equal(outs[0], outs[2], equal_nan=True), "NaN workspace changed the wav"
    assert np.array_equal(outs[1], outs[2], equal_nan=True), "+inf workspace changed the wav"


@pytest.mark.gpu
@pytest.mark.parametrize("precision,fused", [("f16x3", "1"), ("f16x3", "0"), ("bf16x3", "0")])
def test_split_layer_kernels_run_to_run_bitwise(pkg, precision, fused, sched):
    """Repeated forwards are bitwise identical on every split layer-kernel tile (with the
    whole-ResBlock kernel off the 64x256 / 32x256 tiles run every C <= 64 conv).  Guards
    the per-wave vmcnt count of the staged input window (a wait that let a chunk read a
    weight slab before its DMA landed gave nondeterministic errors up to ~6e-4, round 1) and,
    for f16x3, the order-free max of the per-item scale slots and the exclusion of stale LDS
    margin rows from the block maxima: forwards of other configurations (x4 weights, loud
    mels) run between the repeats."""
    from oracle import config as C, prng
    sched("FUSED_RB", fused)
    dev = _dev()
    cfg = C.V1
    sd = C.make_state_dict(cfg, seed=17)
    B, T = 5, 1000
    mel = torch.as_tensor(prng.mel_input(23, (B, cfg.n_mels, T))).to(dev)
    lens = torch.tensor([1000, 731, 1000, 2, 517], dtype=torch.int32, device=dev)
    gen = _gen(pkg, cfg, sd, dev, precision=precision)
    # forwards of other configurations between the repeats leave other values in LDS, in
    # the per-item scale slots and in the cached workspace
    dirt = []
    for preset, seed in (("v2star", 61), ("nonexact", 62)):
        ocfg = C.PRESETS[preset]
        osd = {k: v * 4.0 for k, v in C.make_state_dict(ocfg, seed=seed).items()}
        dirt.append((_gen(pkg, ocfg, osd, dev, precision=precision),
                     torch.as_tensor(30.0 * prng.mel_input(seed, (3, ocfg.n_mels, 333))).to(dev)))
    h = gen.hip_handle(dev)
    outs = []
    for i, n in enumerate((1, 2, 1, 2, 1, 2)):
        h.set_streams(n)
        with torch.no_grad():
            outs.append((gen(mel).cpu().numpy(), gen(mel, lengths=lens).cpu().numpy()))
            og, om = dirt[i % 2]
            og(om)
        torch.cuda.synchronize()
    h.set_streams(2)
    for o in outs[1:]:
        for a, b in zip(outs[0], o):
            assert np.array_equal(a, b), np.abs(a - b).max()


@pytest.mark.gpu
@pytest.mark.parametrize("precision", ["f16x3", "bf16x3", "bf16w"])
@pytest.mark.parametrize("preset,B,T,lens", [("v1", 3, 64, [64, 41, 3]),
                                             ("v2star", 2, 64, [64, 17]),
                                             ("nonexact", 2, 64, [64, 29]),
                                             ("rates248", 3, 36, [36, 21, 5])])
def test_ups_frames_kernel_bitwise(pkg, preset, B, T, lens, precision, sched):
    """The output-frame upsampler kernel (csrc/ups_bf16x3.hip: k = 2u stages, both sample
    classes of a frame per wave) gives the polyphase conv1d_bf16x3 upsampler's result bit
    for bit: the same MFMA sequence per output element, the same split of lrelu(x), the
    same zero padding (and, f16x3, the same per-item input scale).  UPS_FRAMES=2 forces
    it onto every eligible stage (rates 8 and 2 in V1 / V2*, 4 and 2 in the non-exact preset;
    rate 5 stays polyphase); the default (1) keeps the polyphase small-grid tile on these
    small grids; ragged and full batches.  "rates248" puts the rate-2 stage first, so a
    ragged item has an odd number of input frames there (the DPP-paired 16-B store's
    last-frame path)."""
    from oracle import config as C, prng
    dev = _dev()
    cfg = C.PRESETS.get(preset) or C.GenConfig(
        upsample_rates=[2, 4, 8], upsample_kernel_sizes=[4, 8, 16], upsample_initial_channel=256,
        resblock_kernel_sizes=[3, 5], resblock_dilation_sizes=[[1, 3], [1]])
    sd = C.make_state_dict(cfg, seed=31)
    mel = torch.as_tensor(prng.mel_input(31 + T, (B, cfg.n_mels, T))).to(dev)
    ln = torch.tensor(lens, dtype=torch.int32, device=dev)
    outs, names = {}, {}
    for mode in ("1", "2"):
        sched("UPS_FRAMES", mode)  # read when the handle is created
        gen = _gen(pkg, cfg, sd, dev, precision=precision)
        h = gen.hip_handle(dev)
        h.profile_reset()
        h.set_profiling(True)
        with torch.no_grad():
            outs[mode] = (gen(mel).cpu().numpy(), gen(mel, lengths=ln).cpu().numpy())
        torch.cuda.synchronize()
        h.set_profiling(False)
        names[mode] = h.profile_summary()
    n_frames = {m: sum(v["launches"] for k, v in names[m].items() if k.startswith("ups_bf16x3<"))
                for m in names}
    assert n_frames["2"] > n_frames["1"], names
    for a, b in zip(outs["1"], outs["2"]):
        assert np.array_equal(a, b), np.abs(a - b).max()


@pytest.mark.gpu
@pytest.mark.parametrize("precision", ["f16x3", "bf16x3"])
@pytest.mark.parametrize("rb_split", ["1", "0"])
@pytest.mark.parametrize("B,T,lens", [(3, 48, [48, 29, 2]),
                                      (4, 1100, [1100, 1033, 517, 1100])])
def test_conv_post_fused_bitwise(pkg, precision, rb_split, B, T, lens, sched):
    """conv_post + tanh fused into the last C = 32 ResBlock launch (resblock_bf16x3.hip
    conv_post_tail, the default wherever that stage runs one launch per ResBlock) gives the
    separate conv_post4_tanh kernel's wav bit for bit: the same final x on conv_post's
    receptive field, the same (channel, tap) fma order.  RB_CONC=0 keeps the small batch
    on that schedule; ragged batch with whole windows past an item's end (zeroed by the
    host's memset), both split and one-launch k = 11 ResBlocks; also against the oracle.
    [4, 80, 1100] (4400 batch frames >= 4096): the forward runs as two batch halves on two
    streams, each half with its own fused launch."""
    from oracle import config as C, prng
    dev = _dev()
    cfg = C.V1
    sd = C.make_state_dict(cfg, seed=53)
    mel_np = prng.mel_input(53, (B, cfg.n_mels, T))
    mel = torch.as_tensor(mel_np).to(dev)
    ln = torch.tensor(lens, dtype=torch.int32, device=dev)
    sched("RB_CONC", "0")
    sched("RB_SPLIT", rb_split)
    outs, names = {}, {}
    for mode in ("0", "1"):
        sched("FUSE_POST", mode)  # read when the handle is created
        gen = _gen(pkg, cfg, sd, dev, precision=precision)
        h = gen.hip_handle(dev)
        h.profile_reset()
        h.set_profiling(True)
        with torch.no_grad():
            outs[mode] = (gen(mel).cpu().numpy(), gen(mel, lengths=ln).cpu().numpy())
        torch.cuda.synchronize()
        h.set_profiling(False)
        names[mode] = h.profile_summary()
    assert "conv_post4_tanh" in names["0"] and "conv_post4_tanh" not in names["1"], names["1"]
    for a, b in zip(outs["0"], outs["1"]):
        assert np.array_equal(a, b), np.abs(a - b).max()
    full, rag = outs["1"]
    if T <= 48:
        assert np.abs(full - _oracle(cfg, sd, mel_np)).max() < ATOL
    else:  # oracle on a window of the longest item (its receptive field: 15 frames a side)
        a, b = 400, 460
        ref = _oracle(cfg, sd, mel_np[:1, :, a - 15:b + 15])[:, :, 15 * 256:-15 * 256]
        assert np.abs(full[:1, :, a * 256:b * 256] - ref).max() < ATOL
    for i, n in enumerate(lens):
        assert not rag[i, :, C.out_len(cfg, n):].any()


@pytest.mark.gpu
@pytest.mark.parametrize("precision", ["f16x3", "fp32"])
def test_conv_post_kernels(pkg, precision):
    """conv_post + tanh: the 4-samples-per-thread kernel where L % 4 == 0 (V1), the
    LDS-staged one otherwise (rates 5, 5: L = 25 T + 6); both against the oracle on a
    ragged batch, zero past each utterance's length.  (Round 3 proved them bitwise equal on
    the same L: the same (channel, tap) fma order per sample.)"""
    from oracle import config as C, prng
    dev = _dev()
    odd = C.GenConfig(upsample_rates=[5, 5], upsample_kernel_sizes=[10, 10],
                      upsample_initial_channel=64, resblock_kernel_sizes=[3],
                      resblock_dilation_sizes=[[1, 3]])  # L = 25 T + 6: L % 4 == 2
    for cfg, kname in ((C.V1, "conv_post4_tanh"), (odd, "conv_post_tanh")):
        sd = C.make_state_dict(cfg, seed=41)
        mel = prng.mel_input(41, (3, cfg.n_mels, 40))
        gen = _gen(pkg, cfg, sd, dev, precision=precision)
        h = gen.hip_handle(dev)
        h.profile_reset()
        h.set_profiling(True)
        with torch.no_grad():
            full = gen(torch.as_tensor(mel).to(dev)).cpu().numpy()
            rag = gen(torch.as_tensor(mel).to(dev),
                      lengths=torch.tensor([40, 17, 1], dtype=torch.int32, device=dev)).cpu().numpy()
        torch.cuda.synchronize()
        h.set_profiling(False)
        names = h.profile_summary()
        assert kname in names, sorted(names)
        ref = _oracle(cfg, sd, mel)
        assert np.abs(full - ref).max() < ATOL
        L17 = C.out_len(cfg, 17)
        assert np.abs(rag[1, :, :L17] - _oracle(cfg, sd, mel[1:2, :, :17])[0]).max() < ATOL
        assert not rag[1, :, L17:].any() and not rag[2, :, C.out_len(cfg, 1):].any()
