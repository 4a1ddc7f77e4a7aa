"""Small-batch launch paths on the GPU (VERDICT r01 "small-batch latency").

A split-precision layer launch whose tile-3 grid would leave most CUs idle runs on the 64x64
small-grid tile (kernels.h, tile 4; schedule knob SMALL_TILE: -1 auto / 0 never / 1 always).  Every
output element sees the same MFMA sequence on either tile, so the choice must be bitwise
invisible: forced-small, forced-big and auto forwards are compared with torch.equal,
and against the oracle at the north-star 1e-4.
"""
import pytest
import torch

pytestmark = pytest.mark.gpu
ATOL = 1e-4


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    return torch.device("cuda:0")


def _gen(pkg, cfg, sd, dev, precision, knobs):
    """A module whose handle is created under the schedule overrides `knobs`
    (hfg_debug_schedule_set; read when the handle is created, dropped right after)."""
    try:
        for k, v in knobs.items():
            pkg.schedule_override(k, int(v))
        gen = pkg.HiFiGANGenerator(**cfg.kwargs(), precision=precision).eval()
        gen.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()})
        gen = gen.to(dev)
        gen.hip_handle(dev)
    finally:
        pkg.schedule_clear()
    return gen


@pytest.mark.parametrize("precision", ["f16x3", "bf16x3"])
@pytest.mark.parametrize("preset,B,T", [("v1", 1, 96), ("v1", 3, 40), ("v2star", 2, 64), ("v1", 2, 300)])
def test_small_tile_is_bitwise_invisible(pkg, dev, preset, B, T, precision):
    from oracle import config as C, hifigan_torch as H
    cfg = C.PRESETS[preset]
    sd = C.make_state_dict(cfg, seed=31)
    mel = torch.randn(B, 80, T, generator=torch.Generator().manual_seed(B * T))
    outs = {}
    for mode in ("0", "1", "-1"):
        gen = _gen(pkg, cfg, sd, dev, precision, {"SMALL_TILE": mode})
        with torch.no_grad():
            outs[mode] = gen(mel.to(dev))
        torch.cuda.synchronize()
    assert torch.equal(outs["0"], outs["1"])
    assert torch.equal(outs["0"], outs["-1"])
    ref = H.generator_forward(H.to_torch_state(sd), cfg, mel)
    err = (outs["1"].cpu() - ref).abs().max().item()
    print(f"\n{preset} [{B},80,{T}] small tile vs oracle {err:.2e}")
    assert err < ATOL


def test_small_tile_ragged_and_streaming(pkg, dev):
    """Ragged batch (small grids on the short items' stages) equals solo runs bitwise."""
    from oracle import config as C
    cfg = C.V1
    sd = C.make_state_dict(cfg, seed=32)
    gen = _gen(pkg, cfg, sd, dev, "f16x3", {"SMALL_TILE": "-1"})
    lens = [40, 7, 33]
    mel = torch.randn(3, 80, 40, generator=torch.Generator().manual_seed(5))
    with torch.no_grad():
        wav = gen(mel.to(dev), lengths=lens)
        for b, n in enumerate(lens):
            solo = gen(mel[b:b + 1, :, :n].contiguous().to(dev))
            assert torch.equal(wav[b:b + 1, :, :n * 256], solo), b


@pytest.mark.parametrize("precision", ["f16x3", "bf16x3", "fp32"])
@pytest.mark.parametrize("preset,B,T", [("v1", 1, 96), ("v1", 4, 50), ("v2star", 2, 64)])
def test_concurrent_resblocks_are_bitwise_invisible(pkg, dev, precision, preset, B, T):
    """RB_CONC: the ResBlocks of an MRF on concurrent streams, each into its own
    output, and one combine launch ((o_0 + o_1) + o_2) / 3 — the sequential epilogue's
    running sum in the same order, so the wav is bitwise unchanged."""
    from oracle import config as C
    cfg = C.PRESETS[preset]
    sd = C.make_state_dict(cfg, seed=33)
    mel = torch.randn(B, 80, T, generator=torch.Generator().manual_seed(T))
    outs = {}
    for mode in ("0", "1", "-1"):
        gen = _gen(pkg, cfg, sd, dev, precision, {"RB_CONC": mode})
        with torch.no_grad():
            outs[mode] = gen(mel.to(dev), lengths=[T - 3 * b for b in range(B)])
        torch.cuda.synchronize()
    assert torch.equal(outs["0"], outs["1"])
    assert torch.equal(outs["0"], outs["-1"])


def test_concurrent_resblocks_hipgraph(pkg, dev):
    """A captured hipGraph of a small forward (concurrent ResBlocks: fork / join events on
    the capture stream) replays to the eager result."""
    from oracle import config as C
    cfg = C.V1
    sd = C.make_state_dict(cfg, seed=34)
    gen = _gen(pkg, cfg, sd, dev, "f16x3", {"RB_CONC": "1"})
    gen.verify_weights = False
    mel = torch.randn(1, 80, 64, generator=torch.Generator().manual_seed(2)).to(dev)
    with torch.no_grad():
        eager = gen(mel)
        s = torch.cuda.Stream(dev)
        s.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(s):
            gen(mel)
        torch.cuda.current_stream(dev).wait_stream(s)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            out = gen(mel)
        g.replay()
        torch.cuda.synchronize()
    assert torch.equal(out, eager)


@pytest.mark.parametrize("precision", ["fp32", "f16x3", "bf16x3"])
@pytest.mark.parametrize("preset", ["nonexact", "v1"])
def test_ragged_batch_with_concurrent_resblocks_equals_solo(pkg, dev, preset, precision):
    """A ragged batch whose stage lengths are not multiples of 4 (non-exact upsampling:
    5T + 1) through the concurrent-ResBlock schedule (small grids) and its mrf_combine
    launch: every item bitwise equal to the utterance run alone.  (mrf_combine once
    skipped a whole 4-sample group on its first sample's column, losing the next channel
    row's first samples.)"""
    from oracle import config as C
    cfg = C.PRESETS[preset]
    sd = C.make_state_dict(cfg, seed=38)
    mel = torch.randn(3, 80, 77, generator=torch.Generator().manual_seed(14))
    lens = [77, 60, 33]
    gen = _gen(pkg, cfg, sd, dev, precision, {"RB_CONC": "1"})
    with torch.no_grad():
        out = gen(mel.to(dev), lengths=lens)
        for b, n in enumerate(lens):
            solo = gen(mel[b:b + 1, :, :n].to(dev))
            m = solo.shape[-1]
            assert torch.equal(out[b:b + 1, :, :m], solo), (b, n)
            assert not torch.any(out[b, :, m:]), (b, n)  # zero past the item's length
    torch.cuda.synchronize()


@pytest.mark.parametrize("precision", ["bf16x3", "f16x3", "bf16w"])
@pytest.mark.parametrize("preset", ["v1", "nonexact"])
def test_split_resblock_is_bitwise_invisible(pkg, dev, preset, precision):
    """RB_SPLIT=1 (default): a whole-ResBlock launch whose halo recompute the split cuts
    by >= 10 % (k = 11 at C = 32 / 64 in V1) runs as two launches — dilation pairs {1, 3}
    writing x to scratch, then {5} with the MRF epilogue — each window paying only its own
    halo.  The fp32 round trip of x is exact, so the bf16x3 wav is bitwise unchanged (ragged
    batch, and the standalone MRF / ResBlock entry points through the same path).  f16x3 /
    bf16w scale each operand by its block's largest |value|, and the second launch's windows
    differ: only values whose f16 lo half falls below the normal range (< 2^-17 of the
    window's max) can round differently, so the two schedules agree to ~1e-9 of the wav."""
    from oracle import config as C
    cfg = C.PRESETS[preset]
    sd = C.make_state_dict(cfg, seed=40)
    mel = torch.randn(3, 80, 150, generator=torch.Generator().manual_seed(16))
    outs = {}
    for mode in ("0", "1"):
        gen = _gen(pkg, cfg, sd, dev, precision, {"RB_SPLIT": mode, "RB_CONC": "0"})
        conc = _gen(pkg, cfg, sd, dev, precision, {"RB_SPLIT": mode, "RB_CONC": "1"})
        with torch.no_grad():
            outs[mode] = gen(mel.to(dev), lengths=[150, 97, 31])
            outs[mode + "c"] = conc(mel[:1].to(dev))  # concurrent ResBlocks, per-part scratch
        torch.cuda.synchronize()
    if precision == "bf16x3":
        assert torch.equal(outs["0"], outs["1"])
        assert torch.equal(outs["0c"], outs["1c"])
    else:
        for k in ("", "c"):
            d = (outs["0" + k] - outs["1" + k]).abs().max().item()
            print(f"\n{preset} [{precision}] split vs one launch{' (conc)' if k else ''}: {d:.2e}")
            assert d <= 1e-7


@pytest.mark.parametrize("precision", ["f16x3", "bf16x3", "bf16w"])
@pytest.mark.parametrize("preset,B,T,lens", [("v1", 4, 1100, [1100, 513, 3, 1050]),
                                             ("v1", 1, 3000, None),
                                             ("nonexact", 3, 300, [300, 211, 97])])
def test_persistent_resblock_grid_bitwise(pkg, dev, preset, B, T, lens, precision):
    """RB_PERSIST (2, the default: a grid of n_CU blocks; 1: n_CU / stream halves): the C = 64
    ResBlock launches with the 512-column window (one block per CU) run as a persistent grid that walks the windows and copies
    each window's x to LDS beside the previous window's MRF round trip.  Every window's
    arithmetic is the one-window-per-block kernel's, so the wav is bitwise unchanged: ragged
    batches (windows past an item's end skipped), one long item (many windows per block),
    1 and 2 streams; and within 1e-4 of the oracle."""
    from oracle import config as C, hifigan_torch as H
    cfg = C.PRESETS[preset]
    sd = C.make_state_dict(cfg, seed=57)
    mel = torch.randn(B, 80, T, generator=torch.Generator().manual_seed(T + B))
    outs, names = {}, {}
    for mode in ("0", "1", "2"):  # 2: a grid of every CU per half-batch stream
        gen = _gen(pkg, cfg, sd, dev, precision, {"RB_PERSIST": mode, "RB_CONC": "0"})
        h = gen.hip_handle(dev)
        for n in (1, 2):
            h.set_streams(n)
            h.profile_reset()
            h.set_profiling(True)
            with torch.no_grad():
                outs[mode, n] = gen(mel.to(dev), lengths=lens)
            torch.cuda.synchronize()
            h.set_profiling(False)
            names[mode, n] = h.profile_summary()
    assert any("persist" in k for k in names["1", 1]), names["1", 1]
    assert not any("persist" in k for k in names["0", 1])
    for n in (1, 2):
        for m in ("1", "2"):
            assert torch.equal(outs["0", n], outs[m, n]), (m, n, (outs["0", n] - outs[m, n]).abs().max())
    if precision != "bf16w":
        b = 0
        n = T if lens is None else lens[0]
        a, e = min(200, n // 2), min(200, n // 2) + 40
        ref = H.generator_forward(H.to_torch_state(sd), cfg, mel[b:b + 1, :, max(0, a - 15):e + 15])
        hop = C.out_len(cfg, 2) - C.out_len(cfg, 1)
        off = (a - max(0, a - 15)) * hop
        if C.out_len(cfg, 7) == 7 * hop:
            got = outs["1", 1][b:b + 1, :, a * hop:e * hop].cpu()
            assert (got - ref[:, :, off:off + (e - a) * hop]).abs().max().item() < ATOL



@pytest.mark.parametrize("precision", ["f16x3", "bf16x3"])
@pytest.mark.parametrize("rb_split", ["1", "0"])
def test_persistent_grid_with_concurrent_resblocks_bitwise(pkg, dev, precision, rb_split):
    """The production default (persistent C = 64 grids, RB_PERSIST=2) combined with the
    concurrent-ResBlock schedule (RB_CONC=1: each ResBlock on its own stream with per-part
    scratch) and with / without split k = 11 ResBlocks (RB_SPLIT; part 0 writes scratch in
    plain-store mode): bitwise the non-persistent kernel on a one-item batch."""
    from oracle import config as C
    cfg = C.V1
    sd = C.make_state_dict(cfg, seed=58)
    mel = torch.randn(1, 80, 700, generator=torch.Generator().manual_seed(701))
    outs, names = {}, {}
    for mode in ("0", "2"):
        gen = _gen(pkg, cfg, sd, dev, precision,
                   {"RB_PERSIST": mode, "RB_CONC": "1", "RB_SPLIT": rb_split})
        h = gen.hip_handle(dev)
        h.profile_reset()
        h.set_profiling(True)
        with torch.no_grad():
            outs[mode] = gen(mel.to(dev))
        torch.cuda.synchronize()
        h.set_profiling(False)
        names[mode] = h.profile_summary()
    assert any("persist" in k for k in names["2"]), names["2"]
    assert not any("persist" in k for k in names["0"])
    assert any("mrf_combine" in k for k in names["2"]), names["2"]  # the concurrent schedule ran
    assert torch.equal(outs["0"], outs["2"]), (outs["0"] - outs["2"]).abs().max()


@pytest.mark.parametrize("precision", ["f16x3", "bf16x3", "bf16w"])
def test_tall_areg_tile_bitwise(pkg, dev, precision):
    """The 256x128 AREG tile (6: the 256-row stage-0 layer convs of V1, round 6) against tile 5
    (schedule knob AREG_TALL=0): every output element sees the same MFMA sequence (channel groups
    x taps in order, lo*hi, hi*lo, hi*hi), so the wav is bitwise the same — full and ragged
    batches, two streams included."""
    from oracle import config as C
    cfg = C.V1
    sd = C.make_state_dict(cfg, seed=61)
    # 8 items x 1100 frames: each batch-half stream's stage-0 grid (4 x 69 column tiles of 128)
    # stays above the small-grid threshold, so the layer convs run on tiles 6 / 5
    mel = torch.randn(8, 80, 1100, generator=torch.Generator().manual_seed(62))
    lens = [1100, 517, 3, 1034, 1100, 1100, 800, 1099]
    outs, names = {}, {}
    for mode in ("0", "1"):
        gen = _gen(pkg, cfg, sd, dev, precision, {"AREG_TALL": mode})
        h = gen.hip_handle(dev)
        h.profile_reset()
        h.set_profiling(True)
        with torch.no_grad():
            outs[mode] = (gen(mel.to(dev)), gen(mel.to(dev), lengths=lens))
        torch.cuda.synchronize()
        h.set_profiling(False)
        names[mode] = h.profile_summary()
    tall = [k for k in names["1"] if k.startswith("conv1d_bf16x3<") and ", 4, 1, 2, 4, 2," in k]
    assert tall, names["1"]
    assert not any(", 4, 1, 2, 4, 2," in k for k in names["0"])
    for a, b in zip(outs["0"], outs["1"]):
        assert torch.equal(a, b), (a - b).abs().max()


@pytest.mark.parametrize("precision", ["f16x3", "fp32"])
def test_four_resblocks_concurrent_combine(pkg, dev, precision):
    """An MRF of four ResBlocks (the reference constructor takes any list,
    models/hifigan.py:178-190) through the concurrent schedule: mrf_combine's general
    operand path (more than three outputs) and a caller's-stream ResBlock that is not the
    last one (the one with the largest kernel size x dilation count, here k = 7 x 3).
    Bitwise the sequential schedule, ragged items bitwise their solo runs, and the oracle
    within 1e-4."""
    from oracle import config as C, hifigan_torch as H
    cfg = C.GenConfig(upsample_rates=[4, 4], upsample_kernel_sizes=[8, 8],
                      upsample_initial_channel=128, resblock_kernel_sizes=[3, 5, 7, 11],
                      resblock_dilation_sizes=[[1, 3], [1, 2], [1, 3, 5], [1]])
    sd = C.make_state_dict(cfg, seed=41)
    lens = [50, 37]
    mel = torch.randn(2, 80, 50, generator=torch.Generator().manual_seed(41))
    outs = {}
    for mode in ("0", "1"):
        gen = _gen(pkg, cfg, sd, dev, precision, {"RB_CONC": mode})
        with torch.no_grad():
            outs[mode] = gen(mel.to(dev), lengths=lens)
            if mode == "1":
                for b, n in enumerate(lens):
                    solo = gen(mel[b:b + 1, :, :n].contiguous().to(dev))
                    assert torch.equal(outs[mode][b:b + 1, :, :solo.shape[-1]], solo), b
        torch.cuda.synchronize()
    assert torch.equal(outs["0"], outs["1"])
    err = 0.0
    for b, n in enumerate(lens):
        ref = H.generator_forward(H.to_torch_state(sd), cfg, mel[b:b + 1, :, :n])
        err = max(err, (outs["1"][b:b + 1, :, :ref.shape[-1]].cpu() - ref).abs().max().item())
    print(f"\nfour ResBlocks [{precision}] concurrent vs oracle {err:.2e}")
    assert err < ATOL
