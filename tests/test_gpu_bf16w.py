"""bf16 weight storage (HFG_DTYPE_BF16W) on the GPU.

bf16w rounds every conv weight to bf16 when the weights are committed; activations are
still split hi + lo (the f16x3 format: power-of-two-scaled f16 halves), so the kernels run
hi(w)*hi(x) + hi(w)*lo(x) — the NP = 2 instances of the f16x3 kernels, which skip the
lo(w)*hi(x) MFMA (a bf16 value's 8 significant bits fit f16's 11, so lo(w) = 0).  Two checks:

* against the oracle run on the bf16-rounded weights at the north-star 1e-4 (the model
  bf16w computes is the reference Generator with bf16-cast weights, not the fp32 one);
* bitwise against the f16x3 path fed the same pre-rounded weights: there every skipped
  MFMA adds exactly 0 to the accumulator, so dropping it cannot change a bit.
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


def _round_weights(sd):
    return {k: (torch.from_numpy(v).to(torch.bfloat16).float() if k.endswith(".weight")
                else torch.from_numpy(v)) for k, v in sd.items()}


def _gen(pkg, cfg, state, dev, precision):
    gen = pkg.HiFiGANGenerator(**cfg.kwargs(), precision=precision).eval()
    gen.load_state_dict(state)
    return gen.to(dev)


@pytest.mark.parametrize("preset,B,T,lens", [("v1", 2, 120, [120, 77]), ("v1", 1, 48, None),
                                              ("v2star", 3, 64, [64, 31, 50]),
                                              ("nonexact", 2, 40, None)])
def test_bf16w_vs_oracle_and_f16x3(pkg, dev, preset, B, T, lens):
    from oracle import config as C, hifigan_torch as H
    cfg = C.PRESETS[preset]
    sd = C.make_state_dict(cfg, seed=51)
    mel = torch.randn(B, 80, T, generator=torch.Generator().manual_seed(T + B))
    kw = {} if lens is None else {"lengths": lens}
    fp32_state = {k: torch.from_numpy(v) for k, v in sd.items()}
    rounded = _round_weights(sd)
    with torch.no_grad():
        w = _gen(pkg, cfg, fp32_state, dev, "bf16w")(mel.to(dev), **kw)
        x3 = _gen(pkg, cfg, rounded, dev, "f16x3")(mel.to(dev), **kw)
    torch.cuda.synchronize()
    assert torch.equal(w, x3), (w - x3).abs().max().item()
    ref = H.generator_forward(rounded, cfg, mel)
    if lens is None:
        err = (w.cpu() - ref).abs().max().item()
    else:
        err = max((w[b, :, :C.out_len(cfg, n)].cpu()
                   - H.generator_forward(rounded, cfg, mel[b:b + 1, :, :n])[0]).abs().max().item()
                  for b, n in enumerate(lens))
    drift = (ref - H.generator_forward(fp32_state, cfg, mel)).abs().max().item()
    print(f"\n{preset} [{B},80,{T}] bf16w vs bf16-weight oracle {err:.2e} "
          f"(bf16 weights vs fp32 weights: {drift:.2e})")
    assert err < ATOL


def test_bf16w_module_parameters_untouched(pkg, dev):
    """Rounding happens in the handle's copy: the module's parameters stay fp32."""
    from oracle import config as C
    cfg = C.V2STAR
    sd = C.make_state_dict(cfg, seed=52)
    gen = _gen(pkg, cfg, {k: torch.from_numpy(v) for k, v in sd.items()}, dev, "bf16w")
    with torch.no_grad():
        gen(torch.randn(1, 80, 16, device=dev))
    torch.cuda.synchronize()
    w = gen.state_dict()["conv_pre.weight"].cpu()
    assert torch.equal(w, torch.from_numpy(sd["conv_pre.weight"]))
