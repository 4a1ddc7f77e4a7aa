"""Random Generator configurations on the GPU (the reference constructor accepts any
upsample / ResBlock lists, models/hifigan.py:149-222): seeded draws of channel width,
upsample rates and kernel sizes (exact, non-exact, k = u), ResBlock kernel sizes and
dilation lists, batch and ragged lengths.  Every configuration the C ABI accepts must
match the oracle within the north-star 1e-4 in both precisions, with each item of a
ragged batch bitwise equal to its solo run; a configuration it refuses must be refused
at handle creation with a message (never at forward time, never a wrong answer)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
ATOL = 1e-4
N_CFG = 32


def _draw(seed):
    from oracle import config as C
    r = np.random.default_rng(1000 + seed)
    n_up = int(r.integers(1, 5))
    c0 = int(r.choice([32, 64, 128, 256, 512]))
    rates, kernels = [], []
    for _ in range(n_up):
        u = int(r.choice([2, 3, 4, 5, 8]))
        k = int(r.choice([u, 2 * u, 2 * u + 1, 2 * u - 1 if u > 1 else u]))
        rates.append(u)
        kernels.append(max(k, 1))
    n_res = int(r.integers(1, 4))
    ks = [int(r.choice([3, 5, 7, 11])) for _ in range(n_res)]
    dils = [[int(d) for d in r.choice([1, 2, 3, 5], size=int(r.integers(1, 4)))] for _ in range(n_res)]
    cfg = C.GenConfig(upsample_rates=rates, upsample_kernel_sizes=kernels,
                      upsample_initial_channel=c0, resblock_kernel_sizes=ks,
                      resblock_dilation_sizes=dils)
    B = int(r.integers(1, 4))
    T = int(r.integers(3, 33))
    lens = [T] + [int(r.integers(1, T + 1)) for _ in range(B - 1)]
    return cfg, lens


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    return torch.device("cuda:0")


@pytest.mark.parametrize("seed", range(N_CFG))
def test_random_config(pkg, dev, seed):
    """fp32, f16x3 and bf16x3 against the oracle on the fp32 weights; bf16w against the oracle on
    the bf16-rounded weights (the model bf16w computes); every third configuration loads
    its weights in the apply_weight_norm layout (weight_g / weight_v)."""
    from oracle import config as C, hifigan_torch as H
    cfg, lens = _draw(seed)
    wn = seed % 3 == 2
    sd = C.make_weight_norm_state_dict(cfg, seed=seed) if wn else C.make_state_dict(cfg, seed=seed)
    # the plain weights the module folds g * v / ||v|| into (the reference's own fold)
    probe = pkg.HiFiGANGenerator(**cfg.kwargs()).eval()
    if wn:
        probe.apply_weight_norm()
    probe.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()})
    if wn:
        probe.remove_weight_norm()
    plain = {k: v.detach().numpy().copy() for k, v in probe.state_dict().items()}
    rounded = {k: (torch.from_numpy(v).to(torch.bfloat16).float().numpy() if k.endswith(".weight")
                   else v) for k, v in plain.items()}
    T = max(lens)
    mel = torch.randn(len(lens), 80, T, generator=torch.Generator().manual_seed(seed))
    refs_by = {}
    for name, w in (("fp32", plain), ("bf16", rounded)):
        refs_by[name] = [H.generator_forward(H.to_torch_state(w), cfg, mel[b:b + 1, :, :n])
                         for b, n in enumerate(lens)]
    print(f"\nseed {seed}: {cfg} lens {lens} weight_norm {wn}")
    for precision in ("fp32", "f16x3", "bf16x3", "bf16w"):
        refs = refs_by["bf16" if precision == "bf16w" else "fp32"]
        gen = pkg.HiFiGANGenerator(**cfg.kwargs(), precision=precision).eval()
        if wn:
            gen.apply_weight_norm()
        gen.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()})
        gen = gen.to(dev)
        try:
            gen.hip_handle(dev)
        except Exception as e:  # refused configurations: at creation, with a reason
            msg = str(e)
            print(f"  {precision}: refused at creation: {msg}")
            assert msg, "refusal without a message"
            continue
        with torch.no_grad():
            out = gen(mel.to(dev), lengths=lens)
            for b, n in enumerate(lens):
                solo = gen(mel[b:b + 1, :, :n].contiguous().to(dev))
                m = solo.shape[-1]
                assert m == refs[b].shape[-1]
                assert torch.equal(out[b:b + 1, :, :m], solo), (precision, b)
                err = (solo.cpu() - refs[b]).abs().max().item()
                assert err < ATOL, (precision, b, err)
        torch.cuda.synchronize()
        print(f"  {precision}: ok (max err item 0 {(out[0:1, :, :refs[0].shape[-1]].cpu() - refs[0]).abs().max().item():.1e})")
