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
    from oracle import config as C, hifigan_torch as H
    cfg, lens = _draw(seed)
    sd = C.make_state_dict(cfg, seed=seed)
    T = max(lens)
    mel = torch.randn(len(lens), 80, T, generator=torch.Generator().manual_seed(seed))
    refs = [H.generator_forward(H.to_torch_state(sd), cfg, mel[b:b + 1, :, :n])
            for b, n in enumerate(lens)]
    print(f"\nseed {seed}: {cfg} lens {lens}")
    for precision in ("fp32", "bf16x3"):
        gen = pkg.HiFiGANGenerator(**cfg.kwargs(), precision=precision).eval()
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
