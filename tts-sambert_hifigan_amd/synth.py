"""Synthetic workload of the benchmark (BASELINE.json configs 2-5).

No trained checkpoint ships with the reference, so ``bench.py``
runs random-init weights of the named architecture: every parameter drawn from
U(-1/sqrt(fan_in), 1/sqrt(fan_in)), PyTorch's default Conv1d / ConvTranspose1d init
bound (fan_in = size(1) * k, ``models/hifigan.py:177-222``).  Values do not affect
the speed of the path.  This module is product-side (the tests' weight generator
lives under ``oracle/`` and is the checker's, not the benchmark's).
"""
from __future__ import annotations

import zlib
from collections import OrderedDict
from dataclasses import asdict, dataclass, field
from typing import Dict, List, Tuple

import numpy as np


@dataclass
class GenConfig:
    """``HiFiGANGenerator`` constructor arguments (``models/hifigan.py:149-158``)."""
    n_mels: int = 80
    upsample_rates: List[int] = field(default_factory=lambda: [8, 8, 2, 2])
    upsample_kernel_sizes: List[int] = field(default_factory=lambda: [16, 16, 4, 4])
    upsample_initial_channel: int = 512
    resblock_kernel_sizes: List[int] = field(default_factory=lambda: [3, 7, 11])
    resblock_dilation_sizes: List[List[int]] = field(
        default_factory=lambda: [[1, 3, 5], [1, 3, 5], [1, 3, 5]])

    def kwargs(self) -> Dict:
        return asdict(self)


# model_config.yaml:48-57
V1 = GenConfig()
# pinned V2* (V2 width, ResBlock2 kernel / dilation lists)
V2STAR = GenConfig(upsample_initial_channel=128, resblock_kernel_sizes=[3, 5, 7],
                   resblock_dilation_sizes=[[1, 2], [2, 6], [3, 12]])
# test_hifigan_integration.py:147-164: non-exact upsampling (odd k - u)
NONEXACT = GenConfig(upsample_rates=[5, 5, 4, 2], upsample_kernel_sizes=[10, 10, 8, 4])
PRESETS = {"v1": V1, "v2star": V2STAR, "nonexact": NONEXACT}


def param_specs(cfg: GenConfig) -> List[Tuple[str, Tuple[int, ...], int]]:
    """[(state_dict key, shape, fan_in)] in the reference's state_dict order."""
    specs = []
    c0 = cfg.upsample_initial_channel

    def conv(name, cout, cin, k):
        specs.append((name + ".weight", (cout, cin, k), cin * k))
        specs.append((name + ".bias", (cout,), cin * k))

    conv("conv_pre", c0, cfg.n_mels, 7)
    for i, k in enumerate(cfg.upsample_kernel_sizes):
        cin, cout = c0 >> i, c0 >> (i + 1)
        specs.append((f"ups.{i}.weight", (cin, cout, k), cout * k))  # [C_in, C_out, k]
        specs.append((f"ups.{i}.bias", (cout,), cout * k))
    for i in range(len(cfg.upsample_rates)):
        ch = c0 >> (i + 1)
        for j, (kr, dils) in enumerate(zip(cfg.resblock_kernel_sizes,
                                           cfg.resblock_dilation_sizes)):
            for which in ("convs1", "convs2"):
                for m in range(len(dils)):
                    conv(f"mrfs.{i}.resblocks.{j}.{which}.{m}", ch, ch, kr)
    conv("conv_post", 1, c0 >> len(cfg.upsample_rates), 7)
    return specs


def random_state_dict(cfg: GenConfig, seed: int = 0) -> "OrderedDict[str, np.ndarray]":
    """float32 weights with PyTorch's default-init bound, one keyed stream per tensor
    (independent of the order in which tensors are drawn)."""
    sd = OrderedDict()
    for key, shape, fan_in in param_specs(cfg):
        rng = np.random.default_rng([seed, zlib.crc32(key.encode())])
        bound = 1.0 / np.sqrt(fan_in)
        sd[key] = rng.uniform(-bound, bound, size=shape).astype(np.float32)
    return sd


def layer_streaming_bytes_per_frame(cfg: GenConfig) -> int:
    """SURVEY.md §8(d) canonical byte model, fp32, per mel frame: every conv reads its
    input once and writes its output once, each ResBlock conv2 also reads the residual,
    the MRF sum adds (n_res - 1) * 2 passes over C*L, activations / tanh / mean are
    fused.  Weights (once per forward) are added by the caller.  V1: 5,436,736 B."""
    c0 = cfg.upsample_initial_channel
    floats = cfg.n_mels + c0                               # conv_pre in + out
    rate = 1
    c_prev = c0
    n_res = len(cfg.resblock_kernel_sizes)
    pairs = sum(len(d) for d in cfg.resblock_dilation_sizes)
    for i, u in enumerate(cfg.upsample_rates):
        c = c0 >> (i + 1)
        floats += c_prev * rate                            # ups in
        rate *= u
        floats += c * rate                                 # ups out
        floats += (5 * pairs + 2 * (n_res - 1)) * c * rate  # MRF
        c_prev = c
    floats += c_prev * rate + rate                         # conv_post in + out
    return 4 * floats


def param_bytes(cfg: GenConfig) -> int:
    return 4 * sum(int(np.prod(s)) for _, s, _ in param_specs(cfg))
