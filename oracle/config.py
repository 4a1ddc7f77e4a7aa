"""Generator hyper-parameters and parameter enumeration.

TEST INFRASTRUCTURE ONLY (see ``oracle/__init__.py``).

Restates the constructor ``HiFiGANGenerator.__init__`` (``models/hifigan.py:149-222``)
and ``ResBlock.__init__`` (``models/hifigan.py:34-70``) as a list of
``(state_dict key, shape, fan_in)`` in the reference's ``state_dict`` order.
"""
from __future__ import annotations

from collections import OrderedDict
from dataclasses import dataclass, field, asdict
from typing import List

import numpy as np

from . import prng


@dataclass
class GenConfig:
    n_mels: int = 80
    upsample_rates: List[int] = field(default_factory=lambda: [8, 8, 2, 2])
    upsample_kernel_sizes: List[int] = field(default_factory=lambda: [16, 16, 4, 4])
    upsample_initial_channel: int = 512
    resblock_kernel_sizes: List[int] = field(default_factory=lambda: [3, 7, 11])
    resblock_dilation_sizes: List[List[int]] = field(
        default_factory=lambda: [[1, 3, 5], [1, 3, 5], [1, 3, 5]])

    def kwargs(self):
        return asdict(self)


# model_config.yaml:48-57
V1 = GenConfig()
# pinned V2* (V2 channel width + ResBlock2 kernel/dilation lists,
# each dilation realised as a reference conv1/conv2 pair).
V2STAR = GenConfig(upsample_initial_channel=128, resblock_kernel_sizes=[3, 5, 7],
                   resblock_dilation_sizes=[[1, 2], [2, 6], [3, 12]])
# test_hifigan_integration.py:147-164: non-exact upsampling (odd k-u).
NONEXACT = GenConfig(upsample_rates=[5, 5, 4, 2], upsample_kernel_sizes=[10, 10, 8, 4])

PRESETS = {"v1": V1, "v2star": V2STAR, "nonexact": NONEXACT}


def get_padding(kernel_size: int, dilation: int = 1) -> int:
    """models/hifigan.py:21-23"""
    return int((kernel_size * dilation - dilation) / 2)


def param_specs(cfg: GenConfig):
    """[(key, shape, fan_in)] in the reference state_dict order."""
    specs = []
    c0 = cfg.upsample_initial_channel

    def conv(name, cout, cin, k):
        specs.append((name + ".weight", (cout, cin, k), cin * k))
        specs.append((name + ".bias", (cout,), cin * k))

    conv("conv_pre", c0, cfg.n_mels, 7)
    for i, (u, k) in enumerate(zip(cfg.upsample_rates, cfg.upsample_kernel_sizes)):
        cin, cout = c0 // (2 ** i), c0 // (2 ** (i + 1))
        # ConvTranspose1d weight is [C_in, C_out, k]; torch fan_in = size(1) * k
        specs.append((f"ups.{i}.weight", (cin, cout, k), cout * k))
        specs.append((f"ups.{i}.bias", (cout,), cout * k))
    for i in range(len(cfg.upsample_rates)):
        ch = c0 // (2 ** (i + 1))
        for j, (kr, dils) in enumerate(zip(cfg.resblock_kernel_sizes, cfg.resblock_dilation_sizes)):
            for m in range(len(dils)):
                conv(f"mrfs.{i}.resblocks.{j}.convs1.{m}", ch, ch, kr)
            for m in range(len(dils)):
                conv(f"mrfs.{i}.resblocks.{j}.convs2.{m}", ch, ch, kr)
    conv("conv_post", 1, c0 // (2 ** len(cfg.upsample_rates)), 7)
    return specs


def make_state_dict(cfg: GenConfig, seed: int = 0, scale: float = 1.0):
    """PRNG weights with PyTorch default-init bounds (× scale), float32 numpy."""
    sd = OrderedDict()
    for key, shape, fan_in in param_specs(cfg):
        bound = 1.0 / np.sqrt(fan_in)
        sd[key] = prng.uniform_sym(seed, key, shape, bound * scale)
    return sd


def weight_norm_keys(cfg: GenConfig):
    """Modules that ``apply_weight_norm`` wraps (models/hifigan.py:274-283):
    every ``ups`` layer and every ResBlock conv — not conv_pre / conv_post."""
    keys = [f"ups.{i}" for i in range(len(cfg.upsample_rates))]
    for i in range(len(cfg.upsample_rates)):
        for j, dils in enumerate(cfg.resblock_dilation_sizes):
            for m in range(len(dils)):
                keys.append(f"mrfs.{i}.resblocks.{j}.convs1.{m}")
                keys.append(f"mrfs.{i}.resblocks.{j}.convs2.{m}")
    return keys


def make_weight_norm_state_dict(cfg: GenConfig, seed: int = 0):
    """State dict in the ``apply_weight_norm`` layout: weight_g / weight_v for the
    wrapped modules.  ``weight_g`` = ||v|| over dims != 0 times a PRNG
    perturbation in [0.5, 1.5) so the fold g·v/||v|| is exercised."""
    base = make_state_dict(cfg, seed)
    out = OrderedDict()
    wn = set(weight_norm_keys(cfg))
    for key, val in base.items():
        mod, leaf = key.rsplit(".", 1)
        if mod in wn and leaf == "weight":
            v = val
            norm = np.sqrt((v.astype(np.float64) ** 2).reshape(v.shape[0], -1).sum(1))
            pert = 0.5 + prng.uniform01(seed, key + "#g", v.shape[0])
            g = (norm * pert).astype(np.float32).reshape((v.shape[0],) + (1,) * (v.ndim - 1))
            out[mod + ".weight_g"] = g
            out[mod + ".weight_v"] = v
        else:
            out[key] = val
    return out


def out_len(cfg: GenConfig, t: int) -> int:
    """Output length: per stage L_out = (L_in-1)*u - 2*((k-u)//2) + k."""
    length = t
    for u, k in zip(cfg.upsample_rates, cfg.upsample_kernel_sizes):
        length = (length - 1) * u - 2 * ((k - u) // 2) + k
    return length


def flops_per_frame(cfg: GenConfig):
    """Algorithmic MACs per input mel frame for an exact-upsampling config
    (SURVEY.md §8(d)); returns dict of per-layer MACs (per frame)."""
    c0 = cfg.upsample_initial_channel
    macs = {"conv_pre": cfg.n_mels * c0 * 7}
    rate = 1
    for i, (u, k) in enumerate(zip(cfg.upsample_rates, cfg.upsample_kernel_sizes)):
        cin, cout = c0 // 2 ** i, c0 // 2 ** (i + 1)
        rate *= u
        macs[f"ups.{i}"] = cin * cout * k * rate // u  # each input sample × k taps
        mrf = 0
        for kr, dils in zip(cfg.resblock_kernel_sizes, cfg.resblock_dilation_sizes):
            mrf += 2 * len(dils) * cout * cout * kr * rate
        macs[f"mrfs.{i}"] = mrf
    macs["conv_post"] = (c0 // 2 ** len(cfg.upsample_rates)) * 7 * rate
    return macs
