"""PyTorch-CPU fp32 restatement of ``HiFiGANGenerator.forward``.

TEST INFRASTRUCTURE ONLY (see ``oracle/__init__.py``): the large-shape parity
oracle and the CPU baseline (``cpu_baseline.kind = "port"``) on the GPU box.

It issues exactly the ATen op sequence of the reference module tree:

* ``conv_pre``  ``nn.Conv1d(n_mels, C0, 7, padding=3)``        models/hifigan.py:177-183, 238
* per stage i   ``F.leaky_relu(x, 0.1)``                       models/hifigan.py:244
                ``nn.ConvTranspose1d(stride=u, padding=(k-u)//2)`` models/hifigan.py:195-203, 245
                ``MRF.forward``: mean over ResBlocks            models/hifigan.py:116-131
                ``ResBlock.forward``: x += conv2(lrelu(conv1_d(lrelu(x))))  models/hifigan.py:72-86
* ``F.leaky_relu`` → ``conv_post`` ``Conv1d(C, 1, 7, padding=3)`` → ``tanh``  models/hifigan.py:254-256

``nn.Conv1d.forward`` is ``F.conv1d(x, w, b, stride, padding, dilation, groups)``
and ``nn.ConvTranspose1d.forward`` is ``F.conv_transpose1d(x, w, b, stride,
padding, output_padding=0, groups, dilation)``, so with the same weights this
is bitwise identical to the reference on the same thread count
(checked against the committed fixtures by ``tests/test_oracle.py``).
"""
from __future__ import annotations

from typing import Callable, Dict, Optional

import numpy as np
import torch
import torch.nn.functional as F

from .config import GenConfig, get_padding

LRELU_SLOPE = 0.1


def to_torch_state(sd) -> Dict[str, torch.Tensor]:
    """numpy/torch state dict → fp32 CPU tensors; folds weight_g/weight_v
    exactly as torch's weight_norm hook does (``torch._weight_norm(v, g, 0)``,
    the computation ``nn.utils.weight_norm`` installs, models/hifigan.py:274-283)."""
    out = {}
    for k, v in sd.items():
        out[k] = torch.as_tensor(np.asarray(v) if not isinstance(v, torch.Tensor) else v).float()
    for k in list(out.keys()):
        if k.endswith(".weight_g"):
            mod = k[: -len(".weight_g")]
            g, v = out.pop(k), out.pop(mod + ".weight_v")
            out[mod + ".weight"] = torch._weight_norm(v, g, 0)
    return out


@torch.no_grad()
def generator_forward(sd: Dict[str, torch.Tensor], cfg: GenConfig, mel: torch.Tensor,
                      tap: Optional[Callable[[str, torch.Tensor], None]] = None) -> torch.Tensor:
    """mel f32[B, n_mels, T] → wav f32[B, 1, L].  ``tap(name, tensor)`` receives
    the per-stage tensors (conv_pre, ups.i, mrfs.i, wav)."""
    x = F.conv1d(mel, sd["conv_pre.weight"], sd["conv_pre.bias"], 1, 3, 1, 1)
    if tap:
        tap("conv_pre", x)
    n_res = len(cfg.resblock_kernel_sizes)
    for i, (u, k) in enumerate(zip(cfg.upsample_rates, cfg.upsample_kernel_sizes)):
        x = F.leaky_relu(x, LRELU_SLOPE)
        x = F.conv_transpose1d(x, sd[f"ups.{i}.weight"], sd[f"ups.{i}.bias"], u, (k - u) // 2, 0, 1, 1)
        if tap:
            tap(f"ups.{i}", x)
        output = None
        for j, (kr, dils) in enumerate(zip(cfg.resblock_kernel_sizes, cfg.resblock_dilation_sizes)):
            xr = x
            for m, d in enumerate(dils):
                pre = f"mrfs.{i}.resblocks.{j}"
                xt = F.leaky_relu(xr, LRELU_SLOPE)
                xt = F.conv1d(xt, sd[f"{pre}.convs1.{m}.weight"], sd[f"{pre}.convs1.{m}.bias"],
                              1, get_padding(kr, d), d, 1)
                xt = F.leaky_relu(xt, LRELU_SLOPE)
                xt = F.conv1d(xt, sd[f"{pre}.convs2.{m}.weight"], sd[f"{pre}.convs2.{m}.bias"],
                              1, get_padding(kr, 1), 1, 1)
                xr = xr + xt
            output = xr if output is None else output + xr
        x = output / n_res
        if tap:
            tap(f"mrfs.{i}", x)
    x = F.leaky_relu(x, LRELU_SLOPE)
    wav = F.conv1d(x, sd["conv_post.weight"], sd["conv_post.bias"], 1, 3, 1, 1)
    wav = torch.tanh(wav)
    if tap:
        tap("wav", wav)
    return wav
