"""Trained-checkpoint loading for the drop-in Generator.

The reference has no checkpoint I/O of its own (tasks.md:315): its Generator is built
by ``HiFiGANGenerator.__init__`` (models/hifigan.py:149-222) and optionally wrapped in
weight norm by ``apply_weight_norm`` (:274-283).  This module maps the state-dict
layouts a HiFi-GAN vocoder checkpoint comes in onto this package's
``HiFiGANGenerator`` keys (which are the reference's):

* the reference Generator's own ``state_dict`` (plain or weight-normed ``weight_g`` /
  ``weight_v``) — passed through;
* the reference ``HiFiGAN`` wrapper (models/hifigan.py:618-800): ``generator.*`` keys,
  ``msd.*`` / ``mpd.*`` discriminator keys dropped;
* the public HiFi-GAN release layout (jik876/hifi-gan ``generator_v1`` files:
  ``{"generator": sd}``, weight-normed ``conv_pre`` / ``conv_post``, ResBlocks indexed
  flat as ``resblocks.{stage * num_kernels + j}``) — remapped to
  ``mrfs.{stage}.resblocks.{j}`` and its ``conv_pre`` / ``conv_post`` weight norm
  folded (the reference applies none there);
* container dicts ``{"generator" | "state_dict" | "model" | "model_state_dict": sd}``
  and DistributedDataParallel ``module.`` prefixes.

Weight norm is folded with ``torch._weight_norm(v, g, 0)`` — the op the reference's
``weight_norm`` hook runs — so the folded weights are bitwise those the reference
computes at forward time.  Files are read with ``torch.load(weights_only=True)``
(nothing in the file is executed).
"""
from __future__ import annotations

import re
from typing import Dict, Mapping, Optional, Tuple, Union

import torch

_CONTAINER_KEYS = ("generator", "state_dict", "model", "model_state_dict")


def _unwrap(obj) -> Dict[str, torch.Tensor]:
    """The tensor mapping inside a checkpoint.  Known container keys win over the
    "mostly tensors" heuristic, so ``{"state_dict": sd, "step": tensor, "ema": tensor}``
    unwraps to ``sd`` rather than returning the stray tensors."""
    if isinstance(obj, Mapping):
        for key in _CONTAINER_KEYS:
            if key in obj and isinstance(obj[key], Mapping):
                return _unwrap(obj[key])
        tensors = {k: v for k, v in obj.items() if isinstance(v, torch.Tensor)}
        if tensors and len(tensors) >= len(obj) // 2:
            return dict(tensors)
    raise ValueError("no state dict found in the checkpoint (expected a tensor mapping or one of "
                     f"{_CONTAINER_KEYS})")


def fold_weight_norm(sd: Dict[str, torch.Tensor], modules=None) -> Dict[str, torch.Tensor]:
    """Replace every ``<m>.weight_g`` / ``<m>.weight_v`` pair (or only those of ``modules``)
    by ``<m>.weight = torch._weight_norm(v, g, 0)``."""
    out = dict(sd)
    for k in [k for k in sd if k.endswith(".weight_g")]:
        mod = k[: -len(".weight_g")]
        if modules is not None and mod not in modules:
            continue
        v = out.pop(mod + ".weight_v")
        g = out.pop(k)
        out[mod + ".weight"] = torch._weight_norm(v.float(), g.float(), 0)
    return out


def convert_state_dict(obj, num_kernels: int, num_upsamples: int,
                       weight_normed: bool = False) -> Dict[str, torch.Tensor]:
    """Any supported layout → this package's HiFiGANGenerator keys.

    weight_normed: keep ``weight_g`` / ``weight_v`` of the modules the reference
    weight-normalises (ups, ResBlock convs) for a Generator on which
    ``apply_weight_norm()`` was called; otherwise every pair is folded."""
    sd = _unwrap(obj)
    strip = re.compile(r"^(module\.)+")
    sd = {strip.sub("", k): v for k, v in sd.items()}
    if any(k.startswith("generator.") for k in sd):
        # a DDP-wrapped generator inside the wrapper: generator.module.conv_pre.weight
        sd = {strip.sub("", k[len("generator."):]): v for k, v in sd.items()
              if k.startswith("generator.")}
    sd = {k: v for k, v in sd.items() if not k.startswith(("msd.", "mpd."))}
    flat = re.compile(r"^resblocks\.(\d+)\.(.*)$")
    out = {}
    for k, v in sd.items():
        m = flat.match(k)
        if m:  # public-release layout: resblocks.{i * num_kernels + j}
            n = int(m.group(1))
            i, j = divmod(n, num_kernels)
            if i >= num_upsamples:
                raise ValueError(f"{k}: ResBlock index {n} beyond {num_upsamples} stages x "
                                 f"{num_kernels} kernels")
            k = f"mrfs.{i}.resblocks.{j}.{m.group(2)}"
        out[k] = v
    # conv_pre / conv_post carry no weight norm in the reference Generator (:177-183,
    # :216-222): fold it there always; elsewhere unless the target keeps it
    out = fold_weight_norm(out, modules={"conv_pre", "conv_post"})
    if not weight_normed:
        out = fold_weight_norm(out)
    return out


def load_generator_checkpoint(gen, src: Union[str, Mapping], strict: bool = True,
                              map_location: Optional[str] = "cpu"):
    """Load a checkpoint file (``torch.load(..., weights_only=True)``) or mapping into
    ``gen`` (this package's HiFiGANGenerator, or its HiFiGAN wrapper).  Returns the
    ``load_state_dict`` result."""
    target = getattr(gen, "generator", gen)
    obj = torch.load(src, map_location=map_location, weights_only=True) if isinstance(src, str) \
        else src
    wn = any(k.endswith(".weight_g") for k in target.state_dict())
    sd = convert_state_dict(obj, target.num_kernels, target.num_upsamples, weight_normed=wn)
    return target.load_state_dict(sd, strict=strict)
