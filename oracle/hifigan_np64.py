"""Independent numpy float64 restatement of ``HiFiGANGenerator.forward``.

TEST INFRASTRUCTURE ONLY (see ``oracle/__init__.py``).  For small shapes only
(seconds at V1 [1, 80, 32]).  Written from the layer definitions, not from
ATen: Conv1d as a sum of shifted tap-matrix products over a zero-padded input,
ConvTranspose1d as an explicit scatter-add ``y[t*u - p + j] += W[:, :, j]^T x[t]``.

models/hifigan.py:21-23 (get_padding), :72-86 (ResBlock), :116-131 (MRF mean),
:224-261 (Generator.forward).
"""
from __future__ import annotations

import numpy as np

from .config import GenConfig, get_padding


def lrelu(x, slope=0.1):
    return np.where(x >= 0, x, x * slope)


def conv1d(x, w, b, pad, dil):
    """x [B, Cin, L], w [Cout, Cin, k] → [B, Cout, L + 2 pad - dil (k-1)]"""
    bsz, cin, length = x.shape
    cout, _, k = w.shape
    xp = np.zeros((bsz, cin, length + 2 * pad), dtype=np.float64)
    xp[:, :, pad:pad + length] = x
    lout = length + 2 * pad - dil * (k - 1)
    y = np.zeros((bsz, cout, lout), dtype=np.float64)
    for j in range(k):
        y += np.einsum("oc,bct->bot", w[:, :, j], xp[:, :, j * dil: j * dil + lout])
    return y + b[None, :, None]


def conv_transpose1d(x, w, b, stride, pad):
    """x [B, Cin, L], w [Cin, Cout, k] → [B, Cout, (L-1) s - 2 p + k]"""
    bsz, cin, length = x.shape
    _, cout, k = w.shape
    full = (length - 1) * stride + k
    y = np.zeros((bsz, cout, full), dtype=np.float64)
    for j in range(k):
        contrib = np.einsum("co,bct->bot", w[:, :, j], x)  # [B, Cout, L]
        y[:, :, j: j + (length - 1) * stride + 1: stride] += contrib
    lout = full - 2 * pad
    return y[:, :, pad: pad + lout] + b[None, :, None]


def generator_forward(sd, cfg: GenConfig, mel, tap=None):
    """float64 forward; ``tap(name, array)`` sees conv_pre / ups.i / mrfs.i like
    oracle.hifigan_torch.generator_forward."""
    tap = tap or (lambda name, t: None)
    f = {k: np.asarray(v, dtype=np.float64) for k, v in sd.items()}
    for k in list(f):
        if k.endswith(".weight_g"):
            mod = k[: -len(".weight_g")]
            g, v = f.pop(k), f.pop(mod + ".weight_v")
            norm = np.sqrt((v ** 2).reshape(v.shape[0], -1).sum(1)).reshape(g.shape)
            f[mod + ".weight"] = g * v / norm
    x = conv1d(np.asarray(mel, np.float64), f["conv_pre.weight"], f["conv_pre.bias"], 3, 1)
    tap("conv_pre", x)
    n_res = len(cfg.resblock_kernel_sizes)
    for i, (u, k) in enumerate(zip(cfg.upsample_rates, cfg.upsample_kernel_sizes)):
        x = conv_transpose1d(lrelu(x), f[f"ups.{i}.weight"], f[f"ups.{i}.bias"], u, (k - u) // 2)
        tap(f"ups.{i}", x)
        acc = 0.0
        for j, (kr, dils) in enumerate(zip(cfg.resblock_kernel_sizes, cfg.resblock_dilation_sizes)):
            xr = x
            for m, d in enumerate(dils):
                pre = f"mrfs.{i}.resblocks.{j}"
                xt = conv1d(lrelu(xr), f[f"{pre}.convs1.{m}.weight"], f[f"{pre}.convs1.{m}.bias"],
                            get_padding(kr, d), d)
                xt = conv1d(lrelu(xt), f[f"{pre}.convs2.{m}.weight"], f[f"{pre}.convs2.{m}.bias"],
                            get_padding(kr, 1), 1)
                xr = xr + xt
            acc = acc + xr
        x = acc / n_res
        tap(f"mrfs.{i}", x)
    wav = conv1d(lrelu(x), f["conv_post.weight"], f["conv_post.bias"], 3, 1)
    return np.tanh(wav)
