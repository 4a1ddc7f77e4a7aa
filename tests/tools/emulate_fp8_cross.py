"""CPU emulation (float64 accumulation) of candidate split-precision product schemes for
the Generator's convs, against the exact float64 forward — sizing the error of a
cheaper scheme before building it.  Research script (not product, not a test).

  bf16     : bf16(x) * bf16(w)
  bf16x3   : hi*hi + hi*lo + lo*hi in bf16 (the shipped scheme)
  fp8x     : bf16 hi*hi + the two cross terms in fp8 e4m3 with an E8M0 scale per
             32 K-elements (what v_mfma_scale_f32_32x32x64_f8f6f4 would compute)
  fp8x_lo  : bf16 hi*hi + hi*lo in bf16 + lo(x)*hi(w) in fp8 (cross term of the
             activations only in fp8)

usage: python tests/tools/emulate_fp8_cross.py
"""
import os
import sys
import types

import numpy as np
import torch
import torch.nn.functional as F

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..")
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from oracle import config as C, hifigan_torch as H  # noqa: E402
from conftest import golden_case_state, load_golden  # noqa: E402
import json  # noqa: E402


def bf(v):
    return v.to(torch.bfloat16).double()


def q8(v, dim):
    """e4m3 with a power-of-two scale per block of 32 along `dim` (the K index)."""
    v = v.movedim(dim, -1)
    n = v.shape[-1]
    pad = (-n) % 32
    vp = F.pad(v, (0, pad)) if pad else v
    blk = vp.reshape(*vp.shape[:-1], -1, 32)
    amax = blk.abs().amax(-1, keepdim=True).clamp_min(1e-300)
    s = torch.exp2(torch.ceil(torch.log2(amax / 448.0)))
    q = (blk / s).float().to(torch.float8_e4m3fn).double() * s
    q = q.reshape(vp.shape)[..., :n]
    return q.movedim(-1, dim)


def make_shim(scheme):
    def split(v):
        h = bf(v)
        return h, bf(v - h)

    def products(x, w, conv, wdim):
        x = x.double()
        w = w.double()
        if scheme == "exact":
            return conv(x, w)
        if scheme == "bf16":
            return conv(bf(x), bf(w))
        hx, lx = split(x)
        hw, lw = split(w)
        if scheme == "bf16x3":
            return conv(hx, hw) + conv(hx, lw) + conv(lx, hw)
        if scheme == "fp8x":
            return conv(hx, hw) + conv(q8(hx, 1), q8(lw, wdim)) + conv(q8(lx, 1), q8(hw, wdim))
        if scheme == "fp8x_lo":
            return conv(hx, hw) + conv(hx, lw) + conv(q8(lx, 1), q8(hw, wdim))
        raise ValueError(scheme)

    def conv1d(x, w, b, stride, padding, dilation, groups):
        y = products(x, w, lambda a, c: F.conv1d(a, c, None, stride, padding, dilation, groups), 1)
        return y + b.double()[None, :, None]

    def conv_transpose1d(x, w, b, stride, padding, output_padding, groups, dilation):
        y = products(x, w, lambda a, c: F.conv_transpose1d(a, c, None, stride, padding,
                                                          output_padding, groups, dilation), 0)
        return y + b.double()[None, :, None]

    return types.SimpleNamespace(conv1d=conv1d, conv_transpose1d=conv_transpose1d,
                                 leaky_relu=F.leaky_relu)


def run(scheme, sd, cfg, mel):
    saved = H.F
    H.F = make_shim(scheme)
    try:
        sd64 = {k: v.double() for k, v in sd.items()}
        return H.generator_forward(sd64, cfg, mel.double()).numpy()
    finally:
        H.F = saved


def main():
    torch.set_num_threads(8)
    idx = json.load(open(os.path.join(ROOT, "tests", "golden", "golden_index.json")))
    cases = []
    for name in ["g1_v1_b1_t32", "g6_v1_loud2x_b1_t24", "g3_v2star_b2_t32"]:
        cfg, sd = golden_case_state(idx["cases"][name])
        cases.append((name, cfg, H.to_torch_state(sd), torch.from_numpy(load_golden(name)["mel"])))
    from oracle import prng
    sd = H.to_torch_state(C.make_state_dict(C.V1, seed=5))
    cases.append(("v1_rand_t64", C.V1, sd, torch.from_numpy(prng.mel_input(9, (1, 80, 64)))))
    for name, cfg, sd, mel in cases:
        ref = run("exact", sd, cfg, mel)
        row = {}
        for scheme in ["bf16", "bf16x3", "fp8x", "fp8x_lo"]:
            row[scheme] = float(np.abs(run(scheme, sd, cfg, mel) - ref).max())
        print(name, {k: f"{v:.2e}" for k, v in row.items()}, flush=True)


if __name__ == "__main__":
    main()
