"""Where does the split-precision (bf16x3) wav error of the x4 "loud" fixtures come from?
  Runs on the GPU box:

    python tests/tools/diag_precision.py [fixture ...]  > gpurun_out/diag_precision.json

For each fixture: the HIP forward's stage taps (conv_pre, ups.i, mrfs.i) in each precision;
then, on the CPU in float64 (oracle/hifigan_np64.py building blocks), the rest of the
network is run from each tapped stage, so

    wav_err(k) = max | np64_rest(hip_stage_k) - np64_wav |

is the wav error caused by everything up to and including stage k (the stages after k in
exact arithmetic).  The increments between consecutive k attribute the final error to
stages.  Also reports the per-stage relative error against the float64 stage tensors.
Test infrastructure only (reads tests/golden and oracle/).
"""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def _f64(sd):
    from oracle import hifigan_np64 as N  # noqa: F401
    f = {k: np.asarray(v, dtype=np.float64) for k, v in sd.items()}
    for k in list(f):
        if k.endswith(".weight_g"):
            mod = k[: -len(".weight_g")]
            g, v = f.pop(k), f.pop(mod + ".weight_v")
            norm = np.sqrt((v ** 2).reshape(v.shape[0], -1).sum(1)).reshape(g.shape)
            f[mod + ".weight"] = g * v / norm
    return f


def rest_from(f, cfg, name, x):
    """float64 forward from the output of stage `name` to the wav."""
    from oracle.config import get_padding
    from oracle.hifigan_np64 import conv1d, conv_transpose1d, lrelu
    order = ["conv_pre"] + [f"{p}.{i}" for i in range(len(cfg.upsample_rates)) for p in ("ups", "mrfs")]
    pos = order.index(name)
    n_res = len(cfg.resblock_kernel_sizes)
    for nm in order[pos + 1:]:
        kind, i = nm.split(".")
        i = int(i)
        if kind == "ups":
            u, k = cfg.upsample_rates[i], cfg.upsample_kernel_sizes[i]
            x = conv_transpose1d(lrelu(x), f[f"ups.{i}.weight"], f[f"ups.{i}.bias"], u, (k - u) // 2)
        else:
            acc = 0.0
            for j, (kr, dils) in enumerate(zip(cfg.resblock_kernel_sizes,
                                               cfg.resblock_dilation_sizes)):
                xr = x
                for m, d in enumerate(dils):
                    pre = f"mrfs.{i}.resblocks.{j}"
                    xt = conv1d(lrelu(xr), f[f"{pre}.convs1.{m}.weight"],
                                f[f"{pre}.convs1.{m}.bias"], get_padding(kr, d), d)
                    xt = conv1d(lrelu(xt), f[f"{pre}.convs2.{m}.weight"],
                                f[f"{pre}.convs2.{m}.bias"], get_padding(kr, 1), 1)
                    xr = xr + xt
                acc = acc + xr
            x = acc / n_res
    pre_tanh = conv1d(lrelu(x), f["conv_post.weight"], f["conv_post.bias"], 3, 1)
    return np.tanh(pre_tanh), pre_tanh


def main():
    import __graft_entry__ as ge
    from conftest import golden_case_state, load_golden
    from oracle import hifigan_np64 as N
    pkg = ge.load_package()
    pkg.load_library()
    idx = json.load(open(os.path.join(ROOT, "tests", "golden", "golden_index.json")))
    names = sys.argv[1:] or ["g6_v1_loud2x_b1_t24", "g9_v1_loud4x_b1_t24",
                             "g10_v2star_loud4x_b1_t40"]
    dev = torch.device("cuda:0")
    out = {}
    for name in names:
        case = idx["cases"][name]
        cfg, sd = golden_case_state(case)
        g = load_golden(name)
        taps64 = {}
        wav64 = N.generator_forward(sd, cfg, g["mel"], tap=lambda n, t: taps64.__setitem__(n, t))
        f = _f64(sd)
        _, pre64 = rest_from(f, cfg, "mrfs.%d" % (len(cfg.upsample_rates) - 1),
                             taps64["mrfs.%d" % (len(cfg.upsample_rates) - 1)])
        res = {"pre_tanh_maxabs": float(np.abs(pre64).max()),
               "ref_fp32_vs_fp64": float(np.abs(g["wav"] - wav64).max())}
        for precision in ("fp32", "bf16x3"):
            gen = pkg.HiFiGANGenerator(**cfg.kwargs(), precision=precision).eval()
            if any(k.endswith("weight_g") for k in sd):
                gen.apply_weight_norm()
            gen.load_state_dict({k: torch.from_numpy(np.ascontiguousarray(v)) for k, v in sd.items()})
            gen = gen.to(dev)
            with torch.no_grad():
                wav, stages = gen.forward_with_stages(torch.from_numpy(g["mel"]).to(dev))
            torch.cuda.synchronize()
            rows = {}
            for st, t in stages.items():
                h = t.cpu().numpy().astype(np.float64)
                rel = float(np.abs(h - taps64[st]).max() / max(1.0, np.abs(taps64[st]).max()))
                w_k, p_k = rest_from(f, cfg, st, h)
                rows[st] = {"stage_rel_err": rel,
                            "wav_err_through_here": float(np.abs(w_k - wav64).max()),
                            "pre_tanh_err_through_here": float(np.abs(p_k - pre64).max())}
            rows["wav"] = {"wav_err": float(np.abs(wav.cpu().numpy() - wav64).max()),
                           "wav_err_vs_ref32": float(np.abs(wav.cpu().numpy() - g["wav"]).max())}
            res[precision] = rows
        out[name] = res
        print(json.dumps({name: res}), flush=True)


if __name__ == "__main__":
    main()
