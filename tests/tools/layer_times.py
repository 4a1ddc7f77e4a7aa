"""Per-launch kernel times of one V1 [8, 80, 1024] forward, by position in the forward.

GPU box, under rocprofv3 (the program itself after --):
    rocprofv3 --kernel-trace -d gpurun_out/lt -o run --output-format csv -- \
        python tests/tools/layer_times.py run [--precision f16x3] [--streams 1]
then here:
    python tests/tools/layer_times.py show gpurun_out/lt

`run` does 3 warm-up forwards and 8 traced ones on one stream; `show` splits the kernel
trace into forwards (the absmax launch opens each f16x3 forward; else the conv_pre launch),
and prints per position the kernel, its median duration and its algorithmic rate where the
shape is known from the launch order (V1: SURVEY.md §8(d))."""
import csv
import glob
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def run(argv):
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("--precision", default="f16x3")
    ap.add_argument("--streams", type=int, default=1)
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--frames", type=int, default=1024)
    ap.add_argument("--preset", default="v1")
    a = ap.parse_args(argv)
    sys.path.insert(0, ROOT)
    import torch
    import __graft_entry__ as ge
    pkg = ge.load_package()
    import importlib
    S = importlib.import_module(ge.PKG_NAME + ".synth")
    cfg = S.PRESETS[a.preset]
    sd = {k: torch.from_numpy(v) for k, v in S.random_state_dict(cfg, seed=0).items()}
    dev = torch.device("cuda:0")
    gen = pkg.HiFiGANGenerator(**cfg.kwargs(), precision=a.precision).eval()
    gen.load_state_dict(sd)
    h = gen.hip_handle(dev)
    B, T = a.batch, a.frames
    mel = torch.randn(B, cfg.n_mels, T, generator=torch.Generator().manual_seed(1)).to(dev)
    out_len = h.out_len(T)
    wav = torch.empty((B, 1, out_len), dtype=torch.float32, device=dev)
    h.set_streams(a.streams)
    ws_bytes = h.workspace_bytes(B, T)
    ws = torch.empty(ws_bytes, dtype=torch.uint8, device=dev)
    stream = torch.cuda.current_stream(dev)
    for i in range(11):
        h.forward_ws(mel.data_ptr(), B, T, wav.data_ptr(), out_len, ws.data_ptr(), ws_bytes,
                     stream.cuda_stream)
    torch.cuda.synchronize(dev)
    print("ok", float(wav.abs().max()))


def show(d):
    rows = []
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("hfg::", "")
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name))
    rows.sort()
    rows = [r for r in rows if "rocclr" not in r[2]]
    opener = "absmax_kernel" if any(r[2] == "absmax_kernel" for r in rows) else None
    fwds, cur = [], []
    for r in rows:
        if (opener and r[2] == opener) or (not opener and r[2].startswith("conv1d_bf16x3<7, 4")):
            if cur:
                fwds.append(cur)
            cur = []
        cur.append(r)
    if cur:
        fwds.append(cur)
    n = statistics.mode(len(f) for f in fwds)
    fwds = [f[:n] for f in fwds if len(f) >= n][3:]  # drop warm-up forwards
    tot = 0.0
    print(f"{len(fwds)} forwards of {n} launches")
    for i in range(n):
        d_us = statistics.median((f[i][1] - f[i][0]) / 1e3 for f in fwds)
        tot += d_us
        print(f"{i:3d} {d_us:9.1f} us  {fwds[0][i][2]}")
    span = statistics.median((f[-1][1] - f[0][0]) / 1e3 for f in fwds)
    print(f"sum {tot:.1f} us, first start -> last end {span:.1f} us")


if __name__ == "__main__":
    if sys.argv[1] == "run":
        run(sys.argv[2:])
    else:
        show(sys.argv[2])
