"""C1 latency (V1, mel [1, 80, 256]) of the drop-in module: eager and hipGraph replay, median
of 5 rounds of 20 forwards, plus the wav checksum (same-box library A/Bs, round 6).
usage: python profiles/r06/c1_time.py [precision] [frames] [batch] [KNOB=VALUE ...]
(schedule overrides, hfg_debug_schedule_set, applied before the handle is created)"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
import __graft_entry__ as ge  # noqa: E402
import importlib  # noqa: E402

pkg = ge.load_package()
S = importlib.import_module(ge.PKG_NAME + ".synth")
prec = sys.argv[1] if len(sys.argv) > 1 else "f16x3"
T = int(sys.argv[2]) if len(sys.argv) > 2 else 256
B = int(sys.argv[3]) if len(sys.argv) > 3 else 1
dev = torch.device("cuda:0")
cfg = S.PRESETS["v1"]
sd = {k: torch.from_numpy(v) for k, v in S.random_state_dict(cfg, seed=0).items()}
knobs = [a.split("=") for a in sys.argv[4:]]
for k, v in knobs:
    pkg.schedule_override(k, int(v))
gen = pkg.HiFiGANGenerator(**cfg.kwargs(), precision=prec).eval()
gen.load_state_dict(sd)
gen = gen.to(dev)
gen.hip_handle(dev)
pkg.schedule_clear()
mel = torch.randn(B, 80, T, generator=torch.Generator().manual_seed(1234)).to(dev)


def timed(fn, n=20):
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    torch.cuda.synchronize(dev)
    return (time.perf_counter() - t0) / n


with torch.no_grad():
    for _ in range(5):
        gen(mel)
    eager = sorted(timed(lambda: gen(mel)) for _ in range(5))[2]
    s = torch.cuda.Stream(dev)
    s.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(s):
        for _ in range(2):
            gen(mel)
    torch.cuda.current_stream(dev).wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        wav = gen(mel)
    g.replay()
    graph = sorted(timed(g.replay) for _ in range(5))[2]
    ref = gen(mel)
    torch.cuda.synchronize(dev)
    ck = int(pkg._lib.checksum32([ref])[0]) & 0xffffffff
print(f"{prec} B={B} T={T} {' '.join(sys.argv[4:])} eager {eager * 1e3:.3f} ms graph {graph * 1e3:.3f} ms "
      f"graph==eager {bool(torch.equal(wav, ref))} sum {ck:08x}")
