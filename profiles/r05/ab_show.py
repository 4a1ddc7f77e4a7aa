"""Summarise an A/B of profiles/r05/env_ab.sh: value (M samples/s) per variant and run, and
the per-kernel ms/step of the 1-stream pass (mean over runs), f16x3 and bf16x3.
usage: python profiles/r05/ab_show.py TAG"""
import glob
import json
import os
import re
import sys
from collections import defaultdict

tag = sys.argv[1]
d = os.path.join(os.path.dirname(__file__), "..", "..", "gpurun_out", "r05", "ab")
runs = defaultdict(list)
for f in sorted(glob.glob(os.path.join(d, f"{tag}_*_[12].json"))):
    name = re.match(rf"{tag}_(.*)_[12]\.json", os.path.basename(f)).group(1)
    txt = open(f).read().strip().splitlines()
    if not txt:
        continue
    runs[name].append(json.loads(txt[-1]))
for name, rs in runs.items():
    v = [r["value"] / 1e6 for r in rs]
    vb = [r["alt"]["bf16x3"]["value"] / 1e6 for r in rs if "bf16x3" in r.get("alt", {})]
    print(f"{name:12s} f16x3 {' '.join(f'{x:.1f}' for x in v)}  bf16x3 {' '.join(f'{x:.1f}' for x in vb)}")
ks = defaultdict(dict)
for name, rs in runs.items():
    for r in rs:
        for k, kv in r.get("kernels", {}).items():
            ks[k].setdefault(name, []).append(kv["ms_per_step"])
names = list(runs)
print(f"{'kernel (f16x3 pass)':58s} " + " ".join(f"{n:>10s}" for n in names))
for k in sorted(ks, key=lambda k: -max(sum(v) / len(v) for v in ks[k].values())):
    row = ks[k]
    print(f"{k[:58]:58s} " + " ".join(
        f"{sum(row[n]) / len(row[n]):10.4f}" if n in row else f"{'-':>10s}" for n in names))
