"""Print same-box A/B bench runs: python profiles/r03/show_ab.py DIR (files NAME_i.json)."""
import glob
import json
import os
import sys

d = sys.argv[1]
runs = {}
for f in sorted(glob.glob(os.path.join(d, "*.json"))):
    t = open(f).read().strip().splitlines()
    if t:
        runs[os.path.basename(f)[:-5]] = json.loads(t[-1])
names = sorted({k for r in runs.values() for k in r["kernels"]},
               key=lambda k: -max(r["kernels"].get(k, {"ms_per_step": 0})["ms_per_step"] for r in runs.values()))
print(f"{'kernel':60s}" + "".join(f"{n:>12s}" for n in runs))
print(f"{'value ms/step':60s}" + "".join(f"{r['ms_per_step']:12.3f}" for r in runs.values()))
for k in names:
    print(f"{k.split('(')[0][:60]:60s}" + "".join(
        f"{r['kernels'][k]['ms_per_step']:12.3f}" if k in r["kernels"] else f"{'-':>12s}"
        for r in runs.values()))
