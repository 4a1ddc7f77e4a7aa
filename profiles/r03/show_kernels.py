"""Per-kernel ms/step of bench.py JSON lines (the 1-stream profiled pass), side by side.
usage: python profiles/r03/show_kernels.py a.json b.json ..."""
import json
import sys

runs = []
for f in sys.argv[1:]:
    d = json.loads(open(f).read().strip().splitlines()[-1])
    runs.append((f.split("/")[-1].replace(".json", ""), d))
names = []
for _, d in runs:
    for k, v in d["kernels"].items():
        if k not in names and v["ms_per_step"] > 0.05:
            names.append(k)
print(f"{'kernel':58s}" + "".join(f"{n[:10]:>11s}" for n, _ in runs))
print(f"{'value ms/step':58s}" + "".join(f"{d['ms_per_step']:11.3f}" for _, d in runs))
for k in names:
    print(f"{k.split('(')[0][:58]:58s}" + "".join(
        f"{d['kernels'].get(k, {}).get('ms_per_step', 0):11.3f}" for _, d in runs))
