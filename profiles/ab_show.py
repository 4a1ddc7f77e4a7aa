"""Print the A/B runs of profiles/ab_run.sh: ms/step and per-kernel ms.  usage: python profiles/ab_show.py TAG"""
import json
import sys

tag = sys.argv[1] if len(sys.argv) > 1 else "ab"
for f in ("new1", "old1", "new2", "old2"):
    d = json.loads(open(f"gpurun_out/{tag}_{f}.json").read().strip().splitlines()[-1])
    ks = {k.split("(")[0][:34]: round(v["ms_per_step"], 3) for k, v in d["kernels"].items()
          if v["ms_per_step"] > 0.1}
    print(f, round(d["ms_per_step"], 3), ks)
