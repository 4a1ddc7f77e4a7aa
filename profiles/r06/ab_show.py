"""One line per bench JSON: value, ms/step, wav checksum, and the per-kernel-class ms of the
1-stream pass (layer convs, whole ResBlocks, upsamplers, rest).  usage: ab_show.py FILE..."""
import json
import sys

for f in sys.argv[1:]:
    try:
        d = [json.loads(l) for l in open(f) if l.startswith("{")][-1]
    except (IndexError, OSError, ValueError) as e:
        print(f, "no line", e)
        continue
    cls = {"conv": 0.0, "rb": 0.0, "ups": 0.0, "other": 0.0}
    for k, v in d.get("kernels", {}).items():
        c = ("rb" if k.startswith("resblock") else "ups" if k.startswith("ups") or "true" in k.split(",")[7:8]
             else "conv" if k.startswith("conv1d") else "other")
        cls[c] += v["ms_per_step"]
    rf = d.get("roofline", {})
    print(f"{f.split('/')[-1]:28s} {d['value'] / 1e6:7.2f} M/s {d['ms_per_step']:7.3f} ms "
          f"sum {d.get('wav_checksum32')} | conv {cls['conv']:.3f} rb {cls['rb']:.3f} "
          f"ups {cls['ups']:.3f} other {cls['other']:.3f} | dom {rf.get('achieved', 0):.0f} TF")
