"""Per-dispatch durations of the last forward in a rocprofv3 --kernel-trace CSV of bench.py
(--no-profile: the forwards are the only dispatches after warm-up).  Prints position, kernel,
duration, and the gap to the previous dispatch's end on the same queue.
usage: trace_show.py DIR [n_forwards_to_show]"""
import csv
import glob
import sys

files = glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)
rows = []
for f in files:
    with open(f) as fh:
        rows += list(csv.DictReader(fh))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
# a forward starts at the absmax (f16x3 mel scale) launch
starts = [i for i, r in enumerate(rows) if r["Kernel_Name"].startswith("hfg::absmax") or
          "absmax" in r["Kernel_Name"].split("(")[0]]
nshow = int(sys.argv[2]) if len(sys.argv) > 2 else 1
for s in starts[-nshow:]:
    e = next((j for j in starts if j > s), len(rows))
    fw = rows[s:e]
    t0 = int(fw[0]["Start_Timestamp"])
    tot = int(fw[-1]["End_Timestamp"]) - t0
    print(f"forward of {len(fw)} dispatches, {tot / 1e3:.1f} us wall")
    for i, r in enumerate(fw):
        st, en = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        name = r["Kernel_Name"].replace("void hfg::", "").split("(")[0][:58]
        print(f"{i:3d} q{r.get('Queue_Id', r.get('Stream_Id', '?')):>3s} {name:58s} "
              f"{(st - t0) / 1e3:9.1f} {(en - st) / 1e3:8.1f} us")
