"""Per-dispatch time and algorithmic TF/s of the V1 C2 forward ([8, 80, 1024], 1 stream) from a
rocprofv3 --kernel-trace CSV of bench.py --streams 1 --no-profile (mean over the traced forwards;
a forward = the absmax launch + its 44 conv / upsampler / ResBlock launches).
usage: trace_tf.py TRACE_DIR"""
import csv
import glob
import sys

import numpy as np

rows = []
for f in glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True):
    rows += list(csv.DictReader(open(f)))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
st = [i for i, r in enumerate(rows) if "absmax" in r["Kernel_Name"]]
fws = [rows[s:s + 45] for s in st if len(rows[s:s + 45]) == 45]
B, T = 8, 1024
L = [T * 8, T * 64, T * 128, T * 256]


def conv(ci, co, k, l):
    return 2.0 * ci * co * k * l * B


fl = {1: conv(80, 512, 7, T), 2: conv(512, 256, 16, T), 21: conv(256, 128, 16, L[0]),
      35: conv(128, 64, 4, L[1]), 40: conv(64, 32, 4, L[2])}
i = 3
for k in (3, 7, 11):
    for _ in range(6):
        fl[i] = conv(256, 256, k, L[0])
        i += 1
fl[22] = 6 * conv(128, 128, 3, L[1])
i = 23
for k in (7, 11):
    for _ in range(6):
        fl[i] = conv(128, 128, k, L[1])
        i += 1
for base, c, l in ((36, 64, L[2]), (41, 32, L[3])):
    fl[base] = 6 * conv(c, c, 3, l)
    fl[base + 1] = 6 * conv(c, c, 7, l)
    fl[base + 2] = 4 * conv(c, c, 11, l)
    fl[base + 3] = 2 * conv(c, c, 11, l)
fl[44] += 2.0 * 32 * 7 * L[3] * B  # conv_post fused into the last launch
dur = np.array([[int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in fw] for fw in fws]).mean(0) / 1e3
names = [r["Kernel_Name"].replace("void hfg::", "").split("(")[0] for r in fws[-1]]
print(f"{len(fws)} forwards; per-dispatch mean")
for j, (n, d) in enumerate(zip(names, dur)):
    f = fl.get(j, 0.0)
    print(f"{j:3d} {n[:54]:54s} {d:8.1f} us {f / 1e9:7.1f} GF {f / (d * 1e-6) / 1e12 if f else 0:5.0f} TF/s")
print(f"sum {dur.sum():.1f} us, {sum(fl.values()) / 1e12:.3f} TFLOP")
