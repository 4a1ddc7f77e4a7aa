"""Per-kernel SQ counter summary from rocprofv3 --pmc CSVs (profiles/r02_sq.sh).

usage: python profiles/parse_sq.py gpurun_out/sq/p1 gpurun_out/sq/p2

Per kernel (summed over its dispatches): duration, the counters, and derived ratios.
Normalisation (gfx950, 256 CUs x 4 SIMDs, 32 SEs): SQ_BUSY_CYCLES is summed over the
SEs, so clock = SQ_BUSY_CYCLES / 32 / duration; MFMA busy fraction =
SQ_VALU_MFMA_BUSY_CYCLES / (SIMDs x clock x duration)."""
import csv
import glob
import os
import sys
from collections import defaultdict

SIMDS = 1024
SES = 32


def load(d):
    per = defaultdict(lambda: defaultdict(float))
    dur = defaultdict(dict)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("hfg::", "")
            per[k][r["Counter_Name"]] += float(r["Counter_Value"])
            dur[k][r["Dispatch_Id"]] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    return per, {k: sum(v.values()) for k, v in dur.items()}, {k: len(v) for k, v in dur.items()}


def main():
    tot = defaultdict(dict)
    durs, ns = {}, {}
    for d in sys.argv[1:]:
        per, du, n = load(d)
        for k, v in per.items():
            tot[k].update(v)
            durs.setdefault(k, du[k])
            ns.setdefault(k, n[k])
    rows = sorted(tot, key=lambda k: -durs[k])
    for k in rows:
        c = tot[k]
        t = durs[k] * 1e-9
        clk = c.get("SQ_BUSY_CYCLES", 0) / SES / t if t else 0
        mf = c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) / (SIMDS * clk * t) if clk else 0
        wc = c.get("SQ_WAVE_CYCLES", 0)
        print(f"{k}\n  dispatches {ns[k]}  {durs[k] / ns[k] / 1e3:.1f} us each  clock {clk / 1e6:.0f} MHz  "
              f"MFMA busy {mf:.3f}")
        if wc:
            print("  per wave-cycle: " + "  ".join(
                f"{n[3:]} {c[n] / wc:.3f}" for n in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY",
                                                      "SQ_WAIT_INST_LDS", "SQ_ACTIVE_INST_LDS",
                                                      "SQ_ACTIVE_INST_VALU") if n in c))
        if c.get("SQ_INSTS_MFMA"):
            m = c["SQ_INSTS_MFMA"]
            print("  per MFMA: " + "  ".join(
                f"{n[9:]} {c[n] / m:.3f}" for n in ("SQ_INSTS_LDS", "SQ_INSTS_VALU", "SQ_INSTS_VMEM",
                                                     "SQ_INSTS_SALU") if n in c)
                  + f"  bank-conflict/LDS-active {c.get('SQ_LDS_BANK_CONFLICT', 0) / max(c.get('SQ_ACTIVE_INST_LDS', 1), 1):.3f}")


if __name__ == "__main__":
    main()
