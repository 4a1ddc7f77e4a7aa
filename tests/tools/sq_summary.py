"""Summarise the three SQ counter passes of a final set (rocprofv3 --pmc, one pass per
directory sq1/sq2/sq3 of run_counter_collection.csv) per kernel:

  dispatches, mean duration, shader clock (GRBM_GUI_ACTIVE per XCC over the dispatch's
  timestamps: an upper bound, far off for dispatches of a few microseconds),
  MFMA busy (SQ_VALU_MFMA_BUSY_CYCLES over clock cycles x 1024 SIMDs),
  per wave-cycle fractions (SQ_WAIT_ANY, ... / SQ_WAVE_CYCLES),
  per MFMA instruction counts (SQ_INSTS_* / SQ_INSTS_MFMA), LDS bank conflicts per LDS-active.

usage: python tests/tools/sq_summary.py DIR [top_n]   (DIR holds sq1/ sq2/ sq3/)
"""
import csv
import os
import re
import sys
from collections import defaultdict

N_SIMD = 1024  # 256 CUs x 4 SIMDs
N_XCC = 8


def short(name: str) -> str:
    name = re.sub(r"^void ", "", name)
    name = re.sub(r"\(.*\)$", "", name)
    name = name.replace("hfg::", "").replace("(anonymous namespace)::", "")
    return name


def load(d):
    """{(dispatch_id, kernel): {counter: value, '_dur': ns}}"""
    rows = defaultdict(dict)
    f = os.path.join(d, "run_counter_collection.csv")
    if not os.path.exists(f):
        return rows
    with open(f) as fh:
        for r in csv.DictReader(fh):
            k = (r["Dispatch_Id"], short(r["Kernel_Name"]))
            rows[k][r["Counter_Name"]] = rows[k].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
            rows[k]["_dur"] = float(r["End_Timestamp"]) - float(r["Start_Timestamp"])
    return rows


def main():
    d = sys.argv[1]
    top = int(sys.argv[2]) if len(sys.argv) > 2 else 12
    per = defaultdict(lambda: defaultdict(float))  # kernel -> summed counters
    n = defaultdict(int)
    for sub in ("sq1", "sq2", "sq3"):
        for (did, kern), c in load(os.path.join(d, sub)).items():
            if kern.startswith("__amd"):
                continue
            for key, v in c.items():
                per[kern][sub + ":" + key] += v
            if sub == "sq1":
                n[kern] += 1
    order = sorted(per, key=lambda k: -per[k].get("sq1:_dur", 0.0))
    for kern in order[:top]:
        c = per[kern]

        def g(name):
            for sub in ("sq1", "sq2", "sq3"):
                if sub + ":" + name in c:
                    return c[sub + ":" + name]
            return float("nan")

        dur1 = c.get("sq1:_dur", 0.0)
        dur3 = c.get("sq3:_dur", 0.0)
        clock_mhz = g("GRBM_GUI_ACTIVE") / N_XCC / dur3 * 1e3 if dur3 else float("nan")
        dur2 = c.get("sq2:_dur", 0.0)
        busy = (g("SQ_VALU_MFMA_BUSY_CYCLES") / (dur2 * 1e-9 * clock_mhz * 1e6 * N_SIMD)
                if dur2 else float("nan"))
        wc = g("SQ_WAVE_CYCLES")
        mf = g("SQ_INSTS_MFMA") or float("nan")
        print(kern)
        print(f"  dispatches {n[kern]}  {dur1 / max(n[kern], 1) / 1e3:.1f} us each  clock {clock_mhz:.0f} MHz"
              f"  MFMA busy {busy:.3f}")
        print("  per wave-cycle: " + "  ".join(
            f"{k[3:]} {g(k) / wc:.3f}" for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY",
                                                 "SQ_WAIT_INST_LDS", "SQ_ACTIVE_INST_LDS",
                                                 "SQ_ACTIVE_INST_VALU")))
        print(f"  per MFMA: LDS {g('SQ_INSTS_LDS') / mf:.3f}  VALU {g('SQ_INSTS_VALU') / mf:.3f}  "
              f"VMEM {g('SQ_INSTS_VMEM') / mf:.3f}  SALU {g('SQ_INSTS_SALU') / mf:.3f}  "
              f"bank-conflict/LDS-active {g('SQ_LDS_BANK_CONFLICT') / max(g('SQ_ACTIVE_INST_LDS'), 1):.3f}")


if __name__ == "__main__":
    main()
