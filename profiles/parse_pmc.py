"""Turn rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes into per-kernel HBM bytes.

    python profiles/parse_pmc.py <fetch counter_collection.csv> <write counter_collection.csv> \
        [bench json with "kernels"/"roofline"] > profiles/pmc_traffic.json

Corrections (MI355X_MICROARCH.md §HBM, cdna_hip_programming.md §7):
* FETCH_SIZE / WRITE_SIZE are in KiB;
* on gfx950 FETCH_SIZE reports exactly 1/2 of the bytes of a wide coalesced
  streaming read, so fetched bytes = 2 * FETCH_SIZE * 1024;
* WRITE_SIZE is exact for 16-B-per-lane streaming stores (our epilogue stores
  are 4-B per lane, uncalibrated: treat as an estimate).
Output: {kernel_label: {launches, fetch_bytes_per_launch, write_bytes_per_launch,
bytes_per_launch}} with kernel_label = the template-instance name the bench uses.
"""
import csv
import json
import re
import sys
from collections import defaultdict


def label(name: str) -> str:
    name = re.sub(r"^void\s+", "", name)
    name = re.sub(r"^hfg::", "", name)
    return re.sub(r"\(.*\)$", "", name).strip()


def read(path, counter):
    per = defaultdict(list)
    with open(path) as f:
        for row in csv.DictReader(f):
            if row["Counter_Name"] != counter:
                continue
            per[label(row["Kernel_Name"])].append(float(row["Counter_Value"]))
    return per


def main():
    fetch = read(sys.argv[1], "FETCH_SIZE")
    write = read(sys.argv[2], "WRITE_SIZE")
    out = {}
    for k in sorted(set(fetch) | set(write)):
        f = fetch.get(k, [])
        w = write.get(k, [])
        fb = 2.0 * 1024.0 * sum(f) / len(f) if f else None
        wb = 1024.0 * sum(w) / len(w) if w else None
        out[k] = {"launches": max(len(f), len(w)), "fetch_bytes_per_launch": fb,
                  "write_bytes_per_launch": wb,
                  "bytes_per_launch": (fb or 0.0) + (wb or 0.0)}
    if len(sys.argv) > 3:
        bench = json.load(open(sys.argv[3]))
        for k, v in out.items():
            kern = bench.get("kernels", {}).get(k)
            if kern:
                v["bench_ms_per_step"] = kern["ms_per_step"]
    json.dump(out, sys.stdout, indent=1)


if __name__ == "__main__":
    main()
