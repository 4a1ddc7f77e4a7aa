# FETCH_SIZE / WRITE_SIZE calibration per access width (profiles/pmc_calib.hip).
# build here:   hipcc --offload-arch=gfx950 -O3 profiles/pmc_calib.hip -o profiles/pmc_calib
# on the box:   bash profiles/pmc_calib.sh   (writes gpurun_out/pmc_calib.json)
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
rm -rf $R/gpurun_out/calib_fetch $R/gpurun_out/calib_write
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE -d $R/gpurun_out/calib_fetch -o run --output-format csv -- $R/profiles/pmc_calib > $R/gpurun_out/calib_fetch.log 2>&1 && \
timeout -s KILL 60 rocprofv3 --pmc WRITE_SIZE -d $R/gpurun_out/calib_write -o run --output-format csv -- $R/profiles/pmc_calib > $R/gpurun_out/calib_write.log 2>&1 && \
python3 - "$R" <<'EOF'
import csv, glob, json, sys
from collections import defaultdict
R = sys.argv[1]
known = 1 << 30
out = {}
for counter, d in (("FETCH_SIZE", "calib_fetch"), ("WRITE_SIZE", "calib_write")):
    per = defaultdict(list)
    for p in glob.glob(f"{R}/gpurun_out/{d}/**/*counter_collection.csv", recursive=True):
        for row in csv.DictReader(open(p)):
            if row["Counter_Name"] == counter:
                per[row["Kernel_Name"].split("(")[0]].append(float(row["Counter_Value"]))
    for k, v in per.items():
        out.setdefault(k, {})[counter] = {"kib_per_launch": v, "counter_bytes_over_known":
                                          [x * 1024 / known for x in v]}
json.dump(out, open(f"{R}/gpurun_out/pmc_calib.json", "w"), indent=1)
print(json.dumps(out, indent=1))
EOF
