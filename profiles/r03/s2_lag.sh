# Two-stream split with the second half trailing by N launches (HFG_SPLIT_LAG): bitwise
# check against the one-stream forward, then a same-box env A/B of the value pass (GPU box)
O=gpurun_out/lag; mkdir -p $O
HFG_SPLIT_LAG=10 timeout -k 10 300 python -u -m pytest tests/test_gpu_properties.py -m gpu -x -q --timeout 120 --timeout-method thread -k "split or stream" > $O/test.txt 2>&1 || { tail -30 $O/test.txt; exit 1; }
tail -1 $O/test.txt
V0="HFG_SPLIT_LAG=0"
V1="HFG_SPLIT_LAG=5"
V2="HFG_SPLIT_LAG=10"
V3="HFG_SPLIT_LAG=20"
for i in 1 2 3; do
  for v in V0 V1 V2 V3; do
    env ${!v} timeout -k 10 150 python bench.py --no-extra --no-cpu-baseline --no-pmc --steps 20 > $O/${v}_$i.json 2>/dev/null || exit 1
  done
done
python - <<'PY'
import json,glob,os
for f in sorted(glob.glob('gpurun_out/lag/V*.json')):
    d=json.loads(open(f).read().strip().splitlines()[-1]); print(os.path.basename(f), round(d['ms_per_step'],3), round(d['value']/1e6,1))
PY
