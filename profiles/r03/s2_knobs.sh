# Value-pass (2 streams) sweep of the schedule knobs chosen on 1-stream data (GPU box)
O=gpurun_out/knobs; mkdir -p $O
V0="HFG_NONE=0"
V1="HFG_RB64_NARROW=0"
V2="HFG_RB_WN32=8"
V3="HFG_RB_SPLIT=0"
V4="HFG_UPS_SWIZZLE=0"
V5="HFG_RB_SPLIT_MIN=0.95"
for i in 1 2 3; do
  for v in V0 V1 V2 V3 V4 V5; do
    env ${!v} timeout -k 10 150 python bench.py --no-extra --no-cpu-baseline --no-pmc --steps 20 > $O/${v}_$i.json 2>/dev/null || exit 1
  done
done
python - <<'PY'
import json,glob,os
for f in sorted(glob.glob('gpurun_out/knobs/V*.json')):
    d=json.loads(open(f).read().strip().splitlines()[-1]); print(os.path.basename(f), round(d['ms_per_step'],3), round(d['value']/1e6,1))
PY
