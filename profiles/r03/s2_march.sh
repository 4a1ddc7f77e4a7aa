# Marching whole-ResBlock blocks: bitwise test, ResBlock-related parity, then a same-box
# multi-variant A/B (alternated twice) of HFG_RB_NCH / HFG_RB_NCH_BLOCKS / HFG_RB64_NARROW.
O=gpurun_out/march; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_latency_paths.py -m gpu -x -q --timeout 120 --timeout-method thread -k "marching or split" > $O/test.txt 2>&1 || { tail -30 $O/test.txt; exit 1; }
tail -1 $O/test.txt
V0="HFG_RB_NCH=1"
V1="HFG_RB_NCH=2"
V2="HFG_RB_NCH=4 HFG_RB_NCH_BLOCKS=512"
V3="HFG_RB_NCH=3 HFG_RB64_NARROW=2"
V4="HFG_RB_NCH=4 HFG_RB64_NARROW=2 HFG_RB_NCH_BLOCKS=512"
for i in 1 2; do
  for v in V0 V1 V2 V3 V4; do
    env ${!v} timeout -k 10 150 python bench.py --also --no-extra --no-cpu-baseline --no-pmc --steps 20 > $O/${v}_$i.json 2>/dev/null || exit 1
  done
done
python profiles/r03/show_ab.py $O
