# ups.2 (64 rows per class) / ups.1 (512) on the 32-row tile: bitwise tests + same-box env A/B
O=gpurun_out/smallrows; mkdir -p $O
HFG_UPS_SMALL_ROWS=512 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "ups_frames" > $O/test.txt 2>&1 || { tail -30 $O/test.txt; exit 1; }
tail -1 $O/test.txt
V0="HFG_UPS_SMALL_ROWS=0"
V1="HFG_UPS_SMALL_ROWS=64"
V2="HFG_UPS_SMALL_ROWS=512"
for i in 1 2 3; do
  for v in V0 V1 V2; do
    env ${!v} timeout -k 10 150 python bench.py --also --no-extra --no-cpu-baseline --no-pmc --steps 20 --streams 1 > $O/${v}_$i.json 2>/dev/null || exit 1
  done
done
python profiles/r03/show_ab.py $O
