# (1) split-halves stagger A/B (value pass, 2 streams): HFG_SPLIT_STAGGER = 0 (off), 2, 5, 8, 20
# (2) C1 small-grid tile on / off (legs.py c1, eager module forward)
O=gpurun_out/s2stag; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "ups_frames" --timeout 120 --timeout-method thread > $O/parity.txt 2>&1 || { tail -40 $O/parity.txt; exit 1; }
tail -2 $O/parity.txt
for i in 1 2; do
  for n in 0 2 5 8 20; do
    HFG_SPLIT_STAGGER=$n timeout -k 10 150 python bench.py --also --no-extra --no-cpu-baseline --no-pmc --no-profile --steps 30 > $O/st${n}_$i.json 2>/dev/null || exit 1
  done
done
for i in 1 2 3; do
  for st in -1 0; do
    r=$(HFG_SMALL_TILE=$st timeout -k 10 120 python profiles/r03/legs.py c1 2>/dev/null | tail -1) || exit 1
    echo "$i small_tile=$st $r" >> $O/c1_small_tile.txt
  done
done
cat $O/c1_small_tile.txt
echo done
