O=gpurun_out/s2ups6; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "ups_frames" --timeout 120 --timeout-method thread > $O/parity.txt 2>&1 || { tail -40 $O/parity.txt; exit 1; }
tail -2 $O/parity.txt
for i in 1 2; do
  for f in "256 256" "512 256" "256 512" "512 512"; do
    set -- $f
    HFG_UPS_NT=$1 HFG_UPS_NT2=$2 timeout -k 10 150 python bench.py --also --no-extra --no-cpu-baseline --no-pmc --steps 20 --streams 1 > $O/nt$1_$2_$i.json 2>/dev/null || exit 1
  done
done
echo done
