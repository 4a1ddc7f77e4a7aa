O=gpurun_out/s2ups2; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "ups_frames or two_stream" --timeout 120 --timeout-method thread > $O/parity.txt 2>&1 || { tail -40 $O/parity.txt; exit 1; }
tail -2 $O/parity.txt
bash profiles/r03/ab_libs.sh s2ups2/ab pair1 pair0 || exit 1
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/c2 -o run --output-format csv -- \
  python bench.py --steps 5 --warmup 2 --streams 1 --no-extra --no-cpu-baseline --no-pmc --also \
  > $O/c2_bench.json 2> $O/c2_bench.err || exit 1
echo done
