O=gpurun_out/s2planes; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_properties.py -m gpu -x -q -k "ups_frames or max_length or two_stream" --timeout 120 --timeout-method thread > $O/parity.txt 2>&1 || { tail -40 $O/parity.txt; exit 1; }
tail -2 $O/parity.txt
bash profiles/r03/ab_env.sh s2planes/ab "HFG_UPS_PLANES=1" "HFG_UPS_PLANES=0" --streams 1 || exit 1
export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/c2 -o run --output-format csv -- \
  python bench.py --steps 5 --warmup 2 --streams 1 --no-extra --no-cpu-baseline --no-pmc --also \
  > $O/c2_bench.json 2> $O/c2_bench.err || exit 1
echo done
