# same-box A/B of the upsampler changes (XCD swizzle, trailing-column launch)
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_latency_paths.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gputest_ups.log 2>&1 || exit 1
for i in 1 2; do
HFG_UPS_SWIZZLE=0 HFG_SMALL_TILE=0 timeout -k 10 300 python bench.py --no-extra --no-cpu-baseline --no-pmc --also > gpurun_out/bench_ups_off_$i.json 2>/dev/null || exit 1
HFG_SMALL_TILE=0 timeout -k 10 300 python bench.py --no-extra --no-cpu-baseline --no-pmc --also > gpurun_out/bench_ups_swz_$i.json 2>/dev/null || exit 1
timeout -k 10 300 python bench.py --no-extra --no-cpu-baseline --no-pmc --also > gpurun_out/bench_ups_on_$i.json 2>/dev/null || exit 1
done
