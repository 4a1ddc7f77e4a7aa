mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_latency_paths.py tests/test_gpu_parity.py tests/test_gpu_properties.py -m gpu -x -v -s --timeout 120 --timeout-method thread > gpurun_out/gputest_ups.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --no-extra --no-cpu-baseline --also > gpurun_out/bench_ups.json 2> gpurun_out/bench_ups.err
