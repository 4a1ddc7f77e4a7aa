mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_latency_paths.py -m gpu -v -s --timeout 120 --timeout-method thread > gpurun_out/gputest_small.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --batch 1 --frames 256 --no-cpu-baseline --no-pmc --also --steps 20 --streams 1 > gpurun_out/bench_c1.json 2> gpurun_out/bench_c1.err && \
timeout -k 10 300 python bench.py --batch 32 --frames 63 --no-extra --no-cpu-baseline --no-pmc --also --steps 20 --streams 1 > gpurun_out/bench_c5shape.json 2> gpurun_out/bench_c5shape.err
