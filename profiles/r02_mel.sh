mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_mel.py -m gpu -v -s --timeout 120 --timeout-method thread > gpurun_out/gputest_mel.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --no-cpu-baseline --no-pmc --also --steps 5 > gpurun_out/bench_mel.json 2> gpurun_out/bench_mel.err
