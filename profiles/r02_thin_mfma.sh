mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_stages.py tests/test_gpu_parity.py tests/test_gpu_latency_paths.py -m gpu -v -s --timeout 120 --timeout-method thread -k "v2star or V2 or g3 or g8 or g10 or c4" > gpurun_out/gputest_thinm.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --preset v2star --batch 16 --frames 2048 --no-extra --no-cpu-baseline --also --steps 10 > gpurun_out/bench_c4_thinm.json 2> gpurun_out/bench_c4_thinm.err
