mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_stages.py tests/test_gpu_parity.py tests/test_gpu_latency_paths.py -m gpu -v -s --timeout 120 --timeout-method thread -k "v2star or V2 or g3 or g8 or g10 or c4" > gpurun_out/gputest_thinm.log 2>&1 || exit 1
for m in 1 0 -1; do
HFG_THIN_MFMA=$m timeout -k 10 300 python bench.py --preset v2star --batch 16 --frames 2048 --no-extra --no-cpu-baseline --no-pmc --also --steps 10 > gpurun_out/bench_c4_tm$m.json 2>/dev/null || exit 1
done
