# fp32 path: LDS-staged epilogue A/B (HFG_EPI_LDS) + bitwise check
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_latency_paths.py -m gpu -q -x --timeout 120 --timeout-method thread -k "epilogue" > gpurun_out/gputest_epi.log 2>&1 || exit 1
for i in 1 2; do for m in 0 1; do
HFG_EPI_LDS=$m timeout -k 10 300 python bench.py --precision fp32 --no-extra --no-cpu-baseline --no-pmc --also > gpurun_out/bench_epi32_${m}_$i.json 2>/dev/null || exit 1
done; done
