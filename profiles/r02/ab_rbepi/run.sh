# whole-ResBlock LDS-staged MRF epilogue: bitwise checks + same-box A/B (HFG_EPI_LDS toggles
# both epilogues; the layer one was A/B'd alone in profiles/r02/ab_epi)
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_latency_paths.py tests/test_gpu_parity.py tests/test_gpu_stages.py -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/gputest_rbepi.log 2>&1 || exit 1
for i in 1 2; do for m in 0 1; do
HFG_EPI_LDS=$m timeout -k 10 300 python bench.py --no-extra --no-cpu-baseline --no-pmc --also > gpurun_out/bench_rbepi${m}_$i.json 2>/dev/null || exit 1
done; done
