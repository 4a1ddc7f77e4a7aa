#!/bin/bash
# round 4: f16x3 (spread scale slots, exact-column block scales): probe f16 vs bf16 MFMA
# rate, the parity / bitwise suites that name f16x3, then a bench A/B of the precisions
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out/r04
timeout -k 10 120 python -u tests/tools/probe_rates.py > gpurun_out/r04/probe2.json 2> gpurun_out/r04/probe2.err
rc=$?; echo "probe rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 900 python -u -m pytest -v --timeout 300 --timeout-method thread \
  tests/test_gpu_parity.py tests/test_gpu_stages.py tests/test_gpu_latency_paths.py \
  tests/test_gpu_bf16w.py tests/test_gpu_dist.py > gpurun_out/r04/t2.log 2>&1
rc=$?
echo "pytest rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 python -u bench.py --precision f16x3 --also bf16x3 fp32 --no-extra \
  --no-cpu-baseline --no-pmc --steps 20 > gpurun_out/r04/b2.json 2> gpurun_out/r04/b2.err
echo "bench rc=$?"
