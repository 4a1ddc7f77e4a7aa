#!/bin/bash
# round 4: f16x3 after the epilogue-fused unscale, DPP wave max, cheaper amax: GPU suites
# that name f16x3 (output kept: -s), then the bench A/B
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out/r04
timeout -k 10 1000 python -u -m pytest -v -s --timeout 300 --timeout-method thread \
  tests/test_gpu_parity.py tests/test_gpu_stages.py tests/test_gpu_latency_paths.py \
  tests/test_gpu_bf16w.py tests/test_gpu_configs.py tests/test_gpu_glue.py > gpurun_out/r04/t3.log 2>&1
rc=$?
echo "pytest rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 python -u bench.py --precision f16x3 --also bf16x3 --no-extra \
  --no-cpu-baseline --no-pmc --steps 20 > gpurun_out/r04/b3.json 2> gpurun_out/r04/b3.err
echo "bench rc=$?"
