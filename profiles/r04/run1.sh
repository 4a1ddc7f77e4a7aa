#!/bin/bash
# round 4, first f16x3 check: targeted parity tests, then a short bench A/B of the precisions
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out/r04
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_parity.py tests/test_gpu_stages.py \
  -k "golden or stage_outputs or loud or standalone or random_vs" > gpurun_out/r04/t1.log 2>&1
rc=$?
echo "pytest rc=$rc"
# 0: pass, 1: test failures -> still measure; anything else (crash, timeout) -> stop
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 python -u bench.py --precision f16x3 --also bf16x3 fp32 --no-extra \
  --no-cpu-baseline --no-pmc --steps 20 > gpurun_out/r04/b1.json 2> gpurun_out/r04/b1.err
echo "bench rc=$?"
