#!/bin/bash
# round 5, call 10: the fused conv_post tail over all four waves — bitwise / parity tests, then
# a same-box A/B against the previous commit's library (ab/prev.so)
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out/r05
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread \
  tests/test_gpu_parity.py tests/test_gpu_stages.py tests/test_gpu_configs.py \
  -k "conv_post or golden or stage or loud or C5 or C3" > gpurun_out/r05/t10.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r05/t10.log
if [ $rc -ne 0 ]; then exit $rc; fi
bash profiles/r05/lib_ab.sh post4w prev
