#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/areg
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gpu_properties.py tests/test_gpu_latency_paths.py > gpurun_out/areg/pytest2.log 2>&1 &&
HFG_AREG=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gpu_properties.py tests/test_gpu_parity.py tests/test_gpu_configs.py > gpurun_out/areg/pytest3.log 2>&1
