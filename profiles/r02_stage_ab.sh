#!/bin/bash
# AREG straight-line staging (half planes, folded pad/lrelu factors): parity first, then
# same-box A/B against the HEAD build
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/stg
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gpu_latency_paths.py tests/test_gpu_parity.py tests/test_gpu_properties.py > gpurun_out/stg/pytest.log 2>&1 &&
bash profiles/ab_run.sh stg/ab
