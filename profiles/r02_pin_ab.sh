#!/bin/bash
# same-box A/B: pinned B reads in every tap stream (new) vs HEAD (old), then parity
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/pin
bash profiles/ab_run.sh pin/ab --no-pmc &&
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gpu_parity.py tests/test_gpu_latency_paths.py tests/test_gpu_properties.py > gpurun_out/pin/pytest.log 2>&1
