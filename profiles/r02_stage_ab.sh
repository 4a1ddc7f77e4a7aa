#!/bin/bash
# tile-5 A/B runner: parity (latency-path, parity and property GPU tests), then a same-box A/B against
# the HEAD build (profiles/ab_build.sh).  usage: bash profiles/r02_stage_ab.sh TAG
set -o pipefail
TAG=${1:-stg}
mkdir -p gpurun_out/$TAG
export TMPDIR=/tmp
mkdir -p gpurun_out/$TAG
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gpu_latency_paths.py tests/test_gpu_parity.py tests/test_gpu_properties.py > gpurun_out/$TAG/pytest.log 2>&1 &&
bash profiles/ab_run.sh $TAG/ab
