#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/probe
timeout -k 10 200 python -u -m pytest -x -v -s --timeout 120 --timeout-method thread \
  tests/test_gpu_probe.py > gpurun_out/probe/pytest2.log 2>&1
