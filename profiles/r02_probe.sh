#!/bin/bash
# live sustained-MFMA probe + default bench (no extras) to see peak_sustained
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/probe
timeout -k 10 200 python -u -m pytest -x -v -s --timeout 120 --timeout-method thread \
  tests/test_gpu_probe.py > gpurun_out/probe/pytest.log 2>&1 &&
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-extra --no-cpu-baseline --no-pmc \
  > gpurun_out/probe/bench.json 2> gpurun_out/probe/bench.err
