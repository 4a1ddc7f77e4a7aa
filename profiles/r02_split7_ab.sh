#!/bin/bash
# k = 7 ResBlocks split too (HFG_RB_SPLIT_MIN=0.95) vs the default (k = 11 only): bitwise
# test, then a same-box A/B on the same library
set -o pipefail
export TMPDIR=/tmp
T=${1:-split7}
mkdir -p gpurun_out/$T
HFG_RB_SPLIT_MIN=0.95 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gpu_latency_paths.py -k split > gpurun_out/$T/pytest.log 2>&1 || exit 1
for i in 1 2; do
  HFG_RB_SPLIT_MIN=0.95 timeout -k 10 150 python bench.py --also --no-extra --no-cpu-baseline --no-pmc --steps 20 > gpurun_out/$T/ab_new$i.json 2>/dev/null || exit 1
  timeout -k 10 150 python bench.py --also --no-extra --no-cpu-baseline --no-pmc --steps 20 > gpurun_out/$T/ab_old$i.json 2>/dev/null || exit 1
done
