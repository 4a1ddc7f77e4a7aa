#!/bin/bash
# whole-ResBlock split (HFG_RB_SPLIT=1 default) vs one launch: bitwise + parity + stage +
# config-sweep tests, then a same-box A/B on the same library
set -o pipefail
export TMPDIR=/tmp
T=${1:-split}
mkdir -p gpurun_out/$T
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gpu_latency_paths.py tests/test_gpu_parity.py tests/test_gpu_stages.py \
  tests/test_gpu_config_sweep.py tests/test_gpu_glue.py > gpurun_out/$T/pytest.log 2>&1 || exit 1
for i in 1 2; do
  HFG_RB_SPLIT=1 timeout -k 10 150 python bench.py --also --no-extra --no-cpu-baseline --no-pmc --steps 20 > gpurun_out/$T/ab_new$i.json 2>/dev/null || exit 1
  HFG_RB_SPLIT=0 timeout -k 10 150 python bench.py --also --no-extra --no-cpu-baseline --no-pmc --steps 20 > gpurun_out/$T/ab_old$i.json 2>/dev/null || exit 1
done
