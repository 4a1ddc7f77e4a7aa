#!/bin/bash
# same-box A/B of tile 5 (HFG_AREG=1) vs tile 3, same library; then parity
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/areg
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gpu_latency_paths.py -k "areg or lds_staged" > gpurun_out/areg/pytest0.log 2>&1 || exit 1
for i in 1 2; do
  HFG_AREG=1 timeout -k 10 150 python bench.py --also --no-extra --no-cpu-baseline --no-pmc --steps 20 > gpurun_out/areg/new$i.json 2>/dev/null || exit 1
  HFG_AREG=0 timeout -k 10 150 python bench.py --also --no-extra --no-cpu-baseline --no-pmc --steps 20 > gpurun_out/areg/old$i.json 2>/dev/null || exit 1
done
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gpu_parity.py tests/test_gpu_latency_paths.py tests/test_gpu_properties.py > gpurun_out/areg/pytest.log 2>&1
