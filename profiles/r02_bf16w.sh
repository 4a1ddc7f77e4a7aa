#!/bin/bash
# bf16 weight storage (HFG_DTYPE_BF16W): parity tests, then an A/B bench vs bf16x3.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/bf16w
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/test_gpu_bf16w.py tests/test_gpu_parity.py tests/test_gpu_latency_paths.py \
  > gpurun_out/bf16w/pytest.log 2>&1 &&
timeout -k 10 240 python -u bench.py --steps 20 --warmup 5 --no-extra --no-cpu-baseline --no-pmc \
  --also bf16w > gpurun_out/bf16w/bench.json 2> gpurun_out/bf16w/bench.err
