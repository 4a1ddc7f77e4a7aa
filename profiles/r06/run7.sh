#!/bin/bash
# round 6: 256x128 AREG tile (6) for the 256-row layer convs — bitwise / parity tests, then a
# same-box A/B against tile 5 (AREG_TALL=0)
cd "$(dirname "$0")/../.."
O=gpurun_out/r06/run7
mkdir -p $O
timeout -k 10 500 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_latency_paths.py tests/test_gpu_full_output.py tests/test_gpu_stages.py \
  -k "tall or c2_8x80 or stage" > $O/tests.txt 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/tests.txt
if [ $rc -ne 0 ]; then exit $rc; fi
ROUNDS=3 bash profiles/r06/sched_ab.sh tall t5=AREG_TALL=0
