#!/bin/bash
# round 6: C = 32 ResBlocks on 1024-column windows (RB32_WIDE=1) — tests, then a same-box A/B
cd "$(dirname "$0")/../.."
O=gpurun_out/r06/run8
mkdir -p $O
timeout -k 10 300 python -u -m pytest -q --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_latency_paths.py -k "wide_c32" > $O/tests.txt 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/tests.txt
if [ $rc -ne 0 ]; then exit $rc; fi
ROUNDS=2 bash profiles/r06/sched_ab.sh wide w1=RB32_WIDE=1
