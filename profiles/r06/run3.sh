#!/bin/bash
# round 6: upsampler with two raw-input groups in flight — parity / bitwise tests, then a
# same-box A/B against one group in flight (xd1) and the round-5 kernel (r5ups).
cd "$(dirname "$0")/../.."
O=gpurun_out/r06/run3
mkdir -p $O
timeout -k 10 400 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_gpu_full_output.py -k "ups or golden or c2_8x80" > $O/tests.txt 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/tests.txt
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
ROUNDS=3 bash profiles/r06/lib_ab.sh ups xd1 r5ups
ROUNDS=2 bash profiles/r06/sched_ab.sh persist p0=RB_PERSIST=0
