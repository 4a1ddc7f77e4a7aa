#!/bin/bash
# round 6: issue priority raised for the MFMA phases (HFG_PRIO=1, base) vs off (noprio)
cd "$(dirname "$0")/../.."
O=gpurun_out/r06/run4
mkdir -p $O
timeout -k 10 300 python -u -m pytest -q --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_full_output.py -k "f16x3" > $O/tests.txt 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/tests.txt
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
ROUNDS=3 bash profiles/r06/lib_ab.sh prio noprio
