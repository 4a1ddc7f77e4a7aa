#!/bin/bash
# round 6: streaming contract data (stream vs one-shot vs oracle) at default, 2x and 4x scale
cd "$(dirname "$0")/../.."
O=gpurun_out/r06/run5
mkdir -p $O
timeout -k 10 400 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_glue.py > $O/tests.txt 2>&1
echo "pytest rc=$?"; tail -3 $O/tests.txt
