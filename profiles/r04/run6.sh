#!/bin/bash
# rotated ups staging (default build): upsampler parity / bitwise tests, then A/B vs the
# unrotated build and the fma_mix split
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out/r04
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread \
  tests/test_gpu_parity.py -k "ups_frames or golden_fixture_split or random_vs" > gpurun_out/r04/t6.log 2>&1
rc=$?; echo "pytest rc=$rc"
if [ $rc -ne 0 ]; then exit $rc; fi
bash profiles/r04/ab_run.sh rot norot mix
