#!/bin/bash
# round 5, call 9: wide upsampler m-tiles — bitwise test, then the same-box A/B
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out/r05
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread \
  tests/test_gpu_parity.py -k "ups_wide or ups_frames" > gpurun_out/r05/t9.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r05/t9.log
if [ $rc -ne 0 ]; then exit $rc; fi
bash profiles/r05/env_ab.sh upsw "HFG_UPS_WIDE=0" "HFG_UPS_WIDE=2" "HFG_UPS_WIDE=3"
