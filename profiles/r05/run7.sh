#!/bin/bash
# round 5, call 7: persistent C = 64 ResBlock grid (two grid policies) — bitwise tests, A/B
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out/r05
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread \
  tests/test_gpu_latency_paths.py tests/test_gpu_parity.py -k "persistent or run_to_run or split_resblock" \
  > gpurun_out/r05/t7.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r05/t7.log
if [ $rc -ne 0 ]; then exit $rc; fi
bash profiles/r05/env_ab.sh pg "HFG_RB_PERSIST=0" "HFG_RB_PERSIST=1" "HFG_RB_PERSIST=2"
