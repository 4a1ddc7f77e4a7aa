#!/bin/bash
# round 5, call 5: persistent ResBlock grid — bitwise / parity tests, then the same-box A/B
# (persistent grid; CU-masked halves), then block placement + tile-5 stamps
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out/r05
timeout -k 10 900 python -u -m pytest -v --timeout 300 --timeout-method thread \
  tests/test_gpu_latency_paths.py tests/test_gpu_parity.py tests/test_gpu_stages.py tests/test_gpu_glue.py \
  -k "persistent or golden or split or stage or loud or run_to_run or ragged or streaming or conv_post" \
  > gpurun_out/r05/t5.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r05/t5.log
if [ $rc -ne 0 ]; then exit $rc; fi
bash profiles/r05/env_ab.sh pers "HFG_RB_PERSIST=0" "HFG_RB_PERSIST=1" "HFG_CU_SPLIT=1,0" "HFG_CU_SPLIT=1,30" || exit 1
bash profiles/r05/run4.sh
