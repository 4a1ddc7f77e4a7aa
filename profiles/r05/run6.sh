#!/bin/bash
# round 5, call 6: residual-through-LDS layer epilogue + C = 32 persistent ResBlocks — bitwise /
# parity tests, then the same-box A/B
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out/r05
timeout -k 10 900 python -u -m pytest -v --timeout 300 --timeout-method thread \
  tests/test_gpu_latency_paths.py tests/test_gpu_parity.py tests/test_gpu_stages.py \
  -k "persistent or residual_lds or small_tile or golden or split or stage or loud or run_to_run or ragged or conv_post or two_stream" \
  > gpurun_out/r05/t6.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r05/t6.log
if [ $rc -ne 0 ]; then exit $rc; fi
bash profiles/r05/env_ab.sh epi "HFG_RES_LDS=0 HFG_RB_PERSIST=0" "HFG_RES_LDS=1 HFG_RB_PERSIST=0" "HFG_RES_LDS=1 HFG_RB_PERSIST=1" "HFG_RES_LDS=1 HFG_RB_PERSIST=2"
