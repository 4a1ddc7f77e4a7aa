#!/bin/bash
# 64-row ResBlock waves (HFG_RB_WM=2): parity, then A/B vs 32-row; then the conv phase
# stamps and the LDS-read ablations
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out/r04
HFG_RB_WM=2 timeout -k 10 900 python -u -m pytest -v --timeout 300 --timeout-method thread \
  tests/test_gpu_parity.py tests/test_gpu_stages.py tests/test_gpu_latency_paths.py tests/test_gpu_configs.py \
  -k "resblock or mrf or golden or split or stage or loud or C3 or C4 or c4 or c3" > gpurun_out/r04/t14.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r04/t14.log
if [ $rc -ne 0 ]; then exit $rc; fi
bash profiles/r04/env_ab.sh wm "HFG_RB_WM=1" "HFG_RB_WM=2" && bash profiles/r04/run12.sh && bash profiles/r04/run10.sh
