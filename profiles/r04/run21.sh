#!/bin/bash
# k = 7 ResBlocks split in two launches (threshold 0.95 lets them split): parity + env A/B
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out/r04
HFG_RB_SPLIT_TH=0.95 timeout -k 10 900 python -u -m pytest -v --timeout 300 --timeout-method thread \
  tests/test_gpu_parity.py tests/test_gpu_stages.py tests/test_gpu_latency_paths.py \
  -k "resblock or golden or split or stage or loud or two_stream" > gpurun_out/r04/t21.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/r04/t21.log
if [ $rc -ne 0 ]; then exit $rc; fi
bash profiles/r04/env_ab.sh k7split "HFG_RB_SPLIT_TH=0.9" "HFG_RB_SPLIT_TH=0.95"
