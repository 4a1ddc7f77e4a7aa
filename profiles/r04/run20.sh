#!/bin/bash
# batched LDS reads in the tile-5 epilogue: parity, stamps, A/B vs the previous epilogue
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out/r04
timeout -k 10 900 python -u -m pytest -v --timeout 300 --timeout-method thread \
  tests/test_gpu_parity.py tests/test_gpu_stages.py tests/test_gpu_latency_paths.py tests/test_gpu_configs.py \
  -k "golden or split or stage or loud or two_stream or run_to_run or resblock or conv_post or C3 or C4 or ragged" > gpurun_out/r04/t20.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/r04/t20.log
if [ $rc -ne 0 ]; then exit $rc; fi
bash profiles/r04/run15.sh && bash profiles/r04/ab_run.sh bepi prev
