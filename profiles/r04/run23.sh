#!/bin/bash
# persistent ResBlock grid (no prefetch): parity, then A/B vs one block per window
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out/r04
timeout -k 10 900 python -u -m pytest -v --timeout 300 --timeout-method thread \
  tests/test_gpu_parity.py tests/test_gpu_stages.py tests/test_gpu_latency_paths.py tests/test_gpu_configs.py tests/test_gpu_glue.py \
  -k "resblock or mrf or golden or split or stage or loud or two_stream or C3 or C4 or C5 or ragged or stream" > gpurun_out/r04/t23.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/r04/t23.log
if [ $rc -ne 0 ]; then exit $rc; fi
bash profiles/r04/ab_run.sh persist nonpersist
