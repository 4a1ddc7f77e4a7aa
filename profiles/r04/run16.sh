#!/bin/bash
# conv epilogue: loads before stores.  Parity (layer-path tests), phase stamps with store
# ablations, then the same-box A/B against the old epilogue
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out/r04
timeout -k 10 900 python -u -m pytest -v --timeout 300 --timeout-method thread \
  tests/test_gpu_parity.py tests/test_gpu_stages.py tests/test_gpu_latency_paths.py \
  -k "resblock or golden or split or stage or loud or two_stream or run_to_run" > gpurun_out/r04/t16.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r04/t16.log
if [ $rc -ne 0 ]; then exit $rc; fi
bash profiles/r04/run15.sh && bash profiles/r04/ab_run.sh epi oldepi
