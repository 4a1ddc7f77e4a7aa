#!/bin/bash
# margin-filled first conv in the whole-ResBlock kernel: ResBlock / MRF / golden parity, then A/B
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out/r04
timeout -k 10 900 python -u -m pytest -v --timeout 300 --timeout-method thread \
  tests/test_gpu_parity.py tests/test_gpu_stages.py tests/test_gpu_latency_paths.py \
  -k "resblock or mrf or golden or split or stage or loud" > gpurun_out/r04/t9.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r04/t9.log
if [ $rc -ne 0 ]; then exit $rc; fi
bash profiles/r04/ab_run.sh marg nomarg
