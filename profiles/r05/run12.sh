#!/bin/bash
# round 5, call 12: residual layer-conv epilogue with the row tile's residual loaded before its
# first stores (HFG_EPI_RPRE) — epilogue / parity / bitwise tests, then a same-box A/B against
# the previous schedule (ab/rpre0.so)
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out/r05
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread \
  tests/test_gpu_parity.py tests/test_gpu_stages.py tests/test_gpu_configs.py tests/test_gpu_latency_paths.py \
  -k "epilogue or bitwise or golden or stage or loud or C5 or C3 or run_to_run" > gpurun_out/r05/t12.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r05/t12.log
if [ $rc -ne 0 ]; then exit $rc; fi
bash profiles/r05/lib_ab.sh rpre rpre0
