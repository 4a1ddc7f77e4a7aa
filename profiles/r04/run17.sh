#!/bin/bash
# upsampler staging swizzle: bitwise tests, SQ LDS counters (new vs old), same-box A/B
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out/r04
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread \
  tests/test_gpu_parity.py -k "ups or golden_fixture_split or two_stream" > gpurun_out/r04/t17.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/r04/t17.log
if [ $rc -ne 0 ]; then exit $rc; fi
bash profiles/r04/sq_lds.sh "" sqlds_new && bash profiles/r04/sq_lds.sh oldups sqlds_old && bash profiles/r04/ab_run.sh swz oldups
