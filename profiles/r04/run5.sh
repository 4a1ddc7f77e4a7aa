#!/bin/bash
# round 4: re-run the tests that failed in the suite run, then the default bench line
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out/r04
timeout -k 10 600 python -u -m pytest -v -s --timeout 300 --timeout-method thread \
  tests/test_gpu_probe.py tests/test_gpu_properties.py tests/test_gpu_glue.py \
  "tests/test_gpu_parity.py::test_conv_post_kernels" > gpurun_out/r04/t5.log 2>&1
rc=$?
echo "pytest rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 900 python -u bench.py > gpurun_out/r04/b5.json 2> gpurun_out/r04/b5.err
echo "bench rc=$?"
