#!/bin/bash
# full GPU suite + smoke on the working tree (round 5); logs in gpurun_out/r05/
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out/r05
timeout -k 10 1100 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests "$@" \
  > gpurun_out/r05/suite.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/r05/suite.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r05/smoke.log 2>&1
echo "smoke rc=$?"
