#!/bin/bash
# full GPU suite + smoke on the committed tree (round 4)
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out/r04
timeout -k 10 1100 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests \
  > gpurun_out/r04/suite.log 2>&1
rc=$?
echo "pytest rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04/smoke.log 2>&1
echo "smoke rc=$?"
