#!/bin/bash
# round 6: the driver's GPU tier on the committed tree — pytest -m gpu (as the driver runs it) and
# smoke(); logs in gpurun_out/r06/suite/
cd "$(dirname "$0")/../.."
O=gpurun_out/r06/suite
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests/ -x -q -m gpu > $O/gputest.txt 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/gputest.txt
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
echo "smoke rc=$?"; tail -1 $O/smoke.log
