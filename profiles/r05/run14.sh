#!/bin/bash
# round 5, call 14: the end-of-round tree (ablation bits compiled out) — GPU suite, smoke and
# the default bench line, as the driver will run them
cd "$(dirname "$0")/../.."
O=gpurun_out/r05/head
mkdir -p $O
timeout -k 10 1100 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests > $O/gputest.txt 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/gputest.txt
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 900 python -u bench.py > $O/bench.json 2> $O/bench.err
echo "bench rc=$?"
