#!/bin/bash
# round 5, call 8: full GPU suite + smoke + the default bench line on the committed tree
cd "$(dirname "$0")/../.."
bash profiles/r05/suite.sh || exit $?
timeout -k 10 600 python -u bench.py > gpurun_out/r05/bench8.json 2> gpurun_out/r05/bench8.err
echo "bench rc=$?"
