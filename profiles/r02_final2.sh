#!/bin/bash
# round-2 final set at tile 5: full GPU suite + smoke, default bench line, rocprofv3
# kernel stats + FETCH/WRITE PMC passes, two SQ counter passes
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
T=${1:-f2}
mkdir -p $R/gpurun_out/$T
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/$T/pytest.log 2>&1 &&
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$T/smoke.log 2>&1 &&
timeout -k 10 400 python bench.py > gpurun_out/$T/bench.json 2> gpurun_out/$T/bench.err &&
bash profiles/run_rocprof.sh $T &&
bash profiles/r02_sq.sh
