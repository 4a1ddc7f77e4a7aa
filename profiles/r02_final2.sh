#!/bin/bash
# round-2 final set at tile 5: full GPU suite + smoke, default bench line, rocprofv3
# kernel stats + FETCH/WRITE PMC passes, two SQ counter passes
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/f2
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/f2/pytest.log 2>&1 &&
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/f2/smoke.log 2>&1 &&
timeout -k 10 400 python bench.py > gpurun_out/f2/bench.json 2> gpurun_out/f2/bench.err &&
bash profiles/run_rocprof.sh f2 &&
bash profiles/r02_sq.sh
