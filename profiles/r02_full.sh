#!/bin/bash
# full GPU suite + smoke + default bench
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/full
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/full/pytest.log 2>&1 &&
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/full/smoke.log 2>&1 &&
timeout -k 10 400 python bench.py > gpurun_out/full/bench.json 2> gpurun_out/full/bench.err
