#!/bin/bash
# kernel trace (1 stream) + the two SQ counter passes of the C2 bench (profiles/r02_sq.sh)
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
T=${1:-cur}
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_$T -o run --output-format csv -- python3 $R/bench.py --steps 5 --warmup 2 --also --no-cpu-baseline --no-extra --no-pmc --streams 1 > $R/gpurun_out/prof_${T}_bench.json 2> $R/gpurun_out/prof_${T}_bench.err &&
bash $R/profiles/r02_sq.sh
