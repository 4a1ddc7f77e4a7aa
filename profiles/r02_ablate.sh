#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/abl
for f in 0 4 8 12 128 0; do
  HFG_DEBUG_FLAGS=$f timeout -k 10 150 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-extra --no-pmc --also > gpurun_out/abl/f$f.json 2>/dev/null || exit 1
done
