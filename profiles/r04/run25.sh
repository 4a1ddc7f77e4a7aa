#!/bin/bash
# value pass on 1 vs 2 streams (same box, alternated)
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out/r04/ab
for i in 1 2; do
  for s in 2 1; do
    timeout -k 10 200 python -u bench.py --also bf16x3 --no-extra --no-cpu-baseline --no-pmc --no-profile \
      --steps 30 --streams $s > gpurun_out/r04/ab/streams_s${s}_$i.json 2> gpurun_out/r04/ab/streams_s${s}_$i.err || exit 1
  done
done
echo done
