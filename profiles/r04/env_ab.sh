#!/bin/bash
# Same-box A/B of environment settings on the default library: bench (f16x3 + bf16x3) per
# setting, alternated twice.  usage: bash profiles/r04/env_ab.sh TAG "ENV_A" "ENV_B" ...
cd "$(dirname "$0")/../.."
T=$1; shift
mkdir -p gpurun_out/r04/ab
for i in 1 2; do
  j=0
  for e in "$@"; do
    env $e timeout -k 10 200 python -u bench.py --also bf16x3 --no-extra --no-cpu-baseline --no-pmc \
      --steps 20 > gpurun_out/r04/ab/${T}_e${j}_$i.json 2> gpurun_out/r04/ab/${T}_e${j}_$i.err
    rc=$?
    if [ $rc -ne 0 ]; then echo "bench [$e] rc=$rc"; exit $rc; fi
    j=$((j+1))
  done
done
echo "env ab done"
