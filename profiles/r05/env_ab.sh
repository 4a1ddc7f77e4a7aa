#!/bin/bash
# Same-box A/B of environment variants of the default library (round 5): the bench (f16x3
# value pass + the 1-stream per-kernel pass) per variant, alternated twice.
# usage: bash profiles/r05/env_ab.sh TAG "VAR=.. VAR=.." "VAR=.." ...   ("" = the default)
cd "$(dirname "$0")/../.."
T=$1; shift
mkdir -p gpurun_out/r05/ab
for i in 1 2; do
  n=0
  for v in "$@"; do
    n=$((n + 1))
    env $v timeout -k 10 200 python -u bench.py --also --no-extra --no-cpu-baseline --no-pmc \
      --steps 20 > gpurun_out/r05/ab/${T}_v${n}_$i.json 2> gpurun_out/r05/ab/${T}_v${n}_$i.err
    rc=$?
    if [ $rc -ne 0 ]; then echo "bench [$v] rc=$rc"; exit $rc; fi
    echo "$v" > gpurun_out/r05/ab/${T}_v${n}.env
  done
done
echo "ab done"
