#!/bin/bash
# Same-box A/B of schedule overrides (round 6): bench.py with each variant's --sched list,
# alternated ROUNDS times (default 2).  usage: bash profiles/r06/sched_ab.sh TAG NAME=KNOB=V,KNOB=V ...
# (a variant "base" with no overrides always runs first)
cd "$(dirname "$0")/../.."
T=$1; shift
O=gpurun_out/r06/ab
mkdir -p $O
for i in $(seq 1 ${ROUNDS:-2}); do
  for v in base "$@"; do
    n=${v%%=*}; s=""
    if [ "$n" != "$v" ]; then s="--sched $(echo ${v#*=} | tr ',' ' ')"; fi
    timeout -k 10 200 python -u bench.py --also --no-extra --no-cpu-baseline --no-pmc \
      --steps ${STEPS:-20} $s > $O/${T}_${n}_$i.json 2> $O/${T}_${n}_$i.err
    rc=$?
    if [ $rc -ne 0 ]; then echo "bench $n rc=$rc"; exit $rc; fi
    python3 profiles/r06/ab_show.py $O/${T}_${n}_$i.json
  done
done
echo "ab done"
