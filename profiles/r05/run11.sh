#!/bin/bash
# round 5, call 11: the value pass eager vs hipGraph replay, alternated on one box
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out/r05/ab
for i in 1 2; do
  for m in eager graph; do
    f=""; [ $m == graph ] && f="--graph"
    timeout -k 10 200 python -u bench.py --also --no-extra --no-cpu-baseline --no-pmc --steps 20 $f \
      > gpurun_out/r05/ab/graph_${m}_$i.json 2> gpurun_out/r05/ab/graph_${m}_$i.err
    rc=$?; if [ $rc -ne 0 ]; then echo "bench $m rc=$rc"; exit $rc; fi
  done
done
echo "ab done"
