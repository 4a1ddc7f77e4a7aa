#!/bin/bash
# round 6: per-dispatch kernel traces of the C2 forward (1 stream and the 2-stream value pass)
# for a per-launch breakdown (which launches of a kernel instance run below its rate).
cd "$(dirname "$0")/../.."
R=$(pwd)
O=$R/gpurun_out/r06/run2
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for s in 1 2; do
  timeout -k 10 300 rocprofv3 --kernel-trace -d $O/trace_s$s -o run --output-format csv -- \
    python $R/bench.py --steps 3 --warmup 2 --streams $s --no-pmc --no-cpu-baseline --no-extra \
    --no-profile --also > $O/bench_s$s.json 2> $O/bench_s$s.err
  rc=$?; echo "trace s$s rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi
done
