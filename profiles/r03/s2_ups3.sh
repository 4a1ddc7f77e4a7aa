# ups ablation: conversion / loads after group 0 skipped (timing only; HFG_DEBUG_FLAGS)
O=gpurun_out/s2ups3; mkdir -p $O
for i in 1 2; do
  for f in 0 512 1536; do
    HFG_DEBUG_FLAGS=$f timeout -k 10 150 python bench.py --also --no-extra --no-cpu-baseline --no-pmc --steps 20 --streams 1 > $O/dbg${f}_$i.json 2>/dev/null || exit 1
  done
done
echo done
