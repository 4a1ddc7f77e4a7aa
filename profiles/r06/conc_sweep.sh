#!/bin/bash
# RB_CONC auto / forced on / off over small and mid batch shapes (round 6, after the cheaper
# mrf_combine): is the concurrent-ResBlock threshold still right?
cd "$(dirname "$0")/../.."
for i in 1 2; do
  for shape in 62x32 256x4 512x4 1024x2 256x16 2048x1; do
    for m in -1 0 1; do
      timeout -k 10 120 python -u profiles/r06/c1_time.py f16x3 ${shape%x*} ${shape#*x} RB_CONC=$m 2>&1 | tail -1 || exit 1
    done
  done
done
echo "sweep done"
