#!/bin/bash
# per-launch kernel times of the V2* C4 forward [16, 80, 2048], f16x3 vs bf16x3
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r04
for p in f16x3 bf16x3; do
  timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/r04/lt4_$p -o run --output-format csv -- python $R/tests/tools/layer_times.py run --precision $p --preset v2star --batch 16 --frames 2048 > $R/gpurun_out/r04/lt4_$p.log 2>&1 || exit 1
done
echo done
