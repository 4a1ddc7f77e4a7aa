#!/bin/bash
# per-launch kernel times of the V1 forward (f16x3 and bf16x3), by position in the forward
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r04
timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/r04/lt_f16 -o run --output-format csv -- python $R/tests/tools/layer_times.py run --precision f16x3 > $R/gpurun_out/r04/lt_f16.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/r04/lt_bf16 -o run --output-format csv -- python $R/tests/tools/layer_times.py run --precision bf16x3 > $R/gpurun_out/r04/lt_bf16.log 2>&1
echo "rc=$?"
