#!/bin/bash
# Per-launch trace of a [32, 80, 62] f16x3 forward (the C5-sized small batch; round 6)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r06
timeout -k 10 240 rocprofv3 --kernel-trace -d gpurun_out/r06/c5_f16x3 -o run --output-format csv -- python3 tests/tools/layer_times.py run --precision f16x3 --batch 32 --frames 62 > gpurun_out/r06/c5_f16x3.log 2>&1
echo done
