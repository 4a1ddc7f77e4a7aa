#!/bin/bash
# SQ counters per kernel on the C2 bench (1 stream), two --pmc passes (<= 8 SQ each)
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/sq
B="$R/bench.py --steps 2 --warmup 1 --streams 1 --no-profile --no-extra --no-cpu-baseline --no-pmc --also"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS -d $R/gpurun_out/sq/p1 -o run --output-format csv -- python3 $B > $R/gpurun_out/sq/p1.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_VMEM SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_SALU GRBM_GUI_ACTIVE -d $R/gpurun_out/sq/p2 -o run --output-format csv -- python3 $B > $R/gpurun_out/sq/p2.log 2>&1
