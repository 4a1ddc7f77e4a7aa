#!/bin/bash
# round 4: SQ counters of the f16x3 and bf16x3 kernels in one bench (both precisions measured:
# the kernels differ in their last template argument), 3 passes
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
T=r04/sq
mkdir -p $R/gpurun_out/r04
BENCH="python $R/bench.py --steps 2 --warmup 1 --precision f16x3 --also bf16x3 --no-cpu-baseline --no-profile --no-extra --no-pmc"
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY -d $R/gpurun_out/${T}1 -o run --output-format csv -- $BENCH > $R/gpurun_out/${T}1.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VMEM -d $R/gpurun_out/${T}2 -o run --output-format csv -- $BENCH > $R/gpurun_out/${T}2.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE SQ_ACTIVE_INST_VALU SQ_INSTS_SMEM -d $R/gpurun_out/${T}3 -o run --output-format csv -- $BENCH > $R/gpurun_out/${T}3.log 2>&1
echo "rc=$?"
