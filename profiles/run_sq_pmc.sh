# SQ counter passes on the bf16x3 bench (one rocprofv3 run per pass; counters only with --pmc)
# usage: bash profiles/run_sq_pmc.sh TAG
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
T=${1:-sq}
BENCH="python $R/bench.py --steps 1 --warmup 1 --precision ${PREC:-bf16x3} --also --no-cpu-baseline --no-profile --no-extra"
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY -d $R/gpurun_out/${T}1 -o run --output-format csv -- $BENCH > $R/gpurun_out/${T}1.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VMEM -d $R/gpurun_out/${T}2 -o run --output-format csv -- $BENCH > $R/gpurun_out/${T}2.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE SQ_INST_LEVEL_LDS SQ_INSTS_SMEM -d $R/gpurun_out/${T}3 -o run --output-format csv -- $BENCH > $R/gpurun_out/${T}3.log 2>&1
echo done
