# SQ counter passes on the bf16x3 bench (one rocprofv3 run per pass; counters only with --kernel-trace-free --pmc)
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
BENCH="python $R/bench.py --steps 1 --warmup 1 --precision ${PREC:-bf16x3} --also --no-cpu-baseline --no-profile"
timeout -k 10 120 rocprofv3 -L > $R/gpurun_out/rocprof_counters.txt 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY -d $R/gpurun_out/sq1 -o run --output-format csv -- $BENCH > $R/gpurun_out/sq1.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VMEM -d $R/gpurun_out/sq2 -o run --output-format csv -- $BENCH > $R/gpurun_out/sq2.log 2>&1
echo done
