# SQ counters per kernel (one --pmc pass, 8 SQ counters: the block's limit), C2 bench, 1 stream
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES -d $R/gpurun_out/sq_r02 -o run --output-format csv -- python $R/bench.py --steps 2 --warmup 1 --streams 1 --no-profile --no-extra --no-cpu-baseline --no-pmc --also > $R/gpurun_out/sq_r02.log 2>&1
