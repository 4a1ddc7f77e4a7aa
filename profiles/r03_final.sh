#!/bin/bash
# Round-3 profile set (GPU box): GPU suite, smoke, default bench line, 2-rank self-launched
# rehearsal (gloo, both ranks on the one GPU), rocprofv3 kernel stats + FETCH/WRITE PMC passes,
# two SQ counter passes.  Outputs under gpurun_out/r03final/.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r03final
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gputest.txt 2>&1 || { tail -30 $O/gputest.txt; exit 1; }
tail -2 $O/gputest.txt
timeout -k 10 120 python __graft_entry__.py smoke > $O/smoke.log 2>&1 || exit 1
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || exit 1
timeout -k 10 300 python bench.py --gpus 2 --dist-backend gloo --steps 5 --warmup 2 --no-extra --no-cpu-baseline --no-pmc > $O/bench_n2_gloo.json 2> $O/bench_n2_gloo.err || exit 1
cd /tmp && export TMPDIR=/tmp
B="$R/bench.py --steps 5 --warmup 2 --also --no-cpu-baseline --no-extra --no-pmc --streams 1"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 $B > $O/bench_under_rocprof.json 2> $O/prof.err || exit 1
P="$R/bench.py --steps 2 --warmup 1 --also --no-cpu-baseline --no-extra --no-pmc --streams 1 --no-profile"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_fetch -o run --output-format csv -- python3 $P > $O/pmc_fetch.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_write -o run --output-format csv -- python3 $P > $O/pmc_write.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS -d $O/sq/p1 -o run --output-format csv -- python3 $P > $O/sq_p1.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_VMEM SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_SALU GRBM_GUI_ACTIVE -d $O/sq/p2 -o run --output-format csv -- python3 $P > $O/sq_p2.log 2>&1 || exit 1
echo done
