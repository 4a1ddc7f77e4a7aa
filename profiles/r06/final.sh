#!/bin/bash
# round-6 final set on the committed tree: GPU suite + smoke, the default bench line, a
# rocprofv3 kernel-trace/stats run of the same bench (1 stream) and the SQ counter passes.
# Everything lands in gpurun_out/r06/final/ (copied into profiles/r06/final/ afterwards).
cd "$(dirname "$0")/../.."
R=$(pwd)
O=$R/gpurun_out/r06/final
mkdir -p $O
timeout -k 10 1000 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests > $O/gputest.txt 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/gputest.txt
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 900 python -u bench.py > $O/bench.json 2> $O/bench.err
rc=$?; echo "bench rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/rocprof -o run --output-format csv -- \
  python $R/bench.py --steps 20 --warmup 5 --streams 1 --no-pmc --no-cpu-baseline --no-extra --also \
  > $O/bench_under_rocprof.json 2> $O/bench_under_rocprof.err
rc=$?; echo "rocprof rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi
BENCH="python $R/bench.py --steps 2 --warmup 1 --also --no-cpu-baseline --no-profile --no-extra --no-pmc"
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY -d $O/sq1 -o run --output-format csv -- $BENCH > $O/sq1.log 2>&1 && \
timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VMEM -d $O/sq2 -o run --output-format csv -- $BENCH > $O/sq2.log 2>&1 && \
timeout -s KILL 240 rocprofv3 --pmc SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE SQ_ACTIVE_INST_VALU SQ_INSTS_SMEM -d $O/sq3 -o run --output-format csv -- $BENCH > $O/sq3.log 2>&1
echo "sq rc=$?"
