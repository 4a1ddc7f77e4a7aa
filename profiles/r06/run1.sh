#!/bin/bash
# round 6, first GPU call: the new / changed tests (every-sample C2 + C1 vs oracle, schedule
# overrides instead of environment knobs, persistent + concurrent ResBlocks, loud streaming,
# one-collective gather), then the ResBlock operand-rewrite A/B (scalar muls + fma_mixlo split
# vs the round-5 code), then the default bench line.  Logs in gpurun_out/r06/run1/.
cd "$(dirname "$0")/../.."
O=gpurun_out/r06/run1
mkdir -p $O
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_full_output.py tests/test_gpu_latency_paths.py tests/test_gpu_parity.py \
  tests/test_gpu_glue.py tests/test_gpu_mel.py tests/test_gpu_dist.py > $O/tests.txt 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/tests.txt
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
bash profiles/r06/lib_ab.sh rw r5 nomixlo || exit $?
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err
echo "bench rc=$?"
