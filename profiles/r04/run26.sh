#!/bin/bash
# conv_post fused into the last C = 32 ResBlock launch: bitwise test, then value pass A/B
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out/r04/ab
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py -k "conv_post" > gpurun_out/r04/t26.txt 2>&1 || { tail -30 gpurun_out/r04/t26.txt; exit 1; }
tail -3 gpurun_out/r04/t26.txt
for i in 1 2; do
  for f in 1 0; do
    HFG_FUSE_POST=$f timeout -k 10 200 python -u bench.py --also bf16x3 --no-extra --no-cpu-baseline --no-pmc --no-profile \
      --steps 30 > gpurun_out/r04/ab/post_f${f}_$i.json 2> gpurun_out/r04/ab/post_f${f}_$i.err || exit 1
  done
done
for f in gpurun_out/r04/ab/post_*.json; do echo $f; head -c 300 $f; echo; done
