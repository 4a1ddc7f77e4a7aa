#!/bin/bash
# Same-box A/B of library builds (round 5): the bench (f16x3 value pass + 1-stream per-kernel
# pass) with the tree's library and each tts-sambert_hifigan_amd/ab/NAME.so, alternated twice.
# usage: bash profiles/r05/lib_ab.sh TAG NAME...
cd "$(dirname "$0")/../.."
T=$1; shift
L=tts-sambert_hifigan_amd/libhifigan_hip.so
mkdir -p gpurun_out/r05/ab
cp $L /tmp/ab_base.so
for i in 1 2; do
  for n in base "$@"; do
    if [ "$n" == base ]; then cp /tmp/ab_base.so $L; else cp tts-sambert_hifigan_amd/ab/$n.so $L; fi
    timeout -k 10 200 python -u bench.py --also --no-extra --no-cpu-baseline --no-pmc \
      --steps 20 > gpurun_out/r05/ab/${T}_${n}_$i.json 2> gpurun_out/r05/ab/${T}_${n}_$i.err
    rc=$?
    if [ $rc -ne 0 ]; then cp /tmp/ab_base.so $L; echo "bench $n rc=$rc"; exit $rc; fi
  done
done
cp /tmp/ab_base.so $L
echo "ab done"
