#!/bin/bash
# Same-box A/B on the GPU box: bench (f16x3 and bf16x3, value pass + per-kernel pass) with the
# default library and each ab/NAME.so, alternated twice.
# usage: bash profiles/r04/ab_run.sh TAG NAME... [-- bench args]
cd "$(dirname "$0")/../.."
T=$1; shift
names=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do names+=("$1"); shift; done
[ "$1" == "--" ] && shift
L=tts-sambert_hifigan_amd/libhifigan_hip.so
mkdir -p gpurun_out/r04/ab
cp $L /tmp/ab_base.so
for i in 1 2; do
  for n in base "${names[@]}"; do
    if [ "$n" == base ]; then cp /tmp/ab_base.so $L; else cp tts-sambert_hifigan_amd/ab/$n.so $L; fi
    timeout -k 10 200 python -u bench.py --also bf16x3 --no-extra --no-cpu-baseline --no-pmc \
      --steps 20 "$@" > gpurun_out/r04/ab/${T}_${n}_$i.json 2> gpurun_out/r04/ab/${T}_${n}_$i.err
    rc=$?
    if [ $rc -ne 0 ]; then cp /tmp/ab_base.so $L; echo "bench $n rc=$rc"; exit $rc; fi
  done
done
cp /tmp/ab_base.so $L
echo "ab done"
