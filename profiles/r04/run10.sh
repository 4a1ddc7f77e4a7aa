#!/bin/bash
# ablation timings (wrong results, kernel times only): abl.so with HFG_DEBUG_FLAGS
cd "$(dirname "$0")/../.."
L=tts-sambert_hifigan_amd/libhifigan_hip.so
mkdir -p gpurun_out/r04/abl2
cp $L /tmp/base.so && cp tts-sambert_hifigan_amd/ab/abl.so $L
rc=0
for f in 0 2048 4096 6144; do
  HFG_DEBUG_FLAGS=$f timeout -k 10 200 python -u bench.py --no-extra --no-cpu-baseline --no-pmc --also \
    --steps 10 > gpurun_out/r04/abl2/f$f.json 2> gpurun_out/r04/abl2/f$f.err
  rc=$?
  if [ $rc -ne 0 ]; then echo "flags $f rc=$rc"; break; fi
done
cp /tmp/base.so $L
echo "abl rc=$rc"
exit $rc
