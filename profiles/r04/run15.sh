#!/bin/bash
# conv epilogue store ablations on the stamp build (cvtsabl.so): phases per flag
cd "$(dirname "$0")/../.."
L=tts-sambert_hifigan_amd/libhifigan_hip.so
mkdir -p gpurun_out/r04
cp $L /tmp/base.so && cp tts-sambert_hifigan_amd/ab/cvtsabl.so $L
rc=0
for f in 0 8192 16384; do
  HFG_DEBUG_FLAGS=$f timeout -k 10 300 python -u tests/tools/conv_phases.py $L > gpurun_out/r04/cvp_f$f.log 2>&1
  rc=$?
  if [ $rc -ne 0 ]; then echo "flags $f rc=$rc"; break; fi
done
cp /tmp/base.so $L
echo "rc=$rc"
exit $rc
