#!/bin/bash
# ResBlock phase times from the clock-stamp diagnostic build (ab/rbts.so), f16x3 and bf16x3
cd "$(dirname "$0")/../.."
L=tts-sambert_hifigan_amd/libhifigan_hip.so
mkdir -p gpurun_out/r04
cp $L /tmp/base.so && cp tts-sambert_hifigan_amd/ab/rbts.so $L
timeout -k 10 300 python -u tests/tools/rb_phases.py $L --precision f16x3 > gpurun_out/r04/rbp_f16.log 2>&1
rc=$?
if [ $rc -eq 0 ]; then
  timeout -k 10 300 python -u tests/tools/rb_phases.py $L --precision bf16x3 > gpurun_out/r04/rbp_bf16.log 2>&1
  rc=$?
fi
cp /tmp/base.so $L
echo "rc=$rc"
exit $rc
