#!/bin/bash
# tile-5 layer-conv phase times from the clock-stamp diagnostic build (ab/cvts.so)
cd "$(dirname "$0")/../.."
L=tts-sambert_hifigan_amd/libhifigan_hip.so
mkdir -p gpurun_out/r04
cp $L /tmp/base.so && cp tts-sambert_hifigan_amd/ab/cvts.so $L
timeout -k 10 300 python -u tests/tools/conv_phases.py $L > gpurun_out/r04/cvp.log 2>&1
rc=$?
cp /tmp/base.so $L
echo "rc=$rc"; tail -4 gpurun_out/r04/cvp.log
exit $rc
