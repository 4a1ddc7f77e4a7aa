#!/bin/bash
# round 5, call 13: what the k = 7 residual epilogue waits for — layer-conv phase stamps
# (diagnostic build) with the residual read as usual, from an L2-warm row (ablation bit 15),
# or not at all (bit 16)
cd "$(dirname "$0")/../.."
L=tts-sambert_hifigan_amd/libhifigan_hip.so
mkdir -p gpurun_out/r05/phases2
cp $L /tmp/base.so
rc=0
cp tts-sambert_hifigan_amd/ab/cvts.so $L
CVP_TAG=base timeout -k 10 300 python -u tests/tools/conv_phases.py $L > gpurun_out/r05/phases2/cvp_base.log 2>&1 || rc=1
cp tts-sambert_hifigan_amd/ab/cvts_abl.so $L
for f in 0 32768 65536; do
  [ $rc -eq 0 ] || break
  CVP_TAG=abl$f HFG_DEBUG_FLAGS=$f timeout -k 10 300 python -u tests/tools/conv_phases.py $L \
    > gpurun_out/r05/phases2/cvp_abl$f.log 2>&1 || rc=1
done
cp /tmp/base.so $L
echo "phases rc=$rc"
exit $rc
