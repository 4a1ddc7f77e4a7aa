#!/bin/bash
# round 5, call 2: ResBlock / layer-conv phase stamps (diagnostic builds), then the block-stagger
# A/B (real-time spin)
cd "$(dirname "$0")/../.."
L=tts-sambert_hifigan_amd/libhifigan_hip.so
mkdir -p gpurun_out/r05
cp $L /tmp/base.so
cp tts-sambert_hifigan_amd/ab/rbts.so $L
timeout -k 10 300 python -u tests/tools/rb_phases.py $L > gpurun_out/r05/rbp.log 2>&1
rc=$?
cp tts-sambert_hifigan_amd/ab/cvts.so $L
[ $rc -eq 0 ] && timeout -k 10 300 python -u tests/tools/conv_phases.py $L > gpurun_out/r05/cvp.log 2>&1
rc2=$?
cp /tmp/base.so $L
echo "phases rc=$rc/$rc2"
if [ $rc -ne 0 ] || [ $rc2 -ne 0 ]; then exit 1; fi
bash profiles/r05/env_ab.sh stag2 "" "HFG_STAGGER=25,0" "HFG_STAGGER=50,0" "HFG_STAGGER=0,5" "HFG_STAGGER=0,15"
