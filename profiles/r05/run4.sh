#!/bin/bash
# round 5, call 4: block -> CU placement (dispatch_map) and the tile-5 stamps with placement,
# without and with the first-round stagger
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out/r05
timeout -k 10 60 tests/tools/dispatch_map 2048 64 40 > gpurun_out/r05/dmap_2048_64.csv || exit 1
timeout -k 10 60 tests/tools/dispatch_map 1024 150 40 > gpurun_out/r05/dmap_1024_150.csv || exit 1
L=tts-sambert_hifigan_amd/libhifigan_hip.so
cp $L /tmp/base.so
cp tts-sambert_hifigan_amd/ab/cvts.so $L
CVP_TAG=s0 timeout -k 10 300 python -u tests/tools/conv_phases.py $L > gpurun_out/r05/cvp_s0.log 2>&1
rc=$?
[ $rc -eq 0 ] && CVP_TAG=s40 HFG_STAGGER=40,0 timeout -k 10 300 python -u tests/tools/conv_phases.py $L > gpurun_out/r05/cvp_s40.log 2>&1
rc2=$?
cp /tmp/base.so $L
echo "rc=$rc/$rc2"
