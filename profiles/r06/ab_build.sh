#!/bin/bash
# Build a variant of the working tree's library with extra compiler flags into
# tts-sambert_hifigan_amd/ab/NAME.so (same-box A/B: profiles/r06/lib_ab.sh), then restore the
# default build.  usage: bash profiles/r06/ab_build.sh NAME "FLAGS"
set -e
R=$(cd "$(dirname "$0")/../.." && pwd)
N=$1; F=$2
mkdir -p "$R/tts-sambert_hifigan_amd/ab"
HFG_EXTRA_FLAGS="$F" python "$R/tts-sambert_hifigan_amd/build.py" > /dev/null
cp "$R/tts-sambert_hifigan_amd/libhifigan_hip.so" "$R/tts-sambert_hifigan_amd/ab/$N.so"
python "$R/tts-sambert_hifigan_amd/build.py" > /dev/null
echo "built ab/$N.so with [$F]"
