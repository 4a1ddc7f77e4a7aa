# Build the committed HEAD's library as libhifigan_hip.so.old next to the working tree's
# build (same-box A/B of an uncommitted kernel change; see profiles/ab_run.sh).
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
T=$(mktemp -d)
git -C "$R" archive HEAD tts-sambert_hifigan_amd include | tar -x -C "$T"
python "$T/tts-sambert_hifigan_amd/build.py" --force > /dev/null
cp "$T/tts-sambert_hifigan_amd/libhifigan_hip.so" "$R/tts-sambert_hifigan_amd/libhifigan_hip.so.old"
rm -rf "$T"
python "$R/tts-sambert_hifigan_amd/build.py" > /dev/null
