# Same-box A/B on the GPU box: bench with the working tree's library (new) and the
# HEAD build (libhifigan_hip.so.old), alternated twice.  usage: bash profiles/ab_run.sh TAG [bench args]
T=${1:-ab}; shift
L=tts-sambert_hifigan_amd/libhifigan_hip.so
cp $L /tmp/ab_new.so
for i in 1 2; do
  cp /tmp/ab_new.so $L && timeout -k 10 150 python bench.py --also --no-extra --no-cpu-baseline --steps 20 "$@" > gpurun_out/${T}_new$i.json 2>/dev/null || exit 1
  cp $L.old $L && timeout -k 10 150 python bench.py --also --no-extra --no-cpu-baseline --steps 20 "$@" > gpurun_out/${T}_old$i.json 2>/dev/null || exit 1
done
cp /tmp/ab_new.so $L
