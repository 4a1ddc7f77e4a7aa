# Same-box A/B of library variants (tts-sambert_hifigan_amd/libhifigan_hip.so.NAME) on the
# headline bench (1 stream, per-kernel times), alternated twice (GPU box).
# usage: bash profiles/r03/ab_libs.sh TAG name1 name2 ... [-- bench args]
T=$1; shift
V=(); while [ $# -gt 0 ] && [ "$1" != "--" ]; do V+=("$1"); shift; done; [ "$1" = "--" ] && shift
L=tts-sambert_hifigan_amd/libhifigan_hip.so
cp $L /tmp/abl_keep.so; mkdir -p gpurun_out/$T
for i in 1 2 3; do
  for v in "${V[@]}"; do
    cp $L.$v $L
    timeout -k 10 150 python bench.py --also --no-extra --no-cpu-baseline --no-pmc --steps 20 --streams 1 "$@" > gpurun_out/$T/${v}_$i.json 2>/dev/null || { cp /tmp/abl_keep.so $L; exit 1; }
  done
done
cp /tmp/abl_keep.so $L
