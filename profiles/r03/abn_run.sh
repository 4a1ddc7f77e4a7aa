# Same-box comparison of several library builds: bench (1-stream profiled pass included) with
# each tts-sambert_hifigan_amd/libhifigan_hip.so.<variant>, alternated twice.
# usage (GPU box): bash profiles/r03/abn_run.sh TAG variant1 variant2 ...  [-- bench args]
T=$1; shift
V=(); while [ $# -gt 0 ] && [ "$1" != "--" ]; do V+=("$1"); shift; done; [ "$1" = "--" ] && shift
L=tts-sambert_hifigan_amd/libhifigan_hip.so
cp $L /tmp/abn_keep.so
mkdir -p gpurun_out/$T
for i in 1 2; do
  for v in "${V[@]}"; do
    cp $L.$v $L && timeout -k 10 150 python bench.py --also --no-extra --no-cpu-baseline --no-pmc \
      --steps 20 "$@" > gpurun_out/$T/${v}_$i.json 2>/dev/null || { cp /tmp/abn_keep.so $L; exit 1; }
  done
done
cp /tmp/abn_keep.so $L
python profiles/r03/show_kernels.py gpurun_out/$T/*_1.json gpurun_out/$T/*_2.json
