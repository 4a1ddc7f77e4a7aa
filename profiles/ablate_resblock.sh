mkdir -p gpurun_out
for f in 0 16 32 64 128 240; do
  HFG_DEBUG_FLAGS=$f timeout -k 10 120 python bench.py --no-cpu-baseline --also --no-extra --steps 5 > gpurun_out/abl_$f.json 2> gpurun_out/abl_$f.err || exit 1
done
