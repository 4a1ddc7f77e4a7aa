# upsampler ablations (timings only; HFG_DEBUG_FLAGS makes results wrong): 128 = L2-warm
# input loads (always channel group 0), 1 = no input restaging after the first chunk,
# 8 = no epilogue
mkdir -p gpurun_out
for f in 0 128 1 8; do
HFG_DEBUG_FLAGS=$f timeout -k 10 300 python bench.py --no-extra --no-cpu-baseline --no-pmc --also --streams 1 --steps 10 > gpurun_out/bench_upsabl_$f.json 2>/dev/null || exit 1
done
