# whole-ResBlock ablations (timings only; HFG_DEBUG_FLAGS makes results wrong): 16 = no MRF epilogue
mkdir -p gpurun_out
for f in 0 16 0 16; do
HFG_DEBUG_FLAGS=$f timeout -k 10 300 python bench.py --no-extra --no-cpu-baseline --no-pmc --also --streams 1 --steps 10 > gpurun_out/bench_rbabl_$f.json 2>/dev/null || exit 1
done
