for f in 0 1 2 3; do HFG_DEBUG_FLAGS=$f timeout -k 10 120 python bench.py --steps 5 --warmup 2 --precision bf16x3 --also --no-cpu-baseline > gpurun_out/abl_$f.json 2>/dev/null || exit 1; done
