# per-kernel breakdown of the small-batch configs (C1 [1,80,256]; C5-shaped [32,80,63])
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --batch 1 --frames 256 --no-extra --no-cpu-baseline --no-pmc --also --steps 20 --streams 1 > gpurun_out/bench_c1.json 2> gpurun_out/bench_c1.err && \
timeout -k 10 300 python bench.py --batch 32 --frames 63 --no-extra --no-cpu-baseline --no-pmc --also --steps 20 --streams 1 > gpurun_out/bench_c5shape.json 2> gpurun_out/bench_c5shape.err
