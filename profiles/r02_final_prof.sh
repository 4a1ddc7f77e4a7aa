# round-2 profile set: default bench line, rocprofv3 kernel stats + PMC passes
mkdir -p gpurun_out
timeout -k 10 600 python bench.py > gpurun_out/bench_r02.json 2> gpurun_out/bench_r02.err || exit 1
bash profiles/run_rocprof.sh r02
