# rocprofv3 kernel-trace stats + separate FETCH_SIZE / WRITE_SIZE passes of bench.py
# (PMC passes carry no trace domains: MI355X_MICROARCH.md §HBM / gpurun rules).
# usage on the GPU box:  bash profiles/run_rocprof.sh <tag>
# (--streams 1: per-dispatch durations match bench.py's 1-stream roofline pass; --no-pmc:
#  bench.py's own live PMC child passes are not started under the profiler)
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
T=${1:-cur}
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_$T -o run --output-format csv -- python $R/bench.py --steps 5 --warmup 2 --also --no-cpu-baseline --no-extra --no-pmc --streams 1 > $R/gpurun_out/prof_${T}_bench.json 2> $R/gpurun_out/prof_${T}_bench.err && \
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $R/gpurun_out/pmc_fetch_$T -o run --output-format csv -- python $R/bench.py --steps 2 --warmup 1 --also --no-cpu-baseline --no-extra --no-pmc --streams 1 --no-profile > $R/gpurun_out/pmc_fetch_$T.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $R/gpurun_out/pmc_write_$T -o run --output-format csv -- python $R/bench.py --steps 2 --warmup 1 --also --no-cpu-baseline --no-extra --no-pmc --streams 1 --no-profile > $R/gpurun_out/pmc_write_$T.log 2>&1
