# Session-2 re-entry check (GPU box): GPU suite, smoke, default bench, kernel trace of C2.
O=gpurun_out/s2
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gputest.txt 2>&1 || { tail -30 $O/gputest.txt; exit 1; }
tail -3 $O/gputest.txt
timeout -k 10 120 python __graft_entry__.py smoke > $O/smoke.log 2>&1 || exit 1
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err || exit 1
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/c2 -o run --output-format csv -- \
  python bench.py --steps 5 --warmup 2 --streams 1 --no-extra --no-cpu-baseline --no-pmc --also \
  > $O/c2_bench.json 2> $O/c2_bench.err || exit 1
echo done
