# rocprofv3 kernel-trace summaries of the headline workload and every other BASELINE leg
# (GPU box).  usage: bash profiles/r03/prof_legs.sh OUTDIR
O=${1:-gpurun_out/legs}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/c2 -o run --output-format csv -- \
  python bench.py --steps 5 --warmup 2 --streams 1 --no-extra --no-cpu-baseline --no-pmc --also \
  > $O/c2_bench.json || exit 1
for leg in c1 c4 c5 mel stream16; do
  timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $O/$leg -o run --output-format csv -- \
    python profiles/r03/legs.py $leg > $O/$leg.txt || exit 1
done
