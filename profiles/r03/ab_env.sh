# Same-box A/B of one library under two environment settings, alternated twice (GPU box).
# usage: bash profiles/r03/ab_env.sh TAG "ENV_A" "ENV_B" [bench args]   (ENV "-" = none)
T=$1; A=$2; B=$3; shift 3
mkdir -p gpurun_out/$T
for i in 1 2; do
  for v in A B; do
    e=${!v}
    if [ "$e" = "-" ]; then
      timeout -k 10 150 python bench.py --also --no-extra --no-cpu-baseline --no-pmc --steps 20 "$@" > gpurun_out/$T/${v}$i.json 2>/dev/null || exit 1
    else
      env $e timeout -k 10 150 python bench.py --also --no-extra --no-cpu-baseline --no-pmc --steps 20 "$@" > gpurun_out/$T/${v}$i.json 2>/dev/null || exit 1
    fi
  done
done
