# bf16x3 kernel ablations (HFG_DEBUG_FLAGS bits, see csrc/kernels.h): per-kernel ms for each flag set
# usage: bash profiles/ablate_bf16x3.sh TAG "0 1 2 3 4 8 16 31"
T=${1:-abl}
for f in ${2:-0 1 2 4 8 16 3 7 15}; do
  HFG_DEBUG_FLAGS=$f timeout -k 10 120 python bench.py --steps 5 --warmup 2 --precision bf16x3 --no-cpu-baseline --no-extra --also > gpurun_out/${T}_$f.json 2>/dev/null || exit 1
done
