# Whole-ResBlock kernel phase ablation (wrong results: timing only).  HFG_DEBUG_FLAGS bits of
# resblock*_bf16x3: 16 no MRF epilogue, 32 no x loads, 64 no operand writes.
# usage (GPU box): bash profiles/r03/ablate_rb.sh TAG
T=${1:-rbabl}
mkdir -p gpurun_out/$T
for f in 0 16 32 64 112 0; do
  HFG_DEBUG_FLAGS=$f timeout -k 10 150 python bench.py --also --no-extra --no-cpu-baseline --no-pmc \
    --steps 20 > gpurun_out/$T/dbg$f.json 2>/dev/null || exit 1
done
python profiles/r03/show_kernels.py gpurun_out/$T/dbg*.json
