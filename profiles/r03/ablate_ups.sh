# Upsampler phase ablation (wrong results: timing only).  HFG_DEBUG_FLAGS bits of
# conv1d_bf16x3: 8 = no epilogue, 128 = input staging always re-reads channel group 0
# (L2-warm loads), 256 = upsampler staging stores the raw fp32 halves (no leaky_relu, no
# hi/lo split); 1-stream profiled pass, per-kernel ms/step.
# usage (GPU box): bash profiles/r03/ablate_ups.sh TAG
T=${1:-upsabl}
mkdir -p gpurun_out/$T
for f in 0 8 128 256 384 392; do
  HFG_DEBUG_FLAGS=$f timeout -k 10 150 python bench.py --also --no-extra --no-cpu-baseline --no-pmc \
    --steps 20 > gpurun_out/$T/dbg$f.json 2>/dev/null || exit 1
done
python profiles/r03/show_kernels.py gpurun_out/$T/dbg*.json
