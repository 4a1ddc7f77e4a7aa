#!/bin/bash
# round 6: what bounds the upsamplers — timing-only ablations (HFG_ABLATE=1 build, ab/abl.so) of
# the input loads (1024), the staging conversion + LDS store (512), the weight-slab DMA after
# group 0 (131072) and the epilogue stores (262144), per-kernel ms in the 1-stream pass
cd "$(dirname "$0")/../.."
L=tts-sambert_hifigan_amd/libhifigan_hip.so
O=gpurun_out/r06/ab
mkdir -p $O
cp $L /tmp/ab_base.so
cp tts-sambert_hifigan_amd/ab/abl.so $L
for i in 1 2; do
  for f in 0 1024 512 131072 262144 132096; do
    timeout -k 10 200 python -u bench.py --also --no-extra --no-cpu-baseline --no-pmc --steps 10 \
      --sched DEBUG_FLAGS=$f > $O/upsabl_${f}_$i.json 2> $O/upsabl_${f}_$i.err
    rc=$?
    if [ $rc -ne 0 ]; then cp /tmp/ab_base.so $L; echo "bench $f rc=$rc"; exit $rc; fi
    python3 -c "
import json
d=[json.loads(l) for l in open('$O/upsabl_${f}_$i.json') if l.startswith('{')][-1]
print('flags $f', ' '.join(f\"{k.split(',')[0][:12]}..{k[-6:]} {v['ms_per_step']:.3f}\" for k,v in d['kernels'].items() if k.startswith('ups')))"
  done
done
cp /tmp/ab_base.so $L
echo "ablate done"
