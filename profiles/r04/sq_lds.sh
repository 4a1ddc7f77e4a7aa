#!/bin/bash
# one SQ counter pass (LDS bank conflicts + MFMA busy) over a short f16x3 bench with library $1
# (default: the in-tree build), output under gpurun_out/r04/$2
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
L=$R/tts-sambert_hifigan_amd/libhifigan_hip.so
mkdir -p $R/gpurun_out/r04
cp $L /tmp/sq_base.so
if [ -n "$1" ]; then cp $R/tts-sambert_hifigan_amd/ab/$1.so $L; fi
timeout -s KILL 240 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES \
  -d $R/gpurun_out/r04/$2 -o run --output-format csv -- python $R/bench.py --steps 2 --warmup 1 --also --no-cpu-baseline --no-profile --no-extra --no-pmc > $R/gpurun_out/r04/$2.log 2>&1
rc=$?
cp /tmp/sq_base.so $L
echo "sq $2 rc=$rc"
exit $rc
