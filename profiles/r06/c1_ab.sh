#!/bin/bash
# Same-box A/B of library builds on the C1 latency config (profiles/r06/c1_time.py), alternated.
# usage: bash profiles/r06/c1_ab.sh NAME...     (env ROUNDS, default 3; SHAPES, default "256x1":
# space-separated FRAMESxBATCH shapes)
cd "$(dirname "$0")/../.."
L=tts-sambert_hifigan_amd/libhifigan_hip.so
cp $L /tmp/c1ab_base.so
for i in $(seq 1 ${ROUNDS:-3}); do
  for n in base "$@"; do
    if [ "$n" == base ]; then cp /tmp/c1ab_base.so $L; else cp tts-sambert_hifigan_amd/ab/$n.so $L; fi
    for shape in ${SHAPES:-256x1}; do
      echo -n "$n: "
      timeout -k 10 120 python -u profiles/r06/c1_time.py f16x3 ${shape%x*} ${shape#*x} 2>&1 | tail -1
      rc=$?
      if [ $rc -ne 0 ]; then cp /tmp/c1ab_base.so $L; exit $rc; fi
    done
  done
done
cp /tmp/c1ab_base.so $L
echo "c1 ab done"
