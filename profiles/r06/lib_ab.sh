#!/bin/bash
# Same-box A/B of library builds (round 6): bench.py (f16x3 value pass, 2 streams + the 1-stream
# per-kernel pass, wav checksum) with the tree's library ("base") and each
# tts-sambert_hifigan_amd/ab/NAME.so, alternated ROUNDS times (default 2).
# usage: bash profiles/r06/lib_ab.sh TAG NAME...      (env ROUNDS, STEPS)
cd "$(dirname "$0")/../.."
T=$1; shift
L=tts-sambert_hifigan_amd/libhifigan_hip.so
O=gpurun_out/r06/ab
mkdir -p $O
cp $L /tmp/ab_base.so
for i in $(seq 1 ${ROUNDS:-2}); do
  for n in base "$@"; do
    if [ "$n" == base ]; then cp /tmp/ab_base.so $L; else cp tts-sambert_hifigan_amd/ab/$n.so $L; fi
    timeout -k 10 200 python -u bench.py --also --no-extra --no-cpu-baseline --no-pmc \
      --steps ${STEPS:-20} > $O/${T}_${n}_$i.json 2> $O/${T}_${n}_$i.err
    rc=$?
    if [ $rc -ne 0 ]; then cp /tmp/ab_base.so $L; echo "bench $n rc=$rc"; exit $rc; fi
    python3 profiles/r06/ab_show.py $O/${T}_${n}_$i.json
  done
done
cp /tmp/ab_base.so $L
echo "ab done"
