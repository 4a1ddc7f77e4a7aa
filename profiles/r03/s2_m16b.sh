O=gpurun_out/s2m16b; mkdir -p $O
for i in 1 2 3; do
  for m in 1 0; do
    HFG_MFMA16=$m timeout -k 10 150 python bench.py --also --no-extra --no-cpu-baseline --no-pmc --no-profile --steps 30 > $O/m${m}_$i.json 2>/dev/null || exit 1
  done
done
for i in 1 2; do
  for m in 1 0; do
    for leg in c1 c5 stream16; do
      r=$(HFG_MFMA16=$m timeout -k 10 120 python profiles/r03/legs.py $leg 2>/dev/null | tail -1) || exit 1
      echo "$i mfma16=$m $r" >> $O/legs.txt
    done
  done
done
cat $O/legs.txt
echo done
