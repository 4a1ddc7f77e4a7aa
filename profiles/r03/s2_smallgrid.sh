# C1 / C5 / stream16 legs with the small-grid threshold at 256 (default), 160, 96
O=gpurun_out/s2sg; mkdir -p $O; rm -f $O/legs.txt
for i in 1 2 3; do
  for g in 256 384 640; do
    for leg in c1 c5 stream16; do
      r=$(HFG_SMALL_GRID=$g timeout -k 10 120 python profiles/r03/legs.py $leg 2>/dev/null | tail -1) || exit 1
      echo "$i grid=$g $r" >> $O/legs.txt
    done
  done
done
cat $O/legs.txt
echo done
