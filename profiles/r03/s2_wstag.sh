# layer-conv block stagger experiment (HFG_DEBUG_FLAGS = 4096 | n << 16: odd-slot waves start
# n x 512 cycles late), 1-stream bench (per-kernel times) and value pass
O=gpurun_out/s2wstag; mkdir -p $O
for i in 1 2; do
  for n in 0 8 16 32; do
    f=$(( n > 0 ? 4096 + (n << 16) : 0 ))
    HFG_DEBUG_FLAGS=$f timeout -k 10 150 python bench.py --also --no-extra --no-cpu-baseline --no-pmc --steps 20 --streams 1 > $O/n${n}_s1_$i.json 2>/dev/null || exit 1
    HFG_DEBUG_FLAGS=$f timeout -k 10 150 python bench.py --also --no-extra --no-cpu-baseline --no-pmc --no-profile --steps 20 > $O/n${n}_s2_$i.json 2>/dev/null || exit 1
  done
done
echo done
