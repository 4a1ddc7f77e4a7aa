O=gpurun_out/s2prio; mkdir -p $O
bash profiles/r03/ab_libs.sh s2prio/ab prio1 prio0 || exit 1
echo done
