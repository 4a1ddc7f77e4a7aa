O=gpurun_out/s2sched2; mkdir -p $O
bash profiles/r03/ab_libs.sh s2sched2/ab base xt5 xt6 || exit 1
echo done
