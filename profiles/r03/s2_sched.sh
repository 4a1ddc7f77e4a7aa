O=gpurun_out/s2sched; mkdir -p $O
bash profiles/r03/ab_libs.sh s2sched/ab base xt3 xt5 nv1 nv3 st4 st8 || exit 1
echo done
