# C1 leg: kernel + HIP API trace (which copies run per forward)
O=gpurun_out/s2c1; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --kernel-trace --hip-trace -d $GRAFT_REPO_ROOT/$O/t -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/profiles/r03/legs.py c1 > $GRAFT_REPO_ROOT/$O/c1.txt 2>&1 || exit 1
echo done
