cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r06
for p in f16x3 bf16x3; do
  timeout -k 10 240 rocprofv3 --kernel-trace -d gpurun_out/r06/c1_$p -o run --output-format csv -- python3 tests/tools/layer_times.py run --precision $p --batch 1 --frames 256 > gpurun_out/r06/c1_$p.log 2>&1 || exit 1
done
echo done
