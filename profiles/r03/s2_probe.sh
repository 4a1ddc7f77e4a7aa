O=gpurun_out/s2probe; mkdir -p $O
timeout -k 10 60 ./tests/tools/buffer_range_probe > $O/probe.txt 2>&1 || exit 1
cat $O/probe.txt
HFG_FUSED_RB=0 timeout -k 10 300 python -u -m pytest tests/test_gpu_properties.py -m gpu -x -q -k "max_length" --timeout 200 --timeout-method thread > $O/maxlen_nofused.txt 2>&1; tail -2 $O/maxlen_nofused.txt
echo done
