O=gpurun_out/s2post4; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_properties.py -m gpu -x -q -k "conv_post_quad or max_length or golden_fixture or ups_frames" --timeout 120 --timeout-method thread > $O/parity.txt 2>&1 || { tail -40 $O/parity.txt; exit 1; }
tail -2 $O/parity.txt
bash profiles/r03/ab_env.sh s2post4/ab "HFG_POST4=1" "HFG_POST4=0" --streams 1 || exit 1
echo done
