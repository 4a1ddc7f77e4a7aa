O=gpurun_out/s2ups5; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_properties.py -m gpu -x -q -k "ups_frames or max_length or two_stream" --timeout 120 --timeout-method thread > $O/parity.txt 2>&1 || { tail -40 $O/parity.txt; exit 1; }
tail -2 $O/parity.txt
bash profiles/r03/ab_libs.sh s2ups5/ab new old || exit 1
echo done
