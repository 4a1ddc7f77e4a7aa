# tile-5 early input loads for short-tap convs: parity, then same-box library A/B (GPU box)
O=gpurun_out/xe; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_stages.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/test.txt 2>&1 || { tail -30 $O/test.txt; exit 1; }
tail -1 $O/test.txt
bash profiles/r03/ab_libs.sh xe xe0 xe3 xe7 || exit 1
python profiles/r03/show_ab.py gpurun_out/xe
