# ups small-tile occupancy 3 vs 2: bitwise ups test, then same-box A/B (GPU box)
O=gpurun_out/occ; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "ups_frames" > $O/test.txt 2>&1 || { tail -30 $O/test.txt; exit 1; }
tail -1 $O/test.txt
bash profiles/r03/ab_libs.sh occ occ3 occ2 || exit 1
python profiles/r03/show_ab.py gpurun_out/occ
