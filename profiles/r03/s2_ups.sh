# ups frames kernel: parity subset, then same-box A/B against the polyphase path
O=gpurun_out/s2ups; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 120 --timeout-method thread > $O/parity.txt 2>&1 || { tail -40 $O/parity.txt; exit 1; }
tail -3 $O/parity.txt
bash profiles/r03/ab_env.sh s2ups/ab "HFG_UPS_FRAMES=1" "HFG_UPS_FRAMES=0" --streams 1 || exit 1
echo done
