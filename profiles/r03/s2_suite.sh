O=gpurun_out/s2suite; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gputest.txt 2>&1 || { tail -30 $O/gputest.txt; exit 1; }
tail -2 $O/gputest.txt
timeout -k 10 120 python __graft_entry__.py smoke > $O/smoke.log 2>&1 || exit 1
tail -1 $O/smoke.log
echo done
