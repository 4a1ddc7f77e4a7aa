# Last check of the committed tree: GPU suite, smoke, default bench line (GPU box)
O=gpurun_out/finalcheck; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gputest.txt 2>&1 || { tail -30 $O/gputest.txt; exit 1; }
tail -1 $O/gputest.txt
timeout -k 10 120 python __graft_entry__.py smoke > $O/smoke.log 2>&1 || exit 1
tail -1 $O/smoke.log
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || exit 1
python -c "import json;d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]);print(d['value'],d['ms_per_step'],d['roofline']['frac'])"
