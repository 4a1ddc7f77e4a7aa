#!/bin/bash
# round 5, call 15: the driver's multi-rank launch form (torch.distributed.run, 4 ranks) on the
# one-GPU box with the gloo backend (RCCL needs one device per rank): sharding, barrier,
# max-over-ranks timing and the JSON line of an N = 4 run
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out/r05
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 \
  --master-port 29511 bench.py --gpus 4 --steps 5 --warmup 2 --dist-backend gloo \
  > gpurun_out/r05/bench_n4_gloo.json 2> gpurun_out/r05/bench_n4_gloo.err
rc=$?; echo "n4 rc=$rc"; tail -c 600 gpurun_out/r05/bench_n4_gloo.json
exit $rc
