timeout -k 10 300 python bench.py > gpurun_out/bench12.json 2> gpurun_out/bench12.err && \
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 3 --warmup 1 --dist-backend gloo --also > gpurun_out/bench12_n2gloo.json 2> gpurun_out/bench12_n2gloo.err && \
bash profiles/run_rocprof.sh r01
