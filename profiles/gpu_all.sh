#!/bin/bash
# the full GPU test suite + C3* bench through torchrun (1 rank) (GPU box)
set -e
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -q -x --timeout 400 --timeout-method thread -m gpu > gpurun_out/gpu_all.log 2>&1
tail -2 gpurun_out/gpu_all.log
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 1 --steps 5 --warmup 2 --no-cpu > gpurun_out/bench_trun.log 2>&1
tail -1 gpurun_out/bench_trun.log | cut -c1-400
