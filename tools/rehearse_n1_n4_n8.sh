#!/usr/bin/env bash
# The driver's bench commands on the 1-GPU box: N = 1, then N = 4 and N = 8
# as processes sharing the GPU (rehearsals; outputs under gpurun_out/).
set -o pipefail
tools/gpu_step.sh n1 200 python bench.py && \
tools/gpu_step.sh n4 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29513 bench.py --gpus 4 --steps 10 --warmup 3 && \
tools/gpu_step.sh n8 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29514 bench.py --gpus 8 --steps 10 --warmup 3
