#!/usr/bin/env bash
# LL one-shot soaks at the library defaults: an 8-rank virtual node and two
# processes (IPC), exact-sum checks every 5,000 calls.
set -o pipefail
tools/gpu_step.sh soak_ll_vnode8 240 python tools/soak.py --vnode 8 --size-kib 64 --iters 30000 --check-every 5000 && \
tools/gpu_step.sh soak_ll_ipc2 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 tools/soak.py --size-kib 32 --iters 100000 --check-every 5000
