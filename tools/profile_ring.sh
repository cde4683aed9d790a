#!/usr/bin/env bash
# rocprofv3 kernel trace of the ring AllReduce on an n-rank virtual node (one
# GPU): per-launch duration of the fused ring kernel at BASELINE bucket size.
# Run on the GPU box from the repo root.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d "$OUT/prof_ring_trace" -o trace \
  -- python3 "$R/tools/vnode_bench.py" --n 2 4 8 --sizes-mib 128 --iters 10 > "$OUT/prof_ring_trace.log" 2>&1 \
  || { echo "ring trace failed $?"; exit 3; }
echo "ring profile done"
