#!/usr/bin/env bash
# rocprofv3 passes over the ring AllReduce on an n-rank virtual node (one GPU):
#   1. --kernel-trace --stats   per-launch duration of the fused ring kernel,
#                               n = 2 / 4 / 8 at the BASELINE bucket (128 MiB fp32)
#   2. --pmc FETCH_SIZE, 3. --pmc WRITE_SIZE (separate passes): HBM bytes per
#      launch at n = 2 (tools/summarize_ring_profile.py compares them with the
#      algorithmic (6n-4)*S)
# Run on the GPU box from the repo root.  Stops at the first failing pass.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d "$OUT/prof_ring_trace" -o trace \
  -- python3 "$R/tools/vnode_bench.py" --n 2 4 8 --sizes-mib 128 --iters 10 > "$OUT/prof_ring_trace.log" 2>&1 \
  || { echo "ring trace failed $?"; exit 3; }
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $C --kernel-trace -T --output-format csv -d "$OUT/prof_ring_$C" -o pmc \
    --kernel-include-regex "ring_multi" -- python3 "$R/tools/vnode_bench.py" --n 2 --sizes-mib 128 --iters 10 \
    > "$OUT/prof_ring_$C.log" 2>&1 || { echo "ring pmc $C failed $?"; exit 3; }
done
echo "ring profile done"
