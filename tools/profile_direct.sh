#!/usr/bin/env bash
# rocprofv3 kernel trace of the direct AllReduce vs the ring on an n-rank
# virtual node (one GPU): per-launch kernel duration of direct_kernel and
# ring_multi_kernel at small / mid buckets (tools/direct_bench.py), next to
# the wall time per call the bench prints (graph replay).
# Run on the GPU box from the repo root.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
TAG=${DIRECT_TAG:-direct}
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d "$OUT/prof_$TAG" -o trace \
  -- python3 "$R/tools/direct_bench.py" --n ${DIRECT_N:-8} --sizes-kib ${DIRECT_KIB:-32 512 2048} --blocks 128 \
  --calls 50 --algos ${DIRECT_ALGOS:-ring direct oneshot ll} > "$OUT/prof_$TAG.log" 2>&1 || { echo "direct trace failed $?"; exit 3; }
echo "direct profile done"
