#!/usr/bin/env bash
# rocprofv3 passes over the headline bench (run on the GPU box from the repo root):
#   1. --kernel-trace --stats      per-kernel durations (profiles/*_stats.csv)
#   2. --pmc FETCH_SIZE             HBM read side  (separate pass; gfx950: x2 for wide streams)
#   3. --pmc WRITE_SIZE             HBM write side (separate pass)
# Extra args are passed to bench.py.  Stops at the first failing pass.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
TAG=${PROF_TAG:-reduce}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
# the bench's own defaults (50 timed steps after 10 warm-up); --no-hot: no
# same-buffer (cache-assisted) launches of the same kernel in the average
BENCH=(python3 "$R/bench.py" --no-cpu-baseline --no-hot "$@")
timeout -k 10 400 rocprofv3 --kernel-trace --stats -T --output-format csv -d "$OUT/prof_${TAG}_trace" -o trace \
  -- "${BENCH[@]}" > "$OUT/prof_${TAG}_trace.log" 2>&1 || { echo "trace pass failed $?"; exit 3; }
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 400 rocprofv3 --pmc $C --kernel-trace -T --output-format csv -d "$OUT/prof_${TAG}_$C" -o pmc \
    --kernel-include-regex "reduce_" -- "${BENCH[@]}" > "$OUT/prof_${TAG}_$C.log" 2>&1 || { echo "pmc $C failed $?"; exit 3; }
done
echo "profile passes done"
