#!/usr/bin/env bash
# Full GPU suite, smoke, the N = 1 bench and the AllGather direct sweep, each
# under its own limit; stops at the first step that faults or times out.
set -o pipefail
tools/gpu_step.sh tests 800 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread && \
tools/gpu_step.sh smoke 200 python -c "import __graft_entry__ as g; g.smoke()" && \
tools/gpu_step.sh n1 200 python bench.py && \
tools/gpu_step.sh agbench 200 python tools/direct_bench.py --allgather --n 2 4 8 --sizes-kib 4 32 128 512
