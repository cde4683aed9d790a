#!/usr/bin/env bash
# The reference launch shape (2 channels x one 544-thread workgroup) on a
# 2-rank virtual node, 128 MiB fp32, eager, under each hand-off mode (the
# factor study of profiles/r0*_reference_shape_factor_study.json).  Writes
# gpurun_out/factor_<k>.log; run from the repo root on the GPU box.
set -u
mkdir -p gpurun_out
run() {
  local k=$1; shift
  env "$@" MCCS_CHANNELS=2 timeout -k 10 120 python tools/vnode_bench.py --n 2 --sizes-mib 128 --lanes 1 --block 544 \
    --iters 10 > "gpurun_out/factor_$k.log" 2>&1 || { echo "factor $k failed $?"; exit 3; }
}
run 1 MCCS_FIFO_MEMORY=device MCCS_SLICE_STEPS=2 MCCS_FIFO_SLOTS=8 MCCS_LOCALITY=sender
run 2 MCCS_FIFO_MEMORY=uncached MCCS_SLICE_STEPS=2 MCCS_FIFO_SLOTS=8 MCCS_LOCALITY=sender
run 3 MCCS_FIFO_MEMORY=release MCCS_SLICE_STEPS=2 MCCS_FIFO_SLOTS=8 MCCS_LOCALITY=sender
run 4 MCCS_FIFO_MEMORY=device MCCS_FIFO_SLOTS=8 MCCS_LOCALITY=sender
run 5 MCCS_FIFO_MEMORY=device MCCS_SLICE_STEPS=2 MCCS_FIFO_SLOTS=8 MCCS_LOCALITY=receiver
run 6 MCCS_UNUSED=0
echo "factor study done"
