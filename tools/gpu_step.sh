#!/usr/bin/env bash
# Runs GPU steps in order under their own time limits; stops at the first
# step that faults/aborts/times out (exit >= 2, except pytest's 1 = failures).
# usage: tools/gpu_step.sh "<name>" <timeout_s> <cmd...>   (appends to gpurun_out/steps.log)
set -u
name="$1"; shift
tlim="$1"; shift
mkdir -p gpurun_out
start=$(date +%s)
timeout -k 10 "$tlim" "$@" > "gpurun_out/${name}.log" 2>&1
rc=$?
echo "$name rc=$rc secs=$(( $(date +%s) - start ))" | tee -a gpurun_out/steps.log
if [ $rc -ge 2 ]; then
  echo "step $name ended with $rc: stopping" | tee -a gpurun_out/steps.log
  tail -n 40 "gpurun_out/${name}.log"
  exit $rc
fi
exit 0
