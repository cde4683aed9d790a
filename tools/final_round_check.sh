#!/usr/bin/env bash
# Round-end check on the GPU box: full GPU suite, smoke, the N = 1 bench, and
# the documented N > 1 commands as processes on one GPU (the driver's N = 2 /
# N = 8 lines, the N = 4 line with the node gate forced on every connect as on
# a node, configs[3] and configs[4] standalone, and a 5 s budget that must skip
# legs yet still print the line).  Each step under its own limit; stops at the
# first step that faults or times out (tools/gpu_step.sh).  SKIP_TESTS=1 skips
# the suite (when it ran in a call of its own).
rm -f gpurun_out/steps.log
TR="python -m torch.distributed.run --nnodes=1 --master-addr 127.0.0.1"
S=tools/gpu_step.sh
[ -n "$SKIP_TESTS" ] || $S tests 900 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread || exit 1
$S smoke 200 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
$S n1 200 python bench.py || exit 1
$S r_n2 400 $TR --nproc-per-node 2 --master-port 29871 bench.py --gpus 2 || exit 1
$S r_n8 600 $TR --nproc-per-node 8 --master-port 29872 bench.py --gpus 8 || exit 1
MCCS_GATE=1 $S r_n4_gate 600 $TR --nproc-per-node 4 --master-port 29876 bench.py --gpus 4 || exit 1
$S r_n4_fp16 400 $TR --nproc-per-node 4 --master-port 29873 bench.py --gpus 4 --dtype float16 --size-mib 1024 --no-extra || exit 1
MCCS_BENCH_SETUP2_MIN_WORLD=4 $S r_n4_setup2 400 $TR --nproc-per-node 4 --master-port 29874 bench.py --gpus 4 --jobs setup2 || exit 1
MCCS_BENCH_BUDGET_S=5 $S r_budget 400 $TR --nproc-per-node 2 --master-port 29875 bench.py --gpus 2 || exit 1
cat gpurun_out/steps.log
