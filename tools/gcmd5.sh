# round 5 final-code check: GPU suite (incl. the DDP-stream tests), smoke, N=1 bench, rocprof passes,
# host<->device rate, and the N=4 command with the node gate forced on every connect
rm -f gpurun_out/steps.log
TR="python -m torch.distributed.run --nnodes=1 --master-addr 127.0.0.1"
S=tools/gpu_step.sh
$S tests 900 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread || exit 1
$S smoke 200 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
$S n1 200 python bench.py || exit 1
$S e2e 200 python -u tools/e2e_rate.py || exit 1
MCCS_GATE=1 $S bench_n4_gate 600 $TR --nproc-per-node 4 --master-port 29831 bench.py --gpus 4 || exit 1
PROF_TAG=r05 $S prof 900 bash tools/profile_reduce.sh || exit 1
cat gpurun_out/steps.log
