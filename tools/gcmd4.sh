# round 5: host<->device rate, the N = 4 command with the node gate forced on every connect (what a node runs),
# the new DDP-stream tests
rm -f gpurun_out/steps.log
TR="python -m torch.distributed.run --nnodes=1 --master-addr 127.0.0.1"
S=tools/gpu_step.sh
$S ddp 600 python -u -m pytest tests/test_gpu_ddp_stream.py -x -v --timeout 400 --timeout-method thread || exit 1
$S e2e 200 python -u tools/e2e_rate.py || exit 1
MCCS_GATE=1 $S bench_n4_gate 600 $TR --nproc-per-node 4 --master-port 29831 bench.py --gpus 4 || exit 1
cat gpurun_out/steps.log
