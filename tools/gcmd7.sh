# round 5 final code: the documented N > 1 commands as processes on one GPU
rm -f gpurun_out/steps.log
TR="python -m torch.distributed.run --nnodes=1 --master-addr 127.0.0.1"
S=tools/gpu_step.sh
$S r_n2 400 $TR --nproc-per-node 2 --master-port 29871 bench.py --gpus 2 || exit 1
$S r_n8 600 $TR --nproc-per-node 8 --master-port 29872 bench.py --gpus 8 || exit 1
$S r_n4_fp16 400 $TR --nproc-per-node 4 --master-port 29873 bench.py --gpus 4 --dtype float16 --size-mib 1024 --no-extra || exit 1
MCCS_BENCH_SETUP2_MIN_WORLD=4 $S r_n4_setup2 400 $TR --nproc-per-node 4 --master-port 29874 bench.py --gpus 4 --jobs setup2 || exit 1
$S r_budget 400 env MCCS_BENCH_BUDGET_S=5 $TR --nproc-per-node 2 --master-port 29875 bench.py --gpus 2 || exit 1
cat gpurun_out/steps.log
