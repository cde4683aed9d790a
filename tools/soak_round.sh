rm -f gpurun_out/steps.log
TR="python -m torch.distributed.run --nnodes=1 --master-addr 127.0.0.1"
S=tools/gpu_step.sh
$S soak_p2_128 300 $TR --nproc-per-node 2 --master-port 29881 tools/soak.py --iters 20000 --check-every 2000 || exit 1
$S soak_p4_16 300 $TR --nproc-per-node 4 --master-port 29882 tools/soak.py --iters 10000 --size-mib 16 --check-every 2000 || exit 1
$S soak_v8_16 300 python tools/soak.py --vnode 8 --iters 20000 --size-mib 16 --check-every 2000 || exit 1
$S soak_v4_128 300 python tools/soak.py --vnode 4 --iters 5000 --size-mib 128 --check-every 1000 || exit 1
$S soak_ll_v8 240 python tools/soak.py --vnode 8 --size-kib 64 --iters 30000 --check-every 5000 || exit 1
$S soak_ll_p2 240 $TR --nproc-per-node 2 --master-port 29883 tools/soak.py --size-kib 32 --iters 100000 --check-every 5000 || exit 1
$S soak_p2_2m 240 $TR --nproc-per-node 2 --master-port 29884 tools/soak.py --size-kib 2048 --iters 50000 --check-every 5000 || exit 1
cat gpurun_out/steps.log
