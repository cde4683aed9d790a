# round 5: strip A/B check (virtual node, r04 lib vs stripped), depth-A plain vs nt input with rotated and
# same buffers (2 and 3 processes), N=2 / N=8 one-GPU rehearsals with the budget
rm -f gpurun_out/steps.log
TR="python -m torch.distributed.run --nnodes=1 --master-addr 127.0.0.1"
S=tools/gpu_step.sh
for rep in 1 2; do
  MCCS_LIB_PATH=abvar/libmccs_r04.so $S vnode_r04_$rep 200 python -u tools/vnode_bench.py --n 2 4 8 --sizes-mib 16 128 --graph --iters 20 || exit 1
  $S vnode_r05_$rep 200 python -u tools/vnode_bench.py --n 2 4 8 --sizes-mib 16 128 --graph --iters 20 || exit 1
done
V=ch2_reference_ring_sender,ch2_reference_ring_receiver,ch32_reference_ring_sender
for np in 2 3; do
  for rep in 1 2; do
    for rot in 1152 0; do
      $S refdrv_n${np}_plain_rot${rot}_$rep 240 $TR --nproc-per-node $np --master-port $((29600+np*10+rep)) tools/refdrv_bench.py --variants $V --rotate-mib $rot || exit 1
      MCCS_LIB_PATH=abvar/nt_input.so $S refdrv_n${np}_nt_rot${rot}_$rep 240 $TR --nproc-per-node $np --master-port $((29700+np*10+rep)) tools/refdrv_bench.py --variants $V --rotate-mib $rot || exit 1
    done
  done
done
$S bench_n2 400 $TR --nproc-per-node 2 --master-port 29811 bench.py --gpus 2 || exit 1
$S bench_n8 600 $TR --nproc-per-node 8 --master-port 29812 bench.py --gpus 8 || exit 1
cat gpurun_out/steps.log
