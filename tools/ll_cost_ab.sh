# A/B of the LL one-shot's guard prologue (profiles/r06_ll_prefetch_ab.json):
# libmccs_hip.so per variant under abvar/<variant>/ (git-ignored), loaded via
# MCCS_LIB_PATH.  Per variant, interleaved 3x: graph-replayed LL AllReduce
# (32 KiB fp16) on the virtual node at n = 2 / 4 / 8 (tools/guard_control.py
# cost, guard on), and the 2-process N = 2 rehearsal, whose direct sweep
# times the one-slot (deployment-shape) LL launch.
set -e
TR="python -m torch.distributed.run --nnodes=1 --master-addr 127.0.0.1"
for i in 1 2 3; do
 for v in prev new; do
  export MCCS_LIB_PATH=$PWD/abvar/$v/libmccs_hip.so
  timeout -k 10 120 python -c "
import json, sys
sys.path.insert(0, 'tools')
import guard_control as g
out = {n: g.cost(n, 'll', 32 << 10, True)[1:] for n in (2, 4, 8)}
print(json.dumps(out))" > gpurun_out/llab_vnode_${v}_$i.log 2>&1
  timeout -k 10 200 $TR --nproc-per-node 2 --master-port 2992$i bench.py --gpus 2 > gpurun_out/llab_n2_${v}_$i.log 2>&1
  echo "$v $i done"
 done
done
