# A/B of ring step persistence (profiles/r06_step_persist_ab.json): one
# libmccs_hip.so per variant under abvar/<variant>/ (git-ignored; build each
# variant in-tree with __graft_entry__.build() and copy it there), loaded
# through MCCS_LIB_PATH; 2- and 4-process rehearsals on one GPU, interleaved.
#   gpurun -- 'bash tools/ab_step_persist.sh'
set -e
TR="python -m torch.distributed.run --nnodes=1 --master-addr 127.0.0.1"
for i in 1 2 3; do
 for v in start end prev; do
  export MCCS_LIB_PATH=$PWD/abvar/$v/libmccs_hip.so
  timeout -k 10 200 $TR --nproc-per-node 4 --master-port 2990$i bench.py --gpus 4 --dtype float16 --size-mib 1024 --no-extra > gpurun_out/ab2_fp16_${v}_$i.log 2>&1
  timeout -k 10 200 $TR --nproc-per-node 2 --master-port 2991$i bench.py --gpus 2 --no-extra > gpurun_out/ab2_n2_${v}_$i.log 2>&1
  echo "$v $i done"
 done
done
