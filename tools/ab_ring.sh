set -e
for r in 1 2; do
for v in ${AB_VARIANTS:-base inNt inNtOutNt inNtOutWt fifoNt}; do
  if [ $v = base ]; then unset MCCS_LIB_PATH; else export MCCS_LIB_PATH=$PWD/exp/$v.so; fi
  echo "== $v" >> gpurun_out/ab_ring.log
  timeout -k 10 120 python tools/vnode_bench.py --n 2 4 8 --sizes-mib ${AB_SIZES:-128} --iters 20 >> gpurun_out/ab_ring.log 2>&1
done
done
