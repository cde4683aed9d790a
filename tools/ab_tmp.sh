set -e
for r in 1 2; do
for v in old576 old new sleep8; do
echo "== $v" >> gpurun_out/ab3.log
case $v in
 old576) MCCS_LIB_PATH=$PWD/exp/old.so timeout -k 10 100 python tools/vnode_bench.py --block 576 --graph --n 2 4 8 --sizes-mib 4 128 --iters 20 >> gpurun_out/ab3.log 2>&1 ;;
 old) MCCS_LIB_PATH=$PWD/exp/old.so timeout -k 10 100 python tools/vnode_bench.py --block 512 --graph --n 2 4 8 --sizes-mib 4 128 --iters 20 >> gpurun_out/ab3.log 2>&1 ;;
 new) timeout -k 10 100 python tools/vnode_bench.py --graph --n 2 4 8 --sizes-mib 4 128 --iters 20 >> gpurun_out/ab3.log 2>&1 ;;
 sleep8) MCCS_LIB_PATH=$PWD/exp/sleep8.so timeout -k 10 100 python tools/vnode_bench.py --graph --n 2 4 8 --sizes-mib 4 128 --iters 20 >> gpurun_out/ab3.log 2>&1 ;;
esac
done
done
MCCS_LIB_PATH=$PWD/exp/trace.so timeout -k 10 100 python tools/ring_trace.py --n 2 --kib 1024 --show 8 > gpurun_out/tr_1m.log 2>&1
MCCS_LIB_PATH=$PWD/exp/trace.so timeout -k 10 100 python tools/ring_trace.py --n 2 --mib 128 --show 8 > gpurun_out/tr_128m.log 2>&1
MCCS_LIB_PATH=$PWD/exp/trace.so timeout -k 10 100 python tools/ring_trace.py --n 8 --mib 128 --show 16 > gpurun_out/tr_128m8.log 2>&1
