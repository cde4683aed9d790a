# hunt for calls that leave a HIP error on the thread: round-4 library vs round-5, the failing 4-process case
rm -f gpurun_out/steps.log
TR="python -m torch.distributed.run --nnodes=1 --master-addr 127.0.0.1"
S=tools/gpu_step.sh
MCCS_LIB_PATH=abvar/libmccs_r04.so HSA_ENABLE_IPC_MODE_LEGACY=0 $S hunt_r04 300 $TR --nproc-per-node 4 --master-port 29861 tools/stale_error_hunt.py || exit 1
HSA_ENABLE_IPC_MODE_LEGACY=0 $S hunt_r05 300 $TR --nproc-per-node 4 --master-port 29862 tools/stale_error_hunt.py || exit 1
cat gpurun_out/steps.log
