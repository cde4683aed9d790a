#!/usr/bin/env python3
"""Which call leaves a HIP error on the thread?  (round-4 setup failure hunt)

Runs the sequence of tests/ipc_worker.py's failing case (IPC_MODES
direct,oneshot,ll; one rank per process) against the library named by
MCCS_LIB_PATH, and after EVERY call into the library and every torch call of
the sequence reads HIP's per-thread last error with hipPeekAtLastError().
The first call after which it is non-zero is recorded with the error code,
then the error is cleared and the sequence goes on.  Rank 0 prints one JSON
line with every rank's findings.

  MCCS_LIB_PATH=abvar/libmccs_r04.so python -m torch.distributed.run \
      --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29561 tools/stale_error_hunt.py
"""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    import numpy as np
    import torch
    import torch.distributed as dist

    from mccs_amd import _lib
    from mccs_amd import comm as C
    import vnode

    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dev = int(os.environ.get("LOCAL_RANK", rank)) % torch.cuda.device_count()
    torch.cuda.set_device(dev)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    hip = ctypes.CDLL("libamdhip64.so", mode=ctypes.RTLD_GLOBAL)
    found = []

    def peek(what):
        e = hip.hipPeekAtLastError()
        if e:
            found.append({"after": what, "hip_error": e})
            hip.hipGetLastError()

    lib = _lib.load()
    # wrap every library entry point the sequence uses
    for name in list(_lib.SIGNATURES):
        if not hasattr(lib, name):
            continue
        fn = getattr(lib, name)

        def wrapped(*a, _fn=fn, _name=name):
            r = _fn(*a)
            peek(_name)
            return r

        wrapped.argtypes, wrapped.restype = fn.argtypes, fn.restype
        setattr(lib, name, wrapped)

    def exchange(b):
        out = [None] * world
        dist.all_gather_object(out, b)
        return out

    direct_kw = {"direct": dict(direct_bytes=8 << 20, oneshot_bytes=-1, ll_bytes=-1),
                 "oneshot": dict(direct_bytes=-1, oneshot_bytes=8 << 20, ll_bytes=-1),
                 "ll": dict(direct_bytes=-1, oneshot_bytes=8 << 20, ll_bytes=1 << 20)}
    reps = int(os.environ.get("HUNT_REPS", "3"))
    setup_failures = []
    for rep in range(reps):
        for mode, kw in direct_kw.items():
            peek(f"before setup {mode}")
            try:
                comm = C.init_communicator_rank(rank, world, dev, exchange,
                                                C.CommConfig(fifo_memory=C.FIFO_UNCACHED,
                                                             locality=C.LOCALITY_RECEIVER, timeout_ms=20000, **kw))
            except Exception as e:  # noqa: BLE001
                setup_failures.append({"rep": rep, "mode": mode, "error": str(e)[:300]})
                hip.hipGetLastError()
                continue
            for code, count in [(2, 1 << 20), (7, 300007), (6, 1000003), (9, 77777), (7, 3)]:
                rng = np.random.default_rng(count * 31 + rank)
                x = vnode.gen(code, count, rng)
                send = vnode.to_dev(x)
                peek("torch to_dev")
                recv = vnode.to_dev(np.zeros_like(x))
                C.all_reduce(comm, send, recv, count, code, 0)
                comm.sync()
                vnode.from_dev(recv, code)
                peek("torch from_dev")
            sends = [vnode.to_dev(np.ones(100003 + i, np.float32)) for i in range(12)]
            recvs = [vnode.to_dev(np.zeros(100003 + i, np.float32)) for i in range(12)]
            for i in range(12):
                C.all_reduce(comm, sends[i], recvs[i], 100003 + i, 7, 0)
            comm.sync()
            torch.cuda.synchronize()
            peek("torch synchronize")
            comm.destroy()
            peek(f"after destroy {mode}")
            dist.barrier()
    allres = [None] * world
    dist.all_gather_object(allres, {"rank": rank, "stale_errors": found[:50], "n_stale": len(found),
                                    "setup_failures": setup_failures})
    if rank == 0:
        print(json.dumps({"library": os.environ.get("MCCS_LIB_PATH", "mccs_amd/libmccs_hip.so"), "world": world,
                          "reps": reps, "ranks": allres}), flush=True)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
