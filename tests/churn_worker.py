#!/usr/bin/env python3
"""Communicator churn across processes (driven by tests/test_gpu_churn.py).

  python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 \
      --master-port 29513 tests/churn_worker.py

Every cycle: one rank per process connects a communicator of a shape drawn
from the same seed on every rank (IPC export / open of every peer's arena),
runs the int32 known-answer AllReduce on the ring and on the default
small-bucket kernel, then destroys it -- after a barrier with the peers, or
(CHURN_NO_BARRIER=1) right away: the library itself holds a destroyed rank's
arena back until every peer destroyed its side.  Rank 0 prints one JSON line: every
cycle exact, and the largest drop of any rank's free GPU memory from the
end of the first round of shapes (the arena pool warm) to the last cycle.
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    import torch
    import torch.distributed as dist

    from mccs_amd import comm as C
    from test_gpu_churn import INT32, SHAPES, SUM, churn_shapes, kat

    rank = int(os.environ["RANK"])
    world = int(os.environ["WORLD_SIZE"])
    dev = int(os.environ.get("LOCAL_RANK", rank)) % torch.cuda.device_count()
    torch.cuda.set_device(dev)
    dist.init_process_group("gloo", rank=rank, world_size=world)

    def exchange(b):
        out = [None] * world
        dist.all_gather_object(out, b)
        return out

    no_barrier = os.environ.get("CHURN_NO_BARRIER") == "1"
    ok, free = [], []
    shapes = churn_shapes(11, SHAPES, [world])
    for i, (_, cfg) in enumerate(shapes):
        comm = C.init_communicator_rank(rank, world, dev, exchange, C.CommConfig(timeout_ms=20000, **cfg))
        good = True
        for count in (3 << 20, 16 << 10):
            send = torch.full((count,), 2042 + rank, dtype=torch.int32, device=f"cuda:{dev}")
            recv = torch.empty_like(send)
            C.all_reduce(comm, send, recv, count, INT32, SUM)
            comm.sync()
            good = good and bool((recv == kat(world)).all())
        ok.append(good)
        del send, recv
        torch.cuda.synchronize()
        if not no_barrier:
            dist.barrier()
        comm.destroy()
        torch.cuda.empty_cache()
        if i in (SHAPES - 1, len(shapes) - 1):
            dist.barrier()  # every process has released this cycle's buffers (the GPU is shared here)
            free.append(torch.cuda.mem_get_info(dev)[0])
    drift = [None] * world
    dist.all_gather_object(drift, free[0] - free[1])
    oks = [None] * world
    dist.all_gather_object(oks, ok)
    if rank == 0:
        print(json.dumps({"all_ok": all(all(o) for o in oks), "cycles": len(shapes), "max_drift_bytes": max(drift),
                          "drift_per_rank": drift}), flush=True)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
