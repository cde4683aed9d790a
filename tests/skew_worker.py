#!/usr/bin/env python3
"""A peer that reaches the collective late (driven by tests/test_gpu_skew.py).

  python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 \
      --master-port 29517 tests/skew_worker.py

Rank 0 issues an int32 known-answer AllReduce right after connect and waits
in it; rank 1 first sleeps SKEW_S seconds (rank 0 writing a checkpoint, say)
and only then issues its own.  With the library's default watchdog the late
rank must simply be waited for.  Rank 0 prints one JSON line.
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    import torch.distributed as dist

    from mccs_amd import comm as C

    rank = int(os.environ["RANK"])
    world = int(os.environ["WORLD_SIZE"])
    skew = float(os.environ.get("SKEW_S", "35"))
    dev = int(os.environ.get("LOCAL_RANK", rank)) % torch.cuda.device_count()
    torch.cuda.set_device(dev)
    dist.init_process_group("gloo", rank=rank, world_size=world)

    def exchange(b):
        out = [None] * world
        dist.all_gather_object(out, b)
        return out

    comm = C.init_communicator_rank(rank, world, dev, exchange)  # default config: default watchdog
    count = 1 << 20
    send = torch.full((count,), 2042 + rank, dtype=torch.int32, device=f"cuda:{dev}")
    recv = torch.empty_like(send)
    dist.barrier()
    if rank == world - 1:
        time.sleep(skew)
    t0 = time.perf_counter()
    err = None
    try:
        C.all_reduce(comm, send, recv, count, 2, 0)
        comm.sync()
    except Exception as e:  # noqa: BLE001
        err = f"{type(e).__name__}: {e}"
    waited = time.perf_counter() - t0
    ok = err is None and bool((recv == 2042 * world + world * (world - 1) // 2).all())
    res = [None] * world
    dist.all_gather_object(res, {"ok": ok, "err": err, "waited_s": round(waited, 2)})
    if rank == 0:
        print(json.dumps({"skew_s": skew, "ranks": res, "all_ok": all(r["ok"] for r in res)}), flush=True)
    dist.barrier()
    comm.destroy()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
