#!/usr/bin/env python3
"""Diagnostic: does creating / destroying a second communicator change the
ring rate of a live one?  torchrun, n ranks (may share one GPU).
  python -m torch.distributed.run --nproc-per-node 4 tools/ipc_ab.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    import torch.distributed as dist

    from mccs_amd import comm as C
    from mccs_amd import ring_bench as RB

    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    ndev = torch.cuda.device_count()
    device = int(os.environ.get("LOCAL_RANK", rank)) % max(1, ndev)
    torch.cuda.set_device(device)
    dev = torch.device("cuda", device)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    ex = RB._exchange_factory(dist, world)
    n = (64 << 20) // 4
    x = torch.rand(n, device=dev)
    y = torch.empty_like(x)

    def t(cm, label, reps=8):
        el = RB.max_over_ranks(dist, RB._time_steps(torch, dist, cm, lambda: C.all_reduce(cm, x, y, n, C.AllReduceDataType.Float32), 2, reps))
        if rank == 0:
            print(f"{label}: {el / reps * 1e3:.4f} ms", flush=True)

    if os.environ.get("AB_SECOND") == "stream":
        r = C.init_communicator_rank(rank, world, device, ex, C.CommConfig(locality=C.LOCALITY_RECEIVER))
        t(r, "R alone")
        keep = [torch.cuda.Stream() for _ in range(int(os.environ.get("AB_NSTREAMS", "1")))]
        t(r, f"R after creating {len(keep)} torch stream(s)")
        for st in keep:
            with torch.cuda.stream(st):
                torch.ones(1, device=dev).add_(1)
        torch.cuda.synchronize()
        t(r, "R after using them")
        r.destroy()
        dist.barrier()
        dist.destroy_process_group()
        return
    loc2 = C.LOCALITY_SENDER if os.environ.get("AB_SECOND", "s") == "s" else C.LOCALITY_RECEIVER
    r = C.init_communicator_rank(rank, world, device, ex, C.CommConfig(locality=C.LOCALITY_RECEIVER))
    t(r, "R alone")
    t(r, "R alone again")
    s = C.init_communicator_rank(rank, world, device, ex, C.CommConfig(locality=loc2))
    t(r, "R with second comm alive (not run)")
    t(s, "second comm")
    t(r, "R after second comm ran")
    s.destroy()
    t(r, "R after second comm destroyed")
    r.destroy()
    r2 = C.init_communicator_rank(rank, world, device, ex, C.CommConfig(locality=C.LOCALITY_RECEIVER))
    t(r2, "fresh R2")
    r2.destroy()
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
