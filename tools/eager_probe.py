#!/usr/bin/env python3
"""Eager vs graph-replayed AllReduce per call, one rank per process (the
shape of a node), fp16 buckets of the reference's eval sizes.

  python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
      --master-addr 127.0.0.1 --master-port 29541 tools/eager_probe.py

Per size: eager_us = wall time per call of K back-to-back calls (issue +
final sync, max over ranks); issue_us = the host time to issue them (before
the sync), i.e. the host path per call; graph_us = per call of the same
calls captured 20 to a HIP graph and replayed.  eager - graph is the host
path's cost when the host cannot stay ahead of the device.  With --raw the
calls go straight to mccsAllReduce through a prebuilt ctypes signature (no
Python face), to separate the Python layer from the library."""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", type=int, nargs="+", default=[32768, 131072, 524288, 2097152])
    ap.add_argument("--calls", type=int, default=200)
    ap.add_argument("--raw", action="store_true")
    a = ap.parse_args()
    import torch
    import torch.distributed as dist

    from mccs_amd import _lib
    from mccs_amd import comm as C
    from mccs_amd import ring_bench as rb

    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dev = int(os.environ.get("LOCAL_RANK", rank)) % torch.cuda.device_count()
    torch.cuda.set_device(dev)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    share = torch.cuda.device_count() < world
    cfg = C.CommConfig(lanes=rb.shared_gpu_lanes(world) if share else None)
    comm = C.init_communicator_rank(rank, world, dev, rb._exchange_factory(dist, world), cfg)
    lib = _lib.load()
    st = torch.cuda.current_stream()
    rows = []
    for nb in a.sizes:
        n = nb // 2
        x = torch.empty(n, dtype=torch.float16, device="cuda").uniform_(-1, 1)
        y = torch.empty_like(x)
        if a.raw:
            args = (x.data_ptr(), y.data_ptr(), n, 6, 0, comm.handle, st.cuda_stream)
            f = lib.mccsAllReduce

            def call():
                f(*args)
        else:
            def call():
                C.all_reduce(comm, x, y, n, C.AllReduceDataType.Float16, C.AllReduceOpType.Sum, st)
        for _ in range(20):
            call()
        torch.cuda.synchronize()
        comm.sync()
        dist.barrier()
        t0 = time.perf_counter()
        for _ in range(a.calls):
            call()
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        comm.sync()
        t2 = time.perf_counter()
        issue = rb.max_over_ranks(dist, (t1 - t0) / a.calls)
        eager = rb.max_over_ranks(dist, (t2 - t0) / a.calls)
        dist.barrier()
        g = torch.cuda.CUDAGraph()
        gs = torch.cuda.Stream()
        torch.cuda.synchronize()
        with torch.cuda.graph(g, stream=gs):
            for _ in range(20):
                C.all_reduce(comm, x, y, n, C.AllReduceDataType.Float16, C.AllReduceOpType.Sum, gs)
        g.replay()
        torch.cuda.synchronize()
        dist.barrier()
        t0 = time.perf_counter()
        for _ in range(10):
            g.replay()
        torch.cuda.synchronize()
        graph = rb.max_over_ranks(dist, (time.perf_counter() - t0) / 200)
        dist.barrier()
        del g
        rows.append({"bytes": nb, "eager_us": round(eager * 1e6, 2), "issue_us": round(issue * 1e6, 2),
                     "graph_us": round(graph * 1e6, 2), "gap_us": round((eager - graph) * 1e6, 2)})
        del x, y
    if rank == 0:
        print(json.dumps({"tool": "eager_probe", "world": world, "ranks_share_gpu": share, "raw_ctypes": a.raw,
                          "channels": comm.nchannels, "lanes": comm.lanes, "rows": rows}), flush=True)
    torch.cuda.synchronize()
    comm.destroy()
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
