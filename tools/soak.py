#!/usr/bin/env python3
"""Soak of the ring AllReduce: many back-to-back AllReduces (the work FIFO
wraps many times, FIFO steps keep growing), with exact-sum AllReduces checked
bit for bit every --check-every iterations and at the end.

One rank per process (IPC path), launched by torch.distributed.run:
  python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 tools/soak.py --iters 20000
or an n-rank virtual node in this process (fused launches):
  python tools/soak.py --vnode 8 --iters 5000 --size-mib 16
Prints one JSON line; exits non-zero on the first mismatch.
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch

    from mccs_amd import comm as C
    from mccs_amd import ring_bench as rb

    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=5000)
    ap.add_argument("--size-mib", type=int, default=128)
    ap.add_argument("--size-kib", type=int, default=0, help="bucket in KiB (overrides --size-mib; small buckets "
                    "take the library's direct / LL kernels)")
    ap.add_argument("--check-every", type=int, default=1000)
    ap.add_argument("--vnode", type=int, default=0, help="n ranks on cuda:0 in this process")
    args = ap.parse_args()
    n = ((args.size_kib << 10) if args.size_kib else (args.size_mib << 20)) // 4
    code = C.AllReduceDataType.Float32
    dev = torch.device("cuda", 0)
    t0 = time.perf_counter()
    checks = 0
    if args.vnode:
        world = args.vnode
        comms = C.init_all([0] * world)
        xs = [(rb._exact_numerators(torch, n, r, dev).to(torch.float32) / 64.0) for r in range(world)]
        ys = [torch.empty_like(x) for x in xs]
        tot = sum(rb._exact_numerators(torch, n, r, dev) for r in range(world))
        want = (tot.to(torch.float64) / 64.0).to(torch.float32)
        del tot
        for it in range(1, args.iters + 1):
            with C.group():
                for r in range(world):
                    C.all_reduce(comms[r], xs[r], ys[r], n, code, C.AllReduceOpType.Sum)
            if it % args.check_every == 0 or it == args.iters:
                for c in comms:
                    c.sync()
                for r in range(world):
                    if not torch.equal(ys[r], want):
                        raise SystemExit(f"vnode soak: rank {r} mismatch at iteration {it}")
                    ys[r].zero_()
                checks += 1
                print(json.dumps({"iteration": it, "ok": True}), flush=True)
        algo = comms[0].last_algo()
        for c in comms:
            c.destroy()
        rank = 0
    else:
        import torch.distributed as dist

        rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
        dist.init_process_group("gloo")
        share = torch.cuda.device_count() < world
        cfg = C.CommConfig(lanes=rb.shared_gpu_lanes(world) if share else None, timeout_ms=60000)
        dev = torch.device("cuda", int(os.environ.get("LOCAL_RANK", rank)) % torch.cuda.device_count())
        torch.cuda.set_device(dev)
        comm = C.init_communicator_rank(rank, world, dev.index, rb._exchange_factory(dist, world), cfg)
        x = torch.rand(n, device=dev)
        y = torch.empty_like(x)
        for it in range(1, args.iters + 1):
            C.all_reduce(comm, x, y, n, code, C.AllReduceOpType.Sum)
            if it % args.check_every == 0 or it == args.iters:
                ok = rb.exact_sum_ok(torch, C, comm, rank, world, n, torch.float32, code, dev)
                rb.require(dist, ok, f"soak: exact-sum AllReduce at iteration {it}")
                checks += 1
                if rank == 0:
                    print(json.dumps({"iteration": it, "ok": True}), flush=True)
        algo = comm.last_algo()
        comm.destroy()
        dist.destroy_process_group()
    if rank == 0:
        el = time.perf_counter() - t0
        print(json.dumps({"soak": "vnode" if args.vnode else "ipc", "ranks": world, "iters": args.iters,
                          "bytes": n * 4, "algo": algo, "exact_checks": checks, "seconds": round(el, 1),
                          "all_exact": True}), flush=True)


if __name__ == "__main__":
    main()
