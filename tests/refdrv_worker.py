#!/usr/bin/env python3
"""The reference-named kernels driven the way the reference host drives them,
one rank per process (a worker of tests/test_gpu_reference_driver.py).

  python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 \
      --master-port 29513 tests/refdrv_worker.py

No communicator of this library is involved: mccs_amd/refdrive.py restates
the Rust service's host side (the SHM connector's SendBufMeta/RecvBufMeta +
FIFO layout, comm/device.rs, plan.rs's host-mapped work ring with rolling
acks, get_task_schema and launch_plan: grid = #channels, 544-thread blocks).

Each variant (reference ring with the FIFO at the sender, the reference
default; a rotated ring override with the FIFO at the receiver; both again
with every SendBufMeta / RecvBufMeta / FIFO in the reference's own SHM
memory: mlock'ed host pages registered mapped, transport/shm/buffer.rs:17-26,
cuda/alloc.rs:59-99) runs four
cases three times each on the same structures (conn->step persists across
launches, prims_simple.h:318-319,461) and then 1100 back-to-back launches,
so the 1024-entry work ring wraps and flow-controls on workFifoDone
(plan.rs:380-541).  Results are compared bit for bit with the oracle,
workFifoDone with doneAcks, and conn->step across ranks.
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    import torch
    import torch.distributed as dist

    from mccs_amd import refdrive
    from oracle import oracle as orc
    import vnode

    rank, n = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dev = int(os.environ.get("LOCAL_RANK", rank)) % torch.cuda.device_count()
    torch.cuda.set_device(dev)
    dist.init_process_group("gloo", rank=rank, world_size=n)

    def allgather(obj):
        out = [None] * n
        dist.all_gather_object(out, obj)
        return out

    if os.environ.get("REFDRV_BIG") == "1":
        return big_case(torch, dist, refdrive, orc, rank, n, dev, allgather)
    rot = list(range(1, n)) + [0]
    variants = [("ref_sender", 2, None, "sender", "device"),
                ("rotated_receiver", 2, [rot, rot[::-1]], "receiver", "device"),
                ("ref_sender_hostfifo", 2, None, "sender", "host"),
                ("rotated_receiver_hostfifo", 2, [rot, rot[::-1]], "receiver", "host")]
    results = {}
    stream = torch.cuda.Stream()
    for vname, nch, rings, loc, fifo in variants:
        rr = refdrive.RefDrivenRank(rank, n, dev, allgather, nch=nch, rings=rings, locality=loc, fifo=fifo)
        for code, count in ((6, 1 << 20), (7, (1 << 21) + 3), (2, 300007), (6, 777777)):
            rng = np.random.default_rng(count + rank)
            for rep in range(3):
                x = np.full(count, 2042 + rank, np.int32) if code == 2 else vnode.gen(code, count, rng)
                xs = allgather(x)
                send, recv = vnode.to_dev(x), vnode.to_dev(np.zeros_like(x))
                torch.cuda.synchronize()
                dist.barrier()
                rr.all_reduce(send.data_ptr(), recv.data_ptr(), count, code, 0, stream.cuda_stream)
                stream.synchronize()
                k, nthr, ring_used = rr.last_plan
                exp = orc.ring_allreduce(code, 0, xs, nchannels=k, nthreads=nthr, buff_size=rr.buff,
                                         ring_orders=ring_used)
                got = vnode.from_dev(recv, code)
                ok = bool(np.array_equal(got.view(np.uint8), exp.view(np.uint8))) and not rr.aborted()
                ok = ok and nthr == 544 and all(a == rr.ring.chan_next[c] for c, a in enumerate(rr.done_acks()))
                if code == 2:
                    ok = ok and int(exp[0]) == 2042 * n + n * (n - 1) // 2
                results[f"{vname}/dtype{code}/n{count}/rep{rep}"] = {"ok": ok, "steps": rr.steps()}
                del send, recv
        if vname == "ref_sender":
            # every (dtype, op) kernel the reference names, at a ragged count
            # that takes several passes and a tail per slice (the reference-
            # named kernels stream 16 packs per source, bf16 12, bytes 4:
            # a code path of their own, ring_kernel.h kRefUnroll)
            for code in range(10):
                for op in range(4):
                    count = 150001 + 17 * code + op
                    rng = np.random.default_rng(1000 * code + 10 * op + rank)
                    x = vnode.gen(code, count, rng)
                    xs = allgather(x)
                    send, recv = vnode.to_dev(x), vnode.to_dev(np.zeros_like(x))
                    torch.cuda.synchronize()
                    dist.barrier()
                    rr.all_reduce(send.data_ptr(), recv.data_ptr(), count, code, op, stream.cuda_stream)
                    stream.synchronize()
                    k, nthr, ring_used = rr.last_plan
                    exp = orc.ring_allreduce(code, op, xs, nchannels=k, nthreads=nthr, buff_size=rr.buff,
                                             ring_orders=ring_used)
                    got = vnode.from_dev(recv, code)
                    ok = bool(np.array_equal(got.view(np.uint8), exp.view(np.uint8))) and not rr.aborted()
                    results[f"{vname}/all_kernels/dtype{code}/op{op}"] = {"ok": ok, "steps": rr.steps()}
                    del send, recv
        # 1100 back-to-back 4 KiB launches (one channel, one work entry each):
        # the 1024-entry work ring wraps and the host waits on workFifoDone
        count = 1024
        x = np.full(count, 2042 + rank, np.int32)
        send, recv = vnode.to_dev(x), vnode.to_dev(np.zeros_like(x))
        torch.cuda.synchronize()
        dist.barrier()
        for _ in range(1100):
            rr.all_reduce(send.data_ptr(), recv.data_ptr(), count, 2, 0, stream.cuda_stream)
        stream.synchronize()
        got = vnode.from_dev(recv, 2)
        ok = bool(np.all(got == 2042 * n + n * (n - 1) // 2)) and not rr.aborted() and rr.ring.next_available > 1024
        results[f"{vname}/wrap1100"] = {"ok": ok, "steps": rr.steps()}
        rr.close(dist.barrier)
    allres = allgather(results)
    if rank == 0:
        merged = {}
        for k in results:
            steps = [r[k]["steps"] for r in allres]
            merged[k] = all(r[k]["ok"] for r in allres) and all(s == steps[0] for s in steps)
        print(json.dumps({"world": n, "cases": merged, "all_ok": all(merged.values()),
                          "final_steps": allres[0][k]["steps"]}), flush=True)
    dist.barrier()
    dist.destroy_process_group()


def big_case(torch, dist, refdrive, orc, rank, n, dev, allgather):
    """configs[2]'s bucket (128 MiB fp32 per rank), random uniform [-1, 1)
    inputs, reference-driven at the mccs.toml default (2 channels, ring
    0..n-1), at 32 channels, and at 2 channels on host-memory FIFOs (the
    reference SHM transport's own memory): every rank's output bit for bit against the
    oracle's ring order.  Each process regenerates every rank's inputs from
    the same seeds (no bulk exchange)."""
    import numpy as np

    count = (128 << 20) // 4
    g = torch.Generator(device="cuda")

    def inputs_of(r):
        g.manual_seed(9100 + r)
        return torch.rand(count, device="cuda", generator=g) * 2 - 1

    mine = inputs_of(rank)
    host = [inputs_of(r).cpu().numpy() for r in range(n)]
    stream = torch.cuda.Stream()
    results = {}
    for nch, fifo in ((2, "device"), (32, "device"), (2, "host")):
        rr = refdrive.RefDrivenRank(rank, n, dev, allgather, nch=nch, fifo=fifo)
        recv = torch.empty_like(mine)
        torch.cuda.synchronize()
        dist.barrier()
        rr.all_reduce(mine.data_ptr(), recv.data_ptr(), count, 7, 0, stream.cuda_stream)
        stream.synchronize()
        k, nthr, rings = rr.last_plan
        want = orc.ring_allreduce_mt(7, 0, host, nchannels=k, nthreads=nthr, buff_size=rr.buff, ring_orders=rings,
                                     workers=min(16, os.cpu_count() or 1))
        got = recv.cpu().numpy()
        naive = host[0].copy()
        for r in range(1, n):
            naive += host[r]
        results[f"big/ch{nch}/{fifo}"] = {"ok": bool(np.array_equal(got.view(np.uint32), want.view(np.uint32)))
                                   and not rr.aborted() and (n < 3 or not np.array_equal(naive, want)),
                                   "steps": rr.steps(), "grid": k, "block": nthr}
        rr.close(dist.barrier)
    allres = allgather(results)
    if rank == 0:
        merged = {k: all(r[k]["ok"] for r in allres) for k in results}
        print(json.dumps({"world": n, "cases": merged, "all_ok": all(merged.values()),
                          "plans": {k: [results[k]["grid"], results[k]["block"]] for k in results}}), flush=True)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
