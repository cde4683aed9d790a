#!/usr/bin/env python3
"""Multi-process (one rank per process) parity check through IPC-mapped FIFOs.

  python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 \
      --master-port 29511 tests/ipc_worker.py

Driven by tests/test_gpu_ipc.py (a worker, not a test module).

Every rank opens its peers' FIFO arenas with hipIpcOpenMemHandle (the
multi-GPU bench path).  On a one-GPU box all ranks share cuda:0, which still
exercises IPC export/open, the two-phase connect and cross-process flag
hand-offs.  Results are checked against the C oracle (rank 0 gathers inputs).
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def ddp_stream(comm, rank, world, orc, vnode):
    """Two steps of vnode.DDP_STREAM issued back to back on the library's
    default routing, one sync at the end; every bucket checked against the
    oracle and for the kernel the defaults give it."""
    import numpy as np
    import torch
    import torch.distributed as dist

    from mccs_amd import comm as C

    rng = np.random.default_rng(500 + rank)
    cases = []
    for step in range(2):
        for code, nbytes in vnode.DDP_STREAM:
            x = vnode.gen(code, nbytes // vnode.ESIZE[code], rng)
            xs = [None] * world
            dist.all_gather_object(xs, x)
            cases.append((code, xs, vnode.to_dev(x), vnode.to_dev(np.zeros_like(x))))
    algos = []
    for code, xs, send, recv in cases:
        C.all_reduce(comm, send, recv, xs[0].size, code, 0)
        algos.append(comm.last_algo())
    torch.cuda.synchronize()
    comm.sync()
    out = {}
    uncached = comm.fifo_memory != C.FIFO_DEVICE
    for i, (code, xs, send, recv) in enumerate(cases):
        p = vnode.Planner(comm.nchannels, comm.rings())
        nch, nthr, rings = p.select(xs[0].nbytes, 0)
        exp = orc.ring_allreduce(code, 0, xs, nchannels=nch, nthreads=nthr, ring_orders=rings)
        got = vnode.from_dev(recv, code)
        ok = bool(np.array_equal(got.view(np.uint8), exp.view(np.uint8)))
        want = vnode.ddp_expected_algo(xs[0].nbytes, world, uncached)
        out[f"ddp/{algos[i]}/b{i}"] = ok and algos[i] == want
    return out


def seq_stream(comm, rank, world, orc, vnode, nops=40, streams=False):
    """tests/test_gpu_sequence_fuzz.py's random collective sequence (same
    list on every rank), issued back to back on this rank's communicator at
    the library's default routing, one sync at the end, every output checked
    against the oracle.  streams: each collective on one of three streams,
    drawn per rank (the stream waits for the current one, where the inputs
    were copied; the library orders the comm's launches across streams)."""
    import numpy as np
    import torch
    import torch.distributed as dist

    from mccs_amd import comm as C
    from test_gpu_sequence_fuzz import _int_allreduce, sequence

    seq = sequence(np.random.default_rng(9000 + world), nops)
    rng = np.random.default_rng(77 + rank)
    srng = np.random.default_rng(500 + rank)
    pool = [torch.cuda.current_stream(), torch.cuda.Stream(), torch.cuda.Stream()]

    def stream():
        if not streams:
            return None
        st = pool[int(srng.integers(0, 3))]
        st.wait_stream(torch.cuda.current_stream())  # the inputs were copied on the current stream
        return st

    def gathered(x):
        xs = [None] * world
        dist.all_gather_object(xs, x)
        return xs

    checks, algos = [], set()
    for i, o in enumerate(seq):
        if o["kind"] == "ar":
            x = vnode.gen(o["code"], o["count"], rng)
            xs = gathered(x)
            send = vnode.to_dev(x)
            recv = send if o["inplace"] else vnode.to_dev(np.zeros_like(x))
            C.all_reduce(comm, send, recv, o["count"], o["code"], o["op"], stream())
            algos.add(comm.last_algo())
            p = vnode.Planner(comm.nchannels, comm.rings())
            nch, nthr, rings = p.select(x.nbytes, 0)
            exp = orc.ring_allreduce(o["code"], o["op"], xs, nchannels=nch, nthreads=nthr, ring_orders=rings)
            checks.append((f"{i}/ar/code{o['code']}/op{o['op']}/n{o['count']}", recv, exp, o["code"]))
        elif o["kind"] == "ag":
            x = rng.integers(0, 256, o["nbytes"], dtype=np.uint8)
            xs = gathered(x)
            send = vnode.to_dev(x)
            recv = vnode.to_dev(np.zeros(world * o["nbytes"], np.uint8))
            C.all_gather(comm, send, recv, o["nbytes"], stream())
            checks.append((f"{i}/ag/b{o['nbytes']}", recv, orc.ring_allgather(xs), None))
        else:
            batch = []
            for count in o["counts"]:
                x = vnode.gen(o["code"], count, rng)
                batch.append((count, gathered(x), vnode.to_dev(x), vnode.to_dev(np.zeros_like(x))))
            st = stream()
            with C.group():
                for count, xs, send, recv in batch:
                    C.all_reduce(comm, send, recv, count, o["code"], o["op"], st)
            for k, (count, xs, send, recv) in enumerate(batch):
                checks.append((f"{i}.{k}/group/code{o['code']}/op{o['op']}/n{count}", recv,
                               _int_allreduce(xs, o["op"]), o["code"]))
    torch.cuda.synchronize()
    comm.sync()
    out = {}
    for what, t, exp, code in checks:
        got = t.cpu().numpy() if code is None else vnode.from_dev(t, code)
        out[f"seq/{what}"] = bool(np.array_equal(got.view(np.uint8), exp.view(np.uint8)))
    out["seq/algos:" + ",".join(sorted(a for a in algos if a))] = True
    return out


def _streams():
    """Two streams on different hardware queues: HIP maps a process's streams
    onto a few queues (GPU_MAX_HW_QUEUES, 4 here) and runs one queue's
    kernels in order, so two streams of one priority may share a queue and
    never overlap; a queue carries one priority, so these two cannot."""
    import torch

    return torch.cuda.Stream(priority=0), torch.cuda.Stream(priority=-1)


def guard_overlap(comm, rank, world, orc, vnode):
    """A replay beside an eager launch of the same communicator, one rank per
    process (test_gpu_launch_guard.py): each rank captures AllReduce(S -> RX)
    in a graph on stream B, then issues AllReduce(S -> RY) on stream A and
    replays the graph on B at once, no sync and no event between A and B.
    Each rank serialises the two on its launch guard in whatever order its
    GPU queues pick, so rank 0's eager launch may pair with rank 1's replay
    (mccs_hip.h: across processes that order is the caller's to fix); both
    collectives reduce the same send buffer with the same schedule, so every
    pairing gives the oracle's sum -- a wrong one here means two launches of a
    comm overlapped on one rank."""
    import numpy as np
    import torch
    import torch.distributed as dist

    from mccs_amd import comm as C

    out = {}
    for kind, code, count in (("ring", 7, 4 << 20), ("ll", 6, 30001)):
        rng = np.random.default_rng(700 + rank)
        sa, sb = _streams()
        x = vnode.gen(code, count, rng)
        xs = [None] * world
        dist.all_gather_object(xs, x)
        s = vnode.to_dev(x)
        rx, ry = torch.zeros_like(s), torch.zeros_like(s)
        with torch.cuda.stream(sb):
            C.all_reduce(comm, s, rx, count, code, 0, sb)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=sb):
            C.all_reduce(comm, s, rx, count, code, 0, sb)
        torch.cuda.synchronize()
        comm.sync()
        algo = comm.last_algo()
        p = vnode.Planner(comm.nchannels, comm.rings())
        nch, nthr, rings = p.select(count * vnode.ESIZE[code], 0)
        exp = orc.ring_allreduce(code, 0, xs, nchannels=nch, nthreads=nthr, ring_orders=rings)
        w0 = comm.guard_info()["waits"]
        ok = True
        for rep in range(4):
            rx.zero_()
            ry.zero_()
            torch.cuda.synchronize()
            dist.barrier()
            C.all_reduce(comm, s, ry, count, code, 0, sa)
            with torch.cuda.stream(sb):
                g.replay()
            torch.cuda.synchronize()
            comm.sync()
            for t in (rx, ry):
                ok = ok and bool(np.array_equal(vnode.from_dev(t, code).view(np.uint8), exp.view(np.uint8)))
        gi = comm.guard_info()
        out[f"guard/{kind}/{algo}/exact"] = ok
        out[f"guard/{kind}/idle"] = (gi["owner"], gi["confirm"], gi["fin"]) == (0, 0, 0)
        print(json.dumps({"rank": rank, "kind": kind, "algo": algo, "waits": gi["waits"] - w0}), flush=True)
        del g
        torch.cuda.synchronize()
    return out


def main():
    import torch
    import torch.distributed as dist

    from mccs_amd import comm as C
    from oracle import oracle as orc
    import vnode

    rank = int(os.environ["RANK"])
    world = int(os.environ["WORLD_SIZE"])
    dev = int(os.environ.get("LOCAL_RANK", rank)) % torch.cuda.device_count()
    torch.cuda.set_device(dev)
    dist.init_process_group("gloo", rank=rank, world_size=world)

    def exchange(b):
        out = [None] * world
        dist.all_gather_object(out, b)
        return out

    # FIFO memory kind x data placement (receiver-side: remote writes;
    # sender-side: remote reads, the reference SHM layout)
    all_modes = {"uncached": (C.FIFO_UNCACHED, C.LOCALITY_RECEIVER), "device": (C.FIFO_DEVICE, C.LOCALITY_RECEIVER),
                 "sender-uncached": (C.FIFO_UNCACHED, C.LOCALITY_SENDER),
                 "sender-device": (C.FIFO_DEVICE, C.LOCALITY_SENDER),
                 "release": (C.FIFO_UNCACHED_RELEASE, C.LOCALITY_RECEIVER),
                 "sender-release": (C.FIFO_UNCACHED_RELEASE, C.LOCALITY_SENDER),
                 # the direct kernel (two-shot / one-shot) over IPC-mapped arenas
                 "direct": (C.FIFO_UNCACHED, C.LOCALITY_RECEIVER),
                 "oneshot": (C.FIFO_UNCACHED, C.LOCALITY_RECEIVER),
                 # LL one-shot up to 1 MiB (larger buckets: the one-shot)
                 "ll": (C.FIFO_UNCACHED, C.LOCALITY_RECEIVER),
                 # the library defaults, fed a DDP-style bucket stream (vnode.DDP_STREAM)
                 "ddp": (C.FIFO_UNCACHED, C.LOCALITY_RECEIVER),
                 # tests/test_gpu_sequence_fuzz.py's random sequence at the defaults
                 "seq": (C.FIFO_UNCACHED, C.LOCALITY_RECEIVER),
                 "seqs": (C.FIFO_UNCACHED, C.LOCALITY_RECEIVER),
                 # a graph replay beside an eager launch of the same comm (launch guard)
                 "guard": (C.FIFO_UNCACHED, C.LOCALITY_RECEIVER)}
    direct_kw = {"direct": dict(direct_bytes=8 << 20, oneshot_bytes=-1, ll_bytes=-1),
                 "oneshot": dict(direct_bytes=-1, oneshot_bytes=8 << 20, ll_bytes=-1),
                 "ll": dict(direct_bytes=-1, oneshot_bytes=8 << 20, ll_bytes=1 << 20),
                 "guard": dict(direct_bytes=-1, oneshot_bytes=-1, ll_bytes=1 << 20, lanes=2, channel_count=2)}
    names = os.environ.get("IPC_MODES", "uncached,device").split(",")
    results = {}
    # processes sharing one GPU: the library's default lanes; mccsCommConnect
    # shrinks them so every rank's workgroups fit in half the GPU's ring slots
    # (2 ranks x 4 channels x 16 lanes = 128 of 256)
    lanes = None
    for mode in names:
        fifo, loc = all_modes[mode]
        kw = dict(direct_kw.get(mode, {}))
        kw.setdefault("lanes", lanes)
        comm = C.init_communicator_rank(rank, world, dev, exchange,
                                        C.CommConfig(fifo_memory=fifo, locality=loc, timeout_ms=20000, **kw))
        if mode in ("ddp", "seq", "seqs", "guard"):
            if mode == "guard":
                results.update(guard_overlap(comm, rank, world, orc, vnode))
            elif mode == "ddp":
                results.update(ddp_stream(comm, rank, world, orc, vnode))
            else:
                results.update(seq_stream(comm, rank, world, orc, vnode, streams=mode == "seqs"))
            dist.barrier()  # every rank's last kernel is done before any arena returns to the pool
            comm.destroy()
            continue
        cases = [(2, 1 << 20), (7, 300007), (6, 1000003), (9, 77777), (7, 3)]
        nfuzz = int(os.environ.get("IPC_FUZZ", "0"))
        if nfuzz:  # seeded random dtypes / ragged counts, same on every rank
            frng = np.random.default_rng(4242)
            cases = [(int(frng.choice([0, 2, 4, 6, 7, 8, 9])), int(frng.choice([1, 5, 4099, int(frng.integers(1, 3 << 20))])))
                     for _ in range(nfuzz)]
        for code, count in cases:
            rng = np.random.default_rng(count * 31 + rank)
            x = vnode.gen(code, count, rng)
            if code == 2:
                x = np.full(count, 2042 + rank, np.int32)
            xs = [None] * world
            dist.all_gather_object(xs, x)
            send = vnode.to_dev(x)
            recv = vnode.to_dev(np.zeros_like(x))
            ok = True
            try:
                C.all_reduce(comm, send, recv, count, code, 0)
                comm.sync()
                got = vnode.from_dev(recv, code)
                p = vnode.Planner(comm.nchannels, comm.rings())
                nch, nthr, rings = p.select(count * vnode.ESIZE[code], 0)
                exp = orc.ring_allreduce(code, 0, xs, nchannels=nch, nthreads=nthr, ring_orders=rings)
                ok = bool(np.array_equal(got.view(np.uint8), exp.view(np.uint8)))
            except Exception as e:  # noqa: BLE001
                print(f"[rank {rank}] {mode} code={code}: {e}", flush=True)
                ok = False
            if mode in direct_kw:  # the call really took that kernel
                # LL runs on uncached arenas only: where a rank's IPC export of
                # its uncached arena was refused (the library then falls back to
                # a hipMalloc arena + system fences on every rank, api.cpp
                # mccsCommSetupRank) the bucket takes the one-shot instead
                ll_ok = comm.fifo_memory != C.FIFO_DEVICE
                nb = count * vnode.ESIZE[code]
                # above every direct threshold (8 MiB here; IPC_FUZZ draws up to 3M elements) the ring
                want = ("ring" if nb > 8 << 20 else
                        "oneshot" if mode == "ll" and (nb > 1 << 20 or not ll_ok) else mode)
                ok = ok and comm.last_algo() == want
            results[f"{mode}/dtype{code}/n{count}"] = ok
        if mode in direct_kw:  # several launches back to back, fresh inputs each, then one sync
            k = 12
            rng = np.random.default_rng(99 + rank)
            xs_all, sends, recvs = [], [], []
            for i in range(k):
                x = vnode.gen(7, 100003 + i, rng)
                xa = [None] * world
                dist.all_gather_object(xa, x)
                xs_all.append(xa)
                sends.append(vnode.to_dev(x))
                recvs.append(vnode.to_dev(np.zeros_like(x)))
            for i in range(k):
                C.all_reduce(comm, sends[i], recvs[i], 100003 + i, 7, 0)
            comm.sync()
            ok = True
            for i in range(k):
                p = vnode.Planner(comm.nchannels, comm.rings())
                nch, nthr, rings = p.select((100003 + i) * 4, 0)
                exp = orc.ring_allreduce(7, 0, xs_all[i], nchannels=nch, nthreads=nthr, ring_orders=rings)
                ok = ok and bool(np.array_equal(vnode.from_dev(recvs[i], 7).view(np.uint8), exp.view(np.uint8)))
            results[f"{mode}/back_to_back_x{k}"] = ok
        if torch.cuda.device_count() < world:  # co-located processes: lanes shrunk to half the ring slots
            # auto lanes (api.cpp make_comm) capped at half of MI355X's 256 one-per-CU ring slots
            auto = (128 if world == 2 else 64) // comm.nchannels
            want = min(auto, 256 // 2 // (world * comm.nchannels))
            results[f"{mode}/colocated_lanes={comm.lanes}"] = comm.lanes == want
        dist.barrier()  # every rank's last kernel is done before any arena returns to the pool
        comm.destroy()
    allres = [None] * world
    dist.all_gather_object(allres, results)
    if rank == 0:
        merged = {k: all(r.get(k, False) for r in allres) for k in results}
        print(json.dumps({"world": world, "fifo_modes": merged, "all_ok": all(merged.values())}), flush=True)
    dist.barrier()
    dist.destroy_process_group()
    sys.exit(0 if all(results.values()) else 1)


if __name__ == "__main__":
    main()
