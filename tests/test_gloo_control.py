"""CPU, world_size 2 over gloo: the N > 1 control plane of bench.py's ring leg
(connect-handle exchange, all-ranks agreement, max-over-ranks timing) and the
host ring protocol run per rank with the FIFO messages carried by gloo
send/recv between processes (sharding + neighbour exchange of the ring)."""
import os
import socket
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import torch.distributed as dist

    from mccs_amd import ring_bench

    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        ex = ring_bench._exchange_factory(dist, world)
        got = ex(bytes([rank]) * 8)
        ok_exchange = got == [bytes([r]) * 8 for r in range(world)]
        all_true = ring_bench.agree(dist, True)
        one_false = ring_bench.agree(dist, rank != 1)
        mx = ring_bench.max_over_ranks(dist, float(rank) + 0.5)
        # ring allreduce with gloo as the link: rank r holds its chunk sums
        ring_ok = _gloo_ring_allreduce(dist, rank, world)
        init_ok = _init_failure_is_collective(dist, rank, world)
        q.put((rank, ok_exchange, all_true, one_false, mx, ring_ok and init_ok))
    finally:
        dist.destroy_process_group()


def _gloo_ring_allreduce(dist, rank, world):
    """runRing's reduce-scatter + all-gather (all_reduce.h:46-86) with gloo
    point-to-point as the FIFO; result checked against the C oracle."""
    import torch

    from oracle import oracle as orc

    rcs = 256  # elements per chunk; count leaves a ragged last chunk
    count = rcs * world - 5
    xs = [(np.random.default_rng(100 + r).random(count, dtype=np.float32) * 2 - 1) for r in range(world)]
    x = torch.from_numpy(xs[rank].copy())
    out = x.clone()
    nxt, prv = (rank + 1) % world, (rank - 1) % world

    def sl(c):
        lo = min(c * rcs, count)
        return slice(lo, min(lo + rcs, count))

    acc = x[sl((rank - 1) % world)].clone()
    for j in range(2, world + 1):  # reduce-scatter: chunk (rank - j) arrives from prev
        c = (rank - j) % world
        buf = torch.empty(sl(c).stop - sl(c).start, dtype=torch.float32)
        dist.send(acc, nxt) if rank % 2 == 0 else None
        dist.recv(buf, prv)
        if rank % 2 == 1:
            dist.send(acc, nxt)
        acc = x[sl(c)] + buf  # fn(own input, received)
    out[sl(rank)] = acc
    cur = acc
    for j in range(1, world):  # all-gather
        c = (rank - j) % world
        buf = torch.empty(sl(c).stop - sl(c).start, dtype=torch.float32)
        if rank % 2 == 0:
            dist.send(cur, nxt)
            dist.recv(buf, prv)
        else:
            dist.recv(buf, prv)
            dist.send(cur, nxt)
        out[sl(c)] = buf
        cur = buf
    # oracle: 1 channel, 160 threads -> 256-element (1 KiB) granule = rcs
    exp = orc.ring_allreduce(7, 0, xs, nchannels=1, nthreads=160, buff_size=1 << 22)
    return bool(np.array_equal(out.numpy().view(np.uint32), exp.view(np.uint32)))


def _init_failure_is_collective(dist, rank, world):
    """Without a GPU every rank's mccsCommSetupRank fails; each must still
    join the handle exchange and then raise, so no rank blocks in it."""
    import ctypes

    from mccs_amd import _lib, ring_bench
    from mccs_amd import comm as C

    n = ctypes.c_int(0)
    if ctypes.CDLL("libamdhip64.so").hipGetDeviceCount(ctypes.byref(n)) == 0 and n.value > 0:
        return True  # a GPU is present: the failure path is not reachable here
    try:
        C.init_communicator_rank(rank, world, 0, ring_bench._exchange_factory(dist, world))
    except (_lib.MccsError, RuntimeError):
        return True
    return False


@pytest.mark.parametrize("world", [2])
def test_control_plane_world2(world):
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(world))
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, ok_ex, all_true, one_false, mx, ring_ok in res:
        assert ok_ex and all_true and not one_false
        assert mx == world - 0.5
        assert ring_ok, f"rank {rank}: gloo ring != oracle"


class _FakeComm:
    def __init__(self, tag):
        self.tag = tag
        self.destroyed = False

    def destroy(self):
        self.destroyed = True


class _FakeC:
    """Stands in for mccs_amd.comm: creation joins the handle exchange like
    the real init_communicator_rank, nothing else touches a device."""

    def __init__(self):
        self.made = []

    def init_communicator_rank(self, rank, world, device, exchange, cfg):
        exchange(b"h")
        c = _FakeComm(cfg)
        self.made.append(c)
        return c


def _gate_worker(rank, world, port, q):
    sys.path.insert(0, ROOT)
    import torch.distributed as dist

    from mccs_amd import ring_bench as rb

    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        fc, rej = _FakeC(), []
        ex = rb._exchange_factory(dist, world)

        def gate(comm):  # rank 1 sees a wrong sum in every uncached-FIFO mode
            return not (comm.tag == "U" and rank == 1)

        m1 = [("receiver-uncached-fifo", "U"), ("receiver-cached-fifo+system-fences", "D")]
        c1, n1 = rb.make_validated_comm(None, dist, fc, rank, world, 0, None, ex, m1, None,
                                        rejected=rej, gate=gate)
        m2 = [("sender-uncached-fifo", "U"), ("sender-cached-fifo+system-fences", "D")]
        c2, n2 = rb.make_validated_comm(None, dist, fc, rank, world, 0, None, ex, m2, None, rejected=rej, gate=gate)
        c3, n3 = rb.make_validated_comm(None, dist, fc, rank, world, 0, None, ex, m1, None, rejected=[],
                                        gate=lambda c: False)
        # three hand-off modes: relaxed fails on rank 1 only, the release-fence mode passes
        m4 = [("receiver-uncached-fifo", "U"), ("receiver-uncached-fifo+release-fence", "R"),
              ("receiver-cached-fifo+system-fences", "D")]
        rej4 = []
        c4, n4 = rb.make_validated_comm(None, dist, fc, rank, world, 0, None, ex, m4, None, rejected=rej4, gate=gate)
        q.put((rank, n1, n2, n3, [r["kind"] for r in rej], len(fc.made), fc.made[0].destroyed,
               c1.destroyed, c2.destroyed, n4, [r["kind"] for r in rej4]))
    finally:
        dist.destroy_process_group()


def test_bench_gate_rejects_a_mode_on_every_rank_and_records_it():
    """ring_bench.make_validated_comm: a mode that fails the exact-sum gate on
    ANY rank is rejected on all ranks before timing (recorded, its FIFO kind
    skipped afterwards), the next mode is chosen everywhere, and when every
    mode fails no communicator is returned (the bench then exits non-zero)."""
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_gate_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(2))
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, n1, n2, n3, kinds, made, first_destroyed, c1_destroyed, c2_destroyed, n4, kinds4 in res:
        assert n4 == "receiver-uncached-fifo+release-fence" and kinds4 == ["uncached-fifo"]
        assert n1 == "receiver-cached-fifo+system-fences" and n2 == "sender-cached-fifo+system-fences"
        assert n3 is None
        assert kinds == ["uncached-fifo"]
        # m1: U (rejected, destroyed) + D; m2: U skipped, D; m1 again with a fresh list: U + D both
        # rejected; m4: U (rejected) + R
        assert made == 7 and first_destroyed and not c1_destroyed and not c2_destroyed


def _budget_worker(rank, world, port, q):
    sys.path.insert(0, ROOT)
    import torch.distributed as dist

    from mccs_amd import ring_bench as rb

    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        now = [0.0]
        b = rb.Budget(dist, seconds=100, clock=lambda: now[0])
        ran = []
        b.run("a", lambda: ran.append("a"), need_s=10)
        now[0] = 95.0 if rank == 0 else 10.0  # only rank 0's clock says a 10 s leg no longer fits
        b.run("b", lambda: ran.append("b"), need_s=10)
        now[0] = 96.0 if rank == 0 else 11.0
        b.run("c", lambda: ran.append("c"), need_s=1)
        q.put((rank, ran, b.summary()["legs"]))
    finally:
        dist.destroy_process_group()


def test_bench_budget_skips_a_leg_on_every_rank():
    """ring_bench.Budget: the extra legs are collective, so a leg that does not
    fit the budget on ANY rank's clock is skipped on all of them (recorded as
    skipped), and a later leg that fits still runs everywhere."""
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_budget_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(2))
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, ran, legs in res:
        assert ran == ["a", "c"], (rank, ran)
        assert legs["b"]["skipped"] == "budget" and legs["b"]["need_s"] == 10
        assert "wall_s" in legs["a"] and "wall_s" in legs["c"]


def _share_worker(rank, world, port, q):
    sys.path.insert(0, ROOT)
    import torch.distributed as dist

    from mccs_amd import ring_bench as rb

    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        out = []
        # a full node with per-rank device visibility: each process sees ONE
        # device, ordinal 0, yet the bus ids differ -> not sharing
        rb.gpu_bus_id = lambda dev: f"0000:{0x10 + rank:02x}:00.0"
        out.append(rb.ranks_share_gpu(dist, 0, world))
        # a 1-GPU rehearsal: every rank on the same bus id -> sharing
        rb.gpu_bus_id = lambda dev: "0000:75:00.0"
        out.append(rb.ranks_share_gpu(dist, 0, world))
        q.put((rank, out))
    finally:
        dist.destroy_process_group()


def test_bench_decides_gpu_sharing_from_bus_ids():
    """The N > 1 line prices ranks that share a GPU against HBM and spreads
    their lanes; whether they do comes from the ranks' PCI bus ids, not from
    how many devices one process sees (1 under per-rank HIP_VISIBLE_DEVICES
    on a full node)."""
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_share_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(2))
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert [r[1] for r in res] == [[False, True], [False, True]]
