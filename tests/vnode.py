"""Test helper: an n-rank "virtual node" on one GPU (test-only).

All ranks live in this process on cuda:0 (mccsCommInitAll with repeated
devices); their collectives are issued inside one group so the planner fuses
them into a single multi-rank launch (ring blocks of all ranks co-resident,
spinning on each other's FIFO flags in HBM).  The expected result comes from
the C oracle with the same channel selection, schema and ring orders the
planner used (plan.rs:172-302 semantics).
"""
from __future__ import annotations

import numpy as np

from mccs_amd import comm as C

ESIZE = {0: 1, 1: 1, 2: 4, 3: 4, 4: 8, 5: 8, 6: 2, 7: 4, 8: 8, 9: 2}
NPDT = {0: np.int8, 1: np.uint8, 2: np.int32, 3: np.uint32, 4: np.int64, 5: np.uint64, 6: np.float16,
        7: np.float32, 8: np.float64, 9: np.uint16}


def gen(code, count, rng, dist="uniform"):
    npdt = NPDT[code]
    if dist == "exact":
        return (rng.integers(-255, 256, count) / 64.0).astype(npdt)
    if code in (6, 7, 8):
        return (rng.random(count, dtype=np.float32) * 2 - 1).astype(npdt)
    if code == 9:
        f = rng.random(count, dtype=np.float32) * 2 - 1
        return (f.view(np.uint32) >> 16).astype(np.uint16)
    return rng.integers(-5, 6, count).astype(npdt)


def to_dev(x):
    import torch

    return torch.from_numpy(np.ascontiguousarray(x).view(np.uint8).copy()).cuda()


def from_dev(t, code):
    return t.cpu().numpy().view(NPDT[code])


class Planner:
    """Python mirror of the planner's channel selection for expected values."""

    def __init__(self, nch_cfg, rings):
        self.nch = nch_cfg
        self.rings = rings
        self.load = [0] * nch_cfg

    def select(self, total_bytes, elem_bytes_count):
        nch, nthr = C.task_schema(total_bytes, self.nch)
        order = sorted(range(self.nch), key=lambda i: (self.load[i], i))[:nch]
        for i in order:
            self.load[i] += elem_bytes_count
        return nch, nthr, [self.rings[i] for i in order]


def expected_allreduce(orc, inputs, code, op, comm0, planner=None, buff_size=1 << 22):
    count = inputs[0].size
    p = planner or Planner(comm0.nchannels, comm0.rings())
    nch, nthr, rings = p.select(count * ESIZE[code], count * ESIZE[code])
    return orc.ring_allreduce(code, op, inputs, nchannels=nch, nthreads=nthr, buff_size=buff_size,
                              ring_orders=rings)


def run_allreduce(comms, inputs, code, op, inplace=False):
    """One group allreduce across all ranks; returns per-rank numpy outputs."""
    n = len(comms)
    count = inputs[0].size
    send = [to_dev(x) for x in inputs]
    recv = send if inplace else [to_dev(np.zeros_like(x)) for x in inputs]
    with C.group():
        for r in range(n):
            C.all_reduce(comms[r], send[r], recv[r], count, code, op)
    for c in comms:
        c.sync()
    return [from_dev(recv[r], code) for r in range(n)]


def destroy(comms):
    import torch

    torch.cuda.synchronize()
    for c in comms:
        c.destroy()


# A DDP-style bucket stream (tests/test_gpu_ddp_stream.py, tests/ipc_worker.py
# "ddp"): (dtype code, bytes per rank) of one step's buckets -- a small first
# bucket, DDP's 25 MiB buckets, ragged remainders, and sizes on both sides of
# every default direct / LL threshold.
DDP_STREAM = [(7, 24), (6, 16 << 10), (7, 100 << 10), (9, (128 << 10) + 2), (7, 200 << 10),
              (6, 600 << 10), (7, 1 << 20), (7, (1 << 20) + 4), (6, 1536 << 10), (7, 2 << 20),
              (7, 3 << 20), (6, 6 << 20), (7, 8 << 20), (7, (8 << 20) + 4096), (7, 25 << 20),
              (6, 25 << 20), (7, (7 << 20) + 12)]


def ddp_expected_algo(nbytes: int, n: int, uncached: bool = True) -> str:
    """The kernel the library's defaults give a bucket of nbytes per rank
    (api.cpp fill_defaults; LL needs an uncached arena; peer atomics assumed)."""
    import ctypes

    from mccs_amd import _lib

    lib = _lib.load()
    one, two = ctypes.c_int(), ctypes.c_int()
    lib.mccs_direct_defaults(n, ctypes.byref(one), ctypes.byref(two))
    if uncached and nbytes <= lib.mccs_ll_default(n):
        return "ll"
    if one.value > 0 and nbytes <= one.value:
        return "oneshot"
    if two.value > 0 and nbytes <= two.value:
        return "direct"
    return "ring"
