"""Independent numpy model of the reference ring allreduce (test-only).

Simulates every rank executing runRing (reference src/collectives/src/
all_reduce.h:10-87) as a sequence of primitive calls that pass FIFO messages
to the next rank (prims_simple.h send/recvReduceSend/directRecvReduceCopySend/
directRecvCopySend/directRecv, operand order srcs = [user input, received]
from prims_simple.h:174-177).  Arithmetic is numpy's own float16/float32
element ops, so this checks the C oracle's walk and rounding independently.
"""
from __future__ import annotations

from collections import deque

import numpy as np


def _fn(op, x, y):
    if op == "sum":
        with np.errstate(over="ignore"):
            return x + y
    if op == "prod":
        with np.errstate(over="ignore"):
            return x * y
    if op == "max":
        return np.where(x < y, y, x)
    return np.where(x < y, x, y)


def chunk_size_elems(buff_size, itemsize):
    return int(buff_size // 8 // itemsize * 4)


def rank_program(rank_index, n, count, nch, bid, nthreads, buff_size, itemsize):
    """Yields (primitive, offset, nelem) for one channel of one rank (runRing)."""
    chunk = chunk_size_elems(buff_size, itemsize)
    loop = nch * n * chunk
    gran = (nthreads - 32) * 8 // itemsize
    g = 0
    while g < count:
        rcs = min(chunk, -(-(count - g) // (nch * n)))
        rcs = -(-rcs // gran) * gran
        def off(c):
            return g + bid * n * rcs + c * rcs
        def ne(o):
            return min(rcs, count - o)
        c = (rank_index + n - 1) % n
        yield ("send", off(c), ne(off(c)))
        for j in range(2, n):
            c = (rank_index + n - j) % n
            yield ("recvReduceSend", off(c), ne(off(c)))
        c = rank_index
        yield ("recvReduceCopySend", off(c), ne(off(c)))
        for j in range(1, n - 1):
            c = (rank_index + n - j) % n
            yield ("recvCopySend", off(c), ne(off(c)))
        c = (rank_index + 1) % n
        yield ("recv", off(c), ne(off(c)))
        g += loop


def simulate(inputs, op, nch, nthreads, buff_size=1 << 22, ring=None):
    """inputs: list of per-rank 1-D numpy arrays; ring: one send-order list for
    every channel, or a list of per-channel lists (default 0..n-1).
    Returns the list of per-rank outputs."""
    n = len(inputs)
    count = inputs[0].size
    itemsize = inputs[0].dtype.itemsize
    if ring is None:
        rings = [list(range(n))] * nch
    elif isinstance(ring[0], (list, tuple)):
        rings = [list(x) for x in ring]
    else:
        rings = [list(ring)] * nch
    outs = [x.copy() for x in inputs]
    ins = [x.copy() for x in inputs]
    for bid in range(nch):
        ring = rings[bid]
        pos0 = ring.index(0)
        index_of = {r: (ring.index(r) - pos0) % n for r in range(n)}
        nxt = {ring[i]: ring[(i + 1) % n] for i in range(n)}
        fifo = {r: deque() for r in range(n)}  # messages into rank r
        progs = {r: list(rank_program(index_of[r], n, count, nch, bid, nthreads, buff_size, itemsize))
                 for r in range(n)}
        pc = {r: 0 for r in range(n)}
        progressed = True
        while progressed:
            progressed = False
            for r in range(n):
                while pc[r] < len(progs[r]):
                    prim, o, m = progs[r][pc[r]]
                    m = max(m, 0)
                    needs_recv = prim != "send"
                    if needs_recv and not fifo[r]:
                        break
                    recv = fifo[r].popleft() if needs_recv else None
                    sl = slice(o, o + m)
                    if prim == "send":
                        msg = ins[r][sl].copy()
                    elif prim == "recvReduceSend":
                        msg = _fn(op, ins[r][sl], recv)
                    elif prim == "recvReduceCopySend":
                        msg = _fn(op, ins[r][sl], recv)
                        outs[r][sl] = msg
                    elif prim == "recvCopySend":
                        outs[r][sl] = recv
                        msg = recv
                    else:  # recv
                        outs[r][sl] = recv
                        msg = None
                    if msg is not None:
                        fifo[nxt[r]].append(np.asarray(msg, dtype=inputs[0].dtype))
                    pc[r] += 1
                    progressed = True
        assert all(pc[r] == len(progs[r]) for r in range(n)), "ring deadlocked"
    return outs
