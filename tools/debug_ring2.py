#!/usr/bin/env python3
"""More ring diagnostics: allgather small sizes, run-order effects, flag state."""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import torch  # noqa: E402

from mccs_amd import comm as C  # noqa: E402
from oracle import oracle as orc  # noqa: E402
import vnode  # noqa: E402


def allgather(n, nbytes, **cfg):
    comms = C.init_all([0] * n, C.CommConfig(**cfg))
    rng = np.random.default_rng(nbytes)
    inputs = [rng.integers(0, 256, nbytes, dtype=np.uint8) for _ in range(n)]
    send = [vnode.to_dev(x) for x in inputs]
    recv = [vnode.to_dev(np.zeros(n * nbytes, np.uint8)) for _ in range(n)]
    with C.group():
        for r in range(n):
            C.all_gather(comms[r], send[r], recv[r], nbytes)
    for c in comms:
        c.sync()
    exp = orc.ring_allgather(inputs)
    print(f"allgather n={n} nbytes={nbytes} cfg={cfg} lanes={comms[0].lanes} rings0={comms[0].rings()[0]}")
    for r in range(n):
        got = recv[r].cpu().numpy()
        bad = np.nonzero(got != exp)[0]
        if len(bad):
            print(f"  rank {r}: {len(bad)} bad at {bad[:16]} got {got[bad[:8]]} exp {exp[bad[:8]]}")
            if nbytes <= 16:
                print(f"    got {got.tolist()}\n    exp {exp.tolist()}")
    vnode.destroy(comms)


def allreduce(n, code, count, label, **cfg):
    comms = C.init_all([0] * n, C.CommConfig(**cfg))
    rng = np.random.default_rng(n * 10 + code)
    inputs = [vnode.gen(code, count, rng) for _ in range(n)]
    outs = vnode.run_allreduce(comms, inputs, code, 0)
    exp = vnode.expected_allreduce(orc, inputs, code, 0, comms[0])
    nbad = [int(np.count_nonzero(o.view(np.uint8) != exp.view(np.uint8))) for o in outs]
    print(f"{label}: allreduce n={n} code={code} cfg={cfg} fifo_mem={comms[0].fifo_memory} bad bytes per rank {nbad}")
    vnode.destroy(comms)


if __name__ == "__main__":
    for nb in (1, 1000, 4096, 1 << 20):
        allgather(8, nb)
    allgather(8, 1, lanes=1)
    allgather(8, 1000, lanes=1)
    allgather(8, 1000, channel_count=1)
    allreduce(3, 2, 300007, "A-first-uc")
    allreduce(3, 2, 300007, "B-second-uc")
    allreduce(3, 7, 300007, "C-device", fifo_memory=C.FIFO_DEVICE)
    allreduce(3, 2, 300007, "D-after-device-uc")
    allreduce(3, 2, 300007, "E-uc")
    allreduce(3, 7, 300007, "F-device-lanes1", fifo_memory=C.FIFO_DEVICE, lanes=1)
    allreduce(3, 2, 300007, "G-uc")
