#!/usr/bin/env python3
"""Diagnose ring mismatches on a virtual node: where and how outputs differ."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

from mccs_amd import comm as C  # noqa: E402
from oracle import oracle as orc  # noqa: E402
import vnode  # noqa: E402


def run(n, code, count, **cfg):
    comms = C.init_all([0] * n, C.CommConfig(**cfg))
    rng = np.random.default_rng(n * 10 + code)
    inputs = [vnode.gen(code, count, rng) for _ in range(n)]
    outs = vnode.run_allreduce(comms, inputs, code, 0)
    p = vnode.Planner(comms[0].nchannels, comms[0].rings())
    nch, nthr, rings = p.select(count * vnode.ESIZE[code], 0)
    exp, owner = orc.ring_allreduce(code, 0, inputs, nchannels=nch, nthreads=nthr, ring_orders=rings,
                                    want_owner=True)
    print(f"n={n} code={code} count={count} cfg={cfg} nch={nch} nthr={nthr} lanes={comms[0].lanes} "
          f"rings={rings}")
    for r in range(n):
        bad = np.nonzero(outs[r].view(np.uint8 if code in (0, 1) else np.uint32 if vnode.ESIZE[code] == 4
                                      else np.uint16) != exp.view(np.uint8 if code in (0, 1) else np.uint32 if
                                                                  vnode.ESIZE[code] == 4 else np.uint16))[0]
        if len(bad):
            print(f"  rank {r}: {len(bad)} bad, first {bad[:8]}, last {bad[-4:]}, owners {np.unique(owner[bad])}")
            i = bad[0]
            terms = [inputs[q][i] for q in range(n)]
            print(f"    got {outs[r][i]!r} exp {exp[i]!r} inputs {terms} others "
                  f"{[outs[q][i] for q in range(n)]}")
        else:
            print(f"  rank {r}: ok")
    vnode.destroy(comms)


if __name__ == "__main__":
    run(3, 7, 300007)
    run(3, 7, 300007, lanes=1)
    run(3, 7, 300007, fifo_memory=C.FIFO_DEVICE)
    run(3, 7, 300007, channel_count=1)
    run(3, 2, 300007)
    run(4, 7, 300007)
