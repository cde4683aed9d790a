"""GPU: seeded random ring configurations against the oracle.

Each case draws the rank count, dtype, op, element count (ragged, sometimes
tiny, sometimes several FIFO loops), channels, lanes, block size, FIFO depth, FIFO
memory kind, data placement, slicing, an optional ring override and, half of
the time, direct-kernel thresholds and workgroup caps, runs one
grouped AllReduce (or AllGather) on a virtual node and compares every rank
bit for bit with the oracle's restatement of the reference schedule.
"""
import os

import numpy as np
import pytest

from mccs_amd import comm as C
import vnode

pytestmark = pytest.mark.gpu

CASES = int(os.environ.get("MCCS_FUZZ_CASES", "24"))


def _case(seed):
    rng = np.random.default_rng(seed)
    n = int(rng.integers(2, 9))
    code = int(rng.choice([0, 2, 4, 6, 7, 8, 9]))
    op = int(rng.choice([0, 0, 0, 1, 2, 3]))
    esize = vnode.ESIZE[code]
    count = int(rng.choice([1, 3, 127, 4096 + 3, int(rng.integers(1, 1 << 20)), (1 << 22) // esize + 77]))
    cfg = {}
    if rng.random() < 0.5:
        cfg["channel_count"] = int(rng.integers(1, 7))
    if rng.random() < 0.5:
        cfg["lanes"] = int(rng.choice([1, 2, 3]))
    if rng.random() < 0.3:
        cfg["block_threads"] = int(rng.choice([128, 256, 544, 576]))
    if rng.random() < 0.3:
        cfg["fifo_memory"] = C.FIFO_DEVICE
    if rng.random() < 0.3:
        cfg["locality"] = C.LOCALITY_SENDER
    if rng.random() < 0.3:
        cfg["buffer_size"] = int(rng.choice([1 << 20, 1 << 21]))
    if rng.random() < 0.3:
        nch = cfg.setdefault("channel_count", 2)
        cfg["rings"] = [list(rng.permutation(n)) for _ in range(nch)]
    slice2 = bool(rng.random() < 0.25)
    gather = bool(rng.random() < 0.2)
    if rng.random() < 0.3:
        cfg["fifo_slots"] = int(rng.choice([16, 32]))
    fifo_works = bool(rng.random() < 0.3)  # work list through the FIFO even where it fits the launch arguments
    # the direct kernel (LL / one-shot / two-shot / AllGather one-shot) at random
    # thresholds and workgroup caps; results must not change
    blocks = None
    if rng.random() < 0.5:
        cfg["oneshot_bytes"] = int(rng.choice([-1, 64 << 10, 1 << 20, 8 << 20]))
        cfg["direct_bytes"] = int(rng.choice([-1, 1 << 20, 8 << 20, 32 << 20]))
        cfg["ll_bytes"] = int(rng.choice([-1, 16 << 10, 128 << 10, 1 << 20]))
        blocks = int(rng.choice([1, 3, 16, 128]))
    return n, code, op, count, cfg, slice2, gather, fifo_works, blocks, rng


@pytest.mark.parametrize("seed", range(CASES))
def test_random_ring_case(orc, seed, monkeypatch):
    n, code, op, count, cfg, slice2, gather, fifo_works, blocks, rng = _case(1000 + seed)
    if blocks:
        monkeypatch.setenv("MCCS_DIRECT_BLOCKS", str(blocks))
    if slice2:
        monkeypatch.setenv("MCCS_SLICE_STEPS", "2")
    if fifo_works:
        monkeypatch.setenv("MCCS_INLINE_WORKS", "0")
    comms = C.init_all([0] * n, C.CommConfig(**cfg))
    try:
        if gather:
            nbytes = count * vnode.ESIZE[code]
            inputs = [rng.integers(0, 256, nbytes, dtype=np.uint8) for _ in range(n)]
            send = [vnode.to_dev(x) for x in inputs]
            recv = [vnode.to_dev(np.zeros(n * nbytes, np.uint8)) for _ in range(n)]
            with C.group():
                for r in range(n):
                    C.all_gather(comms[r], send[r], recv[r], nbytes)
            for c in comms:
                c.sync()
            exp = orc.ring_allgather(inputs)
            for r in range(n):
                assert np.array_equal(recv[r].cpu().numpy(), exp), (seed, r)
            return
        inputs = [vnode.gen(code, count, rng) for _ in range(n)]
        outs = vnode.run_allreduce(comms, inputs, code, op)
        exp = vnode.expected_allreduce(orc, inputs, code, op, comms[0], buff_size=cfg.get("buffer_size", 1 << 22))
        for r, o in enumerate(outs):
            assert np.array_equal(o.view(np.uint8), exp.view(np.uint8)), (seed, n, code, op, count, cfg, slice2, r)
    finally:
        vnode.destroy(comms)
