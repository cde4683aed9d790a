"""CPU: BASELINE configs[0] -- 2-rank loopback allreduce of 1 KiB fp32 with a
host-side elementwise sum, i.e. the ring FIFO protocol run by host threads
(mccs_host_ring_allreduce), checked bit for bit against the oracle; plus
larger n, channel counts, ring overrides and the allreduce_proto KAT."""
import numpy as np
import pytest

from mccs_amd import comm as C


def _run(n, code, count, nch, nthr, buff=1 << 22, rings=None, op=0, seed=0, inplace=False):
    npdt = {2: np.int32, 6: np.float16, 7: np.float32, 9: np.uint16}[code]
    rng = np.random.default_rng(seed)
    if code == 2:
        xs = [rng.integers(-1000, 1000, count).astype(npdt) for _ in range(n)]
    elif code == 9:
        xs = [((rng.random(count, dtype=np.float32) * 2 - 1).view(np.uint32) >> 16).astype(np.uint16)
              for _ in range(n)]
    else:
        xs = [(rng.random(count, dtype=np.float32) * 2 - 1).astype(npdt) for _ in range(n)]
    ins = [x.copy() for x in xs]
    outs = ins if inplace else [np.zeros_like(x) for x in xs]
    C.host_ring_allreduce(ins, outs, count, code, op, channels=nch, nthreads=nthr, buffer_size=buff, rings=rings)
    return xs, outs


def test_config0_two_rank_loopback_1kib_fp32(orc):
    xs, outs = _run(2, 7, 256, 1, 96)  # schema for 1 KiB: 1 channel, 96 threads
    exp = orc.ring_allreduce(7, 0, xs, nchannels=1, nthreads=96)
    for o in outs:
        assert np.array_equal(o.view(np.uint32), exp.view(np.uint32))
    # n = 2: one add per element, commutative -> also the plain sum
    assert np.array_equal(exp, (xs[0] + xs[1]).astype(np.float32))


@pytest.mark.parametrize("n,code,count,nch,nthr,buff", [
    (3, 6, 100003, 2, 544, 1 << 22), (4, 7, 70001, 2, 288, 1 << 16), (8, 6, 50000, 3, 544, 1 << 20),
    (5, 2, 12345, 1, 160, 1 << 22), (4, 9, 33333, 2, 544, 1 << 22)])
def test_host_ring_matches_oracle(orc, n, code, count, nch, nthr, buff):
    xs, outs = _run(n, code, count, nch, nthr, buff, seed=count)
    exp = orc.ring_allreduce(code, 0, xs, nchannels=nch, nthreads=nthr, buff_size=buff)
    for r, o in enumerate(outs):
        assert np.array_equal(o.view(np.uint8), exp.view(np.uint8)), r


def test_host_ring_overrides_and_inplace(orc):
    rings = [[0, 2, 1, 3], [3, 1, 0, 2]]
    xs, outs = _run(4, 6, 40001, 2, 544, 1 << 18, rings=rings, inplace=True, seed=3)
    exp = orc.ring_allreduce(6, 0, xs, nchannels=2, nthreads=544, buff_size=1 << 18, ring_orders=rings)
    for o in outs:
        assert np.array_equal(o.view(np.uint16), exp.view(np.uint16))


def test_host_ring_kat():
    n, count = 4, (1 << 18) + 9
    ins = [np.full(count, 2042 + r, np.int32) for r in range(n)]
    outs = [np.zeros(count, np.int32) for _ in range(n)]
    C.host_ring_allreduce(ins, outs, count, 2, 0, channels=2, nthreads=544, buffer_size=1 << 16)
    for o in outs:
        assert np.all(o == 2042 * n + n * (n - 1) // 2)


def test_host_ring_pool_across_changing_shapes():
    """Back-to-back calls whose task counts grow and shrink (2x1 .. 8x2
    tasks): parked workers without a task in one call must not run the next
    call's task twice or miss it; every sum exact (integer-valued fp32)."""
    rng = np.random.default_rng(5)
    shapes = [(2, 1), (8, 2), (3, 1), (5, 2), (2, 2), (8, 1), (4, 1)]
    for it in range(140):
        n, nch = shapes[it % len(shapes)]
        count = int(rng.integers(1, 3000))
        send = [rng.integers(-64, 64, count).astype(np.float32) for _ in range(n)]
        recv = [np.empty_like(x) for x in send]
        C.host_ring_allreduce(send, recv, count, C.AllReduceDataType.Float32, channels=nch, nthreads=96)
        exp = np.sum(send, axis=0, dtype=np.float32)
        assert all(np.array_equal(r, exp) for r in recv), (it, n, nch)
