"""GPU parity of the direct AllReduce (two-shot and one-shot) against the oracle.

The direct kernel (mccs_amd/csrc/direct_kernel.h) either sends every ring
chunk to its owner, reduces it there in the ring's order and broadcasts the
result (two-shot), or sends every input everywhere and lets each rank reduce
every chunk in the ring's order (one-shot), so its output must equal the
ring's -- and the oracle's ring-order restatement -- bit for bit, for the
same channels, thread count and rings the planner would have given the ring
(vnode.expected_allreduce).  Runs on the virtual node (all ranks on cuda:0,
one fused launch); every test also asserts that the call really took the
variant under test (Communicator.last_algo).
"""
import numpy as np
import pytest

from mccs_amd import comm as C
import vnode

pytestmark = pytest.mark.gpu
DIRECT_DEFAULTS = True  # conftest: keep the library's direct thresholds

F16, F32, BF16, I32, F64, I8 = 6, 7, 9, 2, 8, 0
DIRECT = 8 << 20
LL_MAX = 1 << 20  # the largest ll_bytes a comm accepts
VARIANTS = ["direct", "oneshot", "ll"]


def _cfg(variant="direct", **kw):
    """One variant per comm.  "ll": the LL one-shot up to LL_MAX, larger
    buckets the one-shot (so every test size has a direct kernel)."""
    kw.setdefault("direct_bytes", DIRECT if variant == "direct" else -1)
    kw.setdefault("oneshot_bytes", DIRECT if variant in ("oneshot", "ll") else -1)
    kw.setdefault("ll_bytes", LL_MAX if variant == "ll" else -1)
    return C.CommConfig(**kw)


def _check(outs, exp):
    for r, o in enumerate(outs):
        assert np.array_equal(o.view(np.uint8), exp.view(np.uint8)), f"rank {r} differs from oracle"


def _algo(comms, want="direct", nbytes=None):
    if want == "ll" and nbytes is not None and nbytes > LL_MAX:
        want = "oneshot"
    assert all(c.last_algo() == want for c in comms), [c.last_algo() for c in comms]


@pytest.mark.parametrize("variant", VARIANTS)
@pytest.mark.parametrize("n", [2, 3, 4, 5, 8])
@pytest.mark.parametrize("code", [F32, F16, BF16])
def test_direct_matches_oracle(orc, n, code, variant):
    comms = C.init_all([0] * n, _cfg(variant))
    try:
        rng = np.random.default_rng(n * 10 + code)
        inputs = [vnode.gen(code, 300007, rng) for _ in range(n)]
        outs = vnode.run_allreduce(comms, inputs, code, 0)
        _algo(comms, variant, inputs[0].nbytes)
        _check(outs, vnode.expected_allreduce(orc, inputs, code, 0, comms[0]))
    finally:
        vnode.destroy(comms)


@pytest.mark.parametrize("variant", VARIANTS)
@pytest.mark.parametrize("code", list(range(10)))
@pytest.mark.parametrize("op", [0, 1, 2, 3])
def test_direct_every_dtype_and_op(orc, code, op, variant):
    n = 4
    comms = C.init_all([0] * n, _cfg(variant))
    try:
        rng = np.random.default_rng(code * 4 + op)
        inputs = [vnode.gen(code, 40013, rng) for _ in range(n)]
        outs = vnode.run_allreduce(comms, inputs, code, op)
        _algo(comms, variant, inputs[0].nbytes)
        _check(outs, vnode.expected_allreduce(orc, inputs, code, op, comms[0]))
    finally:
        vnode.destroy(comms)


@pytest.mark.parametrize("variant", VARIANTS)
@pytest.mark.parametrize("count", [1, 7, 255, 4097, 16385, 65536 * 3 + 5, (2 << 20) - 1])
def test_direct_sizes(orc, count, variant):
    """Tiny buckets (fewer elements than chunks: some owners get none) up to
    the direct capacity (8 MiB of fp32)."""
    n = 8
    comms = C.init_all([0] * n, _cfg(variant))
    try:
        rng = np.random.default_rng(count)
        inputs = [vnode.gen(F32, count, rng) for _ in range(n)]
        outs = vnode.run_allreduce(comms, inputs, F32, 0)
        _algo(comms, variant, inputs[0].nbytes)
        _check(outs, vnode.expected_allreduce(orc, inputs, F32, 0, comms[0]))
    finally:
        vnode.destroy(comms)


@pytest.mark.parametrize("variant", VARIANTS)
@pytest.mark.parametrize("n", [3, 8])
def test_direct_multi_loop_walk(orc, n, variant):
    """A small FIFO buffer (64 KiB: 8 KiB chunks) makes the ring walk several
    loops plus a partial one inside one direct bucket; the kernel's walk must
    follow (all_reduce.h loop / realChunkSize rounding)."""
    buff = 1 << 16
    comms = C.init_all([0] * n, _cfg(variant, buffer_size=buff))
    try:
        rng = np.random.default_rng(n)
        count = 3 * comms[0].nchannels * n * (buff // 8 // 2 * 4 // 2) + 12345
        inputs = [vnode.gen(F16, count, rng) for _ in range(n)]
        outs = vnode.run_allreduce(comms, inputs, F16, 0)
        _algo(comms, variant, inputs[0].nbytes)
        _check(outs, vnode.expected_allreduce(orc, inputs, F16, 0, comms[0], buff_size=buff))
    finally:
        vnode.destroy(comms)


@pytest.mark.parametrize("variant", VARIANTS)
def test_direct_doubled_channels_and_custom_rings(orc, variant):
    n = 8
    rings = C.default_rings(8, 0)
    rings = rings + [list(reversed(r)) for r in rings]  # 14 channels
    comms = C.init_all([0] * n, _cfg(variant, rings=rings))
    try:
        assert comms[0].nchannels == 14
        rng = np.random.default_rng(5)
        inputs = [vnode.gen(BF16, 777777, rng) for _ in range(n)]
        outs = vnode.run_allreduce(comms, inputs, BF16, 0)
        _algo(comms, variant, inputs[0].nbytes)
        _check(outs, vnode.expected_allreduce(orc, inputs, BF16, 0, comms[0]))
    finally:
        vnode.destroy(comms)


@pytest.mark.parametrize("variant", VARIANTS)
def test_direct_in_place(orc, variant):
    n = 4
    comms = C.init_all([0] * n, _cfg(variant))
    try:
        rng = np.random.default_rng(11)
        inputs = [vnode.gen(F32, 500001, rng) for _ in range(n)]
        outs = vnode.run_allreduce(comms, inputs, F32, 0, inplace=True)
        _algo(comms, variant, inputs[0].nbytes)
        _check(outs, vnode.expected_allreduce(orc, inputs, F32, 0, comms[0]))
    finally:
        vnode.destroy(comms)


def test_direct_and_ring_interleaved(orc):
    """Buckets on every side of the thresholds alternate on the same comms:
    the direct launches' running counts, the one-shot parity and the ring's
    FIFO steps all stay in lock-step, every result exact."""
    n = 4
    comms = C.init_all([0] * n, C.CommConfig(direct_bytes=1 << 20, oneshot_bytes=64 << 10, ll_bytes=16 << 10))
    try:
        rng = np.random.default_rng(3)
        for it, count in enumerate([1000, 300000, 262144, 16384, 16385, 262145, 5, 1 << 20, 77777, 3, 4] * 2):
            inputs = [vnode.gen(F32, count, rng) for _ in range(n)]
            outs = vnode.run_allreduce(comms, inputs, F32, 0)
            nb = count * 4
            _algo(comms, "ll" if nb <= 16 << 10 else "oneshot" if nb <= 64 << 10 else "direct" if nb <= (1 << 20)
                  else "ring")
            _check(outs, vnode.expected_allreduce(orc, inputs, F32, 0, comms[0]))
    finally:
        vnode.destroy(comms)


@pytest.mark.parametrize("variant", VARIANTS)
def test_direct_many_back_to_back(orc, variant):
    """Launches without a sync in between, each with its own inputs and
    output (ring_cfg.h's argument for reusing the slots of back-to-back
    launches: a slot overwritten too early shows up as a wrong result), then
    200 more of the same call."""
    import torch

    n, count, k = 8, 65537, 24
    comms = C.init_all([0] * n, _cfg(variant))
    try:
        rng = np.random.default_rng(8)
        inputs = [[vnode.gen(F32, count, rng) for _ in range(n)] for _ in range(k)]
        send = [[vnode.to_dev(x) for x in inp] for inp in inputs]
        recv = [[vnode.to_dev(np.zeros_like(x)) for x in inp] for inp in inputs]
        for i in range(k):
            with C.group():
                for r in range(n):
                    C.all_reduce(comms[r], send[i][r], recv[i][r], count, F32, 0)
        for _ in range(200):
            with C.group():
                for r in range(n):
                    C.all_reduce(comms[r], send[0][r], recv[0][r], count, F32, 0)
        torch.cuda.synchronize()
        for c in comms:
            c.sync()
        _algo(comms, variant)
        for i in range(k):
            exp = vnode.expected_allreduce(orc, inputs[i], F32, 0, comms[0])
            _check([vnode.from_dev(recv[i][r], F32) for r in range(n)], exp)
    finally:
        vnode.destroy(comms)


def test_direct_group_of_two_takes_the_ring(orc):
    """Two AllReduces of one comm in one group are batched for the ring
    (pre_launch_schedule), never split across kernels."""
    import torch

    n, count = 4, 10007
    comms = C.init_all([0] * n, _cfg())
    try:
        rng = np.random.default_rng(21)
        a = [vnode.gen(F32, count, rng) for _ in range(n)]
        b = [vnode.gen(F32, count, rng) for _ in range(n)]
        sa, sb = [vnode.to_dev(x) for x in a], [vnode.to_dev(x) for x in b]
        ra, rb = [vnode.to_dev(np.zeros_like(x)) for x in a], [vnode.to_dev(np.zeros_like(x)) for x in b]
        with C.group():
            for r in range(n):
                C.all_reduce(comms[r], sa[r], ra[r], count, F32, 0)
                C.all_reduce(comms[r], sb[r], rb[r], count, F32, 0)
        torch.cuda.synchronize()
        for c in comms:
            c.sync()
        _algo(comms, "ring")
        p = vnode.Planner(comms[0].nchannels, comms[0].rings())
        ea = vnode.expected_allreduce(orc, a, F32, 0, comms[0], planner=p)
        eb = vnode.expected_allreduce(orc, b, F32, 0, comms[0], planner=p)
        _check([vnode.from_dev(ra[r], F32) for r in range(n)], ea)
        _check([vnode.from_dev(rb[r], F32) for r in range(n)], eb)
    finally:
        vnode.destroy(comms)


@pytest.mark.parametrize("variant", VARIANTS)
def test_direct_captured_in_hip_graph(orc, variant):
    """Direct launches captured into a HIP graph replay with fresh inputs,
    interleaved with eager direct calls (the launch counter lives in device
    memory, so replays and eager launches keep counting together)."""
    import torch

    n, count = 4, 123457
    comms = C.init_all([0] * n, _cfg(variant))
    try:
        rng = np.random.default_rng(13)
        send = [torch.empty(count, dtype=torch.float16, device="cuda") for _ in range(n)]
        recv = [torch.empty_like(x) for x in send]
        s = torch.cuda.Stream()
        with C.group():
            for r in range(n):
                C.all_reduce(comms[r], send[r], recv[r], count, F16, 0, stream=s)
        s.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            for _ in range(2):
                with C.group():
                    for r in range(n):
                        C.all_reduce(comms[r], send[r], recv[r], count, F16, 0, stream=s)
        for it in range(3):
            inputs = [vnode.gen(F16, count, rng) for _ in range(n)]
            for r in range(n):
                send[r].copy_(torch.from_numpy(inputs[r]).cuda())
            torch.cuda.synchronize()
            if it == 1:
                with C.group():
                    for r in range(n):
                        C.all_reduce(comms[r], send[r], recv[r], count, F16, 0, stream=s)
                s.synchronize()
            g.replay()
            torch.cuda.synchronize()
            for c in comms:
                c.sync()
            _algo(comms, variant)
            exp = vnode.expected_allreduce(orc, inputs, F16, 0, comms[0])
            _check([recv[r].cpu().numpy() for r in range(n)], exp)
    finally:
        torch.cuda.synchronize()
        vnode.destroy(comms)


@pytest.mark.parametrize("variant", VARIANTS)
@pytest.mark.parametrize("code,off", [(F16, 2), (F32, 12)])
def test_direct_misaligned_buffers(orc, code, off, variant):
    import torch

    n, count = 3, 100003
    comms = C.init_all([0] * n, _cfg(variant))
    try:
        rng = np.random.default_rng(off)
        inputs = [vnode.gen(code, count, rng) for _ in range(n)]
        nbytes = inputs[0].nbytes
        sbuf = [torch.zeros(nbytes + 64, dtype=torch.uint8, device="cuda") for _ in range(n)]
        rbuf = [torch.zeros(nbytes + 64, dtype=torch.uint8, device="cuda") for _ in range(n)]
        for r in range(n):
            sbuf[r][off:off + nbytes].copy_(torch.from_numpy(inputs[r].view(np.uint8).copy()).cuda())
        with C.group():
            for r in range(n):
                C.all_reduce(comms[r], sbuf[r].data_ptr() + off, rbuf[r].data_ptr() + off, count, code, 0)
        for c in comms:
            c.sync()
        _algo(comms, variant)
        outs = [rbuf[r][off:off + nbytes].cpu().numpy().view(inputs[0].dtype) for r in range(n)]
        _check(outs, vnode.expected_allreduce(orc, inputs, code, 0, comms[0]))
    finally:
        vnode.destroy(comms)


@pytest.mark.parametrize("variant", VARIANTS)
@pytest.mark.parametrize("fifo", [C.FIFO_DEVICE, C.FIFO_UNCACHED_RELEASE])
def test_direct_hand_off_modes(orc, fifo, variant):
    """Cached arena (system-scope release before counting out, acquire after
    a wait) and uncached + release fence."""
    n = 4
    comms = C.init_all([0] * n, _cfg(variant, fifo_memory=fifo))
    try:
        rng = np.random.default_rng(fifo)
        for count in (70001, 1 << 20):
            inputs = [vnode.gen(F32, count, rng) for _ in range(n)]
            outs = vnode.run_allreduce(comms, inputs, F32, 0)
            # a cached arena never takes the LL one-shot
            _algo(comms, "oneshot" if variant == "ll" and fifo == C.FIFO_DEVICE else variant, inputs[0].nbytes)
            _check(outs, vnode.expected_allreduce(orc, inputs, F32, 0, comms[0]))
    finally:
        vnode.destroy(comms)


def test_library_defaults(orc):
    """The library defaults at n = 4: LL one-shot up to 128 KiB per rank,
    one-shot up to 1 MiB, two-shot up to 8 MiB, the ring above."""
    n = 4
    comms = C.init_all([0] * n)
    try:
        assert all(c.direct_enabled() for c in comms)
        rng = np.random.default_rng(44)
        for count, want in ((1000, "ll"), (32768, "ll"), (32769, "oneshot"), (262144, "oneshot"), (262145, "direct"), (2 << 20, "direct"),
                            ((2 << 20) + 1, "ring")):
            inputs = [vnode.gen(F32, count, rng) for _ in range(n)]
            outs = vnode.run_allreduce(comms, inputs, F32, 0)
            _algo(comms, want)
            _check(outs, vnode.expected_allreduce(orc, inputs, F32, 0, comms[0]))
    finally:
        vnode.destroy(comms)


def _allgather(comms, bufs_in, nbytes, inplace):
    """One grouped AllGather; returns each rank's output as bytes."""
    import torch

    n = len(comms)
    outs = []
    with C.group():
        for r in range(n):
            if inplace:  # allgather_proto: send = own segment of the output buffer
                out = torch.zeros(n * nbytes, dtype=torch.uint8, device="cuda")
                out[r * nbytes:(r + 1) * nbytes].copy_(bufs_in[r])
                C.all_gather(comms[r], out[r * nbytes:], out, nbytes)
            else:
                out = torch.zeros(n * nbytes, dtype=torch.uint8, device="cuda")
                C.all_gather(comms[r], bufs_in[r], out, nbytes)
            outs.append(out)
    for c in comms:
        c.sync()
    return [o.cpu().numpy() for o in outs]


@pytest.mark.parametrize("inplace", [False, True])
@pytest.mark.parametrize("n", [2, 3, 8])
@pytest.mark.parametrize("nbytes", [1, 1000, 4096, 65539, 1 << 20])
@pytest.mark.parametrize("variant", ["oneshot", "ll"])
def test_allgather_oneshot(n, nbytes, inplace, variant):
    """AllGather buckets up to oneshot_bytes take the one-shot exchange (up
    to ll_bytes its LL lines): every rank's segment lands in every output
    byte for byte (all_gather.h's result), in place (allgather_proto's
    layout) or not."""
    import torch

    comms = C.init_all([0] * n, _cfg(variant))
    try:
        rng = np.random.default_rng(nbytes + n)
        data = [rng.integers(0, 256, nbytes, dtype=np.uint8) for _ in range(n)]
        bufs = [torch.from_numpy(d).cuda() for d in data]
        outs = _allgather(comms, bufs, nbytes, inplace)
        _algo(comms, variant)
        exp = np.concatenate(data)
        for r, o in enumerate(outs):
            assert np.array_equal(o, exp), f"rank {r}"
    finally:
        vnode.destroy(comms)


def test_allgather_oneshot_back_to_back_and_mixed(orc):
    """AllGathers (one-shot and, above the threshold, ring) and AllReduces
    (LL one-shot, one-shot, two-shot) alternate without syncs in between; every output
    exact (the one-shot slots' parity and the running counts are shared by
    both collectives)."""
    import torch

    n = 4
    comms = C.init_all([0] * n, C.CommConfig(direct_bytes=1 << 20, oneshot_bytes=64 << 10, ll_bytes=8 << 10))
    try:
        rng = np.random.default_rng(77)
        plan = [("ag", 5000), ("ar", 3000), ("ag", 70000), ("ar", 100000), ("ag", 65536), ("ar", 7), ("ag", 1)] * 3
        keep = []
        for kind, size in plan:
            if kind == "ag":
                data = [rng.integers(0, 256, size, dtype=np.uint8) for _ in range(n)]
                src = [torch.from_numpy(d).cuda() for d in data]
                out = [torch.zeros(n * size, dtype=torch.uint8, device="cuda") for _ in range(n)]
                with C.group():
                    for r in range(n):
                        C.all_gather(comms[r], src[r], out[r], size)
                keep.append((kind, size, data, src, out, [c.last_algo() for c in comms]))
            else:
                data = [vnode.gen(F32, size, rng) for _ in range(n)]
                src = [vnode.to_dev(x) for x in data]
                out = [vnode.to_dev(np.zeros_like(x)) for x in data]
                with C.group():
                    for r in range(n):
                        C.all_reduce(comms[r], src[r], out[r], size, F32, 0)
                keep.append((kind, size, data, src, out, [c.last_algo() for c in comms]))
        torch.cuda.synchronize()
        for c in comms:
            c.sync()
        for kind, size, data, src, out, algos in keep:
            if kind == "ag":
                want = "ll" if size <= 8 << 10 else "oneshot" if size <= 64 << 10 else "ring"
                assert algos == [want] * n, (size, algos)
                exp = np.concatenate(data)
                for r in range(n):
                    assert np.array_equal(out[r].cpu().numpy(), exp), (size, r)
            else:
                nb = size * 4
                want = "ll" if nb <= 8 << 10 else "oneshot" if nb <= 64 << 10 else "direct"
                assert algos == [want] * n, (size, algos)
                exp = vnode.expected_allreduce(orc, data, F32, 0, comms[0])
                _check([vnode.from_dev(out[r], F32) for r in range(n)], exp)
    finally:
        vnode.destroy(comms)


@pytest.mark.parametrize("variant", ["oneshot", "ll"])
def test_allgather_oneshot_captured_in_hip_graph(variant):
    import torch

    n, size = 3, 40000
    comms = C.init_all([0] * n, _cfg(variant))
    try:
        rng = np.random.default_rng(5)
        src = [torch.zeros(size, dtype=torch.uint8, device="cuda") for _ in range(n)]
        out = [torch.zeros(n * size, dtype=torch.uint8, device="cuda") for _ in range(n)]
        s = torch.cuda.Stream()
        with C.group():
            for r in range(n):
                C.all_gather(comms[r], src[r], out[r], size, stream=s)
        s.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            for _ in range(2):
                with C.group():
                    for r in range(n):
                        C.all_gather(comms[r], src[r], out[r], size, stream=s)
        for it in range(3):
            data = [rng.integers(0, 256, size, dtype=np.uint8) for _ in range(n)]
            for r in range(n):
                src[r].copy_(torch.from_numpy(data[r]).cuda())
            torch.cuda.synchronize()
            g.replay()
            torch.cuda.synchronize()
            for c in comms:
                c.sync()
            exp = np.concatenate(data)
            for r in range(n):
                assert np.array_equal(out[r].cpu().numpy(), exp), (it, r)
        _algo(comms, variant)
    finally:
        torch.cuda.synchronize()
        vnode.destroy(comms)


@pytest.mark.parametrize("code,count", [(I8, 1), (I8, 13), (F16, 3), (F16, 4099), (F32, 7), (F64, 5),
                                        (BF16, 16385), (I32, 65536)])
@pytest.mark.parametrize("inplace", [False, True])
def test_ll_ragged_and_in_place(orc, code, count, inplace):
    """LL one-shot words (8 bytes) over ragged buckets: a last partial word
    (1-byte and 2-byte types), single-element buckets, in place (a thread
    overwrites only words it has already sent)."""
    n = 5
    comms = C.init_all([0] * n, _cfg("ll"))
    try:
        rng = np.random.default_rng(count * 3 + code)
        inputs = [vnode.gen(code, count, rng) for _ in range(n)]
        outs = vnode.run_allreduce(comms, inputs, code, 0, inplace=inplace)
        _algo(comms, "ll")
        _check(outs, vnode.expected_allreduce(orc, inputs, code, 0, comms[0]))
    finally:
        vnode.destroy(comms)


@pytest.mark.parametrize("inplace", [False, True])
def test_ll_several_words_per_thread(orc, monkeypatch, inplace):
    """One workgroup per rank (MCCS_DIRECT_BLOCKS=1): each thread sends and
    reduces 256 words of a 1 MiB bucket, over the ring's 7 rings at n = 8."""
    monkeypatch.setenv("MCCS_DIRECT_BLOCKS", "1")
    n = 8
    comms = C.init_all([0] * n, _cfg("ll"))
    try:
        rng = np.random.default_rng(99)
        inputs = [vnode.gen(F32, 1 << 18, rng) for _ in range(n)]
        outs = vnode.run_allreduce(comms, inputs, F32, 0, inplace=inplace)
        _algo(comms, "ll")
        _check(outs, vnode.expected_allreduce(orc, inputs, F32, 0, comms[0]))
    finally:
        vnode.destroy(comms)


@pytest.mark.parametrize("variant", VARIANTS)
@pytest.mark.parametrize("code", [F32, F16, BF16])
@pytest.mark.parametrize("op", [0, 2, 3])
def test_direct_nan_and_inf(orc, code, op, variant):
    """NaN / +-Inf inputs through each direct kernel: the same per-type
    operators as the ring (float Max/Min (x < y) ? y : x, half/bf16 fmaxf),
    so the NaN positions and every other bit equal the ring's (the oracle)."""
    n, count = 3, 30011
    comms = C.init_all([0] * n, _cfg(variant))
    try:
        rng = np.random.default_rng(13 * code + op)
        inputs = []
        for _ in range(n):
            x = vnode.gen(code, count, rng)
            f = x.view(np.uint16) if code == BF16 else x
            u = rng.random(count)
            if code == BF16:
                f[u < 0.02], f[(u >= 0.02) & (u < 0.04)], f[(u >= 0.04) & (u < 0.06)] = 0x7FC0, 0x7F80, 0xFF80
            else:
                f[u < 0.02], f[(u >= 0.02) & (u < 0.04)], f[(u >= 0.04) & (u < 0.06)] = np.nan, np.inf, -np.inf
            inputs.append(x)
        outs = vnode.run_allreduce(comms, inputs, code, op)
        _algo(comms, variant, inputs[0].nbytes)
        exp = vnode.expected_allreduce(orc, inputs, code, op, comms[0])

        def isnan(a):
            if code == BF16:
                return np.isnan((a.view(np.uint16).astype(np.uint32) << 16).view(np.float32))
            return np.isnan(a.astype(np.float64))

        en = isnan(exp)
        for r, o in enumerate(outs):
            assert np.array_equal(isnan(o), en), r
            assert np.array_equal(o.view(np.uint8).reshape(count, -1)[~en], exp.view(np.uint8).reshape(count, -1)[~en]), r
    finally:
        vnode.destroy(comms)
