"""GPU parity of the ring AllReduce / AllGather path against the oracle.

Runs an n-rank virtual node on one MI355X (tests/vnode.py): the production
kernels, FIFO protocol, work list and planner, with all ranks' FIFOs in one
GPU's HBM.  Integer and exact-sum inputs are checked against arithmetic
known answers (allreduce_proto main.rs:111); fp inputs bit for bit against
the oracle's ring-order restatement (all_reduce.h summation order, per-hop
rounding in T).  Every rank's output must be identical.
"""
import numpy as np
import pytest

from mccs_amd import comm as C
import vnode

pytestmark = pytest.mark.gpu

F16, F32, BF16, I32, F64, I8 = 6, 7, 9, 2, 8, 0


def _check_all_equal(outs, exp, code):
    for r, o in enumerate(outs):
        assert np.array_equal(o.view(np.uint8), exp.view(np.uint8)), f"rank {r} differs from oracle"


@pytest.mark.parametrize("n", [2, 3, 4, 5, 6, 7, 8])
@pytest.mark.parametrize("code", [F32, F16, BF16])
def test_allreduce_matches_oracle(orc, n, code):
    comms = C.init_all([0] * n)
    try:
        rng = np.random.default_rng(n * 10 + code)
        inputs = [vnode.gen(code, 300007, rng) for _ in range(n)]
        outs = vnode.run_allreduce(comms, inputs, code, 0)
        exp = vnode.expected_allreduce(orc, inputs, code, 0, comms[0])
        _check_all_equal(outs, exp, code)
    finally:
        vnode.destroy(comms)


@pytest.mark.parametrize("doubled", [False, True])
@pytest.mark.parametrize("n", [2, 4, 8])
def test_allreduce_proto_kat(n, doubled):
    """allreduce_proto: int32 Sum, rank r holds 2042+r (scaled to 2 ring loops
    + tail); also with twice the default channels (every ring twice, as the
    bench autotune tries on distinct GPUs)."""
    nch = 2 * len(C.default_rings(n, 0)) if doubled else None
    comms = C.init_all([0] * n, C.CommConfig(channel_count=nch))
    try:
        count = 2 * comms[0].nchannels * n * (1 << 20) // 4 + 999
        inputs = [np.full(count, 2042 + r, dtype=np.int32) for r in range(n)]
        outs = vnode.run_allreduce(comms, inputs, I32, 0)
        for o in outs:
            assert np.all(o == 2042 * n + n * (n - 1) // 2)
    finally:
        vnode.destroy(comms)


@pytest.mark.parametrize("n", [2, 4, 8])
def test_allgather_proto_kat(n):
    """allgather_proto (src/mccs_examples/allgather_proto/src/main.rs:27-115):
    one buffer of n x size bytes per rank, rank r fills its own segment with
    int32 2042 + r and AllGathers IN PLACE (send = buffer + r x size); every
    rank must then hold 2042 + r in segment r (the reference checks the first
    word of each segment; here every word).  size = 1 MiB, as the example's
    --size 1."""
    import torch

    comms = C.init_all([0] * n)
    try:
        size = 1 << 20
        words = size // 4
        bufs = []
        for r in range(n):
            b = torch.zeros(n * words, dtype=torch.int32, device="cuda")
            b[r * words:(r + 1) * words] = 2042 + r
            bufs.append(b)
        with C.group():
            for r in range(n):
                C.all_gather(comms[r], bufs[r][r * words:], bufs[r], size)
        for c in comms:
            c.sync()
        want = torch.arange(n, dtype=torch.int32, device="cuda").repeat_interleave(words) + 2042
        for r in range(n):
            assert torch.equal(bufs[r], want), r
    finally:
        vnode.destroy(comms)


@pytest.mark.parametrize("n", [4, 8])
@pytest.mark.parametrize("code", [F16, F32])
def test_exact_sum_inputs(n, code):
    comms = C.init_all([0] * n)
    try:
        rng = np.random.default_rng(77)
        ks = [rng.integers(-255, 256, 200001) for _ in range(n)]
        inputs = [(k / 64.0).astype(vnode.NPDT[code]) for k in ks]
        outs = vnode.run_allreduce(comms, inputs, code, 0)
        exact = np.sum(np.stack(ks), axis=0) / 64.0
        for o in outs:
            assert np.array_equal(o.astype(np.float64), exact)
    finally:
        vnode.destroy(comms)


@pytest.mark.parametrize("op", [1, 2, 3])
@pytest.mark.parametrize("code", [F32, F16, I32])
def test_allreduce_ops(orc, op, code):
    n = 4
    comms = C.init_all([0] * n)
    try:
        rng = np.random.default_rng(op)
        inputs = [vnode.gen(code, 65537, rng) for _ in range(n)]
        outs = vnode.run_allreduce(comms, inputs, code, op)
        exp = vnode.expected_allreduce(orc, inputs, code, op, comms[0])
        _check_all_equal(outs, exp, code)
    finally:
        vnode.destroy(comms)


@pytest.mark.parametrize("n", [3, 5, 8])
@pytest.mark.parametrize("code", [F16, BF16])
def test_allreduce_prod_half_types(orc, n, code):
    """Prod in fp16 / bf16 through the ring: products of n values in [-1, 1)
    reach fp16 subnormals (below 6.1e-5) and round at every hop, so the
    per-hop rounding and subnormal handling must match the oracle bit for bit
    (the reference keeps subnormals: no fast-math, reduce_kernel.h:287-309)."""
    comms = C.init_all([0] * n)
    try:
        rng = np.random.default_rng(17 * n + code)
        inputs = [vnode.gen(code, 100003, rng) for _ in range(n)]
        outs = vnode.run_allreduce(comms, inputs, code, 1)
        exp = vnode.expected_allreduce(orc, inputs, code, 1, comms[0])
        _check_all_equal(outs, exp, code)
        if code == F16:  # the case is not vacuous
            assert np.count_nonzero(np.abs(exp.astype(np.float32)) < 6.1e-5) > 100
    finally:
        vnode.destroy(comms)


@pytest.mark.parametrize("op", [0, 1, 2, 3])
@pytest.mark.parametrize("code", [F32, F16, BF16, F64])
def test_allreduce_nan_and_inf(orc, code, op):
    """NaN and +-Inf inputs (1 % each) through the ring at n = 3: the
    reference's per-type operators decide what survives -- float / double
    Max/Min are (x < y) ? y : x, so a NaN second operand is dropped; half and
    bf16 Max/Min go through fmaxf / fminf, which drop either NaN
    (reduce_kernel.h:32-46,338-404) -- and Inf - Inf makes NaN in Sum.  The NaN
    positions must match the oracle's and every other element bit for bit
    (NaN payloads are not compared: the reference's hardware makes its own)."""
    n, count = 3, 65537
    comms = C.init_all([0] * n)
    try:
        rng = np.random.default_rng(31 * code + op)
        inputs = []
        for _ in range(n):
            x = vnode.gen(code, count, rng)
            f = x.view(np.uint16) if code == BF16 else x
            special = rng.random(count)
            if code == BF16:  # bf16 bit patterns: NaN 0x7fc0, +Inf 0x7f80, -Inf 0xff80
                f[special < 0.01] = 0x7FC0
                f[(special >= 0.01) & (special < 0.02)] = 0x7F80
                f[(special >= 0.02) & (special < 0.03)] = 0xFF80
            else:
                f[special < 0.01] = np.nan
                f[(special >= 0.01) & (special < 0.02)] = np.inf
                f[(special >= 0.02) & (special < 0.03)] = -np.inf
            inputs.append(x)
        outs = vnode.run_allreduce(comms, inputs, code, op)
        exp = vnode.expected_allreduce(orc, inputs, code, op, comms[0])

        def as_float(a):
            if code == BF16:
                return (a.view(np.uint16).astype(np.uint32) << 16).view(np.float32)
            return a.astype(np.float64)

        en = np.isnan(as_float(exp))
        assert en.any() or op in (2, 3)
        for r, o in enumerate(outs):
            on = np.isnan(as_float(o))
            assert np.array_equal(on, en), (r, np.flatnonzero(on != en)[:8])
            assert np.array_equal(o.view(np.uint8).reshape(count, -1)[~en], exp.view(np.uint8).reshape(count, -1)[~en]), r
    finally:
        vnode.destroy(comms)


@pytest.mark.parametrize("code", list(range(10)))
@pytest.mark.parametrize("op", [0, 2])
def test_allreduce_every_dtype(orc, code, op):
    """All ten mccsDevDataType_t kernels (collectives.h:177-192; the reference
    compiled them, libmccs reached two) through the ring, Sum and Max, n = 3
    (non-commutative fp order), ragged count: bit-exact vs the oracle.  Byte
    types run the 4-pack reduce-copy, 64-bit types two elements per pack."""
    n, count = 3, 250007
    comms = C.init_all([0] * n)
    try:
        rng = np.random.default_rng(code * 10 + op)
        inputs = [vnode.gen(code, count, rng) for _ in range(n)]
        outs = vnode.run_allreduce(comms, inputs, code, op)
        exp = vnode.expected_allreduce(orc, inputs, code, op, comms[0])
        _check_all_equal(outs, exp, code)
    finally:
        vnode.destroy(comms)


@pytest.mark.parametrize("count", [1, 7, 255, 256, 4097, 1 << 20, 5 * (1 << 19) // 2 + 77, (3 << 20) + 5])
def test_allreduce_sizes(orc, count):
    n = 4
    comms = C.init_all([0] * n)
    try:
        rng = np.random.default_rng(count)
        inputs = [vnode.gen(F16, count, rng) for _ in range(n)]
        outs = vnode.run_allreduce(comms, inputs, F16, 0)
        exp = vnode.expected_allreduce(orc, inputs, F16, 0, comms[0])
        _check_all_equal(outs, exp, F16)
    finally:
        vnode.destroy(comms)


def test_allreduce_in_place(orc):
    n = 8
    comms = C.init_all([0] * n)
    try:
        rng = np.random.default_rng(5)
        inputs = [vnode.gen(F32, 1 << 21, rng) for _ in range(n)]
        outs = vnode.run_allreduce(comms, inputs, F32, 0, inplace=True)
        exp = vnode.expected_allreduce(orc, inputs, F32, 0, comms[0])
        _check_all_equal(outs, exp, F32)
    finally:
        vnode.destroy(comms)


def test_repeated_calls_keep_fifo_steps(orc):
    """conn->step persists across launches (prims_simple.h:318-319,461)."""
    n = 4
    comms = C.init_all([0] * n)
    try:
        rng = np.random.default_rng(9)
        for it, count in enumerate([100003, 7, 1 << 20, 33, 250001]):
            inputs = [vnode.gen(F16, count, rng) for _ in range(n)]
            outs = vnode.run_allreduce(comms, inputs, F16, 0)
            exp = vnode.expected_allreduce(orc, inputs, F16, 0, comms[0])
            _check_all_equal(outs, exp, F16)
    finally:
        vnode.destroy(comms)


def test_group_batches_and_chains_works(orc):
    """12 allreduces in one group: >10 elements per channel forces a second
    mccsDevWork chained by workNext (plan.rs:68-90, 424-541; common.h:151-178)."""
    n = 4
    comms = C.init_all([0] * n)
    try:
        rng = np.random.default_rng(12)
        counts = [1000 + 7919 * i for i in range(12)]
        ins = [[vnode.gen(F32, cnt, rng) for _ in range(n)] for cnt in counts]
        sends = [[vnode.to_dev(x) for x in per] for per in ins]
        recvs = [[vnode.to_dev(np.zeros_like(x)) for x in per] for per in ins]
        with C.group():
            for k, cnt in enumerate(counts):
                for r in range(n):
                    C.all_reduce(comms[r], sends[k][r], recvs[k][r], cnt, F32, 0)
        for c in comms:
            c.sync()
        planner = vnode.Planner(comms[0].nchannels, comms[0].rings())
        for k, cnt in enumerate(counts):
            exp = vnode.expected_allreduce(orc, ins[k], F32, 0, comms[0], planner=planner)
            for r in range(n):
                got = vnode.from_dev(recvs[k][r], F32)
                assert np.array_equal(got.view(np.uint32), exp.view(np.uint32)), (k, r)
    finally:
        vnode.destroy(comms)


CONFIGS = [
    dict(lanes=1),
    dict(lanes=3),
    dict(lanes=8, block_threads=256),
    dict(block_threads=576),
    dict(locality=C.LOCALITY_SENDER),
    dict(locality=C.LOCALITY_SENDER, lanes=2),
    dict(fifo_memory=C.FIFO_DEVICE),
    dict(fifo_memory=C.FIFO_UNCACHED_RELEASE),  # release fence before every post
    dict(fifo_memory=C.FIFO_UNCACHED_RELEASE, locality=C.LOCALITY_SENDER, fifo_slots=8),
    dict(buffer_size=1 << 20),
    dict(channel_count=2, rings="default", block_threads=544, lanes=1),  # reference profile
    dict(channel_count=5),
    dict(channel_count=14),  # every ring twice (the bench autotune's doubled channels)
    dict(bridge_streams=1),
    # comm_patterns_override with rings that do not start at rank 0 and are
    # not rotations of each other (ring.index relative to rank 0, userRanks)
    dict(channel_count=2, rings=[[3, 0, 6, 1, 7, 2, 5, 4], [4, 5, 2, 7, 1, 6, 0, 3]]),
    dict(channel_count=3, rings=[[5, 2, 0, 7, 4, 1, 6, 3]] * 3, lanes=2),
    # deeper FIFOs (more slices in flight per lane; same chunk schedule)
    dict(fifo_slots=16),
    dict(fifo_slots=32, lanes=3, buffer_size=1 << 20),
    dict(fifo_slots=16, locality=C.LOCALITY_SENDER, fifo_memory=C.FIFO_DEVICE),
]


@pytest.mark.parametrize("cfg", CONFIGS, ids=[str(c) for c in CONFIGS])
def test_configs(orc, cfg):
    n = 8
    cfg = dict(cfg)
    if cfg.get("rings") == "default":
        cfg["rings"] = [list(range(n))] * cfg["channel_count"]
    comms = C.init_all([0] * n, C.CommConfig(**cfg))
    try:
        rng = np.random.default_rng(len(str(cfg)))
        inputs = [vnode.gen(F16, 777777, rng) for _ in range(n)]
        outs = vnode.run_allreduce(comms, inputs, F16, 0)
        exp = vnode.expected_allreduce(orc, inputs, F16, 0, comms[0], buff_size=cfg.get("buffer_size", 1 << 22))
        _check_all_equal(outs, exp, F16)
    finally:
        vnode.destroy(comms)


@pytest.mark.parametrize("lanes", [33, 64])
@pytest.mark.parametrize("count", [5000, 777777, (37 << 20) // 4 + 3])
def test_wide_lanes(orc, lanes, count):
    """Up to MCCS_MAX_LANES = 64 workgroups per channel (a 2-rank virtual node
    of 2 channels then fills every CU): each lane owns a fixed 256-byte-aligned
    region of a slot group, 32 KiB at 64 lanes; bit-exact, multi-loop sizes
    included."""
    n = 2
    comms = C.init_all([0] * n, C.CommConfig(lanes=lanes, channel_count=2))
    try:
        rng = np.random.default_rng(lanes + count)
        inputs = [vnode.gen(F32, count, rng) for _ in range(n)]
        outs = vnode.run_allreduce(comms, inputs, F32, 0)
        exp = vnode.expected_allreduce(orc, inputs, F32, 0, comms[0])
        _check_all_equal(outs, exp, F32)
    finally:
        vnode.destroy(comms)


def test_single_rank_is_copy():
    import torch

    (c,) = C.init_all([0])
    try:
        x = torch.arange(1000, dtype=torch.float32, device="cuda")
        y = torch.zeros_like(x)
        C.all_reduce(c, x, y, 1000, C.AllReduceDataType.Float32)
        c.sync()
        assert torch.equal(x, y)
    finally:
        vnode.destroy([c])


@pytest.mark.parametrize("n", [2, 4, 8])
@pytest.mark.parametrize("nbytes", [1, 1000, 1 << 20, (5 << 20) + 3])
def test_allgather(orc, n, nbytes):
    comms = C.init_all([0] * n)
    try:
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
        for r in range(n):
            assert np.array_equal(recv[r].cpu().numpy(), exp), r
    finally:
        vnode.destroy(comms)


@pytest.mark.parametrize("cfg", [dict(channel_count=2, rings=[[3, 0, 6, 1, 7, 2, 5, 4], [4, 5, 2, 7, 1, 6, 0, 3]]),
                                 dict(locality=C.LOCALITY_SENDER, lanes=3), dict(lanes=1, block_threads=544)])
def test_allgather_configs(orc, cfg):
    """AllGather (all_gather.h:7-79) under ring overrides (userRanks decide
    every destination offset), sender-side FIFOs and the reference block."""
    n, nbytes = 8, (3 << 20) + 11
    comms = C.init_all([0] * n, C.CommConfig(**cfg))
    try:
        rng = np.random.default_rng(nbytes + len(str(cfg)))
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
            assert np.array_equal(recv[r].cpu().numpy(), exp), r
    finally:
        vnode.destroy(comms)


def test_fused_launch_beyond_residency_fails_loudly():
    """Explicit lanes whose fused vnode launch cannot be co-resident would
    deadlock (every block spins on a peer's flag): refused, not hung."""
    comms = C.init_all([0] * 8, C.CommConfig(lanes=16, block_threads=576))
    try:
        import torch

        x = torch.zeros(1 << 20, device="cuda")
        with pytest.raises(C.MccsError if hasattr(C, "MccsError") else Exception):
            with C.group():
                for c in comms:
                    C.all_reduce(c, x, x, 1 << 20, C.AllReduceDataType.Float32)
    finally:
        vnode.destroy(comms)


def test_bad_usage_fails_loudly():
    comms = C.init_all([0, 0])
    try:
        import torch

        x = torch.zeros(16, device="cuda")
        with pytest.raises(Exception):
            C.all_reduce(comms[0], x, x, 16, 42)  # bad dtype
        with pytest.raises(Exception):
            with C.group():
                C.all_reduce(comms[0], x, x, 16, C.AllReduceDataType.Float32)
                C.all_reduce(comms[0], x, x, 16, C.AllReduceDataType.Float16)  # mixed plan
    finally:
        vnode.destroy(comms)


@pytest.mark.parametrize("code,mib", [(F32, 128), (F16, 1024)], ids=["configs2-fp32-128MiB", "configs3-fp16-1GiB"])
def test_baseline_sizes_exact(code, mib):
    """BASELINE configs[2]/[3] bucket sizes on an 8-rank virtual node through a
    size-independent property: k/64 inputs (|k| <= 255) sum exactly in fp16 and
    fp32 for 8 ranks, so every rank must hold the integer sum / 64 bit for bit
    (the order-independent golden vectors of nccl-tests verifiable.cu:419-520)."""
    import torch

    n = 8
    tdt = {F32: torch.float32, F16: torch.float16}[code]
    count = (mib << 20) // (4 if code == F32 else 2)
    comms = C.init_all([0] * n)
    try:
        i = torch.arange(count, device="cuda", dtype=torch.int64)
        tot = torch.zeros(count, device="cuda", dtype=torch.int64)
        send = []
        for r in range(n):
            k = ((i * 7 + r * 13) % 511) - 255
            tot += k
            send.append((k.to(torch.float32) / 64.0).to(tdt))
            del k
        exp = (tot.to(torch.float64) / 64.0).to(tdt)
        del tot, i
        recv = [torch.empty_like(x) for x in send]
        with C.group():
            for r in range(n):
                C.all_reduce(comms[r], send[r], recv[r], count, code, 0)
        for c in comms:
            c.sync()
        for r in range(n):
            assert torch.equal(recv[r], exp), f"rank {r}"
    finally:
        vnode.destroy(comms)


def test_reference_slicing_matches_oracle(orc, monkeypatch):
    """MCCS_SLICE_STEPS=2: the reference's two 2-step slices per chunk
    (prims_simple.h SliceSteps) instead of the default one 4-step slice; the
    FIFO then holds 4 slices in flight.  Elementwise results cannot depend on
    slicing: still bit-exact."""
    monkeypatch.setenv("MCCS_SLICE_STEPS", "2")
    n = 4
    comms = C.init_all([0] * n)
    try:
        rng = np.random.default_rng(44)
        for count in (7, 300007, (3 << 20) + 5):
            inputs = [vnode.gen(F16, count, rng) for _ in range(n)]
            outs = vnode.run_allreduce(comms, inputs, F16, 0)
            exp = vnode.expected_allreduce(orc, inputs, F16, 0, comms[0])
            _check_all_equal(outs, exp, F16)
    finally:
        vnode.destroy(comms)
        monkeypatch.delenv("MCCS_SLICE_STEPS")
        C.init_all([0])[0].destroy()  # re-arm the device config with the default slicing


@pytest.mark.parametrize("block", [96, 160, 544])
def test_partial_wave_blocks(orc, block):
    """Blocks that are not whole 64-lane waves (the reference's nWarps*32
    sizes: 96 and 544 threads) on slices spanning several row iterations."""
    n = 4
    comms = C.init_all([0] * n, C.CommConfig(block_threads=block, lanes=2))
    try:
        rng = np.random.default_rng(block)
        inputs = [vnode.gen(F32, (3 << 20) + 5, rng) for _ in range(n)]
        outs = vnode.run_allreduce(comms, inputs, F32, 0)
        exp = vnode.expected_allreduce(orc, inputs, F32, 0, comms[0])
        _check_all_equal(outs, exp, F32)
    finally:
        vnode.destroy(comms)


def test_ring_profile_counters(monkeypatch):
    """MCCS_RING_PROFILE=1 arms the per-slice counters read by mccs_ring_profile."""
    monkeypatch.setenv("MCCS_RING_PROFILE", "1")
    comms = C.init_all([0] * 2)
    try:
        C.ring_profile(0, reset=True)
        inputs = [np.ones(1 << 20, np.float32) for _ in range(2)]
        outs = vnode.run_allreduce(comms, inputs, F32, 0)
        assert all(np.all(o == 2.0) for o in outs)
        p = C.ring_profile(0, reset=True)
        assert p["slices"] > 0 and p["work_us"] > 0, p
        assert C.ring_profile(0)["slices"] == 0
    finally:
        vnode.destroy(comms)
        monkeypatch.delenv("MCCS_RING_PROFILE")
        C.init_all([0])[0].destroy()  # disarm


@pytest.mark.parametrize("n,count,bridge,fifo", [(2, 1 << 20, None, False), (2, 1 << 20, None, True),
                                                 (4, 300007, None, False), (2, 77777, 1, False)])
def test_allreduce_captured_in_hip_graph(orc, n, count, bridge, fifo, monkeypatch):
    """AllReduces captured into a HIP graph (torch.cuda.graph) replay with the
    inputs of each replay, interleaved with eager calls on the same comms:
    captured work lists live outside the rolling work FIFO (in the launch
    arguments, or -- fifo=True -- in the graph arena), and the FIFO steps
    persisted in device memory keep eager and replayed launches in
    lock-step."""
    import torch

    if fifo:
        monkeypatch.setenv("MCCS_INLINE_WORKS", "0")

    # bridge=1: launches go to the comm's own stream, joined to the capturing
    # stream by events (libmccs two-stream bridge)
    comms = C.init_all([0] * n, C.CommConfig(bridge_streams=bridge))
    try:
        rng = np.random.default_rng(n * 7 + 1)
        send = [torch.empty(count, dtype=torch.float16, device="cuda") for _ in range(n)]
        recv = [torch.empty_like(x) for x in send]
        s = torch.cuda.Stream()
        # warm-up outside capture (first launch loads the code object)
        with C.group():
            for r in range(n):
                C.all_reduce(comms[r], send[r], recv[r], count, F16, 0, stream=s)
        s.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            for _ in range(2):  # two collectives in one graph
                with C.group():
                    for r in range(n):
                        C.all_reduce(comms[r], send[r], recv[r], count, F16, 0, stream=s)
        for it in range(3):
            inputs = [vnode.gen(F16, count, rng) for _ in range(n)]
            for r in range(n):
                send[r].copy_(torch.from_numpy(inputs[r]).cuda())
            torch.cuda.synchronize()
            if it == 1:  # an eager call between replays advances the same FIFOs
                with C.group():
                    for r in range(n):
                        C.all_reduce(comms[r], send[r], recv[r], count, F16, 0, stream=s)
                s.synchronize()
            g.replay()
            torch.cuda.synchronize()
            for c in comms:
                c.sync()
            exp = vnode.expected_allreduce(orc, inputs, F16, 0, comms[0])
            _check_all_equal([recv[r].cpu().numpy() for r in range(n)], exp, F16)
    finally:
        torch.cuda.synchronize()
        vnode.destroy(comms)


def test_graph_recapture_reuses_the_work_arena(orc, monkeypatch):
    """A server that captures graphs again and again: 150 captures of a group
    of 40 int32 AllReduces (4 chained works on each of 4 channels per rank:
    2,400 arena entries in all, more than the arena's 2048), each graph
    destroyed after use, so its entries return (a HIP user object the graph
    retains).  A graph captured first and kept keeps its entries through all
    of them: torch destroys the captured graph right after instantiation, so
    this also checks that the executable graph holds the user object."""
    import gc

    import torch

    monkeypatch.setenv("MCCS_INLINE_WORKS", "0")  # every captured launch takes arena entries
    n = 2
    comms = C.init_all([0] * n, C.CommConfig(buffer_size=1 << 20, timeout_ms=10000))
    try:
        rng = np.random.default_rng(5)
        s = torch.cuda.Stream()
        count = 1 << 18  # fp16 for the kept graph
        kept_send = [torch.empty(count, dtype=torch.float16, device="cuda") for _ in range(n)]
        kept_recv = [torch.empty_like(x) for x in kept_send]
        with C.group():  # warm-up outside capture
            for r in range(n):
                C.all_reduce(comms[r], kept_send[r], kept_recv[r], count, F16, 0, stream=s)
        s.synchronize()

        def replay_kept():
            inputs = [vnode.gen(F16, count, rng) for _ in range(n)]
            for r in range(n):
                kept_send[r].copy_(torch.from_numpy(inputs[r]).cuda())
            torch.cuda.synchronize()
            kept.replay()
            torch.cuda.synchronize()
            exp = vnode.expected_allreduce(orc, inputs, F16, 0, comms[0], buff_size=1 << 20)
            _check_all_equal([kept_recv[r].cpu().numpy() for r in range(n)], exp, F16)

        kept = torch.cuda.CUDAGraph()
        with torch.cuda.graph(kept, stream=s):
            with C.group():
                for r in range(n):
                    C.all_reduce(comms[r], kept_send[r], kept_recv[r], count, F16, 0, stream=s)
        replay_kept()
        # the throwaway graphs: 40 int32 AllReduces of 4 MiB per rank in one group
        m, icount = 40, 1 << 20
        assert C.task_schema(icount * 4, comms[0].nchannels)[0] == comms[0].nchannels == 4
        isend = [torch.full((icount,), 2042 + r, dtype=torch.int32, device="cuda") for r in range(n)]
        irecv = [[torch.empty(icount, dtype=torch.int32, device="cuda") for _ in range(m)] for _ in range(n)]
        for i in range(150):  # 150 x 4 channels x ceil(40 / 10) works = 2,400 entries per rank
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=s):
                with C.group():
                    for k in range(m):
                        for r in range(n):
                            C.all_reduce(comms[r], isend[r], irecv[r][k], icount, I32, 0, stream=s)
            if i % 50 == 49:
                for r in range(n):
                    for k in range(m):
                        irecv[r][k].zero_()
                g.replay()
                torch.cuda.synchronize()
                assert all(bool((irecv[r][k] == 2042 * 2 + 1).all()) for r in range(n) for k in range(m)), i
            del g
            gc.collect()
        torch.cuda.synchronize()
        replay_kept()
        del kept
    finally:
        torch.cuda.synchronize()
        vnode.destroy(comms)


@pytest.mark.parametrize("n", [2, 4])
@pytest.mark.parametrize("rep", range(3))
def test_one_comm_on_two_streams_runs_in_issue_order(orc, n, rep):
    """A large AllReduce on one stream, then a small one on another, same
    communicators, no sync between: the second must wait for the first (the
    reference runs a communicator's kernels on its one private stream,
    proxy/init.rs:166-175).  Launched concurrently they shared FIFO flags and
    saved steps and returned wrong sums in 2 of 6 of these cases at n = 4."""
    import torch

    comms = C.init_all([0] * n, C.CommConfig(timeout_ms=5000, lanes=1, channel_count=1))
    try:
        rng = np.random.default_rng(3 + rep)
        s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
        cnt_a, cnt_b = 16 << 20, 1 << 18
        xa = [vnode.gen(F32, cnt_a, rng) for _ in range(n)]
        xb = [vnode.gen(F32, cnt_b, rng) for _ in range(n)]
        sa, sb = [vnode.to_dev(x) for x in xa], [vnode.to_dev(x) for x in xb]
        ra, rb = [torch.zeros_like(t) for t in sa], [torch.zeros_like(t) for t in sb]
        torch.cuda.synchronize()
        for stream, cnt, snd, rcv in ((s1, cnt_a, sa, ra), (s2, cnt_b, sb, rb)):
            with C.group():
                for r in range(n):
                    C.all_reduce(comms[r], snd[r], rcv[r], cnt, F32, 0, stream=stream)
        torch.cuda.synchronize()
        for c in comms:
            c.sync()
        ea = vnode.expected_allreduce(orc, xa, F32, 0, comms[0])
        eb = vnode.expected_allreduce(orc, xb, F32, 0, comms[0])
        _check_all_equal([ra[r].cpu().numpy() for r in range(n)], ea, F32)
        _check_all_equal([rb[r].cpu().numpy() for r in range(n)], eb, F32)
    finally:
        torch.cuda.synchronize()
        vnode.destroy(comms)


@pytest.mark.parametrize("code,off", [(F16, 2), (F32, 4), (F32, 12), (BF16, 6)])
def test_allreduce_misaligned_buffers(orc, code, off):
    """User buffers that are not 16-byte aligned take the typed element path
    of the reduce-copy (common_kernel.h:485-550 ReduceCopyMulti) in every
    primitive; results stay bit-identical to the oracle."""
    import torch

    n, count = 3, 100003
    comms = C.init_all([0] * n)
    try:
        rng = np.random.default_rng(off * 10 + code)
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
        outs = [rbuf[r][off:off + nbytes].cpu().numpy().view(inputs[0].dtype) for r in range(n)]
        exp = vnode.expected_allreduce(orc, inputs, code, 0, comms[0])
        _check_all_equal(outs, exp, code)
    finally:
        vnode.destroy(comms)


def test_allreduce_zero_count_is_noop():
    import torch

    comms = C.init_all([0, 0])
    try:
        x = torch.ones(4, device="cuda")
        with C.group():
            for c in comms:
                C.all_reduce(c, x, x, 0, F32, 0)
        for c in comms:
            c.sync()
        assert torch.equal(x, torch.ones(4, device="cuda"))
    finally:
        vnode.destroy(comms)


@pytest.mark.parametrize("depth", [8, 16])
def test_work_fifo_wraps_and_flow_controls(orc, depth, monkeypatch):
    """A tiny work FIFO (plan.rs:380-541: rolling work_queue indices, restart
    at slot 0 on wrap, wait_work_queue on workFifoDone acks) over many calls:
    every call's work list wraps the ring several times and the host must
    wait for the kernel's acks before reusing slots.  (Works that fit the
    launch arguments skip the FIFO: forced off here.)"""
    import torch

    monkeypatch.setenv("MCCS_INLINE_WORKS", "0")
    n = 2
    comms = C.init_all([0] * n, C.CommConfig(work_fifo_depth=depth))
    try:
        rng = np.random.default_rng(depth)
        counts = [1 << 16, 333, (1 << 18) + 7, 5]
        outs_dev, exps = [], []
        for it in range(40):  # ~40 calls x 2 channels >> depth: many wraps, issued back to back
            count = counts[it % len(counts)]
            inputs = [vnode.gen(F32, count, rng) for _ in range(n)]
            send = [vnode.to_dev(x) for x in inputs]
            recv = [vnode.to_dev(np.zeros_like(x)) for x in inputs]
            with C.group():
                for r in range(n):
                    C.all_reduce(comms[r], send[r], recv[r], count, F32, 0)
            outs_dev.append((send, recv))
            exps.append(vnode.expected_allreduce(orc, inputs, F32, 0, comms[0]))
        for c in comms:
            c.sync()
        torch.cuda.synchronize()
        for (send, recv), exp in zip(outs_dev, exps):
            _check_all_equal([vnode.from_dev(recv[r], F32) for r in range(n)], exp, F32)
    finally:
        vnode.destroy(comms)


def test_allreduce_beyond_2pow31_elements():
    """Maximum-size edge: an int8 AllReduce of 2^31 + 5 elements per rank
    (64-bit offsets through the chunk schedule, the work element's count and
    the lane split), checked against a wrapping int8 sum on the device."""
    import torch

    n, count = 2, (1 << 31) + 5
    comms = C.init_all([0] * n)
    try:
        g = torch.Generator(device="cuda")
        xs = []
        for r in range(n):
            g.manual_seed(100 + r)
            xs.append(torch.randint(-8, 8, (count,), dtype=torch.int8, device="cuda", generator=g))
        ys = [torch.empty_like(x) for x in xs]
        with C.group():
            for r in range(n):
                C.all_reduce(comms[r], xs[r], ys[r], count, I8, 0)
        for c in comms:
            c.sync()
        exp = xs[0] + xs[1]
        for r in range(n):
            assert torch.equal(ys[r], exp), r
            assert ys[r][-5:].tolist() == exp[-5:].tolist()
    finally:
        vnode.destroy(comms)


def test_allgather_output_beyond_2pow31_bytes():
    """AllGather whose gathered output passes 2^31 bytes (destination offsets
    rank * sendbytes in 64 bits, all_gather.h:29-79)."""
    import torch

    n, nb = 2, (3 << 29) + 3
    comms = C.init_all([0] * n)
    try:
        g = torch.Generator(device="cuda")
        xs = []
        for r in range(n):
            g.manual_seed(200 + r)
            xs.append(torch.randint(0, 256, (nb,), dtype=torch.uint8, device="cuda", generator=g))
        ys = [torch.empty(n * nb, dtype=torch.uint8, device="cuda") for _ in range(n)]
        with C.group():
            for r in range(n):
                C.all_gather(comms[r], xs[r], ys[r], nb)
        for c in comms:
            c.sync()
        for r in range(n):
            for s in range(n):
                assert torch.equal(ys[r][s * nb:(s + 1) * nb], xs[s]), (r, s)
    finally:
        vnode.destroy(comms)


def test_allgather_captured_in_hip_graph(orc):
    """AllGather recorded into a HIP graph, replayed with new inputs."""
    import torch

    n, nbytes = 4, (1 << 20) + 9
    comms = C.init_all([0] * n)
    try:
        rng = np.random.default_rng(77)
        send = [torch.zeros(nbytes, dtype=torch.uint8, device="cuda") for _ in range(n)]
        recv = [torch.zeros(n * nbytes, dtype=torch.uint8, device="cuda") for _ in range(n)]
        s = torch.cuda.Stream()
        with C.group():
            for r in range(n):
                C.all_gather(comms[r], send[r], recv[r], nbytes, stream=s)
        s.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            with C.group():
                for r in range(n):
                    C.all_gather(comms[r], send[r], recv[r], nbytes, stream=s)
        for _ in range(2):
            inputs = [rng.integers(0, 256, nbytes, dtype=np.uint8) for _ in range(n)]
            for r in range(n):
                send[r].copy_(torch.from_numpy(inputs[r]).cuda())
            torch.cuda.synchronize()
            g.replay()
            torch.cuda.synchronize()
            exp = orc.ring_allgather(inputs)
            for r in range(n):
                assert np.array_equal(recv[r].cpu().numpy(), exp), r
    finally:
        torch.cuda.synchronize()
        vnode.destroy(comms)


def test_zero_count_collectives_are_noops_and_keep_fifo_steps(orc):
    """count = 0 (an empty bucket): mccsAllReduce / mccsAllGather return
    success without launching, inside and outside a group; the FIFO steps are
    untouched, so the next AllReduce on the same communicators is still
    bit-exact (n = 8, fewer elements than ranks next)."""
    import torch

    n = 8
    comms = C.init_all([0] * n)
    try:
        x = [torch.ones(4, device="cuda") for _ in range(n)]
        y = [torch.full((4,), 7.0, device="cuda") for _ in range(n)]
        with C.group():
            for r in range(n):
                C.all_reduce(comms[r], x[r], y[r], 0, F32, 0)
        for r in range(n):
            C.all_gather(comms[r], x[r], y[r], 0)  # outside a group: nothing to launch either
        for c in comms:
            c.sync()
        assert all(bool(torch.all(t == 7.0)) for t in y)
        rng = np.random.default_rng(3)
        for count in (3, 100003):
            inputs = [vnode.gen(F32, count, rng) for _ in range(n)]
            outs = vnode.run_allreduce(comms, inputs, F32, 0)
            exp = vnode.expected_allreduce(orc, inputs, F32, 0, comms[0])
            _check_all_equal(outs, exp, F32)
    finally:
        vnode.destroy(comms)
