"""CPU tests: pin the C oracle (oracle/mccs_oracle.c) before trusting it.

Pins, in order of strength:
  * reference known-answer tests allreduce_proto (src/mccs_examples/
    allreduce_proto/src/main.rs:27,75-116): int32 Sum, rank r holds 2042+r,
    every element == 2042*n + n(n-1)/2; and allgather_proto
    (allgather_proto/src/main.rs:27-115): segment r == 2042 + r;
  * exact-sum fp inputs (values k/64, |k| <= 255) whose sum is exact in any
    order, checked against the float64 sum (nccl-tests verifiable design,
    nccl-tests-mccs/verifiable/verifiable.cu:419-520);
  * IEEE conversions / element ops against numpy and torch CPU;
  * the ring walk against an independent per-rank FIFO simulation
    (tests/ring_sim.py) for fp16/fp32/int32, several n, channel counts,
    thread counts and ring overrides;
  * committed golden fixtures (tests/golden/ring_golden.npz).
"""
import os

import numpy as np
import pytest

import ring_sim  # noqa: E402  (tests/ on sys.path via rootdir conftest)

F16, F32, F64, BF16, I32, I8, U8, I64 = 6, 7, 8, 9, 2, 0, 1, 4
GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def test_half_to_float_exhaustive(orc):
    L = orc.lib()
    bits = np.arange(65536, dtype=np.uint16)
    ref = bits.view(np.float16).astype(np.float32)
    got = np.array([L.oracle_half_to_float(int(b)) for b in bits], dtype=np.float32)
    finite = np.isfinite(ref)
    assert np.array_equal(got[finite].view(np.uint32), ref[finite].view(np.uint32))
    assert np.array_equal(np.isnan(got), np.isnan(ref))


def test_float_to_half_matches_numpy(orc):
    L = orc.lib()
    rng = np.random.default_rng(1)
    vals = np.concatenate([
        rng.standard_normal(20000).astype(np.float32) * 1000,
        rng.standard_normal(5000).astype(np.float32) * 1e-5,  # subnormal range
        np.array([65504, 65519.99, 65520, 65536, -65520, 6.1e-5, 5.96e-8, 2.98e-8, 2.99e-8, 0.0, -0.0,
                  np.inf, -np.inf], dtype=np.float32),
        # exact ties between two halves
        (np.arange(1, 2000, dtype=np.float32) + 0.5) * np.float32(2.0 ** -10),
    ])
    ref = vals.astype(np.float16).view(np.uint16)
    got = np.array([L.oracle_float_to_half(float(v)) for v in vals], dtype=np.uint16)
    assert np.array_equal(got, ref)


def test_float_to_bf16_matches_torch(orc):
    torch = pytest.importorskip("torch")
    L = orc.lib()
    rng = np.random.default_rng(2)
    vals = np.concatenate([rng.standard_normal(20000).astype(np.float32) * 100,
                           np.array([0.0, -0.0, 3.0e38, -3.4e38, 1e-40], dtype=np.float32)])
    ref = torch.from_numpy(vals).to(torch.bfloat16).view(torch.int16).numpy().view(np.uint16)
    got = np.array([L.oracle_float_to_bf16(float(v)) for v in vals], dtype=np.uint16)
    assert np.array_equal(got, ref)


@pytest.mark.parametrize("dtype,npdt", [(F16, np.float16), (F32, np.float32), (F64, np.float64)])
@pytest.mark.parametrize("op", [0, 1, 2, 3])
def test_apply_fp_matches_numpy(orc, dtype, npdt, op):
    rng = np.random.default_rng(3 + op)
    x = (rng.standard_normal(4099) * 50).astype(npdt)
    y = (rng.standard_normal(4099) * 50).astype(npdt)
    got = orc.apply(dtype, op, x, y)
    with np.errstate(over="ignore"):
        ref = [x + y, x * y, np.where(x < y, y, x), np.where(x < y, x, y)][op].astype(npdt)
    assert np.array_equal(got.view(np.uint8), ref.view(np.uint8))


def test_apply_bf16_matches_torch(orc):
    torch = pytest.importorskip("torch")
    rng = np.random.default_rng(4)
    x = torch.from_numpy(rng.standard_normal(5000).astype(np.float32)).to(torch.bfloat16)
    y = torch.from_numpy(rng.standard_normal(5000).astype(np.float32)).to(torch.bfloat16)
    xb = x.view(torch.int16).numpy().view(np.uint16)
    yb = y.view(torch.int16).numpy().view(np.uint16)
    for op, ref in ((0, x + y), (1, x * y), (2, torch.maximum(x, y)), (3, torch.minimum(x, y))):
        got = orc.apply(BF16, op, xb, yb)
        assert np.array_equal(got, ref.view(torch.int16).numpy().view(np.uint16)), op


@pytest.mark.parametrize("dtype,npdt", [(I8, np.int8), (U8, np.uint8), (I32, np.int32), (I64, np.int64)])
def test_apply_int_wraps(orc, dtype, npdt):
    info = np.iinfo(npdt)
    rng = np.random.default_rng(5)
    x = rng.integers(info.min, info.max, 3001, dtype=npdt, endpoint=True)
    y = rng.integers(info.min, info.max, 3001, dtype=npdt, endpoint=True)
    with np.errstate(over="ignore"):
        assert np.array_equal(orc.apply(dtype, 0, x, y), (x + y).astype(npdt))
        assert np.array_equal(orc.apply(dtype, 1, x, y), (x * y).astype(npdt))
    assert np.array_equal(orc.apply(dtype, 2, x, y), np.maximum(x, y))
    assert np.array_equal(orc.apply(dtype, 3, x, y), np.minimum(x, y))


def test_reduce_copy_order(orc):
    # vals = src0; vals = fn(vals, src_i): fp16 association is left to right
    a = np.array([1.0, 2048.0], dtype=np.float16)
    b = np.array([2048.0, 1.0], dtype=np.float16)
    c = np.array([-2048.0, -2048.0], dtype=np.float16)
    (out,) = orc.reduce_copy(F16, 0, [a, b, c])
    ref = ((a + b) + c).astype(np.float16)
    assert np.array_equal(out, ref)
    assert out[0] == 0.0  # (1 + 2048) rounds to 2048 in fp16 before the subtraction


def _schema_py(total_bytes, nch):
    nthr = 512
    while total_bytes < nch * nthr * 64:
        if nch >= 2:
            nch -= 1
        elif nthr % 128 == 0:
            nthr //= 2
        else:
            break
    nthr += 32
    return nch, max(nthr, 96)


@pytest.mark.parametrize("nbytes", [0, 1024, 4096, 16384, 65536, 1 << 17, 1 << 20, 128 << 20, 1 << 30])
@pytest.mark.parametrize("nch", [1, 2, 4, 32])
def test_task_schema(orc, nbytes, nch):
    assert orc.task_schema(nbytes, nch) == _schema_py(nbytes, nch)


def test_task_schema_known_points(orc):
    # 1 KiB -> (1 ch, 96 thr); 128 MiB -> (2 ch, 544 thr)
    assert orc.task_schema(1024, 2) == (1, 96)
    assert orc.task_schema(128 << 20, 2) == (2, 544)
    assert orc.task_schema(1 << 30, 2) == (2, 544)


@pytest.mark.parametrize("n", [2, 3, 4, 8])
def test_allreduce_proto_kat(orc, n):
    # allreduce_proto: buffer = 128 MiB * n bytes of int32; scaled down here to
    # 3 ring loops worth of elements plus a ragged tail (same arithmetic)
    count = 3 * 2 * n * (1 << 20) // 4 + 12345
    inputs = [np.full(count, 2042 + r, dtype=np.int32) for r in range(n)]
    out = orc.ring_allreduce(I32, 0, inputs, nchannels=2, nthreads=544)
    assert np.all(out == 2042 * n + n * (n - 1) // 2)


@pytest.mark.parametrize("n", [2, 3, 8])
def test_allgather_proto_kat(orc, n):
    # allgather_proto (src/mccs_examples/allgather_proto/src/main.rs:27-115):
    # rank r contributes a segment of int32 2042 + r; after the AllGather
    # segment r holds 2042 + r on every rank (1 MiB segments, --size 1)
    words = (1 << 20) // 4
    inputs = [np.full(words, 2042 + r, dtype=np.int32) for r in range(n)]
    out = orc.ring_allgather(inputs).view(np.int32)
    assert np.array_equal(out, np.repeat(np.arange(n, dtype=np.int32) + 2042, words))


@pytest.mark.parametrize("n", [2, 4, 8])
@pytest.mark.parametrize("dtype,npdt", [(F16, np.float16), (F32, np.float32)])
def test_exact_sum_inputs(orc, n, dtype, npdt):
    rng = np.random.default_rng(n)
    count = 70001
    ks = [rng.integers(-255, 256, count) for _ in range(n)]
    inputs = [(k / 64.0).astype(npdt) for k in ks]
    out = orc.ring_allreduce(dtype, 0, inputs, nchannels=2, nthreads=544)
    exact = (np.sum(np.stack(ks), axis=0) / 64.0)
    assert np.array_equal(out.astype(np.float64), exact)


CASES = [
    # n, dtype, count, nch, nthreads, ring
    (2, F32, 256, 1, 96, None),              # the 1 KiB loopback config
    (2, F16, 1000, 1, 96, None),
    (3, F16, 70001, 2, 544, None),
    (4, F16, 5 * (1 << 19) // 2 + 77, 2, 544, None),   # ~2.5 chunks per rank
    (4, F32, 1 << 18, 2, 544, [[0, 2, 1, 3], [3, 1, 2, 0]]),
    (8, F16, 600000, 2, 544, None),
    (8, F32, 123457, 1, 288, [7, 0, 3, 5, 1, 2, 6, 4]),
    (5, I32, 99991, 2, 160, None),
]


@pytest.mark.parametrize("n,dtype,count,nch,nthr,ring", CASES)
def test_ring_oracle_matches_fifo_simulation(orc, n, dtype, count, nch, nthr, ring):
    npdt = orc.NP_DTYPE[dtype]
    rng = np.random.default_rng(count)
    if dtype == I32:
        inputs = [rng.integers(-1 << 20, 1 << 20, count).astype(npdt) for _ in range(n)]
    else:
        inputs = [(rng.random(count, dtype=np.float32) * 2 - 1).astype(npdt) for _ in range(n)]
    got = orc.ring_allreduce(dtype, 0, inputs, nchannels=nch, nthreads=nthr, ring_orders=(
        None if ring is None else (ring if isinstance(ring[0], list) else [ring] * nch)))
    sims = ring_sim.simulate(inputs, "sum", nch, nthr, ring=ring)
    for r in range(n):
        assert np.array_equal(sims[r].view(np.uint8), got.view(np.uint8)), f"rank {r}"


MT_CASES = [
    # (n, dtype, count, nch, nthr, buff, rings): multi-loop walks with a partial
    # last loop (its own realChunkSize), ring overrides, doubled channels
    (8, F32, 7 * 8 * (1 << 17) + 12345, 7, 544, 1 << 20, "default7"),
    (8, F16, 2 * 8 * (1 << 18) * 3 + 999, 2, 544, 1 << 20, None),
    (8, F32, 14 * 8 * (1 << 15) + 77, 14, 544, 1 << 18, "default14"),
    (5, BF16, 300007, 3, 288, 1 << 19, [[4, 1, 0, 3, 2]] * 3),
    (4, I32, 99991, 2, 160, 1 << 20, None),
]


@pytest.mark.parametrize("n,dtype,count,nch,nthr,buff,rings", MT_CASES)
def test_chunk_parallel_oracle_equals_serial(orc, n, dtype, count, nch, nthr, buff, rings):
    """oracle_ring_allreduce_mt (the BASELINE-size checker) evaluates the same
    walk chunk-parallel: identical bytes to the serial restatement."""
    from mccs_amd import comm as C

    if isinstance(rings, str):
        base = C.default_rings(n, 0)
        rings = (base * 2)[:nch]
    npdt = orc.NP_DTYPE[dtype]
    rng = np.random.default_rng(count)
    if dtype == I32:
        inputs = [rng.integers(-1 << 20, 1 << 20, count).astype(npdt) for _ in range(n)]
    elif dtype == BF16:
        inputs = [((rng.random(count, dtype=np.float32) * 2 - 1).view(np.uint32) >> 16).astype(np.uint16)
                  for _ in range(n)]
    else:
        inputs = [(rng.random(count, dtype=np.float32) * 2 - 1).astype(npdt) for _ in range(n)]
    want = orc.ring_allreduce(dtype, 0, inputs, nchannels=nch, nthreads=nthr, buff_size=buff, ring_orders=rings)
    for workers in (1, 7):
        got = orc.ring_allreduce_mt(dtype, 0, inputs, nchannels=nch, nthreads=nthr, buff_size=buff,
                                    ring_orders=rings, workers=workers)
        assert np.array_equal(got.view(np.uint8), want.view(np.uint8)), workers


def test_ring_order_matters_for_fp16(orc):
    """Sanity: the per-hop fp16 rounding is visible (a plain sum would differ)."""
    n = 8
    rng = np.random.default_rng(11)
    inputs = [(rng.random(1 << 16, dtype=np.float32) * 2 - 1).astype(np.float16) for _ in range(n)]
    out = orc.ring_allreduce(F16, 0, inputs, nchannels=2, nthreads=544)
    naive = np.zeros(1 << 16, dtype=np.float16)
    for x in inputs:
        naive = (naive + x).astype(np.float16)
    assert not np.array_equal(out, naive)
    exact = np.sum(np.stack([x.astype(np.float64) for x in inputs]), axis=0)
    # nccl-tests tolerance for fp16, n = 8: 1 + floor(0.75 * 8**0.91) = 5 ulp steps
    # (bit distance is only meaningful away from cancellation)
    big = np.abs(exact) >= 1.0
    dist = np.abs(out.view(np.int16).astype(np.int64) - exact.astype(np.float16).view(np.int16).astype(np.int64))
    assert dist[big].max() <= 5


def test_chunk_owner_map(orc):
    # 1 KiB fp32, n = 2, 1 channel, 96 threads: chunk0 = [0,128) owned by rank 0,
    # chunk1 = [128,256) owned by rank 1
    inputs = [np.zeros(256, np.float32), np.zeros(256, np.float32)]
    _, owner = orc.ring_allreduce(F32, 0, inputs, nchannels=1, nthreads=96, want_owner=True)
    assert np.all(owner[:128] == 0) and np.all(owner[128:] == 1)


def test_golden_ring_fixtures(orc):
    path = os.path.join(GOLDEN, "ring_golden.npz")
    z = np.load(path, allow_pickle=False)
    names = sorted({k.split("__")[0] for k in z.files})
    assert names, "empty fixture file"
    for name in names:
        meta = z[name + "__meta"]
        n, dtype, nch, nthr, op = (int(v) for v in meta[:5])
        inputs = [z[f"{name}__in{r}"] for r in range(n)]
        got = orc.ring_allreduce(dtype, op, inputs, nchannels=nch, nthreads=nthr)
        assert np.array_equal(got.view(np.uint8), z[name + "__out"].view(np.uint8)), name


def _as_f64(a, code):
    if code == 9:
        return (a.astype(np.uint32) << 16).view(np.float32).astype(np.float64)
    return a.astype(np.float64)


@pytest.mark.parametrize("code", [6, 7, 8, 9])
@pytest.mark.parametrize("same_sign", [False, True])
def test_verifiable_generator_sums_exactly(orc, code, same_sign):
    """genInOutFloatSum restatement (verifiable.cu:466-512): for every rank
    count the inputs sum exactly (fp64 holds every partial sum) to the
    generator's own expected output, and the ring oracle reproduces it in
    its summation order bit for bit."""
    for n in range(1, 9):
        ins, want = orc.verifiable_sum(code, n, 30011, seed=977 + n, same_sign=same_sign)
        assert np.array_equal(sum(_as_f64(x, code) for x in ins), _as_f64(want, code)), n
        if n >= 2 and code != 8:
            got = orc.ring_allreduce(code, 0, ins, nchannels=2, nthreads=544)
            assert np.array_equal(got.view(np.uint8), want.view(np.uint8)), n


def test_verifiable_generator_is_index_addressed(orc):
    """Values depend only on (seed, index): generating a sub-range equals the
    same slice of a full generation (so GPU tests can generate in parallel)."""
    ins, want = orc.verifiable_sum(7, 8, 5000, seed=3)
    ins2, want2 = orc.verifiable_sum(7, 8, 1000, seed=3, index0=2500)
    assert np.array_equal(want[2500:3500], want2)
    assert all(np.array_equal(a[2500:3500], b) for a, b in zip(ins, ins2))


def test_nccl_sum_tolerance_values(orc):
    # calcSumFloatTolerance (verifiable.cu:981-1004) at n = 2 / 4 / 8
    assert [orc.sum_float_tolerance(n, 7) for n in (2, 4, 8)] == [2, 3, 4]
    assert [orc.sum_float_tolerance(n, 6) for n in (2, 4, 8)] == [2, 3, 5]
