"""GPU parity: mccs_hip_reduce / mccs_hip_reduce_copy vs the C oracle.

Bit-exact for every dtype and op (the kernel and the oracle apply the same
element functor, reduce_kernel.h semantics, in the same left-to-right order:
common_kernel.h:564-581).  Covers aligned/unaligned pointers, ragged tails,
empty input, 1..8 sources, 1..4 destinations, in-place, every main-loop
variant, and the full 2 x 128 MiB fp32 benchmark size.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

DTYPES = {  # code: (numpy storage, torch dtype name)
    0: (np.int8, "int8"), 1: (np.uint8, "uint8"), 2: (np.int32, "int32"), 3: (np.uint32, "uint32"),
    4: (np.int64, "int64"), 5: (np.uint64, "uint64"), 6: (np.float16, "float16"),
    7: (np.float32, "float32"), 8: (np.float64, "float64"), 9: (np.uint16, "bfloat16"),
}


def rand(code, n, rng):
    npdt = DTYPES[code][0]
    if code in (6, 7, 8):
        return (rng.standard_normal(n) * 4).astype(npdt)
    if code == 9:
        f = (rng.standard_normal(n) * 4).astype(np.float32)
        return (f.view(np.uint32) >> 16).astype(np.uint16)
    info = np.iinfo(npdt)
    lo, hi = (-100, 100) if info.min < 0 else (0, 200)
    return rng.integers(lo, hi, n).astype(npdt)


def to_dev(x, offset_elems=0):
    """Device copy; offset_elems > 0 returns a deliberately misaligned view."""
    import torch

    raw = torch.from_numpy(np.ascontiguousarray(x).view(np.uint8))
    buf = torch.empty(raw.numel() + 64, dtype=torch.uint8, device="cuda")
    off = offset_elems * x.itemsize
    buf[off:off + raw.numel()].copy_(raw)
    return buf, buf.data_ptr() + off


def from_dev(buf, ptr, n, npdt):
    import torch

    off = ptr - buf.data_ptr()
    nbytes = n * np.dtype(npdt).itemsize
    return buf[off:off + nbytes].cpu().numpy().view(npdt)


def run_reduce(srcs_np, ndsts, code, op, misalign=0):
    import mccs_amd
    import torch

    n = srcs_np[0].size
    npdt = DTYPES[code][0]
    s_dev = [to_dev(s, misalign) for s in srcs_np]
    d_dev = [to_dev(np.zeros(n, npdt), misalign) for _ in range(ndsts)]
    mccs_amd.reduce_copy([p for _, p in d_dev], [p for _, p in s_dev], count=n, dtype=code, op=op)
    torch.cuda.synchronize()
    return [from_dev(b, p, n, npdt) for b, p in d_dev]


@pytest.mark.parametrize("code", sorted(DTYPES))
@pytest.mark.parametrize("op", [0, 1, 2, 3])
def test_reduce_two_sources_all_types(orc, code, op):
    rng = np.random.default_rng(100 * code + op)
    n = 100003
    srcs = [rand(code, n, rng) for _ in range(2)]
    (got,) = run_reduce(srcs, 1, code, op)
    (ref,) = orc.reduce_copy(code, op, srcs)
    assert np.array_equal(got.view(np.uint8), ref.view(np.uint8))


@pytest.mark.parametrize("nsrcs,ndsts", [(1, 1), (1, 2), (2, 2), (3, 1), (5, 3), (8, 4)])
@pytest.mark.parametrize("code", [6, 7, 9])
def test_reduce_copy_fan(orc, nsrcs, ndsts, code):
    rng = np.random.default_rng(nsrcs * 10 + ndsts)
    n = 77777
    srcs = [rand(code, n, rng) for _ in range(nsrcs)]
    got = run_reduce(srcs, ndsts, code, 0)
    ref = orc.reduce_copy(code, 0, srcs, ndsts)
    for g, r in zip(got, ref):
        assert np.array_equal(g.view(np.uint8), r.view(np.uint8))


@pytest.mark.parametrize("n", [1, 3, 15, 16, 17, 255, 1023, 4097, (1 << 20) + 5])
@pytest.mark.parametrize("misalign", [0, 1])
def test_reduce_ragged_and_unaligned(orc, n, misalign):
    rng = np.random.default_rng(n)
    srcs = [rand(6, n, rng) for _ in range(2)]
    (got,) = run_reduce(srcs, 1, 6, 0, misalign=misalign)
    (ref,) = orc.reduce_copy(6, 0, srcs)
    assert np.array_equal(got.view(np.uint16), ref.view(np.uint16))


def test_reduce_empty_is_noop():
    import mccs_amd
    import torch

    a = torch.ones(8, device="cuda")
    c = torch.full((8,), 7.0, device="cuda")
    mccs_amd.reduce(c, [a, a], count=0)
    torch.cuda.synchronize()
    assert torch.all(c == 7.0)


def test_reduce_in_place(orc):
    import mccs_amd
    import torch

    rng = np.random.default_rng(9)
    n = 1 << 21
    a = rand(7, n, rng)
    b = rand(7, n, rng)
    ta, tb = torch.from_numpy(a).cuda(), torch.from_numpy(b).cuda()
    mccs_amd.reduce(ta, [ta, tb])
    torch.cuda.synchronize()
    (ref,) = orc.reduce_copy(7, 0, [a, b])
    assert np.array_equal(ta.cpu().numpy().view(np.uint32), ref.view(np.uint32))


def test_invalid_arguments_fail_loudly():
    import mccs_amd
    import torch

    a = torch.ones(8, device="cuda")
    with pytest.raises(mccs_amd.MccsError):
        mccs_amd.reduce(a, [a] * 9)  # > MCCS_REDUCE_MAX_SRCS
    with pytest.raises(mccs_amd.MccsError):
        mccs_amd.reduce(a, [a, a], dtype=42)
    with pytest.raises(mccs_amd.MccsError):
        mccs_amd.reduce(a, [a, a], op=4)  # PreMulSum is not compiled (reference gen_rules.sh:15)


@pytest.mark.parametrize("variant,unroll,policy,bpc,stages,waves", [
    (1, 2, 0, 4, 0, 0), (1, 4, 1, 8, 0, 0), (1, 8, 1, 2, 0, 0), (2, 2, 0, 1, 3, 4), (2, 4, 1, 1, 3, 4),
    (2, 4, 1, 2, 2, 4), (2, 1, 1, 1, 3, 4), (2, 2, 1, 2, 2, 8), (2, 4, 1, 1, 4, 4), (2, 8, 1, 1, 2, 4),
    (2, 4, 2, 1, 3, 5), (2, 4, 1, 1, 3, 6), (2, 2, 2, 2, 3, 6), (2, 4, 0, 1, 2, 6), (2, 1, 2, 1, 2, 8),
    (1, 4, 2, 16, 0, 0), (1, 8, 3, 32, 0, 0), (3, 4, 1, 16, 0, 0), (3, 2, 2, 32, 0, 0), (3, 8, 3, 8, 0, 0),
    (4, 4, 1, 32, 0, 0), (4, 8, 1, 16, 0, 0), (4, 2, 0, 8, 0, 0), (2, 4, 3, 1, 3, 4), (2, 4, 4, 1, 3, 4),
    (2, 4, 5, 1, 3, 4)])
@pytest.mark.parametrize("code", [6, 7, 9])
def test_reduce_variants(orc, variant, unroll, policy, bpc, stages, waves, code):
    import mccs_amd

    rng = np.random.default_rng(variant * 100 + unroll)
    n = (3 << 20) + 123  # many tiles per wave + partial last tile + scalar tail
    srcs = [rand(code, n, rng) for _ in range(2)]
    mccs_amd.tune(variant, unroll, policy, bpc, stages, waves)
    try:
        (got,) = run_reduce(srcs, 1, code, 0)
    finally:
        mccs_amd.tune()
    (ref,) = orc.reduce_copy(code, 0, srcs)
    assert np.array_equal(got.view(np.uint8), ref.view(np.uint8))


def test_reduce_full_benchmark_size(orc):
    """2 x 128 MiB fp32 (BASELINE configs[1]) checked element for element."""
    import mccs_amd
    import torch

    n = (128 << 20) // 4
    g = torch.Generator(device="cuda")
    g.manual_seed(1)
    a = torch.rand(n, device="cuda", generator=g) * 2 - 1
    g.manual_seed(2)
    b = torch.rand(n, device="cuda", generator=g) * 2 - 1
    c = torch.empty_like(a)
    for variant in (1, 2, 3, 4):
        mccs_amd.tune(variant)
        c.zero_()
        mccs_amd.reduce(c, [a, b])
        torch.cuda.synchronize()
        ha, hb = a.cpu().numpy(), b.cpu().numpy()
        ref = np.empty_like(ha)
        orc.reduce_mt(7, 0, [ha, hb], ref, 8)
        assert np.array_equal(c.cpu().numpy().view(np.uint32), ref.view(np.uint32)), variant
    mccs_amd.tune()


def test_reduce_captured_in_hip_graph(orc):
    """The chunk reduce is a plain stream-ordered launch, so a caller can
    capture a bucket of reduces into a hipGraph and replay it (one graph
    launch instead of one host launch per bucket)."""
    import mccs_amd
    import torch

    rng = np.random.default_rng(11)
    n = (1 << 20) + 5
    hs = [[rand(7, n, rng) for _ in range(2)] for _ in range(3)]
    srcs = [[torch.from_numpy(h).cuda() for h in pair] for pair in hs]
    outs = [torch.empty(n, dtype=torch.float32, device="cuda") for _ in range(3)]
    mccs_amd.reduce(outs[0], srcs[0])  # first call outside capture (one-time attribute setup)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s):
            for k in range(3):
                mccs_amd.reduce(outs[k], srcs[k], stream=s)
    for o in outs:
        o.zero_()
    torch.cuda.synchronize()
    g.replay()
    torch.cuda.synchronize()
    for k in range(3):
        (ref,) = orc.reduce_copy(7, 0, hs[k])
        assert np.array_equal(outs[k].cpu().numpy().view(np.uint32), ref.view(np.uint32)), k
    # new inputs in the same buffers: the replay reads them
    for k in range(3):
        srcs[k][0].mul_(2)
    g.replay()
    torch.cuda.synchronize()
    for k in range(3):
        (ref,) = orc.reduce_copy(7, 0, [srcs[k][0].cpu().numpy(), hs[k][1]])
        assert np.array_equal(outs[k].cpu().numpy().view(np.uint32), ref.view(np.uint32)), k


def test_reduce_beyond_2pow31_elements():
    """Maximum-size edge for the standalone chunk reduce: uint8 2^31 + 17
    elements (64-bit pack and tile indices, partial last tile, byte tail)."""
    import mccs_amd
    import torch

    n = (1 << 31) + 17
    g = torch.Generator(device="cuda")
    g.manual_seed(3)
    a = torch.randint(0, 256, (n,), dtype=torch.uint8, device="cuda", generator=g)
    b = torch.randint(0, 256, (n,), dtype=torch.uint8, device="cuda", generator=g)
    c = torch.empty_like(a)
    mccs_amd.reduce(c, [a, b])
    torch.cuda.synchronize()
    assert torch.equal(c, a + b)


@pytest.mark.parametrize("code", [6, 7, 8, 9])
@pytest.mark.parametrize("op", [0, 1, 2, 3])
@pytest.mark.parametrize("nsrcs", [2, 3])
def test_reduce_nan_and_inf(orc, code, op, nsrcs):
    """NaN / +-Inf (2 % each) in every source: the per-type operators of
    reduce_kernel.h decide what survives (float / double Max/Min
    (x < y) ? y : x keep a NaN first operand and drop a NaN second one; half and
    bf16 go through fmaxf / fminf, which drop either).  NaN positions match
    the oracle's and every other element is bit-exact (payloads not compared)."""
    rng = np.random.default_rng(7 * code + op + 100 * nsrcs)
    n = 50021
    srcs = []
    for _ in range(nsrcs):
        x = rand(code, n, rng)
        u = rng.random(n)
        if code == 9:  # bf16 bit patterns
            x[u < 0.02] = 0x7FC0
            x[(u >= 0.02) & (u < 0.04)] = 0x7F80
            x[(u >= 0.04) & (u < 0.06)] = 0xFF80
        else:
            x[u < 0.02] = np.nan
            x[(u >= 0.02) & (u < 0.04)] = np.inf
            x[(u >= 0.04) & (u < 0.06)] = -np.inf
        srcs.append(x)
    (got,) = run_reduce(srcs, 1, code, op)
    (ref,) = orc.reduce_copy(code, op, srcs)

    def isnan(a):
        if code == 9:
            return np.isnan((a.view(np.uint16).astype(np.uint32) << 16).view(np.float32))
        return np.isnan(a)

    assert np.array_equal(isnan(got), isnan(ref))
    keep = ~isnan(ref)
    assert np.array_equal(got.view(np.uint8).reshape(n, -1)[keep], ref.view(np.uint8).reshape(n, -1)[keep])
