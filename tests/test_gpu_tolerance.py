"""Floating-point agreement of the HIP ring with the exact sum, checked on
what the GPU produced, at the BASELINE bucket sizes (8-rank virtual node).

Three properties, each stated with its tolerance:

1. nccl-tests verifiable vectors (the generator the reference vendors,
   genInOutFloatSum, verifiable.cu:466-512, restated in oracle/verifiable.c):
   the inputs sum exactly in any order, so every rank must hold the
   generator's own expected output BIT FOR BIT (tolerance 0).  Committed
   small fixtures (tests/golden/ring_golden.npz, "verifiable" cases) and
   configs[2] (8 x 128 MiB fp32) at full size.
2. Same-sign random inputs, uniform [0, 1): no cancellation, so the
   nccl-tests bit-distance tolerance applies to every element:
   |bits(gpu) - bits(round_T(fp64 sum))| <= calcSumFloatTolerance(8)
   (verifiable.cu:981-1004: fp32 4, fp16 5 at n = 8).
3. Mixed-sign random inputs, uniform [-1, 1): bit distance is meaningless
   near cancellation, so every element is held to the forward error bound
   of recursive summation, |gpu - exact| <= gamma_{n-1} * sum_i |x_i| with
   gamma_k = k*u / (1 - k*u), u = 2^-11 (fp16) / 2^-24 (fp32).
"""
import os
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import pytest

from mccs_amd import comm as C
import vnode

pytestmark = pytest.mark.gpu

F16, F32, BF16 = 6, 7, 9
GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "ring_golden.npz")


def _ring(comms, send, count, code):
    import torch

    recv = [torch.empty_like(x) for x in send]
    with C.group():
        for r, c in enumerate(comms):
            C.all_reduce(c, send[r], recv[r], count, code, 0)
    for c in comms:
        c.sync()
    return recv


def test_verifiable_golden_fixtures_on_gpu():
    z = np.load(GOLDEN, allow_pickle=False)
    names = sorted({k.split("__")[0] for k in z.files if "verifiable" in k})
    assert len(names) >= 3
    for name in names:
        n, dtype, nch, _, op = (int(v) for v in z[name + "__meta"][:5])
        inputs = [z[f"{name}__in{r}"] for r in range(n)]
        comms = C.init_all([0] * n, C.CommConfig(channel_count=nch))
        try:
            outs = vnode.run_allreduce(comms, inputs, dtype, op)
        finally:
            vnode.destroy(comms)
        want = z[name + "__out"]
        for r, o in enumerate(outs):
            assert np.array_equal(o.view(np.uint8), want.view(np.uint8)), f"{name} rank {r}"


def _verifiable_parallel(orc, code, nranks, count, seed, workers=16):
    """Inputs and expected output of the verifiable generator, split over
    threads (the C generator runs without the GIL)."""
    npdt = orc.NP_DTYPE[code]
    ins = [np.empty(count, npdt) for _ in range(nranks)]
    out = np.empty(count, npdt)
    L = orc.lib()
    step = -(-count // workers)

    def part(k):
        lo, hi = k * step, min(count, (k + 1) * step)
        if hi <= lo:
            return
        for r in range(nranks):
            assert L.oracle_verifiable_float_sum(code, 1, nranks, r, seed, lo, hi - lo, 0,
                                                 ins[r][lo:].ctypes.data) == 0
        assert L.oracle_verifiable_float_sum(code, 0, nranks, 0, seed, lo, hi - lo, 0, out[lo:].ctypes.data) == 0

    with ThreadPoolExecutor(workers) as ex:
        list(ex.map(part, range(workers)))
    return ins, out


def test_verifiable_configs2_full_size(orc):
    """configs[2]: 8 ranks x 128 MiB fp32 of verifiable inputs; bit-exact."""
    import torch

    n, count = 8, (128 << 20) // 4
    ins, want = _verifiable_parallel(orc, F32, n, count, seed=0x6D636373)
    comms = C.init_all([0] * n)
    try:
        send = [torch.from_numpy(x).cuda() for x in ins]
        del ins
        recv = _ring(comms, send, count, F32)
        w = torch.from_numpy(want).cuda()
        for r in range(n):
            assert torch.equal(recv[r].view(torch.int32), w.view(torch.int32)), f"rank {r}"
    finally:
        vnode.destroy(comms)


@pytest.mark.parametrize("code,mib", [(F32, 128), (F16, 1024)], ids=["configs2-fp32-128MiB", "configs3-fp16-1GiB"])
def test_random_same_sign_within_nccl_tolerance(orc, code, mib):
    import torch

    n = 8
    tdt, it = {F32: (torch.float32, torch.int32), F16: (torch.float16, torch.int16)}[code]
    count = (mib << 20) // (4 if code == F32 else 2)
    tol = orc.sum_float_tolerance(n, code)
    assert tol == {F32: 4, F16: 5}[code]
    comms = C.init_all([0] * n)
    try:
        g = torch.Generator(device="cuda")
        send = []
        exact = torch.zeros(count, dtype=torch.float64, device="cuda")
        for r in range(n):
            g.manual_seed(7000 + r)
            x = torch.rand(count, device="cuda", generator=g).to(tdt)
            exact += x.double()
            send.append(x)
        ref = exact.to(tdt)
        del exact
        recv = _ring(comms, send, count, code)
        del send
        for r in range(n):
            d = (recv[r].view(it).to(torch.int32) - ref.view(it).to(torch.int32)).abs()
            worst = int(d.max())
            assert worst <= tol, f"rank {r}: max bit distance {worst} > {tol}"
            del d
    finally:
        vnode.destroy(comms)


@pytest.mark.parametrize("code,mib", [(F32, 128), (F16, 1024)], ids=["configs2-fp32-128MiB", "configs3-fp16-1GiB"])
def test_random_mixed_sign_within_forward_error_bound(code, mib):
    import torch

    n = 8
    tdt = {F32: torch.float32, F16: torch.float16}[code]
    u = {F32: 2.0 ** -24, F16: 2.0 ** -11}[code]
    gamma = (n - 1) * u / (1 - (n - 1) * u)
    count = (mib << 20) // (4 if code == F32 else 2)
    comms = C.init_all([0] * n)
    try:
        g = torch.Generator(device="cuda")
        send = []
        exact = torch.zeros(count, dtype=torch.float64, device="cuda")
        absum = torch.zeros(count, dtype=torch.float64, device="cuda")
        for r in range(n):
            g.manual_seed(8000 + r)
            x = (torch.rand(count, device="cuda", generator=g) * 2 - 1).to(tdt)
            xd = x.double()
            exact += xd
            absum += xd.abs()
            send.append(x)
            del xd
        bound = absum.mul_(gamma)
        recv = _ring(comms, send, count, code)
        del send
        for r in range(n):
            err = (recv[r].double() - exact).abs()
            ratio = float((err / bound.clamp_min(1e-300)).max())
            assert bool((err <= bound).all()), f"rank {r}: error / bound = {ratio}"
            del err
    finally:
        vnode.destroy(comms)
