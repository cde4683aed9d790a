"""Bit-exact parity with the oracle at the exact BASELINE shapes, random inputs.

configs[2] (8 ranks x 128 MiB fp32) and configs[3] (8 ranks x 1 GiB fp16) on
the 8-rank virtual node, random uniform [-1, 1) inputs, every byte of every
rank's output compared with the oracle's ring-order restatement
(all_reduce.h:28-86: chunk size, loop size, the partial last loop's own
realChunkSize, chunk k finalised at ring index k, acc = fn(own, received) in
T at every hop).  The order-blind properties of test_gpu_tolerance.py cannot
see a wrong summation order in the tail loop; these can.

Walks covered (C = 4 MiB/8/sizeof(T)*4 elements per chunk):
  configs[2] library default, 7 rings: loop 7*8*C = 28 Mi elems -> one full
             loop + a partial loop (realChunkSize 75,776);
  configs[2] reference default (mccs.toml:19-20: 2 channels, ring 0..7 on
             both, proxy/engine.rs:296-320; 544 threads, plan.rs:602-635;
             one workgroup per channel): 4 full loops;
  configs[2] doubled channels (14 = every ring twice, the bench autotune's
             candidate): one partial loop only;
  configs[3] library default: 9 full loops + a tail (512 Mi / 56 Mi);
  configs[3] reference default: 32 full loops.
Lanes never change results (each lane owns a fixed region of every slice);
the reference profile at 1 GiB runs 8 lanes per channel so the test takes
seconds, not a minute.  The expected bytes come from
oracle.ring_allreduce_mt (the serial walk evaluated chunk-parallel, pinned
to the serial restatement in tests/test_oracle.py).
"""
import os

import pytest

from mccs_amd import comm as C
import vnode

pytestmark = pytest.mark.gpu

F16, F32 = 6, 7
N = 8
REF_RINGS = [list(range(N))] * 2

CASES = [
    ("configs2-fp32-128MiB-default", F32, 128, {}),
    ("configs2-fp32-128MiB-reference", F32, 128, dict(channel_count=2, rings=REF_RINGS, block_threads=544, lanes=1,
                                                      buffer_size=1 << 22)),
    ("configs2-fp32-128MiB-doubled", F32, 128, dict(channel_count=14)),
    ("configs3-fp16-1GiB-default", F16, 1024, {}),
    ("configs3-fp16-1GiB-reference", F16, 1024, dict(channel_count=2, rings=REF_RINGS, block_threads=544, lanes=8,
                                                     buffer_size=1 << 22)),
]


def _walk_loops(count, esize, nch, nthr, buff=1 << 22):
    """(full loops, partial-loop realChunkSize or 0) of all_reduce.h:28-37."""
    chunk = buff // 8 // esize * 4
    loop = nch * N * chunk
    full, rest = divmod(count, loop)
    if not rest:
        return full, 0
    gran = (nthr - 32) * 8 // esize
    rcs = min(chunk, -(-rest // (nch * N)))
    return full, -(-rcs // gran) * gran


@pytest.mark.parametrize("name,code,mib,cfg", CASES, ids=[c[0] for c in CASES])
def test_random_inputs_bit_exact_at_baseline_shape(orc, name, code, mib, cfg):
    import torch

    tdt, it = {F32: (torch.float32, torch.int32), F16: (torch.float16, torch.int16)}[code]
    esize = 4 if code == F32 else 2
    count = (mib << 20) // esize
    comms = C.init_all([0] * N, C.CommConfig(**cfg))
    try:
        planner = vnode.Planner(comms[0].nchannels, comms[0].rings())
        nch, nthr, rings = planner.select(count * esize, count * esize)
        full, tail_rcs = _walk_loops(count, esize, nch, nthr)
        if name.endswith("default") and code == F32:
            assert (nch, full) == (7, 1) and tail_rcs == 75776, (nch, full, tail_rcs)
        if name.endswith("reference"):
            assert nch == 2 and nthr == 544 and comms[0].lanes == cfg["lanes"]
            assert tail_rcs == 0 and full == {F32: 4, F16: 32}[code]
        if name.endswith("doubled"):
            assert nch == 14 and full == 0 and tail_rcs > 0
        if name == "configs3-fp16-1GiB-default":
            assert nch == 7 and full == 9 and tail_rcs > 0

        g = torch.Generator(device="cuda")
        send, host = [], []
        for r in range(N):
            g.manual_seed(0x6D636373 + 31 * r + code)
            x = (torch.rand(count, device="cuda", generator=g) * 2 - 1).to(tdt)
            send.append(x)
            host.append(x.cpu().numpy())
        recv = [torch.empty_like(x) for x in send]
        with C.group():
            for r in range(N):
                C.all_reduce(comms[r], send[r], recv[r], count, code, 0)
        for c in comms:
            c.sync()
        # a plain rank-order sum (rounded in T at every add) as a wrong-order
        # control: it must differ from the oracle, in the tail loop too
        naive = send[0].clone()
        for r in range(1, N):
            naive += send[r]
        del send
        want = orc.ring_allreduce_mt(code, 0, host, nchannels=nch, nthreads=nthr, buff_size=1 << 22,
                                     ring_orders=rings, workers=min(16, os.cpu_count() or 1))
        del host
        w = torch.from_numpy(want).cuda()
        for r in range(N):
            if not torch.equal(recv[r].view(it), w.view(it)):
                bad = (recv[r].view(it) != w.view(it)).nonzero()
                first = int(bad[0])
                raise AssertionError(f"{name}: rank {r} differs from the oracle at {bad.numel()} elements, "
                                     f"first at {first} (full loops {full}, tail realChunkSize {tail_rcs})")
        tail0 = full * nch * N * (4 << 20) // 8 // esize * 4
        assert not torch.equal(naive.view(it), w.view(it)), "order-blind inputs"
        if tail0 < count:
            assert not torch.equal(naive[tail0:].view(it), w[tail0:].view(it)), "order-blind tail"
        del w, recv, naive
    finally:
        vnode.destroy(comms)
