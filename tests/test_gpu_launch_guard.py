"""GPU: a communicator's launches never run beside each other, graph replays included.

VERDICT r05: the host orders a comm's eager launches across streams
(plan.cpp), but a collective captured into a HIP graph runs at replay, which
makes no library call.  Two launches of one comm running at once share its
FIFO flag lines, saved steps and direct control block, and returned wrong sums
(0cee6e4).  The reference cannot hit this: every launch of a comm goes on its
one private stream (src/mccs/src/proxy/init.rs:166-175, plan.rs:659-667).
Here every library launch takes its comm's launch guard on the GPU first
(mccs_amd/csrc/launch_guard.h).  These tests make a replay and an eager
launch -- or two replays -- of the same comms overlap with no dependency
between their streams and no host sync, then check every output bit for bit
against the oracle's ring order, and that the guard really was contended
(its `waits` counter: the overlap happened and was serialised, not avoided by
luck).  A silent wrong sum fails them.
"""
import numpy as np
import pytest

from mccs_amd import comm as C
import vnode

pytestmark = pytest.mark.gpu
DIRECT_DEFAULTS = True  # every test states its own thresholds
F32, F16 = 7, 6
BIG = 8 << 20  # fp32 elements of the long eager / replayed ring AllReduce (32 MiB per rank)


def _streams():
    """Two streams on different hardware queues: HIP maps a process's streams
    onto a few queues (GPU_MAX_HW_QUEUES, 4 here) and runs one queue's
    kernels in order, so two streams of one priority may share a queue and
    never overlap; a queue carries one priority, so these two cannot."""
    import torch

    return torch.cuda.Stream(priority=0), torch.cuda.Stream(priority=-1)


def _cfg(kind):
    # few workgroups per rank: long-running launches, and two of them (one
    # waiting on the guard) stay far inside the GPU's co-resident slots
    return C.CommConfig(timeout_ms=20000, lanes=2, channel_count=2, ll_bytes=1 << 20 if kind == "ll" else -1,
                        oneshot_bytes=8 << 20 if kind == "oneshot" else -1,
                        direct_bytes=8 << 20 if kind == "twoshot" else -1)


def _small_count(kind):
    return {"ll": 30001, "oneshot": 300001, "twoshot": 300001}.get(kind, 1000003)


ALGO = {"ring": "ring", "ll": "ll", "oneshot": "oneshot", "twoshot": "direct"}


def _check(orc, comms, inputs, outs, code, what):
    exp = vnode.expected_allreduce(orc, inputs, code, 0, comms[0])
    for r, o in enumerate(outs):
        got = vnode.from_dev(o, code)
        assert np.array_equal(got.view(np.uint8), exp.view(np.uint8)), f"{what}: rank {r} differs from the oracle"


def _waits(comms):
    return sum(c.guard_info()["waits"] for c in comms)


def _idle(comms):
    for c in comms:
        g = c.guard_info()
        assert (g["owner"], g["confirm"], g["fin"]) == (0, 0, 0), g


def _allreduce(comms, send, recv, count, code, stream):
    with C.group():
        for r, c in enumerate(comms):
            C.all_reduce(c, send[r], recv[r], count, code, 0, stream=stream)


@pytest.mark.parametrize("kind", ["ring", "ll", "oneshot", "twoshot"])
@pytest.mark.parametrize("n", [1, 2, 4])
def test_replay_beside_an_eager_launch(orc, n, kind):
    """A comm's AllReduce captured in a graph on stream B, replayed right after
    an eager AllReduce of the same comms on stream A (no sync, no event between
    the streams): both exact, the guard contended."""
    import torch

    if kind != "ring" and n == 1:
        pytest.skip("a one-rank comm has no direct kernel")
    comms = C.init_all([0] * n, _cfg(kind))
    try:
        rng = np.random.default_rng(60 + n)
        sa, sb = _streams()
        cnt_x = _small_count(kind)
        code_x = F16 if kind == "ll" else F32
        sx = [vnode.to_dev(np.zeros(cnt_x, vnode.NPDT[code_x])) for _ in range(n)]
        rx = [torch.zeros_like(t) for t in sx]
        sy = [vnode.to_dev(np.zeros(BIG, np.float32)) for _ in range(n)]
        ry = [torch.zeros_like(t) for t in sy]
        _allreduce(comms, sx, rx, cnt_x, code_x, sb)  # warm-up outside the capture
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=sb):
            _allreduce(comms, sx, rx, cnt_x, code_x, sb)
        torch.cuda.synchronize()
        for c in comms:
            c.sync()
        assert comms[0].last_algo() == ALGO[kind]
        w0 = _waits(comms)
        for rep in range(4):
            xs = [vnode.gen(code_x, cnt_x, rng) for _ in range(n)]
            ys = [vnode.gen(F32, BIG, rng) for _ in range(n)]
            for r in range(n):
                sx[r].copy_(torch.from_numpy(xs[r].view(np.uint8).copy()))
                sy[r].copy_(torch.from_numpy(ys[r].view(np.uint8).copy()))
            torch.cuda.synchronize()
            _allreduce(comms, sy, ry, BIG, F32, sa)  # eager, stream A
            with torch.cuda.stream(sb):
                g.replay()  # the replay: stream B, nothing orders it after A
            torch.cuda.synchronize()
            for c in comms:
                c.sync()
            _check(orc, comms, xs, rx, code_x, f"replay rep {rep}")
            _check(orc, comms, ys, ry, F32, f"eager rep {rep}")
        assert _waits(comms) > w0, "the replay never met the eager launch on the guard: no overlap was tested"
        _idle(comms)
    finally:
        torch.cuda.synchronize()
        vnode.destroy(comms)


@pytest.mark.parametrize("n", [2, 4])
def test_two_graphs_replayed_on_two_streams(orc, n):
    """Two graphs of the same comms (a long ring AllReduce and an LL one)
    replayed on two streams at once: exact, the guard contended."""
    import torch

    comms = C.init_all([0] * n, _cfg("ll"))
    try:
        rng = np.random.default_rng(80 + n)
        sa, sb = _streams()
        cnt_x = _small_count("ll")
        sx = [vnode.to_dev(np.zeros(cnt_x, np.float16)) for _ in range(n)]
        rx = [torch.zeros_like(t) for t in sx]
        sy = [vnode.to_dev(np.zeros(BIG, np.float32)) for _ in range(n)]
        ry = [torch.zeros_like(t) for t in sy]
        _allreduce(comms, sy, ry, BIG, F32, sa)
        _allreduce(comms, sx, rx, cnt_x, F16, sb)
        torch.cuda.synchronize()
        g1, g2 = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
        with torch.cuda.graph(g1, stream=sa):
            _allreduce(comms, sy, ry, BIG, F32, sa)
        with torch.cuda.graph(g2, stream=sb):
            _allreduce(comms, sx, rx, cnt_x, F16, sb)
        torch.cuda.synchronize()
        w0 = _waits(comms)
        for rep in range(4):
            xs = [vnode.gen(F16, cnt_x, rng) for _ in range(n)]
            ys = [vnode.gen(F32, BIG, rng) for _ in range(n)]
            for r in range(n):
                sx[r].copy_(torch.from_numpy(xs[r].view(np.uint8).copy()))
                sy[r].copy_(torch.from_numpy(ys[r].view(np.uint8).copy()))
            torch.cuda.synchronize()
            with torch.cuda.stream(sa):
                g1.replay()
            with torch.cuda.stream(sb):
                g2.replay()
            torch.cuda.synchronize()
            for c in comms:
                c.sync()
            _check(orc, comms, xs, rx, F16, f"graph 2 rep {rep}")
            _check(orc, comms, ys, ry, F32, f"graph 1 rep {rep}")
        assert _waits(comms) > w0, "the two replays never met on the guard: no overlap was tested"
        _idle(comms)
    finally:
        torch.cuda.synchronize()
        vnode.destroy(comms)


@pytest.mark.parametrize("n", [2, 3])
def test_allgather_replay_beside_an_eager_allreduce(orc, n):
    """The ring AllGather kernel takes the same guard: a captured AllGather
    replayed beside an eager AllReduce of the same comms, both exact."""
    import torch

    comms = C.init_all([0] * n, _cfg("ring"))
    try:
        rng = np.random.default_rng(90 + n)
        sa, sb = _streams()
        size = 1 << 20
        src = [torch.zeros(size, dtype=torch.uint8, device="cuda") for _ in range(n)]
        out = [torch.zeros(n * size, dtype=torch.uint8, device="cuda") for _ in range(n)]
        sy = [vnode.to_dev(np.zeros(BIG, np.float32)) for _ in range(n)]
        ry = [torch.zeros_like(t) for t in sy]
        with C.group():
            for r in range(n):
                C.all_gather(comms[r], src[r], out[r], size, stream=sb)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=sb):
            with C.group():
                for r in range(n):
                    C.all_gather(comms[r], src[r], out[r], size, stream=sb)
        torch.cuda.synchronize()
        w0 = _waits(comms)
        for rep in range(3):
            data = [rng.integers(0, 256, size, dtype=np.uint8) for _ in range(n)]
            ys = [vnode.gen(F32, BIG, rng) for _ in range(n)]
            for r in range(n):
                src[r].copy_(torch.from_numpy(data[r]))
                sy[r].copy_(torch.from_numpy(ys[r].view(np.uint8).copy()))
            torch.cuda.synchronize()
            _allreduce(comms, sy, ry, BIG, F32, sa)
            with torch.cuda.stream(sb):
                g.replay()
            torch.cuda.synchronize()
            for c in comms:
                c.sync()
            exp = np.concatenate(data)
            for r in range(n):
                assert np.array_equal(out[r].cpu().numpy(), exp), f"AllGather rep {rep} rank {r}"
            _check(orc, comms, ys, ry, F32, f"eager rep {rep}")
        assert _waits(comms) > w0, "the replay never met the eager launch on the guard: no overlap was tested"
        _idle(comms)
    finally:
        torch.cuda.synchronize()
        vnode.destroy(comms)


def test_guard_is_free_between_launches(orc):
    """After back-to-back launches of every kind and a sync, each comm's guard
    is free with its counters reset (a count left short would stall the next
    launch until the watchdog)."""
    import torch

    n = 3
    comms = C.init_all([0] * n, C.CommConfig(timeout_ms=20000, ll_bytes=64 << 10, oneshot_bytes=1 << 20,
                                            direct_bytes=4 << 20))
    try:
        rng = np.random.default_rng(5)
        algos = set()
        for count in (1000, 100000, 700000, 3000000, 7):
            xs = [vnode.gen(F32, count, rng) for _ in range(n)]
            s = [vnode.to_dev(x) for x in xs]
            r = [torch.zeros_like(t) for t in s]
            _allreduce(comms, s, r, count, F32, None)
            algos.add(comms[0].last_algo())
            torch.cuda.synchronize()
            for c in comms:
                c.sync()
            _check(orc, comms, xs, r, F32, f"count {count}")
            _idle(comms)
        assert algos == {"ll", "oneshot", "direct", "ring"}, algos
    finally:
        torch.cuda.synchronize()
        vnode.destroy(comms)


@pytest.mark.parametrize("seed", range(4))
def test_random_mix_of_replays_and_eager_launches(orc, seed, monkeypatch):
    """A seeded mix on one set of comms: some collectives (AllReduces, and
    AllGathers about one in five) captured into small graphs (1-3 each), the
    rest issued eagerly, then everything issued in a
    random order on three streams of two priorities with no dependency
    between them and no sync -- each graph replayed once, each eager call
    once.  Size routing picks the LL one-shot, one-shot, two-shot or ring per
    call, so replays and eager launches of every kind meet on the guard in
    whatever order the GPU runs them; every output is the oracle's, bit for
    bit, and the guards end free.  Grids stay small (2 channels x 2 lanes,
    16 direct workgroups per rank): a launch waiting on the guard keeps its
    workgroup slots, and three fused launches of full-GPU grids could keep
    the holder's last workgroups from being dispatched."""
    import torch

    rng = np.random.default_rng(9100 + seed)
    n = int(rng.integers(2, 5))
    monkeypatch.setenv("MCCS_DIRECT_BLOCKS", "16")  # read at communicator creation
    comms = C.init_all([0] * n, C.CommConfig(timeout_ms=20000, lanes=2, channel_count=2, ll_bytes=64 << 10,
                                            oneshot_bytes=1 << 20, direct_bytes=4 << 20))
    streams = [torch.cuda.Stream(priority=0), torch.cuda.Stream(priority=-1), torch.cuda.Stream(priority=0)]
    try:
        ops = []  # (code or None for an AllGather, count / bytes per rank, host inputs, send, recv)
        for _ in range(14):
            if rng.random() < 0.2:
                nbytes = int(np.exp(rng.uniform(np.log(64), np.log(4 << 20))))
                xs = [rng.integers(0, 256, nbytes, dtype=np.uint8) for _ in range(n)]
                ops.append((None, nbytes, xs, [vnode.to_dev(x) for x in xs],
                            [vnode.to_dev(np.zeros(n * nbytes, np.uint8)) for _ in range(n)]))
                continue
            code = int(rng.choice([F32, F16]))
            count = max(1, int(np.exp(rng.uniform(np.log(64), np.log(12 << 20)))) // vnode.ESIZE[code])
            xs = [vnode.gen(code, count, rng) for _ in range(n)]
            send = [vnode.to_dev(x) for x in xs]
            ops.append((code, count, xs, send, [torch.zeros_like(t) for t in send]))

        def issue(i, st):
            code, count, xs, send, recv = ops[i]
            if code is None:
                with C.group():
                    for r, c in enumerate(comms):
                        C.all_gather(c, send[r], recv[r], count, stream=st)
            else:
                _allreduce(comms, send, recv, count, code, st)

        order = [int(i) for i in rng.permutation(len(ops))]
        graphs, eager, k = [], [], 0
        while k < len(order):  # about half the ops go into graphs of 1-3
            take = int(rng.integers(1, 4))
            if rng.random() < 0.5:
                graphs.append(order[k:k + take])
            else:
                eager.extend([i] for i in order[k:k + take])
            k += take
        torch.cuda.synchronize()
        captured = []
        cap = streams[1]
        for members in graphs:
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=cap):
                for i in members:
                    issue(i, cap)
            captured.append(g)
        torch.cuda.synchronize()
        for _, _, _, _, recv in ops:  # the capture ran nothing; start from zeros all the same
            for t in recv:
                t.zero_()
        torch.cuda.synchronize()
        items = [("graph", j) for j in range(len(captured))] + [("eager", e[0]) for e in eager]
        w0 = _waits(comms)
        for pos in rng.permutation(len(items)):
            kind, j = items[int(pos)]
            st = streams[int(rng.integers(0, 3))]
            if kind == "graph":
                with torch.cuda.stream(st):
                    captured[j].replay()
            else:
                issue(j, st)
        torch.cuda.synchronize()
        for c in comms:
            c.sync()
        for i, (code, count, xs, send, recv) in enumerate(ops):
            what = f"seed {seed} n {n} op {i} count {count} code {code}"
            if code is None:
                exp = orc.ring_allgather(xs)
                for r in range(n):
                    assert np.array_equal(recv[r].cpu().numpy(), exp), f"{what}: rank {r} differs from the oracle"
            else:
                _check(orc, comms, xs, recv, code, what)
        _idle(comms)
        print(f"seed {seed} n {n}: {len(captured)} graphs, {len(eager)} eager, guard waits {_waits(comms) - w0}")
        del captured
    finally:
        torch.cuda.synchronize()
        vnode.destroy(comms)


def test_replay_beside_an_eager_launch_across_processes():
    """One rank per process (the deployment shape: one guard per launch, each
    workgroup claims it for itself): two ranks, a ring and an LL bucket, a
    replay racing an eager launch of the same comm on every rank
    (tests/ipc_worker.py guard_overlap)."""
    import json
    import os
    import socket
    import subprocess
    import sys

    here = os.path.dirname(os.path.abspath(__file__))
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2", "--master-addr",
           "127.0.0.1", "--master-port", str(port), os.path.join(here, "ipc_worker.py")]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0", IPC_MODES="guard")
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=env, cwd=os.path.dirname(here))
    # both ranks print to one pipe: their lines can run together, so take
    # every JSON object from the stream (the merged verdict is rank 0's last)
    import re

    lines = [json.loads(m) for m in re.findall(r"\{(?:[^{}]|\{[^{}]*\})*\}", r.stdout)]
    assert r.returncode == 0 and lines, r.stdout[-2000:] + r.stderr[-3000:]
    res = lines[-1]
    assert res["all_ok"], res
    assert {k.split("/")[2] for k in res["fifo_modes"] if k.endswith("/exact")} == {"ring", "ll"}, res
    waits = {(l["rank"], l["kind"]): l["waits"] for l in lines if "waits" in l}
    assert len(waits) == 4 and sum(waits.values()) > 0, waits
