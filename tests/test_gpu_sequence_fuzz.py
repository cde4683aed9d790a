"""GPU: seeded random sequences of collectives on one set of communicators.

The per-case fuzz (test_gpu_ring_fuzz.py) builds fresh communicators for
every collective.  A deployment keeps them: state carried from one launch to
the next -- each lane's saved step in its flag lines, the work FIFO's
position and acknowledgements, the LL lines' launch sequence, the direct
kernels' running counters, one arena shared by the ring and every direct
variant -- is only exercised by many different collectives back to back.
Each case here draws a rank count and a communicator shape, then issues 40
collectives without a sync in between: AllReduces of random dtype, op and
length (1 element to 16 MiB, so the library's default routing sends them to
the LL one-shot, the one-shot, the two-shot or the ring), in place or not,
AllGathers, and groups of several integer AllReduces per communicator (one
launch with several works).  After one sync every output must equal the
oracle's ring-order result bit for bit (integer sums are order-free, so a
group's expected values need no channel plan).  The same sequences also run
with one rank per process (IPC-mapped arenas, tests/ipc_worker.py "seq").
"""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

from mccs_amd import comm as C
import vnode

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
DIRECT_DEFAULTS = True  # conftest: the library's default routing is what is under test
CASES = int(os.environ.get("MCCS_SEQ_CASES", "10"))
OPS = int(os.environ.get("MCCS_SEQ_OPS", "40"))
MAX_BYTES = 16 << 20


def sequence(rng, nops):
    """The same list on every rank: dicts with kind ar / ag / group."""
    ops = []
    for _ in range(nops):
        u = rng.random()
        code = int(rng.choice([0, 2, 4, 6, 7, 8, 9]))
        count = max(1, int(np.exp(rng.uniform(0, np.log(MAX_BYTES)))) // vnode.ESIZE[code])
        if u < 0.7:
            op = int(rng.choice([0, 0, 0, 1, 2, 3]))
            ops.append(dict(kind="ar", code=code, op=op, count=count, inplace=bool(rng.random() < 0.25)))
        elif u < 0.85:
            ops.append(dict(kind="ag", nbytes=count * vnode.ESIZE[code]))
        else:
            code = int(rng.choice([0, 2, 4]))
            ops.append(dict(kind="group", code=code, op=int(rng.choice([0, 2, 3])),
                            counts=[max(1, int(np.exp(rng.uniform(0, np.log(4 << 20)))) // vnode.ESIZE[code])
                                    for _ in range(int(rng.integers(2, 5)))]))
    return ops


def _int_allreduce(xs, op):
    acc = xs[0].copy()
    for x in xs[1:]:
        if op == 0:
            acc = (acc + x).astype(acc.dtype)
        elif op == 2:
            acc = np.maximum(acc, x)
        else:
            acc = np.minimum(acc, x)
    return acc


@pytest.mark.parametrize("seed", range(CASES))
def test_random_collective_sequence(orc, seed):
    import torch

    rng = np.random.default_rng(7000 + seed)
    n = int(rng.integers(2, 9))
    cfg = {}
    if rng.random() < 0.3:
        cfg["channel_count"] = int(rng.integers(1, 7))
    if rng.random() < 0.3:
        cfg["lanes"] = int(rng.choice([1, 2, 4]))
    comms = C.init_all([0] * n, C.CommConfig(**cfg))
    try:
        checks = []  # (what, per-rank device outputs, expected host array, dtype code or None)
        algos = set()
        for i, o in enumerate(sequence(rng, OPS)):
            if o["kind"] == "ar":
                xs = [vnode.gen(o["code"], o["count"], rng) for _ in range(n)]
                send = [vnode.to_dev(x) for x in xs]
                recv = send if o["inplace"] else [vnode.to_dev(np.zeros_like(x)) for x in xs]
                with C.group():
                    for r in range(n):
                        C.all_reduce(comms[r], send[r], recv[r], o["count"], o["code"], o["op"])
                algos.add(comms[0].last_algo())
                checks.append((f"{i} {o}", recv, vnode.expected_allreduce(orc, xs, o["code"], o["op"], comms[0]),
                               o["code"]))
            elif o["kind"] == "ag":
                xs = [rng.integers(0, 256, o["nbytes"], dtype=np.uint8) for _ in range(n)]
                send = [vnode.to_dev(x) for x in xs]
                recv = [vnode.to_dev(np.zeros(n * o["nbytes"], np.uint8)) for _ in range(n)]
                with C.group():
                    for r in range(n):
                        C.all_gather(comms[r], send[r], recv[r], o["nbytes"])
                checks.append((f"{i} {o}", recv, orc.ring_allgather(xs), None))
            else:
                batch = []
                for count in o["counts"]:
                    xs = [vnode.gen(o["code"], count, rng) for _ in range(n)]
                    batch.append((count, xs, [vnode.to_dev(x) for x in xs],
                                  [vnode.to_dev(np.zeros_like(x)) for x in xs]))
                with C.group():
                    for count, xs, send, recv in batch:
                        for r in range(n):
                            C.all_reduce(comms[r], send[r], recv[r], count, o["code"], o["op"])
                for k, (count, xs, send, recv) in enumerate(batch):
                    checks.append((f"{i}.{k} {o['kind']} code={o['code']} op={o['op']} count={count}", recv,
                                   _int_allreduce(xs, o["op"]), o["code"]))
        torch.cuda.synchronize()
        for c in comms:
            c.sync()
        for what, outs, exp, code in checks:
            for r in range(n):
                got = outs[r].cpu().numpy() if code is None else vnode.from_dev(outs[r], code)
                assert np.array_equal(got.view(np.uint8), exp.view(np.uint8)), f"seed {seed} n {n} {cfg} op {what} rank {r}"
        print(f"seed {seed} n {n} {cfg}: single AllReduces took {sorted(algos)}; groups take the ring")
    finally:
        vnode.destroy(comms)


@pytest.mark.parametrize("seed", range(CASES))
def test_random_collective_sequence_mixed_streams(orc, seed):
    """The same kind of sequence with every collective issued on one of three
    streams at random: a communicator's launches still run in issue order
    (a launch on another stream waits for the previous one), so every output
    equals the oracle's.  Inputs are staged and synchronised first: data
    dependencies across streams are the caller's, launch order is the
    library's."""
    import torch

    rng = np.random.default_rng(11000 + seed)
    n = int(rng.integers(2, 9))
    comms = C.init_all([0] * n)
    streams = [torch.cuda.current_stream(), torch.cuda.Stream(), torch.cuda.Stream()]
    try:
        staged = []  # (kind, code, op, count/nbytes, host inputs, send, recv)
        for o in sequence(rng, OPS):
            if o["kind"] == "ar":
                xs = [vnode.gen(o["code"], o["count"], rng) for _ in range(n)]
                send = [vnode.to_dev(x) for x in xs]
                recv = send if o["inplace"] else [vnode.to_dev(np.zeros_like(x)) for x in xs]
                staged.append([("ar", o["code"], o["op"], o["count"], xs, send, recv)])
            elif o["kind"] == "ag":
                xs = [rng.integers(0, 256, o["nbytes"], dtype=np.uint8) for _ in range(n)]
                staged.append([("ag", None, None, o["nbytes"], xs, [vnode.to_dev(x) for x in xs],
                                [vnode.to_dev(np.zeros(n * o["nbytes"], np.uint8)) for _ in range(n)])])
            else:
                batch = []
                for count in o["counts"]:
                    xs = [vnode.gen(o["code"], count, rng) for _ in range(n)]
                    batch.append(("group", o["code"], o["op"], count, xs, [vnode.to_dev(x) for x in xs],
                                  [vnode.to_dev(np.zeros_like(x)) for x in xs]))
                staged.append(batch)
        torch.cuda.synchronize()
        for item in staged:
            st = streams[int(rng.integers(0, 3))]
            with C.group():
                for kind, code, op, cnt, xs, send, recv in item:
                    for r in range(n):
                        if kind == "ag":
                            C.all_gather(comms[r], send[r], recv[r], cnt, stream=st)
                        else:
                            C.all_reduce(comms[r], send[r], recv[r], cnt, code, op, stream=st)
        torch.cuda.synchronize()
        for c in comms:
            c.sync()
        for item in staged:
            for kind, code, op, cnt, xs, send, recv in item:
                if kind == "ag":
                    exp = orc.ring_allgather(xs)
                elif kind == "ar":
                    exp = vnode.expected_allreduce(orc, xs, code, op, comms[0])
                else:
                    exp = _int_allreduce(xs, op)
                for r in range(n):
                    got = recv[r].cpu().numpy() if kind == "ag" else vnode.from_dev(recv[r], code)
                    assert np.array_equal(got.view(np.uint8), exp.view(np.uint8)), (seed, n, kind, code, op, cnt, r)
    finally:
        vnode.destroy(comms)


@pytest.mark.parametrize("seed", range(4))
def test_random_sequence_graph_replay(orc, seed):
    """The whole sequence captured into one HIP graph and replayed three
    times with fresh inputs copied into the same buffers: every replay's
    outputs exact.  State the kernels keep across launches (flag-line steps,
    the LL launch sequence, direct counters) lives in device memory, not in
    the captured arguments, so a replay must see it advance."""
    import torch

    rng = np.random.default_rng(8000 + seed)
    n = int(rng.integers(2, 9))
    comms = C.init_all([0] * n)
    try:
        ops = [o for o in sequence(rng, 30) if o["kind"] != "ag"]
        bufs = []  # per op: (code, op, count, send, recv)
        for o in ops:
            counts = [o["count"]] if o["kind"] == "ar" else o["counts"]
            for count in counts:
                send = [vnode.to_dev(np.zeros(count, vnode.NPDT[o["code"]])) for _ in range(n)]
                recv = send if o.get("inplace") else [vnode.to_dev(np.zeros(count, vnode.NPDT[o["code"]]))
                                                      for _ in range(n)]
                bufs.append((o["kind"], o["code"], o["op"], count, send, recv))

        def issue():
            i = 0
            for o in ops:
                k = 1 if o["kind"] == "ar" else len(o["counts"])
                with C.group():
                    for kind, code, op, count, send, recv in bufs[i:i + k]:
                        for r in range(n):
                            C.all_reduce(comms[r], send[r], recv[r], count, code, op)
                i += k

        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            issue()
        for rep in range(3):
            inputs = []
            for kind, code, op, count, send, recv in bufs:
                xs = [vnode.gen(code, count, rng) for _ in range(n)]
                for r in range(n):
                    send[r].copy_(torch.from_numpy(np.ascontiguousarray(xs[r]).view(np.uint8)).cuda())
                inputs.append(xs)
            g.replay()
            torch.cuda.synchronize()
            for (kind, code, op, count, send, recv), xs in zip(bufs, inputs):
                exp = (vnode.expected_allreduce(orc, xs, code, op, comms[0]) if kind == "ar"
                       else _int_allreduce(xs, op))
                for r in range(n):
                    got = vnode.from_dev(recv[r], code)
                    assert np.array_equal(got.view(np.uint8), exp.view(np.uint8)), (seed, n, rep, kind, code, op,
                                                                                     count, r)
        del g
    finally:
        vnode.destroy(comms)


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("world,mode", [(2, "seq"), (3, "seq"), (4, "seq"), (2, "seqs"), (4, "seqs")])
def test_random_collective_sequence_across_processes(world, mode):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.join(HERE, "ipc_worker.py")]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0", IPC_MODES=mode)  # seqs: random streams per call
    for k in ("MCCS_ONESHOT_BYTES", "MCCS_DIRECT_BYTES", "MCCS_LL_BYTES"):
        env.pop(k, None)
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=env, cwd=os.path.dirname(HERE))
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    lib_lines = "\n".join(l for l in (r.stdout + r.stderr).splitlines() if "mccs" in l.lower() or "hip" in l)[-3000:]
    assert r.returncode == 0 and lines, lib_lines + "\n----\n" + r.stdout[-2000:] + r.stderr[-2000:]
    res = json.loads(lines[-1])
    bad = [k for k, v in res["fifo_modes"].items() if not v]
    assert res["all_ok"] and not bad, bad
    print(f"{world} processes:", [k for k in res["fifo_modes"] if k.startswith("seq/algos")])
