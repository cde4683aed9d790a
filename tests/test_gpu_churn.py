"""GPU: communicator churn -- many create / collective / destroy cycles.

A service (the reference's model: one long-lived process, communicators
created as jobs come and go, src/mccs/src/control.rs) must not grow device
memory with every communicator it has ever built.  FIFO arenas are pooled
rather than freed; with exact-size pooling a 2,000-case fuzz
ran one GPU out of memory.  Here shapes vary cycle by cycle (ranks,
channels, buffer size, FIFO depth, direct thresholds), each cycle runs the
reference's int32 known-answer AllReduce (every rank sends 2042 + rank,
src/mccs_examples/allreduce_proto/src/main.rs:111) on the ring and on the
default small-bucket kernel.  A fixed list of shapes runs ROUNDS times: the
first round fills the arena pool, so from its end to the last round's end
the GPU's free memory must not fall (a leaked arena, event, stream, device
structure or IPC mapping per cycle would).  Across processes every cycle
also opens and closes every peer's arena.
"""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

from mccs_amd import comm as C

pytestmark = pytest.mark.gpu
DIRECT_DEFAULTS = True  # conftest: keep the library defaults (the LL bucket below)
HERE = os.path.dirname(os.path.abspath(__file__))
INT32, SUM = 2, 0
DRIFT_BYTES = 128 << 20  # one leaked arena per cycle would be >= 1 MiB x 36 cycles, mostly far more
SHAPES, ROUNDS = 12, int(os.environ.get("MCCS_CHURN_ROUNDS", "4"))


def churn_shapes(seed, nshapes, n_choices):
    """`nshapes` seeded communicator shapes, the list repeated ROUNDS times."""
    rng = np.random.default_rng(seed)
    out = []
    for _ in range(nshapes):
        out.append((int(rng.choice(n_choices)),
                    dict(channel_count=int(rng.integers(1, 5)),
                         buffer_size=int(rng.choice([1 << 20, 3 << 19, 1 << 21, 1 << 22])),
                         fifo_slots=int(rng.choice([8, 16, 32])),
                         oneshot_bytes=int(rng.choice([256 << 10, 1 << 20, 2 << 20])),
                         direct_bytes=int(rng.choice([-1, 4 << 20, 8 << 20])))))
    return out * ROUNDS


def kat(n):
    return 2042 * n + n * (n - 1) // 2


def test_virtual_node_churn_keeps_memory_flat():
    import torch

    dev = torch.device("cuda", 0)
    counts = (3 << 20, 16 << 10)  # 12 MiB (ring) and 64 KiB (LL one-shot)
    free = []
    shapes = churn_shapes(7, SHAPES, [2, 3, 4])
    for i, (n, cfg) in enumerate(shapes):
        comms = C.init_all([0] * n, C.CommConfig(**cfg))
        try:
            for count in counts:
                send = [torch.full((count,), 2042 + r, dtype=torch.int32, device=dev) for r in range(n)]
                recv = [torch.empty_like(s) for s in send]
                with C.group():
                    for r in range(n):
                        C.all_reduce(comms[r], send[r], recv[r], count, INT32, SUM)
                for c in comms:
                    c.sync()
                for r in range(n):
                    assert bool((recv[r] == kat(n)).all()), (i, n, cfg, count, r)
        finally:
            for c in comms:
                c.destroy()
        del send, recv
        torch.cuda.synchronize()
        torch.cuda.empty_cache()
        if i in (SHAPES - 1, len(shapes) - 1):  # the pool is warm after the first round
            free.append(torch.cuda.mem_get_info(0)[0])
    print(f"virtual node churn: {len(shapes)} cycles, free memory drift over the warm rounds {free[0] - free[1]} B")
    assert free[0] - free[1] < DRIFT_BYTES, f"free memory fell {(free[0] - free[1]) >> 20} MiB over 3 warm rounds"


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("world,no_barrier", [(2, False), (4, False), (2, True), (4, True)])
def test_process_churn_keeps_memory_flat(world, no_barrier):
    """no_barrier: every rank destroys its communicator as soon as its own
    collectives are done, with no barrier among the ranks (the arena release
    protocol, comm.cpp pool, keeps a destroyed arena from a new tenant until
    every peer destroyed its side); the next cycle's communicators may then
    need fresh arenas while the old ones wait, so memory may grow by a few
    arenas, never by one per cycle."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.join(HERE, "churn_worker.py")]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0", CHURN_NO_BARRIER="1" if no_barrier else "0")
    for k in ("MCCS_ONESHOT_BYTES", "MCCS_DIRECT_BYTES", "MCCS_LL_BYTES"):
        env.pop(k, None)
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=env, cwd=os.path.dirname(HERE))
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    lib_lines = "\n".join(l for l in (r.stdout + r.stderr).splitlines() if "mccs" in l.lower() or "hip" in l)[-3000:]
    assert r.returncode == 0 and lines, lib_lines + "\n----\n" + r.stdout[-2000:] + r.stderr[-2000:]
    res = json.loads(lines[-1])
    print(f"process churn, {world} processes:", res)
    assert res["all_ok"], res
    assert res["max_drift_bytes"] < (4 if no_barrier else 1) * DRIFT_BYTES, res
