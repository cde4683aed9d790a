"""GPU: a DDP-style bucket stream at the library's default routing.

VERDICT r04: the suite pins the ring for every GPU module except the direct
kernel's own tests, so the product's default routing of small buckets (LL
one-shot <= 128 KiB, one-shot <= 2 / 1 MiB / 256 KiB, two-shot <= 4 / 8 MiB,
the ring above; include/mccs_hip.h) was never exercised the way a training
step uses it: a burst of buckets of mixed sizes issued back to back, no sync
between them, one wait at the end.  Here the communicators keep every
default (this module sets DIRECT_DEFAULTS), each bucket is checked bit for
bit against the oracle's ring-order restatement, and each call must have
taken the kernel the defaults route it to.  Two shapes: the virtual node (all
ranks on cuda:0, one fused launch per call) and ranks as separate processes
(IPC-mapped arenas, tests/ipc_worker.py "ddp" mode).
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
from vnode import DDP_STREAM as STREAM, ESIZE, ddp_expected_algo as expected_algo

pytestmark = pytest.mark.gpu
DIRECT_DEFAULTS = True  # conftest: keep the library's direct thresholds
HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.mark.parametrize("n", [2, 3, 4, 6, 8])
def test_ddp_bucket_stream_virtual_node(orc, n):
    import torch

    comms = C.init_all([0] * n)
    try:
        rng = np.random.default_rng(100 + n)
        steps = 2
        cases, sends, recvs, algos = [], [], [], []
        for step in range(steps):
            for code, nbytes in STREAM:
                count = nbytes // ESIZE[code]
                inputs = [vnode.gen(code, count, rng) for _ in range(n)]
                s = [vnode.to_dev(x) for x in inputs]
                r = [vnode.to_dev(np.zeros_like(x)) for x in inputs]
                cases.append((code, inputs))
                sends.append(s)
                recvs.append(r)
        # the whole stream back to back, one wait at the end
        for i, (code, inputs) in enumerate(cases):
            with C.group():
                for k in range(n):
                    C.all_reduce(comms[k], sends[i][k], recvs[i][k], inputs[0].size, code, 0)
            algos.append(comms[0].last_algo())
        torch.cuda.synchronize()
        for c in comms:
            c.sync()
        for i, (code, inputs) in enumerate(cases):
            nbytes = inputs[0].nbytes
            assert algos[i] == expected_algo(nbytes, n), (i, nbytes, algos[i])
            exp = vnode.expected_allreduce(orc, inputs, code, 0, comms[0])
            for k in range(n):
                got = vnode.from_dev(recvs[i][k], code)
                assert np.array_equal(got.view(np.uint8), exp.view(np.uint8)), f"bucket {i} ({nbytes} B) rank {k}"
        # every default kernel was exercised by the stream
        assert {"ll", "oneshot", "ring"} <= set(algos)
        if n >= 3:  # two-shot is on from 3 ranks (off at 2: the ring is two hops there)
            assert "direct" in algos
    finally:
        vnode.destroy(comms)


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("world", [2, 4])
def test_ddp_bucket_stream_across_processes(world):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.join(HERE, "ipc_worker.py")]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0", IPC_MODES="ddp")
    for k in ("MCCS_ONESHOT_BYTES", "MCCS_DIRECT_BYTES", "MCCS_LL_BYTES"):
        env.pop(k, None)
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=env, cwd=os.path.dirname(HERE))
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    lib_lines = "\n".join(l for l in (r.stdout + r.stderr).splitlines() if "mccs" in l.lower() or "hip" in l)[-3000:]
    assert r.returncode == 0 and lines, lib_lines + "\n----\n" + r.stdout[-2000:] + r.stderr[-2000:]
    res = json.loads(lines[-1])
    assert res["all_ok"], res
    kinds = {k.split("/")[1] for k in res["fifo_modes"] if k.startswith("ddp/")}
    assert {"ll", "oneshot", "ring"} <= kinds, kinds
