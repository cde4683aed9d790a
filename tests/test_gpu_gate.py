"""GPU: the node gate across processes (tests/gate_worker.py).

Two ranks as two processes on the one-GPU box with the gate forced on
(MCCS_GATE=1): a clean pass keeps every default path; a wrong ring sum
injected on one rank steps both down to the release hand-off through the
ring vote; a wrong one-shot sum injected on the other rank disables the
one-shot on both; a direct launch left hanging (the peer never launches it)
ends at the 5 s watchdog as a vote against every direct variant while the
ring stays usable; thresholds that differ but round to the same arena make
Connect refuse on both; a rank that enters Connect 8 s late is
waited for by the connect-time barrier.  Every AllReduce after a gate is
checked exact and for the kernel it took.
"""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
DIRECT_DEFAULTS = True  # the gate tests the library defaults (conftest otherwise pins the ring)
HERE = os.path.dirname(os.path.abspath(__file__))


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_gate_verdicts_agree_across_processes():
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.join(HERE, "gate_worker.py")]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=env, cwd=os.path.dirname(HERE))
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert r.returncode == 0 and lines, r.stdout[-3000:] + r.stderr[-3000:]
    res = json.loads(lines[-1])
    assert res["all_ok"], res
    assert set(res["cases"]) >= {"clean/gate", "ring/gate", "oneshot/gate", "hang/gate", "mismatch/connect",
                                 "late/gate"}
