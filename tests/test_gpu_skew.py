"""GPU: a peer that reaches the collective 35 s late is waited for.

The FIFO-wait watchdog counts time without progress.  Its default was 30 s
until round 5, so a rank that entered an AllReduce 30 s before its peer (rank
0 writing a checkpoint while the others start the next step) failed the
communicator.  The default is now 10 min, torch's default collective timeout
(include/mccs_hip.h timeout_ms); the test suite itself runs with
MCCS_TIMEOUT_MS=30000 (conftest), which this test removes for its workers.
"""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_late_peer_is_waited_for_at_the_default_watchdog():
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.join(HERE, "skew_worker.py")]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0", SKEW_S="35")
    env.pop("MCCS_TIMEOUT_MS", None)
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=150, env=env, cwd=os.path.dirname(HERE))
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert r.returncode == 0 and lines, r.stdout[-2000:] + r.stderr[-2000:]
    res = json.loads(lines[-1])
    print(res)
    assert res["all_ok"], res
    assert res["ranks"][0]["waited_s"] >= 30, res  # rank 0 really waited past the old default
