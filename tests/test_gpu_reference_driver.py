"""GPU: the reference-named kernels driven the way the reference host drives them.

The Rust service builds every device structure itself and calls the kernel
through collectives-sys; tests/refdrv_worker.py restates
that host side (comm/device.rs, the SHM connector's SendBufMeta/RecvBufMeta
layout, plan.rs work upload and launch_plan) with no communicator of this
library involved, and launches through mccs_hip_launch_coll with the
reference's grid (#channels) and 544-thread blocks.  One rank per process on
the one-GPU box (kernels of one process on one GPU need not run concurrently;
the reference gives each rank its own GPU), FIFO memory shared over IPC.
Results are bit-exact against the oracle, three launches in a row on the same
structures (conn->step persistence), with workFifoDone = doneAcks.
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


@pytest.mark.parametrize("world,big", [(2, False), (3, False), (3, True)], ids=["2", "3", "3-configs2-bucket"])
def test_reference_driven_launch_matches_oracle(world, big):
    """big: configs[2]'s 128 MiB fp32 bucket, random inputs, 2 and 32
    channels (grid = channels, 544 threads), bit-exact at n = 3 where the
    ring order matters (a rank-order sum differs: checked)."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.join(HERE, "refdrv_worker.py")]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0", REFDRV_BIG="1" if big else "0")
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=env, cwd=os.path.dirname(HERE))
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert r.returncode == 0 and lines, r.stdout[-3000:] + r.stderr[-3000:]
    res = json.loads(lines[-1])
    assert res["all_ok"], res
    assert res["world"] == world
