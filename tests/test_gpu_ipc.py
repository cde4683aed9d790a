"""GPU: ring AllReduce across processes through IPC-mapped FIFO arenas.

Two and four ranks in as many processes (tests/ipc_worker.py under
torch.distributed.run), all on cuda:0 of the one-GPU box: exercises
hipIpcGetMemHandle / hipIpcOpenMemHandle, the two-phase connect and
cross-process flag hand-offs in both FIFO memory kinds and both data
placements, bit for bit against the oracle.
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


@pytest.mark.parametrize("world,modes", [(2, "uncached,device,sender-uncached,sender-device,release,sender-release"),
                                         (4, "uncached,sender-uncached"), (2, "direct,oneshot"),
                                         (3, "direct,oneshot,ll"), (4, "direct,oneshot,ll"), (2, "ll")])
def test_multi_process_ring_matches_oracle(world, modes):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.join(HERE, "ipc_worker.py")]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0", IPC_MODES=modes)
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=env, cwd=os.path.dirname(HERE))
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    # the library's own log lines first (a rank's setup error is otherwise cut
    # off by the launcher's long tail)
    lib_lines = "\n".join(l for l in (r.stdout + r.stderr).splitlines() if "mccs" in l.lower() or "hip" in l)[-3000:]
    assert r.returncode == 0 and lines, lib_lines + "\n----\n" + r.stdout[-2000:] + r.stderr[-2000:]
    res = json.loads(lines[-1])
    assert res["all_ok"], res
    assert res["world"] == world
