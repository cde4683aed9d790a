"""GPU: a peer process that exits without destroying its communicator.

Each rank's FIFO arena is pooled at destroy until every peer wrote its
release word (a peer's kernel may post into it after this rank's ended).  A
peer that crashed never writes it; the pool then waits for the peer's exit
instead (csrc/host/comm.cpp pool_refresh: same host and pid namespace, the
process reaped).  Here rank 1 is a child process on the same GPU that
connects and exits without a destroy; rank 0 (this process) destroys, sees its
arena awaited while the child lives, and reusable once the child is reaped.
"""
import ctypes
import os
import subprocess
import sys

import pytest

from mccs_amd import _lib
from mccs_amd import comm as C

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import ctypes, sys
sys.path.insert(0, sys.argv[1])
from mccs_amd import _lib
from mccs_amd import comm as C
lib = _lib.load()
hsize = lib.mccsConnectHandleSize()
mine = (ctypes.c_char * hsize)()
h = ctypes.c_void_p()
cfg, keep = C.CommConfig().to_c(2)
assert lib.mccsCommSetupRank(ctypes.byref(h), 1, 2, 0, ctypes.byref(cfg), mine) == 0
sys.stdout.write(bytes(mine).hex() + "\n"); sys.stdout.flush()
peer = bytes.fromhex(sys.stdin.readline().strip())
rc = lib.mccsCommConnect(h, ctypes.create_string_buffer(peer + bytes(mine), 2 * hsize))
sys.stdout.write(f"connected {rc}\n"); sys.stdout.flush()
sys.stdin.readline()  # rank 0 destroyed its side: exit without a destroy (a crash)
import os; os._exit(0)
"""


def test_exited_peer_releases_the_arena():
    import torch

    torch.cuda.set_device(0)
    lib = _lib.load()
    lib.mccs_test_pool_waiting.restype = ctypes.c_int
    env = dict(os.environ, MCCS_GATE="0", HSA_ENABLE_IPC_MODE_LEGACY="0")
    os.environ["MCCS_GATE"] = "0"  # no node-gate collective: the child never runs one
    child = subprocess.Popen([sys.executable, "-c", CHILD, ROOT], stdin=subprocess.PIPE, stdout=subprocess.PIPE,
                             env=env, text=True)
    try:
        theirs = bytes.fromhex(child.stdout.readline().strip())
        hsize = lib.mccsConnectHandleSize()
        assert len(theirs) == hsize
        mine = (ctypes.c_char * hsize)()
        h = ctypes.c_void_p()
        cfg, keep = C.CommConfig().to_c(2)
        assert lib.mccsCommSetupRank(ctypes.byref(h), 0, 2, 0, ctypes.byref(cfg), mine) == 0
        child.stdin.write(bytes(mine).hex() + "\n")
        child.stdin.flush()
        assert lib.mccsCommConnect(h, ctypes.create_string_buffer(bytes(mine) + theirs, 2 * hsize)) == 0, \
            lib.mccsGetLastErrorString()
        assert child.stdout.readline().strip() == "connected 0"
        before = lib.mccs_test_pool_waiting()
        assert lib.mccsCommDestroy(h) == 0
        assert lib.mccs_test_pool_waiting() == before + 1  # the child is alive: its kernels could still post
        child.stdin.write("exit\n")
        child.stdin.flush()
        assert child.wait(timeout=60) == 0  # reaped
        assert lib.mccs_test_pool_waiting() == before  # exited: nothing can write the arena any more
    finally:
        os.environ.pop("MCCS_GATE", None)
        if child.poll() is None:
            child.kill()
            child.wait()
