"""GPU: communicator setup is immune to HIP errors it did not cause, and
leaves none behind.

HIP keeps a per-thread last error that a failed runtime call sets and only
hipGetLastError() clears.  The library used to report hipGetLastError() as
the status of its own kernel launches (the FIFO arena's cache flush in
mccsCommSetupRank / mccsCommInitAll, the chunk reduce), so an earlier failure
anywhere on the thread -- the caller's, torch's, a handled one of the
library's -- failed setup with mccsUnhandledCudaError.  That is the cause
found for VERDICT r04's lost run (tools/stale_error_probe.py shows it on the
round-4 library: profiles/r05_stale_error_probe.json).  The CPU half of the
diagnosis is tests/test_setup_diag.py.
"""
import ctypes

import numpy as np
import pytest
import torch

from mccs_amd import _lib
from mccs_amd import comm as C

pytestmark = pytest.mark.gpu


@pytest.fixture
def hip():
    h = ctypes.CDLL("libamdhip64.so", mode=ctypes.RTLD_GLOBAL)
    h.hipGetLastError()
    yield h
    h.hipGetLastError()


def _leave_stale_error(hip):
    assert hip.hipSetDevice(9999) != 0
    assert hip.hipPeekAtLastError() != 0, "no stale error to test with"


def _clear_for_torch(hip):
    # torch checks hipGetLastError() after its own launches, so a stale error
    # fails torch's next kernel exactly as it used to fail the library's setup
    # (measured: "HIP error: invalid device ordinal" from torch.full)
    hip.hipGetLastError()


def test_stale_error_does_not_fail_setup_rank(hip):
    torch.cuda.set_device(0)
    lib = _lib.load()
    _leave_stale_error(hip)
    hsize = lib.mccsConnectHandleSize()
    buf = (ctypes.c_char * hsize)()
    h = ctypes.c_void_p()
    cfg, keep = C.CommConfig().to_c(1)
    rc = lib.mccsCommSetupRank(ctypes.byref(h), 0, 1, 0, ctypes.byref(cfg), buf)
    assert rc == 0, lib.mccsGetLastErrorString()
    assert lib.mccsCommDestroy(h) == 0


def test_stale_error_does_not_fail_init_all_or_reduce(hip):
    torch.cuda.set_device(0)
    _leave_stale_error(hip)
    comms = C.init_all([0, 0], C.CommConfig(direct_bytes=-1, oneshot_bytes=-1, ll_bytes=-1))
    _clear_for_torch(hip)
    try:
        n = 4099
        xs = [torch.full((n,), float(r + 1), device="cuda") for r in range(2)]
        ys = [torch.empty_like(x) for x in xs]
        _leave_stale_error(hip)
        with C.group():
            for r in range(2):
                C.all_reduce(comms[r], xs[r], ys[r], n, 7, 0)
        for c in comms:
            c.sync()
        _clear_for_torch(hip)
        assert all(bool((y == 3.0).all()) for y in ys)
    finally:
        for c in comms:
            c.destroy()
    import mccs_amd
    a = torch.ones(1 << 20, device="cuda")
    b = torch.full((1 << 20,), 2.0, device="cuda")
    out = torch.empty_like(a)
    _leave_stale_error(hip)
    mccs_amd.reduce(out, [a, b], dtype=mccs_amd.DataType.Float32, op=mccs_amd.RedOp.Sum)
    _clear_for_torch(hip)
    torch.cuda.synchronize()
    assert bool((out == 3.0).all())


def test_handled_failure_leaves_no_stale_error(hip):
    """A refused IPC open fails Connect with its diagnosis and leaves HIP's
    last error clear, so the caller's next checked launch (torch checks one
    after each kernel) does not inherit it."""
    torch.cuda.set_device(0)
    lib = _lib.load()
    hsize = lib.mccsConnectHandleSize()
    mine = (ctypes.c_char * hsize)()
    h = ctypes.c_void_p()
    cfg, keep = C.CommConfig().to_c(2)
    assert lib.mccsCommSetupRank(ctypes.byref(h), 0, 2, 0, ctypes.byref(cfg), mine) == 0
    peer = bytearray(bytes(mine))
    peer[4:8] = (1).to_bytes(4, "little")  # rank 1
    peer[16:20] = (0x7ffffff0).to_bytes(4, "little")  # another pid
    peer[56:120] = bytes(64)  # an IPC handle that names nothing
    hip.hipGetLastError()
    rc = lib.mccsCommConnect(h, bytes(mine) + bytes(peer))
    err = lib.mccsGetLastErrorString().decode()
    assert rc != 0 and "IPC open of rank 1's arena: IpcOpenMemHandle -> hip" in err, (rc, err)
    assert hip.hipPeekAtLastError() == 0, "the library left its handled failure on the thread"
    assert lib.mccsCommDestroy(h) == 0
    x = torch.arange(1000, device="cuda", dtype=torch.float32)
    assert float((x * 2).sum()) == float(np.arange(1000).sum() * 2)
