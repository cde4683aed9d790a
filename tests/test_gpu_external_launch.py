"""mccs_hip_launch_coll (the external-planner launch, plan.rs:638-669) with two
ranks of ONE GPU in ONE process: the second rank's launch is refused while the
first is still running (the two kernels spin on each other's flags, so
separate launches of co-located ranks would deadlock until the watchdog).
The running kernel is then ended through its abortFlag (mccsCommAbort)."""
import ctypes
import time

import numpy as np
import pytest

from mccs_amd import _lib
from mccs_amd import abi
from mccs_amd import comm as C

pytestmark = pytest.mark.gpu

FUNC_ALLREDUCE, F32 = 4, 7
INVALID_USAGE = 5  # mccsInvalidUsage


def _works(nch, send, recv, count, nthr):
    works = (abi.mccsDevWork * nch)()
    for c in range(nch):
        w = works[c]
        e = w.elems[0]
        e.isUsed, e.nWarps = 1, nthr // 32
        e.sendbuff, e.recvbuff, e.count = send, recv, count
        e.bid, e.nChannels = c, nch
        w.header.type = 1  # mccsDevWorkTypeColl
        w.header.isLast, w.header.inFifo, w.header.doneAcks = 1, 0, 0
    return works


@pytest.fixture(autouse=True)
def _ref_watchdog():
    """The reference-named kernels' watchdog defaults to 10 min (no late
    peer may trip it in a deployment); a hang here should end in 30 s."""
    lib = _lib.load()
    assert lib.mccs_hip_set_ref_watchdog(30000) == 0
    yield
    lib.mccs_hip_set_ref_watchdog(30000)


def test_ref_watchdog_is_settable():
    """mccs_hip_set_ref_watchdog governs the reference-named kernels: a rank
    launched without its peer gives up after the set 300 ms (abortFlag
    raised, the kernel ends), and 0 restores the 10 min default."""
    import torch

    lib = _lib.load()
    comms = C.init_all([0, 0], C.CommConfig(lanes=1, fifo_slots=8))
    try:
        nch, nthr, count = comms[0].nchannels, 544, 1 << 16
        x, y = torch.ones(count, device="cuda"), torch.zeros(count, device="cuda")
        wb = torch.frombuffer(bytearray(bytes(_works(nch, x.data_ptr(), y.data_ptr(), count, nthr))),
                              dtype=torch.uint8).cuda()
        torch.cuda.synchronize()
        assert lib.mccs_hip_set_ref_watchdog(300) == 0
        st = torch.cuda.Stream()
        t0 = time.perf_counter()
        assert lib.mccs_hip_launch_coll(FUNC_ALLREDUCE, F32, 0, comms[0].dev_comm(), (1 << nch) - 1, wb.data_ptr(),
                                        nch, nthr, st.cuda_stream) == 0
        st.synchronize()  # no peer ever runs: only the watchdog ends it
        waited = time.perf_counter() - t0
        assert 0.25 < waited < 10, waited
        with pytest.raises(_lib.MccsError, match="abortFlag 1"):
            comms[0].sync()
        assert lib.mccs_hip_set_ref_watchdog(0) == 0 and lib.mccs_hip_set_ref_watchdog(-1) == 0
    finally:
        torch.cuda.synchronize()
        for c in comms:
            c.destroy()


def test_colocated_external_launch_refused_while_peer_runs():
    import torch

    lib = _lib.load()
    f = lib.mccs_hip_launch_coll
    f.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p,
                  ctypes.c_uint, ctypes.c_uint, ctypes.c_void_p]
    f.restype = ctypes.c_int
    comms = C.init_all([0, 0], C.CommConfig(lanes=1, timeout_ms=20000, fifo_slots=8))
    try:
        nch, nthr, count = comms[0].nchannels, 544, 1 << 20
        xs = [torch.ones(count, device="cuda") for _ in range(2)]
        ys = [torch.zeros(count, device="cuda") for _ in range(2)]
        wbufs = [torch.frombuffer(bytearray(bytes(_works(nch, xs[r].data_ptr(), ys[r].data_ptr(), count, nthr))),
                                  dtype=torch.uint8).cuda() for r in range(2)]
        st = torch.cuda.Stream()  # non-blocking: the abort below must not wait for the kernel
        torch.cuda.synchronize()
        rc0 = f(FUNC_ALLREDUCE, F32, 0, comms[0].dev_comm(), (1 << nch) - 1, wbufs[0].data_ptr(), nch, nthr,
                st.cuda_stream)
        assert rc0 == 0
        time.sleep(0.05)  # rank 0 now spins on rank 1's flags
        rc1 = f(FUNC_ALLREDUCE, F32, 0, comms[1].dev_comm(), (1 << nch) - 1, wbufs[1].data_ptr(), nch, nthr,
                st.cuda_stream)
        assert rc1 == INVALID_USAGE, rc1
        comms[0].abort()  # raises rank 0's abortFlag: its control waves end the kernel
        t0 = time.perf_counter()
        st.synchronize()
        assert time.perf_counter() - t0 < 10, "the aborted kernel did not end promptly"
        assert np.all(ys[0].cpu().numpy() != 2.0)  # never completed: no peer
        with pytest.raises(_lib.MccsError):
            comms[0].sync()  # the aborted communicator reports its failure ...
    finally:
        torch.cuda.synchronize()
        for c in comms:
            c.destroy()
    # ... and only that one: error bits live in each communicator's own abort
    # line, so a fresh communicator in the same process syncs clean (a
    # process-wide error word once failed the next test's first AllReduce)
    import vnode

    fresh = C.init_all([0, 0])
    try:
        outs = vnode.run_allreduce(fresh, [np.ones(4096, np.float32)] * 2, F32, 0)
        assert all(np.all(o == 2.0) for o in outs)
    finally:
        vnode.destroy(fresh)


def test_external_launch_refuses_a_deeper_fifo_communicator():
    """The reference-named kernels index the reference's 8 FIFO slots; a
    library communicator built with 16 (the default) is refused before
    anything is launched (its peers would index another slot ring)."""
    import torch

    lib = _lib.load()
    comms = C.init_all([0, 0], C.CommConfig(lanes=1))
    try:
        nch, nthr, count = comms[0].nchannels, 544, 1 << 10
        x, y = torch.ones(count, device="cuda"), torch.zeros(count, device="cuda")
        wb = torch.frombuffer(bytearray(bytes(_works(nch, x.data_ptr(), y.data_ptr(), count, nthr))),
                              dtype=torch.uint8).cuda()
        rc = lib.mccs_hip_launch_coll(FUNC_ALLREDUCE, F32, 0, comms[0].dev_comm(), (1 << nch) - 1, wb.data_ptr(), nch,
                                      nthr, torch.cuda.current_stream().cuda_stream)
        assert rc == INVALID_USAGE, rc
        torch.cuda.synchronize()
        assert torch.all(y == 0)
    finally:
        for c in comms:
            c.destroy()
