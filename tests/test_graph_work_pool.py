"""Graph work arena reuse, on the fake runtime (CPU).

Launches captured into a HIP graph keep their work lists in the comm's
graph work arena (2048 entries), since a graph replays the same arguments
forever.  Until round 5 the entries were never returned, so a process that
captured graphs again and again (a server re-capturing per batch shape)
exhausted the arena and could capture no more collectives on that comm.  Now
each captured launch holds a contiguous range that returns when its graph is
destroyed (a HIP user object the graph retains, rt().GraphOnDestroy).  The
fake runtime lets a stream "capture" into a numbered graph and "destroys"
graphs on request (mccs_test_fake_capture / mccs_test_fake_destroy_graph);
tests/test_gpu_ring.py checks the same on the GPU, including that an
executable graph keeps its range after torch destroys the captured graph.
"""
import ctypes

import pytest

from mccs_amd import _lib
from mccs_amd import comm as C

F32, SUM = 7, 0
STREAM = 0x5000  # a fake stream handle


@pytest.fixture
def lib(monkeypatch):
    lib = _lib.load()
    monkeypatch.setenv("MCCS_TEST_HOOKS", "1")
    monkeypatch.setenv("MCCS_GATE", "0")
    monkeypatch.setenv("MCCS_INLINE_WORKS", "0")  # every launch's works go through an arena
    lib.mccs_test_fake_capture.argtypes = [ctypes.c_void_p, ctypes.c_int]
    lib.mccs_test_fake_destroy_graph.argtypes = [ctypes.c_int]
    assert lib.mccs_test_fake_runtime(0) == 0
    assert lib.mccs_test_fake_runtime(2) == 0
    yield lib
    lib.mccs_test_fake_capture(STREAM, 0)
    lib.mccs_test_fake_runtime(0)


def _capture_until_full(lib, comms, graph, limit=10000):
    """Captures AllReduces into `graph` until the arena refuses one; returns
    how many were captured."""
    lib.mccs_test_fake_capture(STREAM, graph)
    k = 0
    try:
        while k < limit:
            with C.group():
                for r, c in enumerate(comms):
                    C.all_reduce(c, 0x10000000 * (r + 1), 0x10000000 * (r + 1) + 0x8000000, 64 << 20, F32, SUM,
                                 stream=STREAM)
            k += 1
    except _lib.MccsError as e:
        assert "graph work arena exhausted" in str(e), e
    finally:
        lib.mccs_test_fake_capture(STREAM, 0)
    return k


def _capture(lib, comms, graph, k):
    lib.mccs_test_fake_capture(STREAM, graph)
    try:
        for _ in range(k):
            with C.group():
                for r, c in enumerate(comms):
                    C.all_reduce(c, 0x10000000 * (r + 1), 0x10000000 * (r + 1) + 0x8000000, 64 << 20, F32, SUM,
                                 stream=STREAM)
    finally:
        lib.mccs_test_fake_capture(STREAM, 0)


def test_destroyed_graphs_return_their_work_entries(lib):
    comms = C.init_all([0, 1], C.CommConfig(buffer_size=1 << 20))
    try:
        per_launch = comms[0].nchannels  # one work per channel at 64 MiB
        full = _capture_until_full(lib, comms, 1)
        assert full == 2048 // per_launch, (full, per_launch)
        # every captured launch registered one release per comm
        assert lib.mccs_test_fake_destroy_graph(1) == 2 * full
        # the arena is whole again: as many captures fit as the first time
        assert _capture_until_full(lib, comms, 2) == full
        assert lib.mccs_test_fake_destroy_graph(2) == 2 * full
        # eager launches are unaffected throughout
        with C.group():
            for r, c in enumerate(comms):
                C.all_reduce(c, 0x10000000 * (r + 1), 0x10000000 * (r + 1) + 0x8000000, 1 << 20, F32, SUM, stream=0)
    finally:
        for c in comms:
            c.destroy()


def _capture_group(lib, comms, graph, m):
    """One launch of m grouped AllReduces per comm: ceil(m / 10) chained works
    per channel (MCCS_MAX_WORK_ELEMENTS = 10)."""
    lib.mccs_test_fake_capture(STREAM, graph)
    try:
        with C.group():
            for _ in range(m):
                for r, c in enumerate(comms):
                    C.all_reduce(c, 0x10000000 * (r + 1), 0x10000000 * (r + 1) + 0x8000000, 64 << 20, F32, SUM,
                                 stream=STREAM)
    finally:
        lib.mccs_test_fake_capture(STREAM, 0)


def test_released_ranges_coalesce(lib):
    """The arena filled one-work-per-channel launch at a time; a launch of
    two chained works per channel needs twice that contiguously, which only
    the released ranges of a destroyed graph, merged, provide."""
    comms = C.init_all([0, 1], C.CommConfig(buffer_size=1 << 20))
    try:
        q = 2048 // comms[0].nchannels // 4
        _capture(lib, comms, 1, q)
        _capture(lib, comms, 2, q)
        _capture_until_full(lib, comms, 3)
        with pytest.raises(_lib.MccsError, match="graph work arena exhausted"):
            _capture_group(lib, comms, 4, 12)
        assert lib.mccs_test_fake_destroy_graph(2) == 2 * q
        _capture_group(lib, comms, 5, 12)
    finally:
        for g in range(1, 6):
            lib.mccs_test_fake_destroy_graph(g)
        for c in comms:
            c.destroy()


def test_graph_outliving_its_comm(lib):
    """A graph destroyed after its communicator: the release runs against the
    shared pool, not the freed comm."""
    comms = C.init_all([0, 1], C.CommConfig(buffer_size=1 << 20))
    _capture(lib, comms, 1, 3)
    for c in comms:
        c.destroy()
    assert lib.mccs_test_fake_destroy_graph(1) == 6
