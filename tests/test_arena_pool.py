"""The process-wide FIFO arena pool (csrc/host/comm.cpp), on the fake runtime.

Arenas are pooled by (device, memory type) instead of freed, so the library
never re-allocates a range it owns as another memory type.
Exact-size pooling kept one arena per communicator shape: a 2,000-case ring
fuzz (every case a new shape) ran one MI355X out of memory at case 876.  Now a
request rounds up to a size class and takes the smallest pooled arena of at
least that size (at most twice it), and an allocation the device refuses for
lack of memory releases the pooled uncached arenas and retries once.
"""
import ctypes

import pytest

from mccs_amd import _lib
from mccs_amd import comm as C

OOM = 2  # hipErrorOutOfMemory


@pytest.fixture
def lib(monkeypatch):
    lib = _lib.load()
    monkeypatch.setenv("MCCS_TEST_HOOKS", "1")
    monkeypatch.setenv("MCCS_GATE", "0")
    lib.mccs_test_fake_fail.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.c_int]
    lib.mccs_test_pool_waiting.restype = ctypes.c_int
    assert lib.mccs_test_fake_runtime(0) == 0
    assert lib.mccs_test_fake_runtime(2) == 0
    yield lib
    lib.mccs_test_fake_runtime(0)


def _calls(lib):
    n = lib.mccs_test_fake_calls(None, 0, 0)
    buf = ctypes.create_string_buffer(n + 1)
    lib.mccs_test_fake_calls(buf, n + 1, 1)
    return [x for x in buf.value.decode().splitlines() if x]


def _pooled(lib):
    b, e, p = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
    assert lib.mccs_test_fake_live(ctypes.byref(b), ctypes.byref(e), ctypes.byref(p)) == 0
    return p.value


def _cycle(lib, **cfg):
    """Creates and destroys a 2-rank communicator; returns the arena
    allocations it made (MallocUncached calls)."""
    _calls(lib)
    comms = C.init_all([0, 1], C.CommConfig(**cfg))
    n = _calls(lib).count("MallocUncached")
    for c in comms:
        c.destroy()
    return n


def test_nearby_shapes_share_pooled_arenas(lib):
    # ring only (no direct slots): arena = flags + channels x 2 x buffer_size
    base = dict(direct_bytes=-1, oneshot_bytes=-1, ll_bytes=-1)
    assert _cycle(lib, channel_count=4, **base) == 2
    assert _pooled(lib) == 2
    # the same shape again and a smaller one (within 2x) reuse them
    assert _cycle(lib, channel_count=4, **base) == 0
    assert _cycle(lib, channel_count=3, **base) == 0
    assert _pooled(lib) == 2
    # a much smaller shape does not pin a 4x larger arena: new allocations
    assert _cycle(lib, channel_count=1, **base) == 2
    assert _pooled(lib) == 4


def test_many_shapes_keep_the_pool_bounded(lib):
    """Sixty distinct ring shapes, created and destroyed one after another,
    leave a handful of pooled arenas, not one per shape."""
    shapes = [dict(channel_count=ch, buffer_size=bs, fifo_slots=fs, direct_bytes=-1, oneshot_bytes=-1, ll_bytes=-1)
              for ch in (1, 2, 3, 4, 5, 6) for bs in (1 << 20, 3 << 19, 1 << 21, 5 << 19, 1 << 22)
              for fs in (16, 32)]
    allocs = sum(_cycle(lib, **s) for s in shapes)
    assert allocs <= 30 and _pooled(lib) == allocs, (allocs, _pooled(lib))


def test_out_of_memory_releases_pooled_uncached_arenas(lib):
    base = dict(direct_bytes=-1, oneshot_bytes=-1, ll_bytes=-1)
    _cycle(lib, channel_count=1, **base)
    assert _pooled(lib) == 2
    # a shape no pooled arena fits, on a device that is out of memory: the
    # pooled arenas go back to the runtime and the allocation is retried
    assert lib.mccs_test_fake_fail(b"MallocUncached", 1, OOM) == 0
    _calls(lib)
    comms = C.init_all([0, 1], C.CommConfig(channel_count=6, **base))
    trace = _calls(lib)
    assert trace.count("MallocUncached") == 3, trace  # rank 0: refused, retried; rank 1
    i = trace.index("MallocUncached")
    assert "Free" in trace[i:trace.index("MallocUncached", i + 1)], trace
    assert all(c.fifo_memory == C.FIFO_UNCACHED for c in comms), "the retry must keep the uncached arena"
    assert _pooled(lib) == 1  # device 0's went back; device 1 had memory
    for c in comms:
        c.destroy()
    assert _pooled(lib) == 3


def test_arena_waits_for_every_peer_release(lib):
    """A peer's kernel may post into this rank's arena after this rank's own
    kernel ended, so a destroyed communicator's arena is reused only after
    every peer destroyed its side (each writes the tenancy's epoch into the
    arena's release word for its rank).  Until then a new communicator gets a
    fresh arena -- the destroy contract no longer rests on the caller."""
    from test_rank_per_process import _connect_per_process

    comms, _ = _connect_per_process(lib, 2)  # one rank per "process", devices 0 and 1
    comms[0].destroy()
    assert lib.mccs_test_pool_waiting() == 1  # rank 0's arena: rank 1 may still post into it
    _calls(lib)
    fresh = C.init_all([0, 1])
    assert _calls(lib).count("MallocUncached") == 2, "rank 0's unreleased arena was handed out again"
    for c in fresh:
        c.destroy()  # in-process ranks release each other
    assert lib.mccs_test_pool_waiting() == 1
    comms[1].destroy()  # rank 1 releases rank 0's arena (rank 0 released rank 1's at its own destroy)
    assert lib.mccs_test_pool_waiting() == 0
    _calls(lib)
    again = [C.init_all([0, 1]) for _ in range(2)]
    assert _calls(lib).count("MallocUncached") == 0  # all four pooled arenas are free again
    for cs in again:
        for c in cs:
            c.destroy()


def test_refused_connect_does_not_strand_the_arena(lib):
    """an arena is marked shared when SetupRank exports it, so its
    destroy pools it until every peer writes its release word -- but a peer
    writes that word only if its Connect mapped the arena.  A handle set the
    ranks refuse is refused by every rank before any IPC open, so those arenas
    go back to the pool free (a service retrying failed connects used to lose
    one arena per attempt on every rank)."""
    from test_rank_per_process import PID_OFFSET

    n = 2
    hsize = lib.mccsConnectHandleSize()
    hs, bufs = [], []
    for r in range(n):
        buf = (ctypes.c_char * hsize)()
        h = ctypes.c_void_p()
        cfg, keep = C.CommConfig().to_c(n)
        assert lib.mccsCommSetupRank(ctypes.byref(h), r, n, r, ctypes.byref(cfg), buf) == 0
        del keep
        hs.append(h)
        bufs.append(bytearray(buf))
    bufs[1][0:4] = (0x12345678).to_bytes(4, "little")  # rank 1's handle is not a connect handle
    for r in range(n):
        mine = []
        for q in range(n):
            b = bytearray(bufs[q])
            if q != r:
                b[PID_OFFSET:PID_OFFSET + 4] = (0x7ffffff0 - q).to_bytes(4, "little")
            mine.append(bytes(b))
        allh = ctypes.create_string_buffer(b"".join(mine), hsize * n)
        assert lib.mccsCommConnect(hs[r], allh) == 4  # mccsInvalidArgument, on every rank
    for h in hs:
        assert lib.mccsCommDestroy(h) == 0
    assert lib.mccs_test_pool_waiting() == 0
    _calls(lib)
    again = C.init_all([0, 1])
    assert _calls(lib).count("MallocUncached") == 0  # both arenas were reusable at once
    for c in again:
        c.destroy()


def test_exited_peer_is_not_awaited(lib):
    """a peer that crashed after connecting, or whose Connect
    failed before it mapped this rank's arena, never writes its release word,
    and the arena stayed pooled for the life of the process.  A peer of the
    same host and pid namespace that has exited (and been reaped) can no
    longer write the arena, so the pool stops awaiting it.  The fake runtime
    marks a fake peer pid exited on request."""
    from test_rank_per_process import _connect_per_process

    comms, _ = _connect_per_process(lib, 2)  # rank 0 sees rank 1 as pid 0x7ffffff0 - 1, and vice versa
    comms[0].destroy()
    assert lib.mccs_test_pool_waiting() == 1  # rank 1 is alive: its kernels may still post
    assert lib.mccs_test_fake_process_exit(0x7ffffff0 - 1) == 0
    assert lib.mccs_test_pool_waiting() == 0  # rank 1 exited: nothing can write rank 0's arena
    comms[1].destroy()  # rank 0 wrote its release into rank 1's arena at its own destroy
    assert lib.mccs_test_pool_waiting() == 0
    _calls(lib)
    again = C.init_all([0, 1])
    assert _calls(lib).count("MallocUncached") == 0  # both arenas reusable
    for c in again:
        c.destroy()


def test_failed_ipc_open_then_peer_exit(lib):
    """Rank 1's Connect fails opening rank 0's arena (after the handle check,
    so both arenas were exported and stay awaited); rank 0 connected.  Rank 1
    never mapped rank 0's arena and never writes its word: rank 0's arena is
    reusable once rank 1's process has exited, and not before."""
    from test_rank_per_process import PID_OFFSET

    n = 2
    hsize = lib.mccsConnectHandleSize()
    hs, bufs = [], []
    for r in range(n):
        buf = (ctypes.c_char * hsize)()
        h = ctypes.c_void_p()
        cfg, keep = C.CommConfig().to_c(n)
        assert lib.mccsCommSetupRank(ctypes.byref(h), r, n, r, ctypes.byref(cfg), buf) == 0
        del keep
        hs.append(h)
        bufs.append(bytearray(buf))

    def handles(r):
        out = []
        for q in range(n):
            b = bytearray(bufs[q])
            if q != r:
                b[PID_OFFSET:PID_OFFSET + 4] = (0x7ffffff0 - q).to_bytes(4, "little")
            out.append(bytes(b))
        return ctypes.create_string_buffer(b"".join(out), hsize * n)

    assert lib.mccsCommConnect(hs[0], handles(0)) == 0
    assert lib.mccs_test_fake_fail(b"IpcOpenMemHandle", 1, 1) == 0
    assert lib.mccsCommConnect(hs[1], handles(1)) != 0
    assert b"IPC open of rank 0" in lib.mccsGetLastErrorString()
    assert lib.mccsCommDestroy(hs[1]) == 0  # its arena: rank 0 mapped it and releases it at its destroy
    assert lib.mccsCommDestroy(hs[0]) == 0
    assert lib.mccs_test_pool_waiting() == 1  # rank 0's arena: rank 1 (alive) never wrote its word
    assert lib.mccs_test_fake_process_exit(0x7ffffff0 - 1) == 0
    assert lib.mccs_test_pool_waiting() == 0


def test_peer_in_another_pid_namespace_is_awaited(lib):
    """A peer pid names a process of this host only within this process's pid
    namespace: a peer whose handle carries another namespace is awaited by
    its release word alone, even if a process of that number exits here."""
    from test_rank_per_process import PID_OFFSET

    n = 2
    hsize = lib.mccsConnectHandleSize()
    hs, bufs = [], []
    for r in range(n):
        buf = (ctypes.c_char * hsize)()
        h = ctypes.c_void_p()
        cfg, keep = C.CommConfig().to_c(n)
        assert lib.mccsCommSetupRank(ctypes.byref(h), r, n, r, ctypes.byref(cfg), buf) == 0
        del keep
        hs.append(h)
        bufs.append(bytearray(buf))
    pidns = int.from_bytes(bufs[1][hsize - 8:hsize], "little")  # ConnectHandle.pidns, the last field
    assert pidns != 0, "this host exposes /proc/self/ns/pid"
    bufs[1][hsize - 8:hsize] = (pidns ^ 1).to_bytes(8, "little")  # rank 1 "in another namespace"
    for r in range(n):
        mine = []
        for q in range(n):
            b = bytearray(bufs[q])
            if q != r:
                b[PID_OFFSET:PID_OFFSET + 4] = (0x7ffffff0 - q).to_bytes(4, "little")
            mine.append(bytes(b))
        assert lib.mccsCommConnect(hs[r], ctypes.create_string_buffer(b"".join(mine), hsize * n)) == 0
    assert lib.mccsCommDestroy(hs[0]) == 0
    assert lib.mccs_test_fake_process_exit(0x7ffffff0 - 1) == 0
    assert lib.mccs_test_pool_waiting() == 1  # rank 1's pid means nothing here: wait for its word
    assert lib.mccsCommDestroy(hs[1]) == 0  # its word arrives
    assert lib.mccs_test_pool_waiting() == 0
