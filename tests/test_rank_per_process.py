"""The N > 1 bench's path on a node, on CPU: one rank per process, each on its
own GPU (mccsCommSetupRank + handle exchange + mccsCommConnect, what every
torchrun rank of the driver's SCALE run executes).

No run of this repo has had two GPUs, so the branches Connect takes only for
peers on other devices -- peer access to each of them, no co-residency lane
shrink, peer atomics looked up by PCI bus id, no vote without the gate -- ran
nowhere.  These tests install the recording fake device runtime (host memory,
no kernels: csrc/host/rt.cpp) with one fake GPU per rank, relabel every other
rank's handle as another process's (the fake maps IPC inside this one), and
check what a node would get: the same channels, lanes and rings as the
one-process path (mccsCommInitAll, the reference's service model), and every
FIFO connection wired end to end -- the buffer, tail and head a rank writes
for its ring successor are the ones that successor reads (the reference's
SHM connector pairing, transport/shm/transporter.rs:87-183,278-365).
"""
import ctypes

import pytest

from mccs_amd import _lib
from mccs_amd import abi
from mccs_amd import comm as C

DIRECT_DEFAULTS = True  # conftest: keep the library's routing defaults here
PID_OFFSET = 16  # ConnectHandle: magic, rank, nranks, device, pid (comm.h)
F32, SUM = 7, 0


@pytest.fixture
def lib(monkeypatch):
    lib = _lib.load()
    monkeypatch.setenv("MCCS_TEST_HOOKS", "1")
    # the fake runs no kernel, so the gate's sums could never match
    # (tests/test_gate_host.py covers the gate's host logic)
    monkeypatch.setenv("MCCS_GATE", "0")
    lib.mccs_test_fake_fail.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.c_int]
    yield lib
    lib.mccs_test_fake_runtime(0)


def _fresh(lib, ndev):
    assert lib.mccs_test_fake_runtime(0) == 0
    assert lib.mccs_test_fake_runtime(ndev) == 0


def _log(lib):
    n = lib.mccs_test_fake_log(None, 0, 0)
    buf = ctypes.create_string_buffer(n + 1)
    lib.mccs_test_fake_log(buf, n + 1, 1)
    out = []
    for line in buf.value.decode().splitlines():
        kind, *kv = line.split()
        out.append((kind, dict(x.split("=", 1) for x in kv)))
    return out


def _connect_per_process(lib, n, config=None, devices=None):
    """Every rank set up on its own fake device, then connected with the
    others' handles marked as other processes'.  Returns (comms, per-rank
    fake log of its Connect)."""
    devices = devices or list(range(n))
    hsize = lib.mccsConnectHandleSize()
    hs, bufs = [], []
    for r in range(n):
        buf = (ctypes.c_char * hsize)()
        h = ctypes.c_void_p()
        cfg, keep = (config or C.CommConfig()).to_c(n)
        rc = lib.mccsCommSetupRank(ctypes.byref(h), r, n, devices[r], ctypes.byref(cfg), buf)
        del keep
        assert rc == 0, lib.mccsGetLastErrorString()
        hs.append(h)
        bufs.append(bytearray(buf))
    _log(lib)
    logs = []
    for r in range(n):
        mine = []
        for q in range(n):
            b = bytearray(bufs[q])
            if q != r:
                b[PID_OFFSET:PID_OFFSET + 4] = (0x7ffffff0 - q).to_bytes(4, "little")
            mine.append(bytes(b))
        allh = ctypes.create_string_buffer(b"".join(mine), hsize * n)
        rc = lib.mccsCommConnect(hs[r], allh)
        assert rc == 0, (r, lib.mccsGetLastErrorString())
        logs.append(_log(lib))
    comms = [C.Communicator(h.value) for h in hs]
    for c in comms:
        c._load_info()
    return comms, logs


def _views(c):
    """Per channel: (recv buffer, send buffer, recv tail, recv head, send head,
    send tail) -- the connector view the kernels load (ring_cfg.h)."""
    base = c.dev_comm()
    views = (ctypes.c_void_p * (6 * abi.MCCS_MAX_NCHANNELS)).from_address(
        base + ctypes.sizeof(abi.mccsDevCommAndChannels))
    return [tuple(views[6 * ch:6 * ch + 6]) for ch in range(c.nchannels)]


def _check_wiring(comms):
    """A rank's send side on channel ch is its ring successor's receive side:
    same FIFO buffer, same tail (sender posts, receiver polls), same head
    (receiver returns credits, sender polls)."""
    n = len(comms)
    rings = comms[0].rings()
    assert all(c.rings() == rings for c in comms), "ranks disagree on the rings"
    views = [_views(c) for c in comms]
    for ch, ring in enumerate(rings):
        assert sorted(ring) == list(range(n))
        for i, a in enumerate(ring):
            b = ring[(i + 1) % n]
            ra, sa = views[a][ch], views[b][ch]
            assert all(ra) and all(sa), (ch, a)
            assert ra[1] == sa[0], f"channel {ch}: rank {a} sends into a buffer rank {b} does not read"
            assert ra[5] == sa[2], f"channel {ch}: rank {a} posts a tail rank {b} does not poll"
            assert ra[4] == sa[3], f"channel {ch}: rank {b} returns credits rank {a} does not poll"


@pytest.mark.parametrize("n", [2, 4, 8])
def test_rank_per_gpu_matches_the_one_process_path(lib, n):
    """Channels, lanes and rings equal mccsCommInitAll's over the same
    devices (no co-residency shrink on distinct GPUs), and every connection
    is wired end to end."""
    _fresh(lib, n)
    ref = C.init_all(list(range(n)), C.CommConfig())
    want = [(c.nchannels, c.lanes, c.block_threads, c.rings()) for c in ref]
    _check_wiring(ref)
    for c in ref:
        c.destroy()
    comms, logs = _connect_per_process(lib, n)
    try:
        assert [(c.nchannels, c.lanes, c.block_threads, c.rings()) for c in comms] == want
        _check_wiring(comms)
        for r, ev in enumerate(logs):
            # peer access from this rank's GPU to every other rank's
            peers = {int(kv["peer"]) for k, kv in ev if k == "peer" and int(kv["dev"]) == r}
            assert peers == set(range(n)) - {r}, (r, ev)
            # no gate ran, so no vote: the count-based direct variants stay off
            # on distinct GPUs (every rank must route a bucket alike)
            assert not comms[r].direct_enabled()
            assert comms[r].gate_info()["ran"] is False
    finally:
        for c in comms:
            c.destroy()
    blocks, events, pooled = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
    lib.mccs_test_fake_live(ctypes.byref(blocks), ctypes.byref(events), ctypes.byref(pooled))
    assert blocks.value == pooled.value and events.value == 0, "destroy left more than the pooled arenas"


@pytest.mark.parametrize("locality", [C.LOCALITY_RECEIVER, C.LOCALITY_SENDER])
def test_rank_per_gpu_wiring_either_locality(lib, locality):
    """The FIFO at the receiver (default) or at the sender (the reference SHM
    default): wired end to end either way."""
    _fresh(lib, 4)
    comms, _ = _connect_per_process(lib, 4, C.CommConfig(locality=locality))
    try:
        _check_wiring(comms)
    finally:
        for c in comms:
            c.destroy()


def test_rank_per_gpu_launch_stays_on_its_device(lib):
    """Each process launches its own rank on its own GPU: one ring launch per
    rank, grid = channels x lanes, every communicator of it on that device,
    the works in the launch arguments, no host wait before the launch."""
    _fresh(lib, 8)
    comms, _ = _connect_per_process(lib, 8)
    try:
        for r, c in enumerate(comms):
            C.all_reduce(c, 0x10000000 * (r + 1), 0x10000000 * (r + 1) + 0x8000000, 1 << 20, F32, SUM, stream=0)
            ev = _log(lib)
            launches = [kv for k, kv in ev if k == "launch"]
            assert len(launches) == 1, ev
            kv = launches[0]
            assert int(kv["dev"]) == r and kv["comms_on_dev"] == "1" and kv["kind"] == "ring"
            assert kv["grid"] == f"{c.nchannels * c.lanes}x1"
            assert kv["inline_works"] == str(c.nchannels)
            assert not any(k == "host_wait" for k, _ in ev)
            assert c.last_algo() == "ring"
    finally:
        for c in comms:
            c.destroy()


def _algo(comms, count):
    out = []
    for r, c in enumerate(comms):
        C.all_reduce(c, 0x10000000 * (r + 1), 0x10000000 * (r + 1) + 0x8000000, count, F32, SUM, stream=0)
        out.append(c.last_algo())
    return out


def test_rank_per_gpu_counted_variants_need_the_vote(lib):
    """Routing on distinct GPUs without the gate (MCCS_GATE=0): the LL
    one-shot makes no remote atomics and every rank decides it alike from the
    handles (same ll_bytes, every arena uncached), so 16 KiB still takes it;
    a 1 MiB bucket, one-shot-sized at n = 2, takes the ring, because the
    count-based variants need peer atomics that only the vote confirms on
    every rank.  Processes sharing one GPU need no vote: the one-shot runs."""
    _fresh(lib, 2)
    comms, _ = _connect_per_process(lib, 2)
    try:
        assert _algo(comms, 4 << 10) == ["ll", "ll"]
        assert _algo(comms, 256 << 10) == ["ring", "ring"]
    finally:
        for c in comms:
            c.destroy()
    _fresh(lib, 1)
    comms, _ = _connect_per_process(lib, 2, devices=[0, 0])
    try:
        assert _algo(comms, 4 << 10) == ["ll", "ll"]
        assert _algo(comms, 256 << 10) == ["oneshot", "oneshot"]
    finally:
        for c in comms:
            c.destroy()


def test_one_rank_on_a_device_arena_moves_every_rank(lib):
    """A rank whose uncached arena cannot be exported falls back to a plain
    device arena (system fences).  Its peers learn it from its handle, so
    every rank runs the same hand-off and none takes the LL one-shot (its
    polled lines need uncached arenas on both ends): a rank that routed
    alone would leave its peers waiting in another kernel."""
    _fresh(lib, 4)
    assert lib.mccs_test_fake_fail(b"IpcGetMemHandle", 3, 1) == 0  # rank 2's export
    comms, _ = _connect_per_process(lib, 4)
    try:
        assert [c.fifo_memory for c in comms] == [C.FIFO_DEVICE] * 4
        _check_wiring(comms)
        assert _algo(comms, 4 << 10) == ["ring"] * 4
    finally:
        for c in comms:
            c.destroy()
