"""The one-process multi-GPU path on CPU.

The reference deploys one service process that drives every GPU of the node
(src/mccs/src/transport/shm/transporter.rs:76-78; launches per device in
src/mccs/src/proxy/plan.rs:638-669).  Here that path is mccsCommInitAll over
distinct devices + a grouped collective + mccsCommSync.  Its hazard is the
deadlock class DESIGN.md records for ranks launched separately: ring blocks of
different ranks spin on each other's flags, so every rank's kernel must be in
flight before the host waits on any of them, and ranks sharing a GPU must be
one launch.  These tests install the recording fake device runtime
(csrc/host/rt.cpp, mccs_test_fake_runtime: host memory, no kernels run) with
8 devices and check the order of launches, stream waits and host waits the
library issues.
"""
import ctypes

import pytest

from mccs_amd import _lib
from mccs_amd import comm as C

F32, SUM = 7, 0


def _parse(line):
    kind, *kv = line.split()
    return kind, dict(x.split("=", 1) for x in kv)


@pytest.fixture
def fake(monkeypatch):
    lib = _lib.load()
    monkeypatch.setenv("MCCS_TEST_HOOKS", "1")  # the hook is refused without it
    # the fake runs no kernel, so the node gate's sums would never match:
    # these tests look at launches (tests/test_gate_host.py covers the gate)
    monkeypatch.setenv("MCCS_GATE", "0")

    def install(ndev):
        assert lib.mccs_test_fake_runtime(ndev) == 0

    yield install
    lib.mccs_test_fake_runtime(0)


def test_fake_runtime_hook_is_refused_without_opt_in(monkeypatch):
    monkeypatch.delenv("MCCS_TEST_HOOKS", raising=False)
    assert _lib.load().mccs_test_fake_runtime(4) == 5  # mccsInvalidUsage: HIP stays installed


def _log(clear=True):
    lib = _lib.load()
    n = lib.mccs_test_fake_log(None, 0, 0)
    assert n >= 0, "fake runtime not installed"
    buf = ctypes.create_string_buffer(n + 1)
    lib.mccs_test_fake_log(buf, n + 1, 1 if clear else 0)
    return [_parse(x) for x in buf.value.decode().splitlines() if x]


def _allreduce_group(comms, count=1 << 20):
    with C.group():
        for r, c in enumerate(comms):
            # "device" buffers are never touched by the fake; distinct fake addresses
            C.all_reduce(c, 0x10000000 * (r + 1), 0x10000000 * (r + 1) + 0x8000000, count, F32, SUM, stream=0)


def _check_launch_phase(ev, ndev, ranks_per_dev, lanes_x_ch):
    launches = [(i, kv) for i, (k, kv) in enumerate(ev) if k == "launch"]
    assert sorted(int(kv["dev"]) for _, kv in launches) == list(range(ndev)), ev
    for _, kv in launches:
        gx, gy = (int(v) for v in kv["grid"].split("x"))
        assert gy == ranks_per_dev and gx == lanes_x_ch
        assert kv["comms_on_dev"] == "1", "a fused launch carries a communicator of another device"
    last = max(i for i, _ in launches)
    waits = [i for i, (k, _) in enumerate(ev) if k == "host_wait"]
    assert not waits or min(waits) > last, f"host waited before every rank was launched: {ev}"
    for k, kv in ev:
        if k == "stream_wait":
            assert kv["event_dev"] == kv["dev"], f"cross-device stream dependency between launches: {kv}"
    return launches


def test_init_all_eight_devices_one_launch_per_device(fake):
    fake(8)
    comms = C.init_all(list(range(8)), C.CommConfig(buffer_size=1 << 20))
    try:
        ev = _log()
        # every device can reach every other device's FIFO arena
        peers = {(int(kv["dev"]), int(kv["peer"])) for k, kv in ev if k == "peer"}
        assert peers == {(a, b) for a in range(8) for b in range(8) if a != b}
        lanes, nch = comms[0].lanes, comms[0].nchannels
        assert nch == 7 and lanes == 9  # 7 arc-disjoint directed Hamiltonian cycles: all 7 links per GPU
        _allreduce_group(comms)
        ev = _log()
        launches = _check_launch_phase(ev, 8, 1, nch * lanes)
        assert len(launches) == 8
        # one work per ring: the 7 works travel in the launch arguments
        assert all(kv["inline_works"] == "7" for _, kv in launches), launches
        for c in comms:
            c.sync()
        ev = _log()
        assert [k for k, _ in ev if k == "launch"] == []
        assert {int(kv["dev"]) for k, kv in ev if k == "host_wait"} == set(range(8))
    finally:
        for c in comms:
            c.destroy()


def test_back_to_back_groups_issue_without_host_waits(fake):
    fake(8)
    comms = C.init_all(list(range(8)), C.CommConfig(buffer_size=1 << 20))
    try:
        _log()
        for _ in range(3):
            _allreduce_group(comms)
        ev = _log()
        assert sum(1 for k, _ in ev if k == "launch") == 24
        assert not any(k == "host_wait" for k, _ in ev), "stream-ordered collectives made the host wait"
    finally:
        for c in comms:
            c.destroy()


@pytest.mark.parametrize("n,nch,lanes", [(2, 4, 32), (4, 6, 10), (8, 7, 9)])
def test_default_channels_and_lanes(fake, n, nch, lanes):
    """One rank per device: n = 2 runs 4 channels of its ring x 32 lanes
    (128 workgroups), n = 4 its 6 directed rings x 10, n = 8 its 7
    arc-disjoint rings x 9 (lanes)."""
    fake(n)
    comms = C.init_all(list(range(n)), C.CommConfig())
    try:
        assert [(c.nchannels, c.lanes) for c in comms] == [(nch, lanes)] * n
    finally:
        for c in comms:
            c.destroy()


@pytest.mark.parametrize("n", [2, 3, 8])
def test_connector_views_match_the_peers(fake, n):
    """The per-channel connector views communicator launches load
    (ring_cfg.h mccsRingConnView, right after mccsDevCommAndChannels in the
    device communicator's allocation) hold exactly the prev-recv / next-send
    mccsDevConnInfo addresses the reference-named kernels read through
    mccsDevChannel.peers (the fake runtime keeps device memory in host RAM)."""
    from mccs_amd import abi

    fake(n)
    comms = C.init_all(list(range(n)), C.CommConfig())
    try:
        for c in comms:
            base = c.dev_comm()
            dc = abi.mccsDevCommAndChannels.from_address(base)
            views = (ctypes.c_void_p * (6 * abi.MCCS_MAX_NCHANNELS)).from_address(
                base + ctypes.sizeof(abi.mccsDevCommAndChannels))
            for ch in range(c.nchannels):
                chan = dc.channels[ch]
                peers = (abi.mccsDevChannelPeer * n).from_address(chan.peers)
                r = peers[chan.ring.prev].recv[0]
                s = peers[chan.ring.next].send[0]
                want = [r.buffs[0], s.buffs[0], r.tail, r.head, s.head, s.tail]
                assert list(views[6 * ch:6 * ch + 6]) == want and all(want), (c.rank, ch)
    finally:
        for c in comms:
            c.destroy()


def test_work_list_falls_back_to_the_fifo(fake, monkeypatch):
    """Works go through the reference's work FIFO when they do not fit the
    launch arguments: several collectives of a group on one channel (chained
    works, or one work of several elements), or MCCS_INLINE_WORKS=0."""
    fake(8)
    comms = C.init_all(list(range(8)), C.CommConfig(buffer_size=1 << 20))
    try:
        _log()
        with C.group():
            # 12 grouped 4 MiB AllReduces, each on all 7 channels: 12 elements per
            # channel = 2 chained works (MCCS_MAX_WORK_ELEMENTS = 10 per work)
            for _ in range(12):
                for r, c in enumerate(comms):
                    C.all_reduce(c, 0x10000000 * (r + 1), 0x10000000 * (r + 1) + 0x8000000, 1 << 20, F32, SUM,
                                 stream=0)
        launches = [kv for k, kv in _log() if k == "launch"]
        assert len(launches) == 8 and all(kv["inline_works"] == "0" for kv in launches), launches
        # two grouped AllReduces: one work per channel, but of two elements; an
        # inline work carries its header and ONE element (ring_cfg.h mccsInlineWork)
        with C.group():
            for _ in range(2):
                for r, c in enumerate(comms):
                    C.all_reduce(c, 0x10000000 * (r + 1), 0x10000000 * (r + 1) + 0x8000000, 1 << 20, F32, SUM,
                                 stream=0)
        launches = [kv for k, kv in _log() if k == "launch"]
        assert len(launches) == 8 and all(kv["inline_works"] == "0" for kv in launches), launches
        # MCCS_INLINE_WORKS=0 is read when a communicator is created
        monkeypatch.setenv("MCCS_INLINE_WORKS", "0")
        off = C.init_all(list(range(8)), C.CommConfig(buffer_size=1 << 20))
        _log()
        _allreduce_group(off)
        launches = [kv for k, kv in _log() if k == "launch"]
        assert len(launches) == 8 and all(kv["inline_works"] == "0" for kv in launches), launches
        for c in off:
            c.destroy()
    finally:
        for c in comms:
            c.destroy()


def test_colocated_ranks_are_fused_per_device(fake):
    """Two ranks per device (4 devices): one launch per device, blockIdx.y = rank slot."""
    fake(4)
    devs = [0, 0, 1, 1, 2, 2, 3, 3]
    comms = C.init_all(devs, C.CommConfig(buffer_size=1 << 20, lanes=2))
    try:
        _log()
        _allreduce_group(comms)
        ev = _log()
        launches = _check_launch_phase(ev, 4, 2, comms[0].nchannels * 2)
        assert len(launches) == 4
        # 2 ranks x 7 channels = 14 works > MCCS_INLINE_WORKS (8): the work FIFO
        assert all(kv["inline_works"] == "0" for _, kv in launches), launches
    finally:
        for c in comms:
            c.destroy()


def test_two_stream_bridge_stays_on_each_device(fake):
    """bridge_streams = 1 (libmccs user event -> comm stream -> backend event,
    collectives.rs:86,134): every stream wait joins streams of one device."""
    fake(8)
    comms = C.init_all(list(range(8)), C.CommConfig(buffer_size=1 << 20, bridge_streams=1))
    try:
        _log()
        _allreduce_group(comms)
        ev = _log()
        _check_launch_phase(ev, 8, 1, comms[0].nchannels * comms[0].lanes)
        assert sum(1 for k, _ in ev if k == "stream_wait") >= 8
    finally:
        for c in comms:
            c.destroy()


def test_external_launch_refuses_blocks_without_a_control_wave():
    """mccs_hip_launch_coll: blocks of <= 64 threads have no control wave; the
    argument check refuses them before any HIP call (no GPU needed)."""
    lib = _lib.load()
    f = lib.mccs_hip_launch_coll
    f.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p,
                  ctypes.c_uint, ctypes.c_uint, ctypes.c_void_p]
    f.restype = ctypes.c_int
    invalid_argument, allreduce = 4, 4  # mccsInvalidArgument, mccsFuncAllReduce
    assert f(allreduce, F32, SUM, 0x1000, 1, 0x2000, 1, 64, None) == invalid_argument
    assert f(allreduce, F32, SUM, 0x1000, 1, 0x2000, 1, 608, None) == invalid_argument


def test_comm_events_ride_on_the_launch(fake, monkeypatch):
    """A communicator launch carries its comm event as the dispatch's stop
    event (hipExtLaunchKernel): a hipEventRecord behind the kernel is a marker
    packet that cost ~3 us of device time per launch on MI355X
    (tools/launch_cost.hip).  mccsCommSync then waits on that event.  Extra
    records remain only where something consumes them: the two-stream
    bridge's user events."""
    fake(8)
    for inline in ("1", "0"):  # launch-argument works, then the work FIFO (read at creation)
        monkeypatch.setenv("MCCS_INLINE_WORKS", inline)
        comms = C.init_all(list(range(8)), C.CommConfig(buffer_size=1 << 20))
        try:
            _log()
            _allreduce_group(comms)
            ev = _log()
            launches = [kv for k, kv in ev if k == "launch"]
            assert len(launches) == 8 and all(kv["stop_event"] != "0" for kv in launches), launches
            assert not any(k == "record" for k, _ in ev), ev
            for c in comms:
                c.sync()
            waits = [kv["what"] for k, kv in _log() if k == "host_wait"]
            assert waits.count("event") == 8 and "device" not in waits, waits
        finally:
            for c in comms:
                c.destroy()
    monkeypatch.delenv("MCCS_INLINE_WORKS")
    comms = C.init_all(list(range(8)), C.CommConfig(buffer_size=1 << 20, bridge_streams=1))
    try:
        _log()
        _allreduce_group(comms)
        ev = _log()
        assert sum(1 for k, _ in ev if k == "record") == 8  # the user events of the bridge
        assert all(kv["stop_event"] != "0" for k, kv in ev if k == "launch")
    finally:
        for c in comms:
            c.destroy()


@pytest.mark.parametrize("inline", ["1", "0"])
def test_fused_ranks_record_their_events_only_when_consumed(fake, monkeypatch, inline):
    """Ranks sharing a device run as one launch: the first comm's event rides
    on it; the others' events are recorded only when consumed (here: not), and
    their mccsCommSync waits on the launching comm's event (not the device:
    ADVICE r03).  Works in the launch arguments or in the work FIFO alike (a
    FIFO launch used to record every fused slot's event: a marker packet and
    ~1.5 us of host time each)."""
    monkeypatch.setenv("MCCS_INLINE_WORKS", inline)
    fake(4)
    comms = C.init_all([0, 0, 1, 1, 2, 2, 3, 3], C.CommConfig(buffer_size=1 << 20, lanes=2, channel_count=1,
                                                              rings=[[0, 1, 2, 3, 4, 5, 6, 7]]))
    try:
        _log()
        _allreduce_group(comms)
        ev = _log()
        assert sum(1 for k, _ in ev if k == "launch") == 4
        assert not any(k == "record" for k, _ in ev), ev
        for c in comms:
            c.sync()
        waits = [kv["what"] for k, kv in _log() if k == "host_wait"]
        assert waits.count("event") == 8 and waits.count("device") == 0, waits
    finally:
        for c in comms:
            c.destroy()


def test_direct_allreduce_plans(fake):
    """With a direct threshold, one AllReduce of at most that many bytes per
    rank launches the direct kernel (one launch per device, the ring walk's
    channels and thread count in its arguments); a larger one, or two
    AllReduces of one comm in a group, the ring."""
    fake(8)
    comms = C.init_all(list(range(8)), C.CommConfig(direct_bytes=4 << 20))
    try:
        _log()
        _allreduce_group(comms, count=1 << 20)  # 4 MiB fp32: direct
        ev = _log()
        launches = [kv for k, kv in ev if k == "launch"]
        assert len(launches) == 8 and all(kv["kind"] == "direct" for kv in launches), launches
        nch, nthr = C.task_schema(4 << 20, comms[0].nchannels)
        for kv in launches:
            assert kv["grid"].endswith("x1") and kv["block"] == "512" and kv["comms_on_dev"] == "1"
            assert (int(kv["nch"]), int(kv["nthr"]), int(kv["count"])) == (nch, nthr, 1 << 20)
        assert all(c.last_algo() == "direct" for c in comms)
        _allreduce_group(comms, count=(1 << 20) + 1)  # one element over: ring
        ev = _log()
        assert [kv["kind"] for k, kv in ev if k == "launch"] == ["ring"] * 8
        assert all(c.last_algo() == "ring" for c in comms)
        with C.group():  # two AllReduces of each comm: batched for the ring
            for r, c in enumerate(comms):
                for j in range(2):
                    C.all_reduce(c, 0x10000000 * (r + 1) + j * 0x1000000, 0x10000000 * (r + 1) + 0x8000000, 1000, F32,
                                 SUM, stream=0)
        ev = _log()
        assert [kv["kind"] for k, kv in ev if k == "launch"] == ["ring"] * 8
        for c in comms:
            c.sync()
    finally:
        for c in comms:
            c.destroy()


def test_direct_defaults_and_fused_ranks(fake, monkeypatch):
    """Library defaults at n = 2: one-shot up to 2 MiB, the ring above
    (two-shot off at 2 ranks); fused ranks on one device share one direct
    launch; without peer atomics every AllReduce takes the ring."""
    for k in ("MCCS_ONESHOT_BYTES", "MCCS_DIRECT_BYTES"):
        monkeypatch.delenv(k, raising=False)
    fake(2)
    comms = C.init_all([0, 0, 0, 0, 1, 1, 1, 1], C.CommConfig(direct_bytes=1 << 20))
    plain = none = None
    try:
        _log()
        _allreduce_group(comms, count=1000)
        launches = [kv for k, kv in _log() if k == "launch"]
        assert len(launches) == 2 and all(kv["kind"] == "direct" for kv in launches)
        assert all(kv["grid"].endswith("x4") and kv["comms_on_dev"] == "1" for kv in launches)
        for c in comms:
            c.sync()
        plain = C.init_all([0, 1])
        assert all(c.direct_enabled() for c in plain)
        for count, want in ((1000, "oneshot"), (524288, "oneshot"), (524289, "ring")):
            _log()
            _allreduce_group(plain, count=count)
            assert [kv["kind"] for k, kv in _log() if k == "launch"] == (["direct"] * 2 if want != "ring" else
                                                                         ["ring"] * 2)
            assert [c.last_algo() for c in plain] == [want] * 2
        for c in plain:
            c.sync()
        monkeypatch.setenv("MCCS_TEST_NO_P2P_ATOMICS", "1")
        none = C.init_all([0, 1])
        assert not any(c.direct_enabled() for c in none)
        _log()
        _allreduce_group(none, count=1000)
        assert [kv["kind"] for k, kv in _log() if k == "launch"] == ["ring"] * 2
        for c in none:
            c.sync()
    finally:
        for c in comms + (plain or []) + (none or []):
            c.destroy()


def test_oneshot_below_its_threshold(fake):
    """Buckets up to oneshot_bytes take the one-shot variant, larger ones up
    to direct_bytes the two-shot one, the rest the ring; pieces stay within
    4..64 KiB."""
    fake(8)
    comms = C.init_all(list(range(8)), C.CommConfig(direct_bytes=4 << 20, oneshot_bytes=256 << 10))
    try:
        for count, want, mode in ((1000, "oneshot", "oneshot"), (65536, "oneshot", "oneshot"),
                                  (65537, "direct", "twoshot"), (1 << 20, "direct", "twoshot"),
                                  ((1 << 20) + 1, "ring", None)):
            _log()
            _allreduce_group(comms, count=count)
            launches = [kv for k, kv in _log() if k == "launch"]
            assert len(launches) == 8
            assert all(c.last_algo() == want for c in comms), (count, [c.last_algo() for c in comms])
            if mode:
                for kv in launches:
                    assert kv["kind"] == "direct" and kv["mode"] == mode
                    for p in (int(kv["piece"]), int(kv["piece2"])):
                        assert 1024 <= p <= 16384  # fp32 elements: 4..64 KiB
        for c in comms:
            c.sync()
    finally:
        for c in comms:
            c.destroy()


@pytest.mark.parametrize("n,oneshot,direct", [(4, 1 << 20, 8 << 20), (8, 256 << 10, 8 << 20), (3, 1 << 20, 4 << 20),
                                              (2, 2 << 20, None)])
def test_direct_default_thresholds(fake, monkeypatch, n, oneshot, direct):
    for k in ("MCCS_ONESHOT_BYTES", "MCCS_DIRECT_BYTES"):
        monkeypatch.delenv(k, raising=False)
    assert C.direct_defaults(n) == (oneshot, direct or -1)
    fake(n)
    comms = C.init_all(list(range(n)))
    try:
        cases = [(oneshot // 4, "oneshot"), (oneshot // 4 + 1, "direct" if direct else "ring")]
        if direct:
            cases += [(direct // 4, "direct"), (direct // 4 + 1, "ring")]
        for count, want in cases:
            _allreduce_group(comms, count=count)
            assert [c.last_algo() for c in comms] == [want] * n, (count, want)
        for c in comms:
            c.sync()
    finally:
        for c in comms:
            c.destroy()


def test_allgather_oneshot_plans(fake):
    """AllGather buckets up to oneshot_bytes per rank take the direct kernel's
    AllGather mode; larger ones the ring."""
    fake(8)
    comms = C.init_all(list(range(8)), C.CommConfig(oneshot_bytes=64 << 10, direct_bytes=-1))
    try:
        for nbytes, kind, algo in ((1000, "direct", "oneshot"), (65536, "direct", "oneshot"), (65537, "ring", "ring")):
            _log()
            with C.group():
                for r, c in enumerate(comms):
                    C.all_gather(c, 0x10000000 * (r + 1), 0x10000000 * (r + 1) + 0x8000000, nbytes, stream=0)
            launches = [kv for k, kv in _log() if k == "launch"]
            assert [kv["kind"] for kv in launches] == [kind] * 8
            if kind == "direct":
                assert all(kv["mode"] == "ag-oneshot" and int(kv["count"]) == nbytes for kv in launches)
            assert [c.last_algo() for c in comms] == [algo] * 8
        for c in comms:
            c.sync()
    finally:
        for c in comms:
            c.destroy()


@pytest.mark.parametrize("n,count,rings", [(8, 1 << 20, None), (8, 3_000_001, None), (4, 777, None),
                                           (3, 1_234_567, None), (8, 2_500_000, "doubled")])
def test_direct_ownership_matches_the_oracle(fake, orc, n, count, rings):
    """The host's per-rank element counts (the kernel's hand-off thresholds)
    equal the oracle's chunk ownership for the same walk (channels, threads,
    rings, 4 MiB FIFO buffer), including multi-loop walks and 2 x channels."""
    import numpy as np

    fake(n)
    ring_list = None
    if rings == "doubled":
        base = C.default_rings(n, 0)
        ring_list = base + [list(reversed(r)) for r in base]
    comms = C.init_all(list(range(n)), C.CommConfig(direct_bytes=64 << 20, oneshot_bytes=-1, rings=ring_list))
    try:
        _log()
        _allreduce_group(comms, count=count)
        launches = [kv for k, kv in _log() if k == "launch"]
        assert launches and all(kv["mode"] == "twoshot" for kv in launches)
        owned = [int(v) for v in launches[0]["owned"].split(",")]
        nch, nthr = C.task_schema(count * 4, comms[0].nchannels)
        zeros = [np.zeros(count, np.float32) for _ in range(n)]
        _, owner = orc.ring_allreduce(7, 0, zeros, nchannels=nch, nthreads=nthr, ring_orders=comms[0].rings()[:nch],
                                      want_owner=True)
        assert owned == np.bincount(owner, minlength=n).tolist()
        for c in comms:
            c.sync()
    finally:
        for c in comms:
            c.destroy()


def test_ll_below_its_threshold(fake):
    """Buckets up to ll_bytes take the LL one-shot (one 8-byte word per
    thread: grid = words / 512), larger ones the one-shot; a cached arena
    (FIFO_DEVICE) never takes LL; the LL slot is exactly 2 x ll_bytes."""
    fake(8)
    comms = C.init_all(list(range(8)), C.CommConfig(direct_bytes=-1, oneshot_bytes=256 << 10, ll_bytes=32 << 10))
    cached = None
    try:
        for count, want in ((1, "ll"), (1000, "ll"), (8192, "ll"), (8193, "oneshot")):
            _log()
            _allreduce_group(comms, count=count)
            launches = [kv for k, kv in _log() if k == "launch"]
            assert len(launches) == 8
            assert all(c.last_algo() == want for c in comms), (count, [c.last_algo() for c in comms])
            for kv in launches:
                assert kv["kind"] == "direct" and kv["mode"] == want
                if want == "ll":
                    assert int(kv["gx"]) == max(1, (count * 4 + 4095) // 4096)
                    assert int(kv["llslot"]) == 64 << 10
        for c in comms:
            c.sync()
        cached = C.init_all(list(range(8)), C.CommConfig(direct_bytes=-1, oneshot_bytes=256 << 10, ll_bytes=32 << 10,
                                                         fifo_memory=C.FIFO_DEVICE))
        _allreduce_group(cached, count=1000)
        assert all(c.last_algo() == "oneshot" for c in cached)
        for c in cached:
            c.sync()
    finally:
        for c in comms + (cached or []):
            c.destroy()


def test_ll_allgather_plans(fake):
    """AllGathers up to ll_bytes per rank take the LL lines (mode ll-ag),
    larger ones up to oneshot_bytes the one-shot exchange."""
    fake(8)
    comms = C.init_all(list(range(8)), C.CommConfig(oneshot_bytes=64 << 10, direct_bytes=-1, ll_bytes=16 << 10))
    try:
        for nbytes, want, mode in ((1000, "ll", "ll-ag"), (16 << 10, "ll", "ll-ag"), ((16 << 10) + 1, "oneshot", "ag-oneshot")):
            _log()
            with C.group():
                for r, c in enumerate(comms):
                    C.all_gather(c, 0x10000000 * (r + 1), 0x10000000 * (r + 1) + 0x8000000, nbytes, stream=0)
            launches = [kv for k, kv in _log() if k == "launch"]
            assert launches and all(kv["mode"] == mode for kv in launches), (nbytes, launches[:1])
            assert all(c.last_algo() == want for c in comms)
        for c in comms:
            c.sync()
    finally:
        for c in comms:
            c.destroy()


def test_ll_runs_without_peer_atomics(fake, monkeypatch):
    """Without peer atomics the count-based direct variants are off, but the
    LL one-shot (no remote atomics) still takes the buckets up to ll_bytes;
    larger ones the ring."""
    monkeypatch.setenv("MCCS_TEST_NO_P2P_ATOMICS", "1")
    fake(2)
    comms = C.init_all([0, 1], C.CommConfig(ll_bytes=64 << 10))
    try:
        assert not any(c.direct_enabled() for c in comms)
        for count, want in ((1000, "ll"), (16384, "ll"), (16385, "ring")):
            _log()
            _allreduce_group(comms, count=count)
            kinds = [kv.get("mode", kv["kind"]) for k, kv in _log() if k == "launch"]
            assert kinds == (["ll"] * 2 if want == "ll" else ["ring"] * 2), (count, kinds)
            assert [c.last_algo() for c in comms] == [want] * 2
        for c in comms:
            c.sync()
    finally:
        for c in comms:
            c.destroy()


def test_fused_rank_sync_waits_on_the_launch_not_the_device(fake):
    """Rank slots k >= 1 of a fused launch record no event of their own; their
    mccsCommSync waits on the launching comm's stop event instead of the whole
    device, which would also wait on other communicators' spinning kernels
    (ADVICE r03).  Destroying the launching comm first falls back safely (to
    the rank's own event or the device, never the freed event)."""
    fake(2)
    comms = C.init_all([0, 0, 1, 1], C.CommConfig(buffer_size=1 << 20, lanes=1))
    try:
        _log()
        _allreduce_group(comms)
        _log()
        for c in comms:
            c.sync()
        waits = [kv for k, kv in _log() if k == "host_wait"]
        assert waits and all(kv["what"] in ("event", "memcpy") for kv in waits), waits
        # the launching comm of each device goes first: its fused peer falls back to a device wait
        _allreduce_group(comms)
        comms[0].destroy()
        comms[2].destroy()
        _log()
        comms[1].sync()
        waits = [kv for k, kv in _log() if k == "host_wait"]
        # never a wait on the destroyed comm's event (the fake reports such an event's device as -1)
        assert waits and all(kv["dev"] != "-1" for kv in waits), waits
    finally:
        for c in (comms[1], comms[3]):
            c.destroy()


def test_launch_on_another_stream_waits_for_the_previous_one(fake):
    """A communicator's launches run in issue order whatever stream each one
    is issued on (the reference runs them on one private stream,
    proxy/init.rs:166-175): a launch on another stream than the comm's
    previous one waits for that launch's event first; on the same stream the
    stream order is enough and nothing is added."""
    fake(2)
    comms = C.init_all([0, 1], C.CommConfig(buffer_size=1 << 20))
    try:
        def group(stream):
            with C.group():
                for r, c in enumerate(comms):
                    C.all_reduce(c, 0x10000000 * (r + 1), 0x10000000 * (r + 1) + 0x8000000, 1 << 20, F32, SUM,
                                 stream=stream)

        group(0x7000)
        _log()
        group(0x7000)  # same stream: no wait
        assert not any(k == "stream_wait" for k, _ in _log())
        group(0x7100)  # another stream: waits for the previous launch on every device
        ev = _log()
        waits = [kv for k, kv in ev if k == "stream_wait"]
        assert sorted(int(kv["dev"]) for kv in waits) == [0, 1], ev
        assert all(kv["stream"] == str(0x7100) and kv["event_dev"] == kv["dev"] for kv in waits), waits
        for d in (0, 1):  # on each device the wait is queued before that device's launch
            w = next(i for i, (k, kv) in enumerate(ev) if k == "stream_wait" and kv["dev"] == str(d))
            l = next(i for i, (k, kv) in enumerate(ev) if k == "launch" and kv["dev"] == str(d))
            assert w < l, ev
    finally:
        for c in comms:
            c.destroy()


def test_recreated_stream_at_the_same_address_is_another_stream(fake):
    """HIP gives a destroyed stream's address to the next stream created
    (tools/stream_id_probe.c: six create/destroy rounds, one address, ids
    2..7), and a stream destroyed with work still queued keeps running it.  So
    a comm's next launch on a new stream at the old address must still wait
    for the previous launch: streams are compared by id, not address."""
    fake(2)
    comms = C.init_all([0, 1], C.CommConfig(buffer_size=1 << 20))
    lib = _lib.load()
    lib.mccs_test_fake_recreate_stream.argtypes = [ctypes.c_void_p]
    try:
        def group(stream):
            with C.group():
                for r, c in enumerate(comms):
                    C.all_reduce(c, 0x10000000 * (r + 1), 0x10000000 * (r + 1) + 0x8000000, 1 << 20, F32, SUM,
                                 stream=stream)

        group(0x7000)
        _log()
        group(0x7000)
        assert not any(k == "stream_wait" for k, _ in _log())
        assert lib.mccs_test_fake_recreate_stream(0x7000) == 0
        group(0x7000)  # same address, new stream: waits on every device
        waits = [kv for k, kv in _log() if k == "stream_wait"]
        assert sorted(int(kv["dev"]) for kv in waits) == [0, 1], waits
    finally:
        for c in comms:
            c.destroy()


def test_launch_larger_than_the_work_fifo_is_refused(fake, monkeypatch):
    """A group whose works cannot all sit in the work FIFO at once (the one
    kernel reads them all) is refused up front with the reason, instead of
    waiting for acknowledgements that cannot come."""
    from mccs_amd._lib import MccsError

    monkeypatch.setenv("MCCS_INLINE_WORKS", "0")
    fake(2)
    comms = C.init_all([0, 1], C.CommConfig(buffer_size=1 << 20, work_fifo_depth=8))
    try:
        with pytest.raises(MccsError, match="more than the work FIFO's 8: split the group"):
            with C.group():
                for _ in range(25):  # 25 elements per channel: 3 chained works on each of 4 channels = 12
                    for r, c in enumerate(comms):
                        C.all_reduce(c, 0x10000000 * (r + 1), 0x10000000 * (r + 1) + 0x8000000, 1 << 20, F32, SUM,
                                     stream=0)
        _log()
        _allreduce_group(comms)  # the comms stay usable
        assert sum(1 for k, _ in _log() if k == "launch") == 2
    finally:
        for c in comms:
            c.destroy()


def test_capture_leaves_the_eager_issue_order_alone(fake):
    """a launch captured into a graph used to overwrite the comm's
    latest-launch record (stream, event, sync owner) although a capture
    launches nothing; the next eager launch on a third stream then skipped
    its wait for the eager launch before the capture.  Eager on stream A,
    capture on stream C, eager on stream B: B must wait on A's launch."""
    fake(2)
    comms = C.init_all([0, 1], C.CommConfig(buffer_size=1 << 20))
    lib = _lib.load()
    lib.mccs_test_fake_capture.argtypes = [ctypes.c_void_p, ctypes.c_int]
    try:
        def group(stream):
            with C.group():
                for r, c in enumerate(comms):
                    C.all_reduce(c, 0x10000000 * (r + 1), 0x10000000 * (r + 1) + 0x8000000, 1 << 20, F32, SUM,
                                 stream=stream)

        group(0x7000)  # eager on A
        _log()
        assert lib.mccs_test_fake_capture(0x7200, 1) == 0
        group(0x7200)  # captured on C
        assert lib.mccs_test_fake_capture(0x7200, 0) == 0
        cap = _log()
        assert [kv["stream"] for k, kv in cap if k == "launch"] == [str(0x7200)] * 2, cap
        assert not any(k == "stream_wait" for k, _ in cap), "a captured launch waited on an event outside its graph"
        group(0x7100)  # eager on B: ordered after A's launch on every device
        ev = _log()
        waits = [kv for k, kv in ev if k == "stream_wait"]
        assert sorted(int(kv["dev"]) for kv in waits) == [0, 1], ev
        assert all(kv["stream"] == str(0x7100) for kv in waits), waits
    finally:
        for c in comms:
            c.destroy()


@pytest.mark.parametrize("n", [1, 3, 8])
def test_launches_carry_the_guard_order(fake, n):
    """Every launch names its rank slots in the order of their launch guards'
    addresses (launch_guard.h: fused launches take their guards in that one
    order, so two of them can never each hold a guard the other waits for);
    the guard line sits at MCCS_GUARD_OFF in each comm's device allocation."""
    fake(1)
    comms = C.init_all([0] * n, C.CommConfig(buffer_size=1 << 20))
    try:
        for count in (1 << 20, 1000):  # ring, then a direct-sized bucket (LL at n >= 2)
            _log()
            _allreduce_group(comms, count)
            launch = [kv for k, kv in _log() if k == "launch"]
            assert len(launch) == 1
            order = int(launch[0]["guard_order"])
            slots = [(order >> (4 * i)) & 15 for i in range(n)]
            assert sorted(slots) == list(range(n))
            devs = [c.dev_comm() for c in comms]
            assert [devs[k] for k in slots] == sorted(devs)
            assert launch[0]["no_guard"] == "0"
    finally:
        for c in comms:
            c.destroy()


def test_guard_test_hook_is_read_at_connect(fake, monkeypatch):
    """MCCS_LAUNCH_GUARD=0 (with MCCS_TEST_HOOKS=1) turns the guard off for
    communicators connected afterwards: the GPU test's control case."""
    fake(1)
    monkeypatch.setenv("MCCS_LAUNCH_GUARD", "0")
    comms = C.init_all([0] * 2, C.CommConfig(buffer_size=1 << 20))
    try:
        for count in (1 << 20, 1000):
            _log()
            _allreduce_group(comms, count)
            assert [kv["no_guard"] for k, kv in _log() if k == "launch"] == ["1"]
    finally:
        for c in comms:
            c.destroy()
