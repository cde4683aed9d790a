"""CPU: host logic of the reference-driven harness (mccs_amd/refdrive.py) --
plan.rs's work-ring reservation and rolling acknowledgements (plan.rs:380-541)
against a simulated kernel, and the configuration-only variants the bench
times.  No GPU."""
import pytest

from mccs_amd import comm as C
from mccs_amd import refdrive


class _SimKernel:
    """Launches run in order, one per host poll of workFifoDone (the kernel
    writes doneAcks to each of its channels' done words, common.h:153-155)."""

    def __init__(self, nch, stuck=False):
        self.done = [0] * nch
        self.pending = []
        self.stuck = stuck

    def read(self):
        if self.pending and not self.stuck:
            chans, acks, _ = self.pending.pop(0)
            for c in chans:
                self.done[c] = acks
        return list(self.done)

    def write(self, c, v):
        self.done[c] = v


@pytest.mark.parametrize("depth,nch,ks", [(16, 3, [3]), (16, 4, [1, 2, 3, 4]), (64, 7, [7, 5, 1])])
def test_work_ring_never_splits_a_launch_and_never_reuses_unacked_slots(depth, nch, ks):
    ring = refdrive.WorkRing(nch, depth)
    sim = _SimKernel(nch)
    held = {}  # slot -> launch id still pending
    wraps = 0
    for i in range(40 * depth):
        k = ks[i % len(ks)]
        chans = list(range(k))
        before = ring.next_available
        start, acks = ring.reserve(chans, sim.read, sim.write, timeout_s=5)
        if start != before:
            wraps += 1
            assert start % depth == 0  # wrapped to the ring start
        assert (start % depth) + k <= depth  # one launch's works are contiguous
        done_ids = {lid for lid in held.values() if all(lid != p[2] for p in sim.pending)}
        for s in range(start, start + k):
            lid = held.get(s % depth)
            assert lid is None or lid in done_ids, f"slot {s % depth} reused before launch {lid} was acknowledged"
        for s in range(start, start + k):
            held[s % depth] = i
        assert acks == (start + k) & 0xFFFFFFFF
        sim.pending.append((chans, acks, i))
    assert wraps > 0 or depth % k == 0


def test_reference_ack_arithmetic_lets_the_host_overwrite_an_unread_work():
    """The reference quirk the default avoids (plan.rs:461-470): with
    DoneAcks = first + k + 1, one acknowledged launch also releases the
    first entry of the launch after it.  A host that runs a full ring ahead
    then reuses that entry while its launch is still pending."""
    depth, nch = 16, 4
    ks = [1, 2, 3, 4]
    ring = refdrive.WorkRing(nch, depth, reference_acks=True)
    sim = _SimKernel(nch)
    held, hit = {}, False
    for i in range(40 * depth):
        k = ks[i % len(ks)]
        start, acks = ring.reserve(list(range(k)), sim.read, sim.write, timeout_s=5)
        pending = {p[2] for p in sim.pending}
        hit = hit or any(held.get(s % depth) in pending for s in range(start, start + k))
        for s in range(start, start + k):
            held[s % depth] = i
        sim.pending.append((list(range(k)), acks, i))
    assert hit


def test_work_ring_flow_control_stops_at_depth_without_acknowledgements():
    depth, nch = 16, 2
    ring = refdrive.WorkRing(nch, depth)
    sim = _SimKernel(nch, stuck=True)
    n = 0
    with pytest.raises(RuntimeError, match="no acknowledgement"):
        for _ in range(depth):
            ring.reserve([0, 1], sim.read, sim.write, timeout_s=0.05)
            n += 1
    assert n * 2 <= depth + 2


def test_work_ring_counters_wrap_u32():
    ring = refdrive.WorkRing(2, 16)
    ring.next_available = ring.acked_min = 0xFFFFFFF0
    ring.chan_next = [0xFFFFFFF0, 0xFFFFFFF0]
    sim = _SimKernel(2)
    sim.done = [0xFFFFFFF0, 0xFFFFFFF0]
    for _ in range(40):
        start, acks = ring.reserve([0, 1], sim.read, sim.write, timeout_s=5)
        sim.pending.append(([0, 1], acks, 0))
        assert 0 <= start <= 0xFFFFFFFF and (start % 16) + 2 <= 16


@pytest.mark.parametrize("n", [2, 4, 8])
def test_configuration_only_variants(n):
    vs = refdrive.default_variants(n, C.default_rings)
    names = [v["name"] for v in vs]
    assert names[:5] == ["ch2_reference_ring_sender", "ch2_reference_ring_receiver",
                         "ch2_reference_ring_sender_hostfifo", "ch32_reference_ring_sender",
                         "ch32_reference_ring_sender_hostfifo"]
    # the shipped 2-channel shape under each config-only choice: locality and
    # the reference's own host-memory FIFOs
    assert [(v["locality"], v["fifo"]) for v in vs[:3]] == [("sender", "device"), ("receiver", "device"),
                                                           ("sender", "host")]
    for v in vs:
        assert 1 <= v["nch"] <= 32 and v["locality"] in ("sender", "receiver") and v["fifo"] in ("device", "host")
        if v["rings"] is not None:
            assert len(v["rings"]) == v["nch"]
            for r in v["rings"]:
                assert sorted(r) == list(range(n))
    spread = vs[5]["rings"]
    # the spread variants cycle over every distinct default ring equally often
    uniq = {tuple(r) for r in spread}
    assert all(sum(1 for r in spread if tuple(r) == u) == len(spread) // len(uniq) for u in uniq)
    if n == 8:
        assert len(uniq) == 7 and vs[5]["nch"] == 28


def test_variants_capped_when_ranks_share_a_gpu():
    vs = refdrive.default_variants(8, C.default_rings, 16)
    assert [v["nch"] for v in vs] == [2, 2, 2, 16, 16, 14, 14]
    assert all(v["nch"] * 8 <= 128 for v in vs)


def test_reference_rings_are_the_engine_default():
    assert refdrive.reference_rings(4, 2) == [[0, 1, 2, 3], [0, 1, 2, 3]]


def test_host_segment_roundtrip_without_gpu(monkeypatch):
    """The host connector's segment: shm_open + ftruncate (zeroed) + mmap +
    mlock, registered through hipHostRegister (faked here: no GPU); a peer
    opening the name sees the creator's bytes; the name is unlinked once
    every rank mapped it."""
    import ctypes
    import uuid

    calls = []

    class FakeHip:
        def hipHostRegister(self, p, n, flags):
            calls.append(("reg", n, flags))
            return 0

        def hipHostGetDevicePointer(self, out, p, flags):
            out._obj.value = p.value
            return 0

        def hipHostUnregister(self, p):
            calls.append(("unreg",))
            return 0

    monkeypatch.setattr(refdrive, "hip", lambda: FakeHip())
    name = f"/mccs_test_{uuid.uuid4().hex[:12]}"
    a = refdrive.HostSegment(name, 3 * 4096 + 5, create=True)
    try:
        assert a.nbytes == 4 * 4096 and a.dev == a.host
        assert bytes((ctypes.c_char * 64).from_address(a.host)) == bytes(64)
        ctypes.memset(a.host + 4096, 0x5A, 16)
        b = refdrive.HostSegment(name, 3 * 4096 + 5, create=False)
        assert bytes((ctypes.c_char * 16).from_address(b.host + 4096)) == b"\x5a" * 16
        a.unlink()
        with pytest.raises(OSError):
            refdrive.HostSegment(name, 4096, create=False)
        b.close()
    finally:
        a.close()
    assert calls.count(("reg", 4 * 4096, refdrive.hipHostRegisterMapped)) == 2 and calls.count(("unreg",)) == 2
