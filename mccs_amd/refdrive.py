"""Reference-driven launches ("depth A" of the drop-in).

The reference's Rust service builds every device structure itself and calls
the kernel by symbol.  This module restates exactly that
host side for the reference-named kernels of libmccs_hip.so, with no
communicator of this library involved, so the number an UNCHANGED service
gets can be timed and its results checked:

* transport/shm/transporter.rs:49-183 + transport/meta.rs:7-67 (the SHM
  connector): per channel a 4096-byte SendBufMeta (head at offset 0), a
  4096-byte RecvBufMeta (tail at offset 0) and one FIFO of buffer_size bytes
  (8 slots of buffer_size/8).  Head lives with the sender, tail with the
  receiver; the FIFO data with the sender (`Locality::Sender`, the reference
  default) or with the receiver (`mccs.toml [shm] locality`).  `fifo`
  selects the memory:
    "device" -- device memory of the owning GPU, shared with the peers over
      IPC: the xGMI connector that replaces the host-pinned SHM buffers
      (§8(f) 2);
    "host"   -- the reference's own SHM memory: page-aligned host memory,
      mlock'ed (transport/shm/buffer.rs:17-26) and registered mapped with
      hipHostRegister + hipHostGetDevicePointer in every process that
      touches it (cuda/alloc.rs:59-99, shm/transporter.rs:102-106).  The
      reference service is one process, so a plain System.alloc suffices
      there; the ranks here are processes, so each rank's segment is a POSIX
      shared-memory object that its peers map too.  This is the deployment
      an UNCHANGED Rust service runs;
* comm/device.rs:35-183 (CommDevResources::new, conn_info_to_dev):
  mccsDevCommAndChannels, per-channel peers arrays, userRanks,
  ring prev/next/index, abortFlag, workFifoDone (host-mapped,
  device.rs:56-64);
* plan.rs:172-302 (compute_coll_work, select_best_channels: least-loaded
  channels first), plan.rs:380-541 (wait_work_queue, upload_work: the
  host-mapped work ring, wrap to the ring start, isLast / inFifo /
  doneAcks, rolling acks), plan.rs:602-669 (get_task_schema, launch_plan:
  grid = #channels, block = nthreads, e.g. 544).

The launch goes through mccs_hip_launch_coll (the kernel symbol plus
hipLaunchKernel, the call plan.rs:659-666 makes with cudaLaunchKernel).
The reference-named kernels run the reference hand-off policy (system-scope
release/acquire, 2-step slices, 8 FIFO slots, 30 s watchdog on abortFlag).
"""
from __future__ import annotations

import ctypes
import os
import time

from . import _lib as L
from . import abi

FUNC_ALLREDUCE = 4  # mccsFuncAllReduce
META = 4096  # SendBufMeta / RecvBufMeta, each padded to a page (meta.rs:7-67)
WORK_DEPTH = 1024  # entries of the host-mapped work ring (power of two; the reference has 65536)
ESIZE = {0: 1, 1: 1, 2: 4, 3: 4, 4: 8, 5: 8, 6: 2, 7: 4, 8: 8, 9: 2}

_hip = None


def hip() -> ctypes.CDLL:
    global _hip
    if _hip is None:
        h = ctypes.CDLL("libamdhip64.so")
        vp, sz = ctypes.c_void_p, ctypes.c_size_t
        h.hipHostMalloc.argtypes = [ctypes.POINTER(vp), sz, ctypes.c_uint]
        h.hipHostGetDevicePointer.argtypes = [ctypes.POINTER(vp), vp, ctypes.c_uint]
        h.hipHostFree.argtypes = [vp]
        h.hipMemcpy.argtypes = [vp, vp, sz, ctypes.c_int]
        h.hipMemset.argtypes = [vp, ctypes.c_int, sz]
        h.hipMalloc.argtypes = [ctypes.POINTER(vp), sz]
        h.hipFree.argtypes = [vp]
        h.hipSetDevice.argtypes = [ctypes.c_int]
        h.hipHostRegister.argtypes = [vp, sz, ctypes.c_uint]
        h.hipHostUnregister.argtypes = [vp]
        _hip = h
    return _hip


_libc = None


def libc() -> ctypes.CDLL:
    global _libc
    if _libc is None:
        c = ctypes.CDLL(None, use_errno=True)
        vp, sz = ctypes.c_void_p, ctypes.c_size_t
        c.shm_open.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.c_uint]
        c.shm_unlink.argtypes = [ctypes.c_char_p]
        c.ftruncate.argtypes = [ctypes.c_int, ctypes.c_long]
        c.posix_fallocate.argtypes = [ctypes.c_int, ctypes.c_long, ctypes.c_long]
        c.mmap.argtypes = [vp, sz, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_long]
        c.mmap.restype = vp
        c.munmap.argtypes = [vp, sz]
        c.mlock.argtypes = [vp, sz]
        c.munlock.argtypes = [vp, sz]
        c.close.argtypes = [ctypes.c_int]
        _libc = c
    return _libc


PAGE = 4096
hipHostRegisterMapped = 0x2


class HostSegment:
    """One rank's SHM connector memory as the reference allocates it: page
    aligned host memory, mlock'ed (buffer.rs:17-26: System.alloc + mlock),
    registered mapped for the current device (DeviceHostMapped::register,
    cuda/alloc.rs:59-99).  `create=True` makes the POSIX shm object (zeroed by
    ftruncate); peers open it by name.  `dev` is the device address the
    kernels use; `host` the CPU address."""

    def __init__(self, name: str, nbytes: int, create: bool):
        c = libc()
        self.name, self.nbytes = name.encode(), (nbytes + PAGE - 1) // PAGE * PAGE
        self.host = self.dev = None
        self._fd, self._registered, self._locked, self._owner = -1, False, False, create
        flags = (0o100 | 0o200 | 2) if create else 2  # O_CREAT|O_EXCL|O_RDWR / O_RDWR
        self._fd = c.shm_open(self.name, flags, 0o600)
        if self._fd < 0:
            raise OSError(ctypes.get_errno(), f"shm_open({name})")
        try:
            if create and c.ftruncate(self._fd, self.nbytes) != 0:
                raise OSError(ctypes.get_errno(), "ftruncate")
            # reserve the pages now: a full /dev/shm then fails here (ENOSPC)
            # instead of a SIGBUS at the first touch of an unbacked page
            if create:
                rc = c.posix_fallocate(self._fd, 0, self.nbytes)
                if rc != 0:
                    raise OSError(rc, f"posix_fallocate({self.nbytes} bytes of /dev/shm)")
            p = c.mmap(None, self.nbytes, 0x1 | 0x2, 0x01, self._fd, 0)  # PROT_READ|WRITE, MAP_SHARED
            if p in (None, ctypes.c_void_p(-1).value):
                raise OSError(ctypes.get_errno(), "mmap")
            self.host = p
            # mlock as the reference does; an ordinary user's RLIMIT_MEMLOCK
            # may refuse it, and hipHostRegister pins the pages anyway
            self._locked = c.mlock(p, self.nbytes) == 0
            _ok(hip().hipHostRegister(p, self.nbytes, hipHostRegisterMapped), "hipHostRegister(mapped)")
            self._registered = True
            dp = ctypes.c_void_p()
            _ok(hip().hipHostGetDevicePointer(ctypes.byref(dp), ctypes.c_void_p(p), 0), "hipHostGetDevicePointer")
            self.dev = dp.value or p  # cuda/alloc.rs:80-82: fall back to the host address
        except Exception:
            self.close()
            raise

    def unlink(self) -> None:
        if self._owner:
            libc().shm_unlink(self.name)
            self._owner = False

    def close(self) -> None:
        c = libc()
        if self._registered:
            hip().hipHostUnregister(ctypes.c_void_p(self.host))
            self._registered = False
        if self.host:
            if self._locked:
                c.munlock(ctypes.c_void_p(self.host), self.nbytes)
            c.munmap(ctypes.c_void_p(self.host), self.nbytes)
            self.host = None
        if self._fd >= 0:
            c.close(self._fd)
            self._fd = -1
        self.unlink()


def _ok(rc: int, what: str) -> None:
    if rc != 0:
        raise RuntimeError(f"{what}: hipError {rc}")


def _rolling_less(a: int, b: int) -> bool:
    """plan.rs:695-704 rolling_less_u32."""
    return ((a - b) & 0xFFFFFFFF) >= 0x80000000


def _rolling_min(a: int, b: int) -> int:
    return a if _rolling_less(a, b) else b


def reference_rings(n: int, nch: int) -> list[list[int]]:
    """proxy/engine.rs:296-320 default: ring 0 -> 1 -> ... -> n-1 on every channel."""
    return [list(range(n)) for _ in range(nch)]


class WorkRing:
    """plan.rs's work-FIFO bookkeeping (upload_work's slot reservation,
    wait_work_queue's rolling acknowledgements, plan.rs:380-541), host-only so
    it is unit-tested on CPU.  One work per selected channel per launch.

    Acknowledgement value: plan.rs:461-470 gives a channel's single (first
    and last) work DoneAcks(new_subsequent_start + 1) = first + k + 1, one
    entry PAST the launch's last entry.  Once that launch is read, the
    host's acked_min therefore also covers the first entry of the NEXT
    launch, which may not have been read yet: a host a full ring ahead can
    overwrite it (tests/test_refdrive_host.py reproduces the overwrite).
    By default the acknowledgement here is the launch's end, first + k
    (exact; NCCL's doneAcks is likewise one past the channel's last work);
    `reference_acks=True` keeps the reference arithmetic."""

    def __init__(self, nch: int, depth: int = WORK_DEPTH, reference_acks: bool = False):
        assert depth & (depth - 1) == 0
        self.nch, self.depth = nch, depth
        self.reference_acks = reference_acks
        self.next_available = 0
        self.chan_next = [0] * nch
        self.acked_min = 0

    def _wait(self, target: int, read_done, write_done, timeout_s: float) -> None:
        """plan.rs:380-422."""
        if not _rolling_less((self.acked_min + self.depth) & 0xFFFFFFFF, target & 0xFFFFFFFF):
            return
        t0 = time.monotonic()
        while True:
            ackd = read_done()
            ackd_all = self.next_available
            for c in range(self.nch):
                if ackd[c] != self.chan_next[c]:
                    ackd_all = _rolling_min(ackd_all, ackd[c])
            for c in range(self.nch):
                if ackd[c] == self.chan_next[c]:
                    write_done(c, ackd_all)
            self.acked_min = ackd_all
            if not _rolling_less((self.acked_min + self.depth) & 0xFFFFFFFF, target & 0xFFFFFFFF):
                return
            if time.monotonic() - t0 > timeout_s:
                raise RuntimeError("reference-driven work ring: no acknowledgement (kernel stuck?)")
            time.sleep(0)

    def reserve(self, chans, read_done, write_done, timeout_s: float = 60.0):
        """Slots for one launch over `chans` (ascending channel ids): returns
        (first slot counter, doneAcks).  Wraps to the ring start rather than
        splitting a launch's works, and waits until the slots are acknowledged
        (upload_work, plan.rs:424-443)."""
        k = len(chans)
        mask = self.depth - 1
        start = self.next_available
        if ((start + k - 1) & mask) < (start & mask):
            start = (start + mask) & ~mask & 0xFFFFFFFF
            self.next_available = start
        self._wait(start + k, read_done, write_done, timeout_s)
        acks = (start + k + (1 if self.reference_acks else 0)) & 0xFFFFFFFF
        for c in chans:
            self.chan_next[c] = acks
        self.next_available = (start + k) & 0xFFFFFFFF
        return start, acks


class RefDrivenRank:
    """One rank's device structures, built as the Rust service builds them.

    `allgather(obj) -> list` exchanges picklable objects between the ranks
    (torch.distributed.all_gather_object over gloo in the bench).  `rings`:
    one send order per channel (comm_patterns_override, config.rs:32-47);
    default the reference ring on every channel."""

    def __init__(self, rank: int, n: int, device: int, allgather, nch: int = 2, rings=None,
                 buff_size: int = 1 << 22, locality: str = "sender", fifo: str = "device",
                 watchdog_ms: int | None = None):
        if not 2 <= n or not 1 <= nch <= abi.MCCS_MAX_NCHANNELS or locality not in ("sender", "receiver") \
                or fifo not in ("device", "host"):
            raise ValueError("bad reference-driven configuration")
        self.rank, self.n, self.device, self.nch, self.buff = rank, n, device, nch, buff_size
        self.rings = [list(r) for r in (rings or reference_rings(n, nch))]
        if len(self.rings) != nch or any(sorted(r) != list(range(n)) for r in self.rings):
            raise ValueError("each channel needs a ring over every rank")
        self.locality, self.fifo = locality, fifo
        self.lib = L.load()
        h = hip()
        _ok(h.hipSetDevice(device), "hipSetDevice")
        # the reference kernels' watchdog on this device: 10 min unless the
        # caller (or MCCS_TIMEOUT_MS) sets one -- the tests and the bench bound
        # a hang to seconds
        if watchdog_ms is None and os.environ.get("MCCS_TIMEOUT_MS"):
            watchdog_ms = int(os.environ["MCCS_TIMEOUT_MS"])
        if watchdog_ms is not None:
            L.check(self.lib.mccs_hip_set_ref_watchdog(int(watchdog_ms)), "mccs_hip_set_ref_watchdog")
        self._dev_allocs, self._host_allocs, self._opened, self._segs = [], [], [], []
        # -- connector memory: [SendBufMeta][RecvBufMeta][FIFO] per channel, one allocation
        self.stride = 2 * META + buff_size
        self._mine = 0
        if fifo == "host":
            self._init_host_connector(allgather)
        else:
            self._init_device_connector(allgather)
        self._build_device_structs()

    def _init_device_connector(self, allgather) -> None:
        h, rank, n, device, nch = hip(), self.rank, self.n, self.device, self.nch
        # every rank joins the handle exchange even after a local failure (an
        # empty handle), so a peer's error never leaves the others blocked in it
        mine, handle, local_err = ctypes.c_void_p(), (ctypes.c_char * 64)(), None
        try:
            L.check(self.lib.mccsMemAllocShared(device, self.stride * nch, ctypes.byref(mine), handle),
                    "mccsMemAllocShared")
            self._mine = mine.value
            _ok(h.hipMemset(self._mine, 0, self.stride * nch), "hipMemset")
        except Exception as e:  # noqa: BLE001
            local_err = e
        handles = allgather(b"" if local_err else bytes(handle))
        if local_err or any(not x for x in handles):
            self.close()
            raise RuntimeError(f"reference-driven connector setup failed ({local_err or 'on another rank'})")
        self.base = [0] * n
        try:
            for r in range(n):
                if r == rank:
                    self.base[r] = self._mine
                    continue
                p = ctypes.c_void_p()
                L.check(self.lib.mccsMemOpenShared(device, handles[r], ctypes.byref(p)), "mccsMemOpenShared")
                self.base[r] = p.value
                self._opened.append(p.value)
        except Exception:
            self.close()  # no collective here: the caller agrees on the failure
            raise

    def _init_host_connector(self, allgather) -> None:
        """Every rank's [SendBufMeta][RecvBufMeta][FIFO] x channels in host
        memory (the reference SHM transport): this rank creates its segment,
        then maps and registers every peer's.  Two exchanges, both joined by
        every rank whatever fails locally: the names, then "all mapped" (after
        which the names are unlinked; the mappings keep the memory)."""
        import uuid

        rank, n = self.rank, self.n
        nbytes = self.stride * self.nch
        name, local_err = f"/mccs_refdrv_{uuid.uuid4().hex[:16]}_{rank}", None
        try:
            self._segs.append(HostSegment(name, nbytes, create=True))
        except Exception as e:  # noqa: BLE001
            local_err = e
        names = allgather("" if local_err else name)
        self.base = [0] * n
        # only the ring neighbours' segments are touched (each channel's prev
        # and next): an 8-rank, 32-channel rank maps 2 of 7 peers' 128 MiB
        neigh = set()
        for ring in self.rings:
            pos = ring.index(rank)
            neigh.update((ring[(pos + 1) % n], ring[(pos - 1) % n]))
        if not local_err and all(names):
            try:
                for r in range(n):
                    if r == rank:
                        self.base[r] = self._segs[0].dev
                        continue
                    if r not in neigh:
                        continue
                    seg = HostSegment(names[r], nbytes, create=False)
                    self._segs.append(seg)
                    self.base[r] = seg.dev
            except Exception as e:  # noqa: BLE001
                local_err = e
        oks = allgather(local_err is None and all(names))
        for s in self._segs:
            s.unlink()
        if not all(oks):
            self.close()
            raise RuntimeError(f"reference-driven host connector setup failed ({local_err or 'on another rank'})")

    def _build_device_structs(self) -> None:
        h, rank, n, nch, buff_size, locality = hip(), self.rank, self.n, self.nch, self.buff, self.locality
        # -- host-mapped sync: work ring + workFifoDone (device.rs:56-64)
        self.h_work, self.d_work = self._host_mapped(abi.MCCS_WORK_SIZE * WORK_DEPTH)
        self.h_done, self.d_done = self._host_mapped(4 * abi.MCCS_MAX_NCHANNELS)
        ctypes.memset(self.h_done, 0, 4 * abi.MCCS_MAX_NCHANNELS)
        self.d_abort = self._dev_alloc(64)
        _ok(h.hipMemset(self.d_abort, 0, 64), "hipMemset")  # the reference leaves it uninitialised
        # -- mccsDevCommAndChannels (device.rs:81-183)
        hc = abi.mccsDevCommAndChannels()
        hc.comm.rank, hc.comm.nRanks = rank, n
        hc.comm.buffSizes[0] = buff_size
        hc.comm.abortFlag = self.d_abort
        self.d_peers = []
        for c in range(nch):
            ring = self.rings[c]
            pos = ring.index(rank)
            user_ranks = [ring[(pos + i) % n] for i in range(n)]
            prev, nxt = user_ranks[n - 1], user_ranks[1]
            peers = (abi.mccsDevChannelPeer * n)()
            s = peers[nxt].send[0]
            s.buffs[0] = self._fifo(c, rank if locality == "sender" else nxt)
            s.head = self._send_meta(c, rank)
            s.tail = self._recv_meta(c, nxt)
            rv = peers[prev].recv[0]
            rv.buffs[0] = self._fifo(c, prev if locality == "sender" else rank)
            rv.tail = self._recv_meta(c, rank)
            rv.head = self._send_meta(c, prev)
            ch = hc.channels[c]
            ch.peers = self._upload(bytes(peers))
            self.d_peers.append(ch.peers)
            ch.ring.prev, ch.ring.next = prev, nxt
            ch.ring.userRanks = self._upload(b"".join(int(u).to_bytes(4, "little", signed=True) for u in user_ranks))
            ch.ring.index = (pos - ring.index(0)) % n  # engine.rs:274-286
            ch.workFifoDone = self.d_done + 4 * c
        self.d_comm = self._upload(bytes(hc))
        # -- planner state (plan.rs)
        self.ring = WorkRing(nch)
        self.launches = 0
        self._works = {}

    # memory helpers ---------------------------------------------------------
    def _fifo(self, c, r):
        return self.base[r] + c * self.stride + 2 * META

    def _send_meta(self, c, r):
        return self.base[r] + c * self.stride

    def _recv_meta(self, c, r):
        return self.base[r] + c * self.stride + META

    def _host_mapped(self, nbytes):
        hp, dp = ctypes.c_void_p(), ctypes.c_void_p()
        _ok(hip().hipHostMalloc(ctypes.byref(hp), nbytes, 0x2), "hipHostMalloc(mapped)")
        self._host_allocs.append(hp.value)
        _ok(hip().hipHostGetDevicePointer(ctypes.byref(dp), hp, 0), "hipHostGetDevicePointer")
        return hp.value, dp.value

    def _dev_alloc(self, nbytes):
        p = ctypes.c_void_p()
        _ok(hip().hipMalloc(ctypes.byref(p), nbytes), "hipMalloc")
        self._dev_allocs.append(p.value)
        return p.value

    def _upload(self, b: bytes) -> int:
        p = self._dev_alloc(len(b))
        buf = ctypes.create_string_buffer(b, len(b))
        _ok(hip().hipMemcpy(p, buf, len(b), 1), "hipMemcpy H2D")
        return p

    # plan.rs ---------------------------------------------------------------
    def _read_done(self):
        return list((ctypes.c_uint32 * abi.MCCS_MAX_NCHANNELS).from_address(self.h_done))

    def _write_done(self, c, v):
        (ctypes.c_uint32 * abi.MCCS_MAX_NCHANNELS).from_address(self.h_done)[c] = v

    def all_reduce(self, send_ptr: int, recv_ptr: int, count: int, dtype: int, op: int, stream: int) -> None:
        """One AllReduce task through plan.rs's path (one work element per
        selected channel), launched on `stream`.  count = 0 launches nothing."""
        if count == 0:
            return
        nbytes = count * ESIZE[dtype]
        sch, nthr = ctypes.c_int(), ctypes.c_int()
        self.lib.mccs_task_schema(nbytes, self.nch, ctypes.byref(sch), ctypes.byref(nthr))
        k, nthr = sch.value, nthr.value
        # select_best_channels (plan.rs:292-302): least loaded first, ties by
        # id; the loads belong to the plan being built (one task per plan
        # here), so they start at zero: channels 0..k-1, which also map to the
        # set bits of channelMask in ascending order
        load = [0] * self.nch
        chans = sorted(sorted(range(self.nch), key=lambda i: (load[i], i))[:k])
        mask_q = WORK_DEPTH - 1
        start, acks = self.ring.reserve(chans, self._read_done, self._write_done)
        key = (send_ptr, recv_ptr, count, k, nthr)
        works = self._works.get(key)
        if works is None:  # work_elem_conversion (plan.rs:550-600), built once per shape
            works = []
            for nth in range(k):
                w = abi.mccsDevWork()
                w.header.type = 1  # mccsDevWorkTypeColl
                w.header.isLast, w.header.inFifo = 1, 1
                e = w.elems[0]
                e.isUsed, e.nWarps = 1, nthr // 32
                e.sendbuff, e.recvbuff, e.count = send_ptr, recv_ptr, count
                e.bid, e.nChannels = nth, k
                works.append(w)
            if len(self._works) > 64:
                self._works.clear()
            self._works[key] = works
        for nth in range(k):
            w = works[nth]
            w.header.doneAcks = acks
            ctypes.memmove(self.h_work + ((start + nth) & mask_q) * abi.MCCS_WORK_SIZE, ctypes.addressof(w),
                           abi.MCCS_WORK_SIZE)
        channel_mask = 0
        for c in chans:
            channel_mask |= 1 << c
        rc = self.lib.mccs_hip_launch_coll(FUNC_ALLREDUCE, dtype, op, self.d_comm, channel_mask,
                                           self.d_work + (start & mask_q) * abi.MCCS_WORK_SIZE, k, nthr, stream)
        L.check(rc, "mccs_hip_launch_coll")
        self.launches += 1
        self.last_plan = (k, nthr, [self.rings[c] for c in chans])

    def aborted(self) -> bool:
        v = ctypes.c_int32()
        _ok(hip().hipMemcpy(ctypes.byref(v), self.d_abort, 4, 2), "hipMemcpy D2H")
        return v.value != 0

    def steps(self) -> list[int]:
        """conn->step of this rank's send and recv connectors, per channel."""
        out = []
        for c in range(self.nch):
            ring = self.rings[c]
            pos = ring.index(self.rank)
            pr = (abi.mccsDevChannelPeer * self.n)()
            _ok(hip().hipMemcpy(ctypes.byref(pr), self.d_peers[c], ctypes.sizeof(pr), 2), "hipMemcpy D2H")
            out += [int(pr[ring[(pos + 1) % self.n]].send[0].step), int(pr[ring[(pos - 1) % self.n]].recv[0].step)]
        return out

    def done_acks(self) -> list[int]:
        return list((ctypes.c_uint32 * abi.MCCS_MAX_NCHANNELS).from_address(self.h_done))[:self.nch]

    def close(self, barrier=None) -> None:
        """Unmaps the peers' memory; `barrier()` (all ranks) before freeing our
        own, which the peers may still have mapped.  Safe on a partly built
        rank."""
        h = hip()
        for name in ("_opened", "_dev_allocs", "_host_allocs", "_segs"):
            if not hasattr(self, name):
                setattr(self, name, [])
        if not hasattr(self, "_mine"):
            self._mine = 0
        h.hipDeviceSynchronize()
        for p in self._opened:
            self.lib.mccsMemCloseShared(self.device, ctypes.c_void_p(p))
        self._opened = []
        # host connector: our mappings only (a peer's pages live on until its
        # own close unmaps them; every name was unlinked after setup)
        for s in self._segs:
            s.close()
        self._segs = []
        if barrier is not None:
            barrier()
        if self._mine:
            self.lib.mccsMemFreeShared(self.device, ctypes.c_void_p(self._mine))
            self._mine = 0
        for p in self._dev_allocs:
            h.hipFree(ctypes.c_void_p(p))
        for p in self._host_allocs:
            h.hipHostFree(ctypes.c_void_p(p))
        self._dev_allocs, self._host_allocs = [], []


# ---------------------------------------------------------------------------
# Timing harness shared by bench.py (config.reference_driven, N > 1) and
# tools/refdrv_bench.py (the 2-process rehearsal on one GPU).

def exact_inputs(torch, count: int, rank: int, dtype, device):
    """Values k/64 with |k| <= 127: every partial sum of <= 8 ranks is exact
    in fp16 and fp32, so the result is independent of the summation order."""
    i = torch.arange(count, dtype=torch.int64, device=device)
    return (((i * 7 + rank * 13) % 255) - 127).to(torch.float32).div_(64.0).to(dtype)


def expected_exact(torch, count: int, world: int, dtype, device):
    acc = torch.zeros(count, dtype=torch.float64, device=device)
    for r in range(world):
        acc += exact_inputs(torch, count, r, torch.float64, device)
    return acc.to(dtype)


def default_variants(world: int, default_rings, max_channels: int = 32) -> list[dict]:
    """The configurations an unchanged service can run by configuration alone:
    mccs.toml's channel_count = 2 (the shipped default), MCCS_MAX_NCHANNELS =
    32 on the reference ring, and the same 32-channel budget over this
    library's link-spreading rings given as comm_patterns_override, with the
    FIFO data at the sender (the reference SHM layout) or the receiver
    (`mccs.toml [shm] locality = receiver`, config only).  `fifo`: "device"
    (the xGMI connector: FIFOs in the owning GPU's HBM) or "host" (the
    reference's own SHM memory, mlock'ed host pages registered mapped: what
    an unchanged service allocates).  `max_channels` caps the budget where
    ranks share one GPU (a rehearsal: every rank's workgroups must be
    resident at once)."""
    cap = max(2, min(32, max_channels))
    base = default_rings(world, 0)
    uniq = []
    for r in base:
        if r not in uniq:
            uniq.append(r)
    spread = (uniq * cap)[:max(1, cap // len(uniq)) * len(uniq)]
    return [
        {"name": "ch2_reference_ring_sender", "nch": 2, "rings": None, "locality": "sender", "fifo": "device"},
        {"name": "ch2_reference_ring_receiver", "nch": 2, "rings": None, "locality": "receiver", "fifo": "device"},
        {"name": "ch2_reference_ring_sender_hostfifo", "nch": 2, "rings": None, "locality": "sender",
         "fifo": "host"},
        {"name": f"ch{cap}_reference_ring_sender", "nch": cap, "rings": None, "locality": "sender", "fifo": "device"},
        {"name": f"ch{cap}_reference_ring_sender_hostfifo", "nch": cap, "rings": None, "locality": "sender",
         "fifo": "host"},
        {"name": f"ch{len(spread)}_spread_rings_sender", "nch": len(spread), "rings": spread, "locality": "sender",
         "fifo": "device"},
        {"name": f"ch{len(spread)}_spread_rings_receiver", "nch": len(spread), "rings": spread,
         "locality": "receiver", "fifo": "device"},
    ]


# Send/recv pairs the timed loop rotates through, per rank: at least this
# many bytes, as bench.py's N = 1 loop rotates (bench.py --rotate-mib), so
# no call finds its input in the 256 MB last-level cache from the call
# before (a same-buffer loop flatters plain input loads).
ROTATE_BYTES = 1152 << 20


def time_reference_driven(torch, dist, rank: int, world: int, device: int, nbytes: int, variants: list[dict],
                          warmup: int = 3, steps: int = 10, group=None, rotate_bytes: int = ROTATE_BYTES,
                          watchdog_ms: int | None = None) -> list[dict]:
    """Times every variant at `nbytes` fp32 per rank (algbw = nbytes / t per
    AllReduce, max over ranks), each gated by an exact-sum check on every
    rank.  Step i uses send/recv pair i mod P, P = ceil(rotate_bytes /
    2 nbytes) (1 = one pair reused: the same-buffer figure).  Ranks must be
    one per process; `dist` carries the handle exchange and barriers (gloo)."""
    dtype, code = torch.float32, 7
    count = nbytes // 4
    dev = torch.device("cuda", device)
    npairs = max(1, -(-rotate_bytes // (2 * nbytes))) if rotate_bytes > 0 else 1
    sends = [exact_inputs(torch, count, rank, dtype, dev) for _ in range(npairs)]
    recvs = [torch.empty_like(sends[0]) for _ in range(npairs)]
    send, recv = sends[0], recvs[0]
    want = expected_exact(torch, count, world, dtype, dev)
    from ._streams import side_stream

    stream = side_stream(torch, device, slot=1)

    def allgather(obj):
        out = [None] * world
        dist.all_gather_object(out, obj, group=group)
        return out

    def barrier():
        dist.barrier(group=group)

    def max_over_ranks(v: float) -> float:
        t = torch.tensor([v], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
        return float(t.item())

    def agree(ok: bool) -> bool:
        return max_over_ranks(0.0 if ok else 1.0) == 0.0

    # Every rank runs the same sequence of collectives whatever fails
    # locally: a failure is recorded, agreed on, and the variant skipped on
    # all ranks together.
    out = []
    for v in variants:
        res = {"variant": v["name"], "channels": v["nch"], "locality": v["locality"],
               "fifo": v.get("fifo", "device"), "buffer_pairs_rotated": npairs}
        rr, err = None, None
        try:
            rr = RefDrivenRank(rank, world, device, allgather, nch=v["nch"], rings=v["rings"],
                               locality=v["locality"], fifo=v.get("fifo", "device"), watchdog_ms=watchdog_ms)
        except Exception as e:  # noqa: BLE001
            err = f"setup: {type(e).__name__}: {e}"[:300]
        if agree(err is None):
            try:
                recv.zero_()
                torch.cuda.synchronize(dev)
                barrier()
                rr.all_reduce(send.data_ptr(), recv.data_ptr(), count, code, 0, stream.cuda_stream)
                stream.synchronize()
                k, nthr, _ = rr.last_plan
                res.update(grid=k, block=nthr)
                ok = bool(torch.equal(recv, want)) and not rr.aborted()
            except Exception as e:  # noqa: BLE001  (a refused launch: the peers' kernels hit the watchdog)
                err, ok = f"gate: {type(e).__name__}: {e}"[:300], False
            ok = agree(ok)
            res["exact"] = ok
            if ok:
                el = float("inf")
                try:
                    for i in range(warmup):
                        rr.all_reduce(sends[i % npairs].data_ptr(), recvs[i % npairs].data_ptr(), count, code, 0,
                                      stream.cuda_stream)
                    stream.synchronize()
                except Exception as e:  # noqa: BLE001
                    err = f"warmup: {type(e).__name__}: {e}"[:300]
                barrier()
                try:
                    for r_ in recvs:
                        r_.zero_()
                    torch.cuda.synchronize(dev)
                    barrier()
                    t0 = time.perf_counter()
                    for i in range(steps):
                        rr.all_reduce(sends[i % npairs].data_ptr(), recvs[i % npairs].data_ptr(), count, code, 0,
                                      stream.cuda_stream)
                    stream.synchronize()
                    el = time.perf_counter() - t0
                    # every pair the timed loop wrote holds the exact sum
                    ok2 = all(bool(torch.equal(recvs[i], want)) for i in range(min(steps, npairs))) and \
                        not rr.aborted()
                except Exception as e:  # noqa: BLE001
                    err, ok2 = f"timing: {type(e).__name__}: {e}"[:300], False
                el = max_over_ranks(el)
                ok2 = agree(ok2)
                res["exact_after_timing"] = ok2
                if ok2 and el != float("inf"):
                    ms = el / steps * 1e3
                    res.update(ms_per_allreduce=round(ms, 4),
                               algbw_GBps=round(nbytes / (ms * 1e-3) / 1e9, 2),
                               busbw_GBps=round(nbytes / (ms * 1e-3) / 1e9 * 2 * (world - 1) / world, 2),
                               steps=steps)
        if err:
            res["error"] = err
        try:
            if rr is not None:
                rr.close(barrier)
            else:
                barrier()  # the peers' close() waits here before freeing
        except Exception as e:  # noqa: BLE001
            res.setdefault("error", f"close: {e}"[:300])
        out.append(res)
    return out
