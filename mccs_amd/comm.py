"""Communicators and collectives: the Python face of libmccs.

Mirrors the reference application API (src/libmccs/src/lib.rs:19-27):

  reference (Rust libmccs)                      here
  ------------------------------------------    ---------------------------------------------
  init_communicator_rank(id, rank, n, dev, ip)  init_communicator_rank(rank, n, dev, exchange)
  all_reduce(comm, send, recv, size, dtype,     all_reduce(comm, send, recv, size, dtype,
             op, stream) -> Result<(), Error>              op, stream)  (raises MccsError)
  all_gather(comm, send, recv, size, stream)    all_gather(comm, send, recv, size, stream)
  AllReduceDataType {Float16, Int32}            AllReduceDataType (+ Float32: the one API delta,
                                                SURVEY §8(b); + the other kernel dtypes)
  AllReduceOpType {Sum, Prod, ...}              AllReduceOpType

`size` is an element count (src/ipc/mccs/src/command.rs:71-80).  Everything
below is a thin ctypes layer over include/mccs_hip.h; the work happens in
libmccs_hip.so (HIP kernels + C++ planner).  There is no fallback path.
"""
from __future__ import annotations

import contextlib
import ctypes
import enum
import time
from dataclasses import dataclass

from . import _lib
from ._lib import DataType, RedOp, _CommConfig

_P = ctypes.POINTER
_vp, _ci, _sz = ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t


class AllReduceDataType(enum.IntEnum):
    """ipc::mccs::command::AllReduceDataType (command.rs:28-31) + Float32 and the
    remaining kernel dtypes; values are mccsDevDataType_t codes."""

    Float16 = DataType.Float16
    Int32 = DataType.Int32
    Float32 = DataType.Float32
    Int8 = DataType.Int8
    Uint8 = DataType.Uint8
    Uint32 = DataType.Uint32
    Int64 = DataType.Int64
    Uint64 = DataType.Uint64
    Float64 = DataType.Float64
    Bfloat16 = DataType.Bfloat16


class AllReduceOpType(enum.IntEnum):
    """command.rs:33-42 (PreMulSum/SumPostDiv are declared there but no kernel
    exists for them in the reference either: gen_rules.sh:15)."""

    Sum = 0
    Prod = 1
    Max = 2
    Min = 3
    PreMulSum = 4
    SumPostDiv = 5


LOCALITY_SENDER, LOCALITY_RECEIVER = 0, 1
# MCCS_FIFO_*: uncached arena (relaxed hand-offs), plain device arena
# (system-scope release/acquire), uncached arena + release fence before posts
FIFO_UNCACHED, FIFO_DEVICE, FIFO_UNCACHED_RELEASE = 0, 1, 2


@dataclass
class CommConfig:
    """comm_default_config (mccs.toml:18-20) + MI355X knobs.  None = the
    library default (mccsCommConfigDefault, which also honours the MCCS_*
    environment overrides)."""

    channel_count: int | None = None
    buffer_size: int | None = None
    lanes: int | None = None
    block_threads: int | None = None
    locality: int | None = None
    fifo_memory: int | None = None
    timeout_ms: int | None = None
    work_fifo_depth: int | None = None
    bridge_streams: int | None = None
    rings: list | None = None  # comm_patterns_override: channel_count x nranks send orders
    fifo_slots: int | None = None  # FIFO slots per connection: 8 (reference), 16, 32
    direct_bytes: int | None = None  # largest bucket (bytes per rank) for the direct two-shot kernel; < 0 never
    oneshot_bytes: int | None = None  # largest bucket for the one-shot variant; < 0 never
    ll_bytes: int | None = None  # largest bucket for the LL one-shot (uncached arenas); < 0 never

    def to_c(self, nranks: int):
        c = _CommConfig()
        _lib.load().mccsCommConfigDefault(ctypes.byref(c))
        for f, _ in _CommConfig._fields_:
            if f in ("rings", "reserved"):
                continue
            v = getattr(self, f)
            if v is not None:
                setattr(c, f, int(v))
        keep = None
        if self.rings is not None:
            flat = [int(x) for ring in self.rings for x in ring]
            if len(flat) != len(self.rings) * nranks:
                raise ValueError("each ring must list every rank once")
            keep = (_ci * len(flat))(*flat)
            c.rings = ctypes.cast(keep, _P(_ci))
            c.channel_count = len(self.rings)
        return c, keep


def _sig():
    return _lib.load()


def _ptr(x) -> int:
    return x.data_ptr() if hasattr(x, "data_ptr") else int(x)


def _stream(s) -> int:
    if s is None:
        import torch

        return torch.cuda.current_stream().cuda_stream
    return s.cuda_stream if hasattr(s, "cuda_stream") else int(s)


class Communicator:
    """One rank of a communicator (reference: MccsCommunicatorHandle)."""

    def __init__(self, handle: int):
        self._h = ctypes.c_void_p(handle)
        self._load_info()

    def _load_info(self) -> None:
        """(Re)reads the comm's profile; mccsCommConnect may shrink the lanes of
        co-located processes and settle the hand-off mode."""
        info = (_ci * 7)()
        _lib.check(_sig().mccsCommInfo(self._h, info), "mccsCommInfo")
        (self.rank, self.nranks, self.device, self.nchannels, self.lanes, self.block_threads,
         self.fifo_memory) = list(info)

    @property
    def handle(self) -> int:
        return self._h.value

    def gate_info(self) -> dict:
        """Outcome of the node gate (mccsCommGateInfo): whether it ran, the
        hand-off the comm now runs (MCCS_FIFO_*), the MCCS_GATE_* bits that
        failed and the direct variants it disabled."""
        info = (ctypes.c_int * 4)()
        _lib.check(_sig().mccsCommGateInfo(self._h, info), "mccsCommGateInfo")
        return {"ran": bool(info[0]), "fifo_mode": info[1], "failed": info[2], "disabled": info[3]}

    def guard_info(self) -> dict:
        """The comm's launch guard (mccsCommGuardInfo, launch_guard.h): the
        holder's token (0 = free), the fused-launch confirm word, finished
        workgroups of the holder, and how many workgroups ever waited for
        another launch of this comm."""
        out = (ctypes.c_uint64 * 4)()
        _lib.check(_sig().mccsCommGuardInfo(self._h, out), "mccsCommGuardInfo")
        return {"owner": out[0], "confirm": out[1], "fin": out[2], "waits": out[3]}

    def rings(self) -> list[list[int]]:
        out = []
        for ch in range(self.nchannels):
            arr = (_ci * self.nranks)()
            _lib.check(_sig().mccsCommRing(self._h, ch, arr), "mccsCommRing")
            out.append(list(arr))
        return out

    def last_algo(self) -> str | None:
        """"ring", "direct" (two-shot) or "oneshot": the algorithm of the latest
        launch (None before one)."""
        a = _sig().mccsCommLastAlgo(self._h)
        return {0: "ring", 1: "direct", 2: "oneshot", 3: "ll"}.get(a)

    def direct_enabled(self) -> bool:
        """Whether AllReduces may take the direct kernel (a direct region is
        configured and every device pair supports peer atomics)."""
        return bool(_sig().mccsCommDirectEnabled(self._h))

    def dev_comm(self) -> int:
        p = ctypes.c_void_p()
        _lib.check(_sig().mccsCommDevComm(self._h, ctypes.byref(p)), "mccsCommDevComm")
        return p.value

    def all_reduce(self, send_buf, recv_buf, size: int, data_type=AllReduceDataType.Float32,
                   op_type=AllReduceOpType.Sum, stream=None) -> None:
        all_reduce(self, send_buf, recv_buf, size, data_type, op_type, stream)

    def all_gather(self, send_buf, recv_buf, size: int, stream=None) -> None:
        all_gather(self, send_buf, recv_buf, size, stream)

    def sync(self) -> None:
        """Waits for the comm's launches; raises on a device-side timeout/abort."""
        _lib.check(_sig().mccsCommSync(self._h), "mccsCommSync")

    def abort(self) -> None:
        _lib.check(_sig().mccsCommAbort(self._h), "mccsCommAbort")

    def destroy(self) -> None:
        """mccsCommDestroy: frees the comm once its last launch completed.  No
        barrier with the peers is needed: the FIFO arena is reused only after
        every peer destroyed its side (include/mccs_hip.h)."""
        if self._h.value:
            _lib.check(_sig().mccsCommDestroy(self._h), "mccsCommDestroy")
            self._h = ctypes.c_void_p(0)


def init_all(devices: list[int], config: CommConfig | None = None) -> list[Communicator]:
    """One process drives len(devices) ranks (the reference's one-service-per-host
    model).  Devices may repeat: ranks sharing a GPU must issue collectives
    inside `group()` so they run as one launch."""
    lib = _sig()
    n = len(devices)
    cfg, keep = (config or CommConfig()).to_c(n)
    hs = (_vp * n)()
    devs = (_ci * n)(*devices)
    _lib.check(lib.mccsCommInitAll(hs, n, devs, ctypes.byref(cfg)), "mccsCommInitAll")
    del keep
    return [Communicator(hs[i]) for i in range(n)]


def init_communicator_rank(rank: int, nranks: int, device: int, exchange, config: CommConfig | None = None):
    """One rank per process.  `exchange(bytes) -> list[bytes]` all-gathers the
    per-rank connect handles (e.g. over torch.distributed/gloo); it replaces
    the reference's bootstrap ring + exchange engine."""
    lib = _sig()
    cfg, keep = (config or CommConfig()).to_c(nranks)
    hsize = lib.mccsConnectHandleSize()
    mine = (ctypes.c_char * hsize)()
    h = ctypes.c_void_p()
    t0 = time.perf_counter()
    rc = lib.mccsCommSetupRank(ctypes.byref(h), rank, nranks, device, ctypes.byref(cfg), mine)
    detail = _lib.last_error() if rc != 0 else ""
    t1 = time.perf_counter()
    del keep
    # every rank joins the exchange even after a local failure (its diagnosis
    # in place of a handle), so a peer's error never leaves the others blocked
    # in it, and every rank can say which rank failed and why
    allh = exchange(bytes(mine) if rc == 0 else b"ERR:" + detail.encode())
    if rc != 0:
        raise _lib.MccsError(rc, "mccsCommSetupRank", detail)
    comm = Communicator(h.value)
    if len(allh) != nranks or any(len(x) != hsize for x in allh):
        comm.destroy()
        failed = [(r, x[4:].decode(errors="replace")) for r, x in enumerate(allh) if x[:4] == b"ERR:"]
        if failed:
            raise RuntimeError("connect-handle exchange: " +
                               "; ".join(f"rank {r} failed mccsCommSetupRank: {d}" for r, d in failed))
        raise RuntimeError("connect-handle exchange: a peer sent malformed data")
    buf = ctypes.create_string_buffer(b"".join(allh), hsize * nranks)
    t2 = time.perf_counter()
    rc = lib.mccsCommConnect(h, buf)
    if rc != 0:
        detail = _lib.last_error()
        comm.destroy()
        raise _lib.MccsError(rc, "mccsCommConnect", detail)
    comm._load_info()
    # this rank's wall time per phase (the N > 1 bench line reports it per rank);
    # connect includes the node gate when it runs
    comm.connect_timing = {"setup_s": round(t1 - t0, 4), "exchange_s": round(t2 - t1, 4),
                           "connect_s": round(time.perf_counter() - t2, 4)}
    return comm


def all_reduce(comm: Communicator, send_buf, recv_buf, size: int, data_type=AllReduceDataType.Float32,
               op_type=AllReduceOpType.Sum, stream=None) -> None:
    """libmccs::all_reduce (collectives.rs:75-138): stream-ordered, returns after launch."""
    rc = _sig().mccsAllReduce(_ptr(send_buf), _ptr(recv_buf), int(size), int(data_type), int(op_type),
                              comm._h, _stream(stream))
    _lib.check(rc, "mccsAllReduce")


def all_gather(comm: Communicator, send_buf, recv_buf, size: int, stream=None) -> None:
    """libmccs::all_gather: `size` bytes per rank; recv holds nranks*size bytes."""
    rc = _sig().mccsAllGather(_ptr(send_buf), _ptr(recv_buf), int(size), comm._h, _stream(stream))
    _lib.check(rc, "mccsAllGather")


@contextlib.contextmanager
def group():
    """ProxyCommand::GroupCall: collectives inside are launched together at exit."""
    lib = _sig()
    _lib.check(lib.mccsGroupStart(), "mccsGroupStart")
    try:
        yield
    finally:
        _lib.check(lib.mccsGroupEnd(), "mccsGroupEnd")


def default_rings(nranks: int, channels: int = 0) -> list[list[int]]:
    """Default ring orders (host-only; no GPU needed)."""
    out = (_ci * (32 * nranks))()
    k = _sig().mccs_default_rings(nranks, channels, out, 32)
    return [list(out[c * nranks:(c + 1) * nranks]) for c in range(k)]


def host_ring_allreduce(sendbufs, recvbufs, count: int, data_type, op_type=AllReduceOpType.Sum,
                        channels: int = 1, nthreads: int = 96, buffer_size: int = 1 << 22, rings=None) -> None:
    """BASELINE configs[0]: the ring protocol on host threads over host memory
    (numpy arrays or raw host pointers; no GPU)."""
    n = len(sendbufs)
    arr = ctypes.c_void_p * max(1, n)
    sp = arr(*[x.ctypes.data if hasattr(x, "ctypes") else int(x) for x in sendbufs])
    rp = arr(*[x.ctypes.data if hasattr(x, "ctypes") else int(x) for x in recvbufs])
    ro = None
    if rings is not None:
        flat = [int(v) for r in rings for v in r]
        ro = (_ci * len(flat))(*flat)
    rc = _sig().mccs_host_ring_allreduce(n, sp, rp, int(count), int(data_type), int(op_type), channels, nthreads,
                                         buffer_size, ro)
    _lib.check(rc, "mccs_host_ring_allreduce")


def ring_profile(device: int = 0, reset: bool = True) -> dict:
    """Per-slice timing of the ring kernels on `device` (MCCS_RING_PROFILE=1
    set before communicator init): slices, mean µs waiting for peer flags,
    mean µs streaming + draining (work_us), of which drain_us is the tail
    after thread 0's wave issued its last store (store drain + barrier)."""
    out = (ctypes.c_ulonglong * 4)()
    _lib.check(_sig().mccs_ring_profile(device, out, 1 if reset else 0), "mccs_ring_profile")
    n = max(1, out[0])
    return {"slices": out[0], "wait_us": out[1] / n / 100.0, "work_us": out[2] / n / 100.0,
            "drain_us": out[3] / n / 100.0}


def direct_defaults(nranks: int) -> tuple[int, int]:
    """(oneshot_bytes, direct_bytes) the library uses by default for n ranks
    (-1 = off); host-only."""
    a, b = _ci(), _ci()
    _sig().mccs_direct_defaults(int(nranks), ctypes.byref(a), ctypes.byref(b))
    return a.value, b.value


def ll_default(nranks: int) -> int:
    """ll_bytes the library uses by default for n ranks (-1 = off); host-only."""
    return int(_sig().mccs_ll_default(int(nranks)))


def task_schema(total_bytes: int, channels: int) -> tuple[int, int]:
    a, b = _ci(), _ci()
    _sig().mccs_task_schema(total_bytes, channels, ctypes.byref(a), ctypes.byref(b))
    return a.value, b.value


__all__ = ["AllReduceDataType", "AllReduceOpType", "CommConfig", "Communicator", "init_all",
           "init_communicator_rank", "all_reduce", "all_gather", "group", "default_rings", "task_schema",
           "direct_defaults", "ll_default",
           "host_ring_allreduce", "ring_profile",
           "RedOp", "DataType"]
