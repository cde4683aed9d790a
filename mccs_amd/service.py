"""Application <-> backend split of libmccs (the reference's mCCS service model).

In mCCS the collectives run inside a backend (the service, src/mccs) and the
application only holds IPC-mapped views of buffers the backend allocated
(libmccs memory.rs:12-37).  Stream order crosses the process boundary through
interprocess events: the application records its per-stream event before a
request and waits on the communicator's backend event after it
(collectives.rs:86,134).  The backend makes its comm stream wait on the
application's event before launching (proxy/engine.rs:1185-1189).

This module keeps those semantics on top of libmccs_hip.so's bridge C-ABI
(mccsMemAllocShared / mccsEventCreateShared / mccsCommEventHandle /
mccsCommWaitEvent ...).  The request channel is a plain
multiprocessing.Connection: the reference's shared-memory command queues,
daemon and control plane are out of scope.

  backend process:   Backend(devices).serve(conn)
  application:       client = Client(conn); comms = client.init_all(n) ...
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass

from . import _lib
from . import comm as C

HANDLE = 64  # MCCS_IPC_HANDLE_BYTES


def _sig():
    return _lib.load()


def _h() -> ctypes.Array:
    return (ctypes.c_char * HANDLE)()


@dataclass
class DevicePtr:
    """libmccs DevicePtr: the application's mapping plus the backend's id."""
    ptr: int
    backup_mem: int  # backend allocation id (the backend's own pointer)
    device: int
    nbytes: int


class Backend:
    """The backend side: owns communicators, allocations and opened user events."""

    def __init__(self):
        self.comms: list[C.Communicator] = []
        self.allocs: dict[int, tuple[int, int]] = {}  # backend ptr -> (device, nbytes)
        self.user_events: dict[tuple[int, int], int] = {}  # (rank, app stream id) -> opened event

    # -- requests -----------------------------------------------------------
    def init_all(self, devices: list[int], config: dict | None = None) -> list[bytes]:
        self.comms = C.init_all(devices, C.CommConfig(**(config or {})))
        out = []
        for c in self.comms:
            h = _h()
            _lib.check(_sig().mccsCommEventHandle(c._h, h), "mccsCommEventHandle")
            out.append(bytes(h))
        return out

    def cuda_malloc(self, device: int, nbytes: int) -> tuple[bytes, int]:
        p = ctypes.c_void_p()
        h = _h()
        _lib.check(_sig().mccsMemAllocShared(device, nbytes, ctypes.byref(p), h), "mccsMemAllocShared")
        self.allocs[p.value] = (device, nbytes)
        return bytes(h), p.value

    def register_stream(self, rank: int, stream_id: int, event_handle: bytes) -> None:
        ev = ctypes.c_void_p()
        _lib.check(_sig().mccsEventOpenShared(self.comms[rank].device, event_handle, ctypes.byref(ev)),
                   "mccsEventOpenShared")
        self.user_events[(rank, stream_id)] = ev.value

    def all_reduce(self, calls: list[tuple]) -> None:
        """calls: (rank, send_backup, recv_backup, count, dtype, op, stream_id) per
        rank; ranks sharing a GPU are issued as one group (one fused launch)."""
        for rank, _s, _r, _n, _d, _o, sid in calls:
            _lib.check(_sig().mccsCommWaitEvent(self.comms[rank]._h, self.user_events[(rank, sid)]),
                       "mccsCommWaitEvent")
        with C.group():
            for rank, s, r, n, d, o, _sid in calls:
                st = ctypes.c_void_p()
                _lib.check(_sig().mccsCommStream(self.comms[rank]._h, ctypes.byref(st)), "mccsCommStream")
                C.all_reduce(self.comms[rank], s, r, n, d, o, st.value)

    def shutdown(self) -> None:
        import torch

        torch.cuda.synchronize()
        for c in self.comms:
            c.destroy()
        for ev in self.user_events.values():
            _sig().mccsEventDestroyShared(ev)
        for p, (dev, _n) in self.allocs.items():
            _sig().mccsMemFreeShared(dev, p)

    def serve(self, conn) -> None:
        """Request loop: (name, args) -> ("ok", result) | ("err", message)."""
        while True:
            name, args = conn.recv()
            if name == "shutdown":
                self.shutdown()
                conn.send(("ok", None))
                return
            try:
                conn.send(("ok", getattr(self, name)(*args)))
            except Exception as e:  # noqa: BLE001  (reported to the application)
                conn.send(("err", f"{type(e).__name__}: {e}"))


class Client:
    """The application side, mirroring libmccs (communicator.rs, memory.rs,
    collectives.rs) over a backend connection."""

    def __init__(self, conn):
        self.conn = conn
        self.backend_events: list[int] = []
        self.devices: list[int] = []
        self.stream_events: dict[tuple[int, int], int] = {}

    def _call(self, name, *args):
        self.conn.send((name, args))
        kind, val = self.conn.recv()
        if kind != "ok":
            raise RuntimeError(f"backend {name}: {val}")
        return val

    def init_all(self, devices: list[int], config: dict | None = None) -> list[int]:
        """InitCommunicator: returns rank ids; opens each comm's backend event."""
        handles = self._call("init_all", devices, config)
        self.devices = list(devices)
        for dev, h in zip(devices, handles):
            ev = ctypes.c_void_p()
            _lib.check(_sig().mccsEventOpenShared(dev, h, ctypes.byref(ev)), "mccsEventOpenShared")
            self.backend_events.append(ev.value)
        return list(range(len(devices)))

    def cuda_malloc(self, device: int, nbytes: int) -> DevicePtr:
        h, backup = self._call("cuda_malloc", device, nbytes)
        p = ctypes.c_void_p()
        _lib.check(_sig().mccsMemOpenShared(device, h, ctypes.byref(p)), "mccsMemOpenShared")
        return DevicePtr(p.value, backup, device, nbytes)

    def register_stream(self, rank: int, stream: int) -> None:
        ev = ctypes.c_void_p()
        h = _h()
        _lib.check(_sig().mccsEventCreateShared(self.devices[rank], ctypes.byref(ev), h), "mccsEventCreateShared")
        self.stream_events[(rank, stream)] = ev.value
        self._call("register_stream", rank, stream, bytes(h))

    def all_reduce(self, calls: list[tuple]) -> None:
        """calls: (rank, send: DevicePtr, recv: DevicePtr, count, dtype, op, stream).
        Stream-ordered like libmccs::all_reduce: returns once the backend has
        launched; later work on `stream` waits for the result."""
        for rank, *_rest, stream in calls:
            _lib.check(_sig().mccsEventRecordShared(self.stream_events[(rank, stream)], stream),
                       "mccsEventRecordShared")
        self._call("all_reduce", [(rank, s.backup_mem, r.backup_mem, int(n), int(d), int(o), stream)
                                  for rank, s, r, n, d, o, stream in calls])
        for rank, *_rest, stream in calls:
            _lib.check(_sig().mccsStreamWaitShared(stream, self.backend_events[rank]), "mccsStreamWaitShared")

    def close(self, ptrs: list[DevicePtr] = ()) -> None:
        for p in ptrs:
            _sig().mccsMemCloseShared(p.device, p.ptr)
        for ev in list(self.stream_events.values()) + self.backend_events:
            _sig().mccsEventDestroyShared(ev)
        self._call("shutdown")


def backend_main(conn) -> None:
    """Entry point of a backend process (multiprocessing spawn target)."""
    Backend().serve(conn)
