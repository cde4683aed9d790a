"""In-process multi-device legs of the N > 1 bench line (rank 0, ranks 1..N-1
parked at a barrier).

* in_process_multi_device: the reference's own service model -- ONE process
  drives every GPU of the node (src/mccs/src/control.rs:244-282; the SHM
  connector is an in-process pointer, transport/shm/transporter.rs:76-78):
  mccsCommInitAll over devices 0..N-1 (peer access between every pair), one
  grouped AllReduce = one launch per device, exact-sum gated, algbw at the
  bucket size of the line.
* xgmi_calibration: what the links give this library's own copy kernel
  (mccs_hip_reduce_copy, 1 source -> 1 destination, the register streaming
  loop) when one side of the copy is a peer GPU's HBM: one link alone in
  each direction (pull = read the peer, push = write the peer), both
  directions of one link at once, every link of device 0 at once, and the
  ring's load -- every device pushing to every peer at once.  The ring's
  roofline is then priced against the measured per-direction rate beside
  the spec figure.

Both run only when this process sees at least `world` GPUs; on a box whose
ranks share one GPU they report "n/a".  Every exception is caught and
recorded: these legs never fail the line.
"""
from __future__ import annotations

import ctypes
import time

from ._streams import side_stream


def _hip():
    from .refdrive import hip

    h = hip()
    h.hipDeviceCanAccessPeer.argtypes = [ctypes.POINTER(ctypes.c_int), ctypes.c_int, ctypes.c_int]
    h.hipDeviceEnablePeerAccess.argtypes = [ctypes.c_int, ctypes.c_uint]
    return h


def enable_peer_access(torch, devices) -> None:
    """hipDeviceEnablePeerAccess between every ordered pair of distinct devices
    (already-enabled is fine)."""
    h = _hip()
    for a in devices:
        for b in devices:
            if a == b:
                continue
            can = ctypes.c_int(0)
            if h.hipDeviceCanAccessPeer(ctypes.byref(can), a, b) != 0 or not can.value:
                raise RuntimeError(f"device {a} cannot access device {b}")
            with torch.cuda.device(a):
                rc = h.hipDeviceEnablePeerAccess(b, 0)
            if rc not in (0, 704):  # 704 = hipErrorPeerAccessAlreadyEnabled
                raise RuntimeError(f"hipDeviceEnablePeerAccess({a} -> {b}) = {rc}")
    h.hipGetLastError()


def _exact(torch, n, rank, dev):
    i = torch.arange(n, device=dev, dtype=torch.int64)
    return ((i * 7 + rank * 13) % 511) - 255  # k/64, |k| <= 255: exact sums for <= 8 ranks


def in_process_multi_device(torch, C, world: int, nbytes: int, warmup: int = 3, steps: int = 10,
                            devices=None, config=None) -> dict:
    """One process, `world` ranks on `devices` (default 0..world-1): exact-sum
    gate, then `steps` grouped AllReduces of nbytes fp32 per rank.  `config`:
    the CommConfig (default: the library's)."""
    devices = list(devices if devices is not None else range(world))
    n = nbytes // 4
    comms = C.init_all(devices, config)
    try:
        xs, ys, sts = [], [], []
        for r, d in enumerate(devices):
            dev = torch.device("cuda", d)
            xs.append((_exact(torch, n, r, dev).to(torch.float32) / 64.0))
            ys.append(torch.empty_like(xs[-1]))
            sts.append(side_stream(torch, d, slot=0))
        for d in set(devices):
            torch.cuda.synchronize(d)

        def step():
            with C.group():
                for r in range(world):
                    C.all_reduce(comms[r], xs[r], ys[r], n, C.AllReduceDataType.Float32, C.AllReduceOpType.Sum,
                                 stream=sts[r])

        def sync_all():
            for s in sts:
                s.synchronize()
            for c in comms:
                c.sync()

        step()
        sync_all()
        ok = True
        for r, d in enumerate(devices):
            dev = torch.device("cuda", d)
            tot = torch.zeros(n, dtype=torch.int64, device=dev)
            for q in range(world):
                tot += _exact(torch, n, q, dev)
            ok = ok and bool(torch.equal(ys[r], (tot.to(torch.float64) / 64.0).to(torch.float32)))
            del tot
        res = {"devices": devices, "channels": comms[0].nchannels, "lanes": comms[0].lanes,
               "fifo_memory": comms[0].fifo_memory, "exact_sum_full_size": ok}
        if not ok:
            return res
        for _ in range(warmup):
            step()
        sync_all()
        t0 = time.perf_counter()
        for _ in range(steps):
            step()
        sync_all()
        per = (time.perf_counter() - t0) / steps
        res.update(ms_per_allreduce=round(per * 1e3, 4), algbw_GBps=round(nbytes / per / 1e9, 3),
                   busbw_GBps=round(nbytes / per / 1e9 * 2 * (world - 1) / world, 3), steps=steps)
        return res
    finally:
        for d in set(devices):
            torch.cuda.synchronize(d)
        for c in comms:
            c.destroy()


def xgmi_calibration(torch, devices, nbytes: int = 64 << 20, reps: int = 10) -> dict:
    """Link bandwidth seen by this library's copy kernel: GB/s of bytes that
    crossed a link (wall time over `reps` launches per job after a warm-up),
    with one side of every copy in a peer GPU's HBM.  `devices[0]` is the
    local GPU.  Uses mccs_hip_reduce_copy with the register streaming loop
    (the access pattern of the ring's reduce-copy): a 1 -> k copy writes k
    peers at once (push), a k -> 1 reduce reads k peers at once (pull), so
    no device runs more than two launches at a time (a process's streams
    share its 4 hardware queues; mccs_amd/_streams.py)."""
    import importlib

    R = importlib.import_module(__package__ + ".reduce")  # the module (the package exports a function `reduce`)
    devices = list(devices)
    nd = len(devices)
    distinct = len(set(devices)) == nd
    if distinct:
        enable_peer_access(torch, devices)
    n = nbytes // 4
    bufs = {}

    def buf(i, tag):
        """A buffer in the HBM of devices[i] (indices, so a one-GPU smoke run
        with repeated devices exercises the same code)."""
        if (i, tag) not in bufs:
            bufs[(i, tag)] = torch.empty(n, dtype=torch.float32, device=torch.device("cuda", devices[i])).fill_(1.0)
        return bufs[(i, tag)]

    saved = R.get_tune()

    def timed(jobs, blocks_per_cu):
        """jobs: (launching device index, dst list, src list, stream slot);
        all concurrently.  Returns GB/s of link bytes: a job moves
        max(len(dsts), len(srcs)) x nbytes across links."""
        R.tune(1, 4, 1, blocks_per_cu, 0, 0)
        streams = [side_stream(torch, devices[i], slot=slot) for i, _, _, slot in jobs]  # the legs' streams, reused

        def run(k):
            for (i, dsts, srcs, _), st in zip(jobs, streams):
                with torch.cuda.device(devices[i]):
                    for _ in range(k):
                        R.reduce_copy(dsts, srcs, count=n, stream=st)
        run(1)
        for d in set(devices):
            torch.cuda.synchronize(d)
        t0 = time.perf_counter()
        run(reps)
        for d in set(devices):
            torch.cuda.synchronize(d)
        el = time.perf_counter() - t0
        moved = sum(max(len(dsts), len(srcs)) for _, dsts, srcs, _ in jobs) * nbytes * reps
        return moved / el / 1e9

    def groups(idx):  # at most 4 destinations per launch (MCCS_REDUCE_MAX_DSTS)
        idx = list(idx)
        return [idx[k:k + 4] for k in range(0, len(idx), 4)]

    out = {"bytes_per_copy": nbytes, "reps": reps, "kernel": "mccs_hip_reduce_copy (REG loop, nt)",
           "peers_distinct_gpus": distinct, "unit": "GB/s of bytes crossing links"}
    try:
        peers = range(1, nd)
        out["one_link"] = {
            "peer": devices[1],
            "pull_GBps": round(timed([(0, [buf(0, "dst")], [buf(1, "src")], 0)], 4), 2),
            "push_GBps": round(timed([(0, [buf(1, "dst")], [buf(0, "src")], 0)], 4), 2),
            # both directions of that link at once (each side pushes)
            "bidirectional_push_GBps_total": round(
                timed([(0, [buf(1, "dst")], [buf(0, "src")], 0), (1, [buf(0, "dst")], [buf(1, "src")], 0)], 4), 2),
        }
        # every peer of device 0 alone, push and pull (link uniformity)
        out["per_peer"] = [{"peer": devices[q],
                            "pull_GBps": round(timed([(0, [buf(0, "dst")], [buf(q, "src")], 0)], 4), 2),
                            "push_GBps": round(timed([(0, [buf(q, "dst")], [buf(0, "src")], 0)], 4), 2)}
                           for q in peers]
        # every link of device 0 at once: one reduce reading all peers; pushes
        # to all peers from a 1 -> 4 and a 1 -> 3 copy on two streams
        pg = groups(peers)
        out["all_links_of_dev0"] = {
            "pull_GBps_total": round(timed([(0, [buf(0, "dsum")], [buf(q, "src") for q in peers], 0)], 4), 2),
            "push_GBps_total": round(timed([(0, [buf(q, "dst0") for q in g], [buf(0, "src")], k)
                                            for k, g in enumerate(pg)], 4 // len(pg) or 1), 2),
        }
        # the ring's load: every device pushes to every peer at once
        jobs = []
        for a in range(nd):
            others = [b for b in range(nd) if b != a]
            for k, g in enumerate(groups(others)):
                jobs.append((a, [buf(b, f"dst{a}") for b in g], [buf(a, "src")], k))
        tot = timed(jobs, max(1, 4 // max(1, len(groups(range(nd - 1))))))
        links = nd * (nd - 1)
        out["all_to_all_push"] = {"GBps_total": round(tot, 2), "directed_links": links,
                                  "GBps_per_link_direction": round(tot / links, 2)}
        out["per_link_direction_GBps"] = out["all_to_all_push"]["GBps_per_link_direction"]
    except Exception as e:  # recorded, never fatal
        out["error"] = f"{type(e).__name__}: {e}"[:300]
    finally:
        R.tune(saved["variant"], saved["unroll"], saved["policy"], saved["blocks_per_cu"], saved["stages"],
               saved["waves"])
        bufs.clear()
        for d in set(devices):
            torch.cuda.synchronize(d)
        torch.cuda.empty_cache()
    return out
