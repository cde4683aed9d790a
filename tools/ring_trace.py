#!/usr/bin/env python3
"""Slice timeline of the ring engine on a virtual node (one GPU).

Needs a -DMCCS_RING_TRACE build:
  tools/build_variant.sh trace -DMCCS_RING_TRACE
  MCCS_LIB_PATH=exp/trace.so python tools/ring_trace.py --n 2 --lanes 16 --mib 128
Prints, per rank slot and slice of lane 0 of channel 0 (s_memrealtime, 10 ns
ticks, relative to the first event): when the control wave made the slice
ready, when data waves started / finished issuing / drained, when it was
posted, and the detection latency (our ready of t+1 - prev's post of t).
"""
import argparse
import ctypes
import json
import os
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

EV = {1: "ready", 2: "start", 3: "issued", 4: "drained", 5: "added", 6: "post", 7: "enter", 8: "exit",
      9: "loaded", 10: "conn"}


def main():
    import torch

    from mccs_amd import _lib
    from mccs_amd import comm as C

    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=2)
    ap.add_argument("--lanes", type=int, default=0)
    ap.add_argument("--mib", type=int, default=128)
    ap.add_argument("--kib", type=int, default=0, help="bucket size in KiB (overrides --mib)")
    ap.add_argument("--show", type=int, default=12, help="slices printed per rank")
    ap.add_argument("--per-wave", action="store_true", help="per data wave split of each slice (rank 0)")
    ap.add_argument("--channels", type=int, default=0, help="channel count (0: default)")
    ap.add_argument("--ref-shape", action="store_true", help="the reference launch shape (see below)")
    args = ap.parse_args()
    lib = _lib.load()
    fn = lib.mccs_ring_trace_ar_sum
    fn.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
    fn.restype = ctypes.c_int
    n = args.n
    kw = {"channel_count": args.channels} if args.channels else {}
    if args.ref_shape:
        # the reference launch shape through the library: 2 channels x one
        # 544-thread workgroup, 8 slots of a 4 MiB buffer, 2-step slices,
        # cached FIFOs with system-scope fences (kRefCfg)
        os.environ["MCCS_SLICE_STEPS"] = "2"
        kw = dict(channel_count=2, block_threads=544, fifo_slots=8, buffer_size=4 << 20,
                  fifo_memory=C.FIFO_DEVICE)
        args.lanes = 1
    comms = C.init_all([0] * n, C.CommConfig(lanes=args.lanes, **kw))
    cnt = ((args.kib << 10) if args.kib else (args.mib << 20)) // 4
    xs = [torch.randn(cnt, device="cuda") for _ in range(n)]
    ys = [torch.empty_like(x) for x in xs]

    def once():
        with C.group():
            for r in range(n):
                C.all_reduce(comms[r], xs[r], ys[r], cnt, C.AllReduceDataType.Float32)
        for c in comms:
            c.sync()
        torch.cuda.synchronize()

    once()
    R, W, S, E = 8, 10, 256, 11  # ring_kernel.h kTrace*
    words = R * W * S * E
    buf = (ctypes.c_ulonglong * words)()
    assert fn(buf, words) == words  # clear
    once()
    fn(buf, words)
    import numpy as np

    a = np.ctypeslib.as_array(buf).reshape(R, W, S, E)
    nz = np.argwhere(a)
    k = len(nz)
    ev = defaultdict(lambda: defaultdict(list))  # (rank) -> (t, ev) -> [(ts, wave)]
    t0 = int(a[a > 0].min()) if k else 0
    for rank, wave, t, e in nz:
        ev[int(rank)][(int(t), EV[int(e)])].append((int(a[rank, wave, t, e]) - t0, int(wave)))
    rings = comms[0].rings()
    out = {"events": k, "n": n, "lanes": comms[0].lanes, "channels": comms[0].nchannels}
    print(json.dumps(out))
    for r in sorted(ev):
        first = {e: min((x for x, _ in ev[r].get((0, e), [])), default=None) for e in ("enter", "loaded", "conn")}
        print(f"rank {r}: enter {first['enter']} loaded {first['loaded']} conn {first['conn']} "
              f"exit {max(x for x, _ in ev[r][(0, 'exit')])}")
    nsl = max(t for r in ev for (t, e) in ev[r] if e not in ("enter", "exit", "loaded", "conn")) + 1 if k else 0
    lat, per = [], []
    for r in sorted(ev):
        prev = rings[0][(rings[0].index(r) - 1) % n]
        print(f"rank {r} (prev {prev})  t: ready start[min,max] issued[min,max] drained[max] post  | detect")
        for t in range(nsl):
            g = ev[r]
            rd = min((x for x, _ in g.get((t, "ready"), [])), default=None)
            st = [x for x, _ in g.get((t, "start"), [])]
            iss = [x for x, _ in g.get((t, "issued"), [])]
            dr = [x for x, _ in g.get((t, "drained"), [])]
            po = min((x for x, _ in g.get((t, "post"), [])), default=None)
            ppost = min((x for x, _ in ev[prev].get((t - 1, "post"), [])), default=None) if t else None
            det = rd - ppost if (rd is not None and ppost is not None) else None
            if det is not None and t > 2:
                lat.append(det)
            if po is not None and st and t > 2:
                per.append(po - min(st))
            if t < args.show:
                print(f"  {t:3d}: {rd} {min(st) if st else None},{max(st) if st else None} "
                      f"{min(iss) if iss else None},{max(iss) if iss else None} {max(dr) if dr else None} {po} | {det}")
    if lat:
        lat.sort()
        per.sort()
        print(json.dumps({"detect_ticks_median": lat[len(lat) // 2], "detect_ticks_p90": lat[9 * len(lat) // 10],
                          "start_to_post_ticks_median": per[len(per) // 2]}))
    if args.per_wave:
        # where a slice's time goes, per data wave (rank 0): start -> issued
        # (streaming), issued -> drained (the drain), drained -> added (waiting
        # for the other waves to count out of the previous slice), and the
        # slice's span from its first start to its post
        g = ev[0]
        rows = []
        for t in range(3, nsl):
            st = dict((w, x) for x, w in g.get((t, "start"), []))
            iss = dict((w, x) for x, w in g.get((t, "issued"), []))
            dr = dict((w, x) for x, w in g.get((t, "drained"), []))
            ad = dict((w, x) for x, w in g.get((t, "added"), []))
            po = min((x for x, _ in g.get((t, "post"), [])), default=None)
            waves = sorted(set(st) & set(iss) & set(dr) & set(ad))
            if not waves or po is None:
                continue
            s0 = min(st[w] for w in waves)
            rows.append({"t": t, "span": po - s0,
                         "start_skew": max(st[w] for w in waves) - s0,
                         "stream": [iss[w] - st[w] for w in waves],
                         "drain": [dr[w] - iss[w] for w in waves],
                         "countout_wait": [ad[w] - dr[w] for w in waves]})
        for r in rows[: args.show]:
            print(json.dumps(r))
        if rows:
            import statistics as stt
            print(json.dumps({
                "per_wave_summary_ticks": {
                    "span_median": stt.median(r["span"] for r in rows),
                    "start_skew_median": stt.median(r["start_skew"] for r in rows),
                    "stream_median": stt.median(x for r in rows for x in r["stream"]),
                    "stream_max_median": stt.median(max(r["stream"]) for r in rows),
                    "drain_median": stt.median(x for r in rows for x in r["drain"]),
                    "countout_wait_median": stt.median(x for r in rows for x in r["countout_wait"]),
                    "slices": len(rows)}}))
    for c in comms:
        c.destroy()


if __name__ == "__main__":
    main()
