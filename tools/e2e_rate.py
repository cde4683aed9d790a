#!/usr/bin/env python3
"""End-to-end bucket rate including host<->device copies (recorded in DESIGN.md).

In deployment mCCS buckets come from and return to host memory (the
reference's IPC / gdrcopy path).  This times, on one MI355X:
  pinned host a, b (128 MiB fp32 each) --H2D--> device --reduce--> c --D2H--> pinned host
and reports each phase and the whole path: serial on one stream, and chunked
over three streams (H2D of chunk k+1 under the reduce of chunk k and the D2H
of chunk k-1).  Device-resident reduce rate is the headline; this is not.
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch

    import mccs_amd

    mib = int(sys.argv[1]) if len(sys.argv) > 1 else 128
    n = (mib << 20) // 4
    dev = torch.device("cuda", 0)
    ha = torch.rand(n).pin_memory()
    hb = torch.rand(n).pin_memory()
    hc = torch.empty(n).pin_memory()
    da, db, dc = (torch.empty(n, device=dev) for _ in range(3))
    s = torch.cuda.current_stream()

    def timed(fn, iters=10):
        fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for _ in range(iters):
            fn()
        e1.record(s)
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / iters / 1e3

    t_h2d = timed(lambda: (da.copy_(ha, non_blocking=True), db.copy_(hb, non_blocking=True)))
    t_red = timed(lambda: mccs_amd.reduce(dc, [da, db]))
    t_d2h = timed(lambda: hc.copy_(dc, non_blocking=True))
    t_all = timed(lambda: (da.copy_(ha, non_blocking=True), db.copy_(hb, non_blocking=True),
                           mccs_amd.reduce(dc, [da, db]), hc.copy_(dc, non_blocking=True)))
    torch.cuda.synchronize()
    assert torch.equal(hc, ha + hb)

    # chunked three-stream pipeline: H2D of chunk k+1 (copy-in stream) runs
    # under the reduce of chunk k (compute stream) and the D2H of chunk k-1
    # (copy-out stream); PCIe is full duplex, so the bucket costs about its
    # H2D time instead of H2D + reduce + D2H.  Events order the streams.
    s_in, s_out = torch.cuda.Stream(), torch.cuda.Stream()

    def pipelined(chunk_elems):
        starts = list(range(0, n, chunk_elems))
        ev_in = [torch.cuda.Event() for _ in starts]
        ev_red = [torch.cuda.Event() for _ in starts]
        for k, lo in enumerate(starts):
            hi = min(n, lo + chunk_elems)
            with torch.cuda.stream(s_in):
                da[lo:hi].copy_(ha[lo:hi], non_blocking=True)
                db[lo:hi].copy_(hb[lo:hi], non_blocking=True)
                ev_in[k].record(s_in)
            s.wait_event(ev_in[k])
            mccs_amd.reduce(dc[lo:hi], [da[lo:hi], db[lo:hi]], stream=s)
            ev_red[k].record(s)
            s_out.wait_event(ev_red[k])
            with torch.cuda.stream(s_out):
                hc[lo:hi].copy_(dc[lo:hi], non_blocking=True)
        s.wait_stream(s_out)  # the bucket is done when its last D2H is

    pipe = {}
    for cmib in (4, 16, 32):
        hc.zero_()
        t = timed(lambda: pipelined((cmib << 20) // 4))
        torch.cuda.synchronize()
        assert torch.equal(hc, ha + hb)
        pipe[cmib] = t
    best = min(pipe, key=pipe.get)
    nb = n * 4
    print(json.dumps({
        "bucket_MiB": mib,
        "h2d_GBps": round(2 * nb / t_h2d / 1e9, 2),
        "reduce_device_GBps": round(3 * nb / t_red / 1e9, 2),
        "d2h_GBps": round(nb / t_d2h / 1e9, 2),
        "end_to_end_ms": round(t_all * 1e3, 3),
        "end_to_end_bucket_GBps": round(nb / t_all / 1e9, 2),
        "end_to_end_host_bytes_GBps": round(3 * nb / t_all / 1e9, 2),
        "pipelined_ms_by_chunk_MiB": {k: round(v * 1e3, 3) for k, v in pipe.items()},
        "pipelined_best_chunk_MiB": best,
        "pipelined_bucket_GBps": round(nb / pipe[best] / 1e9, 2),
        "note": "serial: one stream; pipelined: chunked H2D / reduce / D2H on three streams; "
                "PCIe Gen5 x16 spec 63 GB/s per direction",
    }))


if __name__ == "__main__":
    main()
