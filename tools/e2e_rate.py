#!/usr/bin/env python3
"""End-to-end bucket rate including host<->device copies (recorded in DESIGN.md).

In deployment mCCS buckets come from and return to host memory (the
reference's IPC / gdrcopy path).  This times, on one MI355X:
  pinned host a, b (128 MiB fp32 each) --H2D--> device --reduce--> c --D2H--> pinned host
and reports each phase and the whole pipeline (serial, one stream), plus the
overlapped variant (H2D of the next bucket on a copy stream while the current
one is reduced).  Device-resident reduce rate is the headline; this is not.
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
    nb = n * 4
    print(json.dumps({
        "bucket_MiB": mib,
        "h2d_GBps": round(2 * nb / t_h2d / 1e9, 2),
        "reduce_device_GBps": round(3 * nb / t_red / 1e9, 2),
        "d2h_GBps": round(nb / t_d2h / 1e9, 2),
        "end_to_end_ms": round(t_all * 1e3, 3),
        "end_to_end_bucket_GBps": round(nb / t_all / 1e9, 2),
        "end_to_end_host_bytes_GBps": round(3 * nb / t_all / 1e9, 2),
        "note": "serial on one stream; PCIe Gen5 x16 spec 63 GB/s per direction",
    }))


if __name__ == "__main__":
    main()
