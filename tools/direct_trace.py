#!/usr/bin/env python3
"""Phase timeline of the direct AllReduce on the virtual node.

  VARIANT_SRCS=direct tools/build_variant.sh dtrace -DMCCS_DIRECT_TRACE
  MCCS_LIB_PATH=exp/dtrace.so python tools/direct_trace.py [--n 2 8] [--kib 32 512]

For each (n, size, variant) it runs a few calls, then one traced call, and
prints per rank slot the microseconds (s_memrealtime, 100 MHz) from the
earliest workgroup-0 start of the launch to each phase mark of workgroup 0:
start, phase-1 stores issued, counted out, first wait passed, phase-2 done,
counted out, second wait passed, end (direct_kernel.h kDt*; one-shot has no
phase 3).
"""
import argparse
import ctypes
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

EVENTS = ["start", "phase1", "counted1", "wait2", "phase2", "counted2", "wait3", "end", "prologue", "piece1",
          "piece3", "-"]
NE = len(EVENTS)


def main():
    import torch

    from mccs_amd import _lib
    from mccs_amd import comm as C

    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, nargs="+", default=[2, 8])
    ap.add_argument("--kib", type=int, nargs="+", default=[32, 512])
    a = ap.parse_args()
    lib = _lib.load()
    fn = lib.mccs_direct_trace
    fn.restype = ctypes.c_int
    fn.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
    buf = (ctypes.c_ulonglong * (16 * NE))()
    if fn(buf, 16 * NE) < 0:
        sys.exit("this libmccs_hip.so has no direct trace: build it with -DMCCS_DIRECT_TRACE")
    rows = []
    for n in a.n:
        cap = max(a.kib) << 10
        for variant, kw in (("direct", dict(direct_bytes=cap, oneshot_bytes=-1, ll_bytes=-1)),
                            ("direct-cached", dict(direct_bytes=cap, oneshot_bytes=-1, ll_bytes=-1, fifo_memory=C.FIFO_DEVICE)),
                            ("oneshot", dict(direct_bytes=-1, oneshot_bytes=min(cap, 64 << 20), ll_bytes=-1))):
            comms = C.init_all([0] * n, C.CommConfig(**kw))
            for kib in a.kib:
                cnt = (kib << 10) // 2
                xs = [torch.randn(cnt, device="cuda").half() for _ in range(n)]
                ys = [torch.empty_like(x) for x in xs]

                def once():
                    with C.group():
                        for r in range(n):
                            C.all_reduce(comms[r], xs[r], ys[r], cnt, 6, 0)

                for _ in range(5):
                    once()
                torch.cuda.synchronize()
                fn(buf, 16 * NE)
                once()
                torch.cuda.synchronize()
                assert comms[0].last_algo() == variant.split("-")[0]
                fn(buf, 16 * NE)
                t = [[buf[s * NE + e] for e in range(NE)] for s in range(n)]
                t0 = min(row[0] for row in t)
                per = [dict(sorted(((EVENTS[e], round((row[e] - t0) / 100.0, 2)) for e in range(NE) if row[e]),
                                   key=lambda kv: kv[1])) for row in t]
                rec = {"n": n, "kib": kib, "variant": variant, "slots_us": per}
                rows.append(rec)
                print(json.dumps(rec), flush=True)
            torch.cuda.synchronize()
            for c in comms:
                c.destroy()
    print(json.dumps({"tool": "direct_trace", "rows": rows}))


if __name__ == "__main__":
    main()
