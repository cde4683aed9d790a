#!/usr/bin/env python3
"""Virtual-node ring allreduce timing on ONE GPU (all ranks share its HBM).

Not the xGMI number: every rank's FIFO traffic lands in the same HBM, so this
measures protocol overhead and per-lane streaming, not link bandwidth.
  python tools/vnode_bench.py [--sizes-mib 128] [--n 2 4 8]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch

    from mccs_amd import comm as C

    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, nargs="+", default=[2, 4, 8])
    ap.add_argument("--sizes-mib", type=int, nargs="+", default=[1, 16, 128])
    ap.add_argument("--sizes-kib", type=int, nargs="+", default=None, help="bucket sizes in KiB (override MiB)")
    ap.add_argument("--lanes", type=int, nargs="+", default=[0])
    ap.add_argument("--block", type=int, default=0)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--bridge", type=int, default=0, help="CommConfig.bridge_streams (0 = library default)")
    ap.add_argument("--profile", action="store_true", help="per-slice wait/stream timing (MCCS_RING_PROFILE)")
    ap.add_argument("--graph", action="store_true", help="also time the same calls captured in one HIP graph")
    ap.add_argument("--allgather", action="store_true", help="time AllGather (size = bytes per rank) instead")
    args = ap.parse_args()
    if args.profile:
        os.environ["MCCS_RING_PROFILE"] = "1"
    for n in args.n:
        for lanes in args.lanes:
            # the ring at every size (the direct kernel has tools/direct_bench.py)
            comms = C.init_all([0] * n, C.CommConfig(lanes=lanes, block_threads=args.block,
                                                          bridge_streams=args.bridge or None,
                                                          direct_bytes=-1, oneshot_bytes=-1, ll_bytes=-1))
            for kib in (args.sizes_kib or [m << 10 for m in args.sizes_mib]):
                cnt = (kib << 10) // 4
                xs = [torch.randn(cnt, device="cuda") for _ in range(n)]
                ys = [torch.empty(n * cnt if args.allgather else cnt, device="cuda") for _ in xs]

                def call(r, st=None):
                    if args.allgather:
                        C.all_gather(comms[r], xs[r], ys[r], cnt * 4, stream=st)
                    else:
                        C.all_reduce(comms[r], xs[r], ys[r], cnt, C.AllReduceDataType.Float32, stream=st)

                def once():
                    with C.group():
                        for r in range(n):
                            call(r)

                once()
                for c in comms:
                    c.sync()
                torch.cuda.synchronize()
                if args.profile:
                    C.ring_profile(0, reset=True)
                t0 = time.perf_counter()
                for _ in range(args.iters):
                    once()
                for c in comms:
                    c.sync()
                torch.cuda.synchronize()
                dt = (time.perf_counter() - t0) / args.iters
                prof = C.ring_profile(0, reset=True) if args.profile else None
                graph_ms = None
                if args.graph:  # the same iters calls as one graph replay (no host path per call)
                    st = torch.cuda.Stream()
                    g = torch.cuda.CUDAGraph()
                    torch.cuda.synchronize()
                    with torch.cuda.graph(g, stream=st):
                        for _ in range(args.iters):
                            with C.group():
                                for r in range(n):
                                    call(r, st)
                    g.replay()
                    torch.cuda.synchronize()
                    t0 = time.perf_counter()
                    g.replay()
                    torch.cuda.synchronize()
                    graph_ms = (time.perf_counter() - t0) / args.iters * 1e3
                    del g
                print(json.dumps({"coll": "allgather" if args.allgather else "allreduce", "n": n, "lanes": comms[0].lanes, "channels": comms[0].nchannels,
                                  "block": comms[0].block_threads, "bridge": args.bridge, "KiB": kib, "ms": round(dt * 1e3, 4),
                                  "algbw_GBps": round((kib << 10) / dt / 1e9, 2), "slice_profile": prof,
                                  "graph_ms": round(graph_ms, 4) if graph_ms else None,
                                  "graph_algbw_GBps": round((kib << 10) / graph_ms / 1e6, 2) if graph_ms else None}),
                      flush=True)
                del xs, ys
            torch.cuda.synchronize()
            for c in comms:
                c.destroy()


if __name__ == "__main__":
    main()
