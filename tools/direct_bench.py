#!/usr/bin/env python3
"""Direct (two-shot, one-shot) vs ring AllReduce per call on the virtual node (all
ranks on ONE GPU, one fused launch per call).

Not the xGMI number: every rank's traffic lands in one GPU's HBM.  What it
shows is the protocol's fixed cost per call -- flag round trips, launch,
workgroup count -- which is what decides the threshold below which the
direct kernel should take a bucket.
  python tools/direct_bench.py [--n 2 4 8] [--sizes-kib 32 128 ...] [--blocks 32 128]
Per (n, size): ring / direct us per call, eager (back-to-back calls, one
sync) and graph-replayed (20 calls per graph).
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
    from mccs_amd._streams import side_stream

    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, nargs="+", default=[2, 4, 8])
    ap.add_argument("--sizes-kib", type=int, nargs="+", default=[32, 128, 512, 2048, 8192, 32768])
    ap.add_argument("--blocks", type=int, nargs="+", default=[128])
    ap.add_argument("--calls", type=int, default=100)
    ap.add_argument("--dtype", default="float16")
    ap.add_argument("--oneshot-max-kib", type=int, default=2048)
    ap.add_argument("--algos", nargs="+", default=["ring", "direct", "oneshot", "ll"],
                    help="variants to time (rocprof passes isolate one kernel mode each)")
    ap.add_argument("--allgather", action="store_true", help="time AllGather (size = bytes per rank): ring vs one-shot")
    args = ap.parse_args()
    dt = getattr(torch, args.dtype)
    code = {torch.float16: 6, torch.float32: 7, torch.bfloat16: 9}[dt]
    es = torch.empty(0, dtype=dt).element_size()
    rows = []
    st = side_stream(torch, 0, slot=1)
    for n in args.n:
        top = max(args.sizes_kib) << 10
        cfgs = {"ring": C.CommConfig(direct_bytes=-1, oneshot_bytes=-1, ll_bytes=-1),
                "direct": C.CommConfig(direct_bytes=top, oneshot_bytes=-1, ll_bytes=-1),
                "oneshot": C.CommConfig(direct_bytes=-1, ll_bytes=-1, oneshot_bytes=min(top, args.oneshot_max_kib << 10)),
                "ll": C.CommConfig(direct_bytes=-1, oneshot_bytes=-1, ll_bytes=1 << 20)}
        if len(args.blocks) == 1:
            os.environ["MCCS_DIRECT_BLOCKS"] = str(args.blocks[0])
        sets = {a: C.init_all([0] * n, cfg) for a, cfg in cfgs.items()}
        for a in [a for a in sets if a not in args.algos]:
            for c in sets.pop(a):
                c.destroy()
        for kib in args.sizes_kib:
            cnt = (kib << 10) // es
            xs = [torch.randn(cnt, device="cuda").to(dt) for _ in range(n)]
            ys = [torch.empty(n * cnt if args.allgather else cnt, dtype=dt, device="cuda") for _ in xs]
            row = {"n": n, "bytes": kib << 10}
            for algo, comms in sets.items():
                if algo == "oneshot" and kib > args.oneshot_max_kib or algo == "ll" and kib > 1024:
                    continue
                if args.allgather and algo == "direct":
                    continue
                for blocks in (args.blocks if algo != "ring" else [0]):
                    if blocks and len(args.blocks) > 1:
                        # MCCS_DIRECT_BLOCKS is read when a communicator is created
                        os.environ["MCCS_DIRECT_BLOCKS"] = str(blocks)
                        for c in comms:
                            c.destroy()
                        comms = sets[algo] = C.init_all([0] * n, cfgs[algo])

                    def once():
                        with C.group():
                            for r in range(n):
                                if args.allgather:
                                    C.all_gather(comms[r], xs[r], ys[r], cnt * es, stream=st)
                                else:
                                    C.all_reduce(comms[r], xs[r], ys[r], cnt, code, 0, stream=st)

                    for _ in range(5):
                        once()
                    st.synchronize()
                    assert comms[0].last_algo() == algo, (algo, comms[0].last_algo())
                    t0 = time.perf_counter()
                    for _ in range(args.calls):
                        once()
                    st.synchronize()
                    eager = (time.perf_counter() - t0) / args.calls
                    g = torch.cuda.CUDAGraph()
                    with torch.cuda.graph(g, stream=st):
                        for _ in range(20):
                            once()
                    g.replay()
                    torch.cuda.synchronize()
                    t0 = time.perf_counter()
                    for _ in range(5):
                        g.replay()
                    torch.cuda.synchronize()
                    graph = (time.perf_counter() - t0) / 100
                    del g
                    for c in comms:
                        c.sync()
                    key = algo if not blocks else f"{algo}_g{blocks}"
                    row[key + "_eager_us"] = round(eager * 1e6, 2)
                    row[key + "_graph_us"] = round(graph * 1e6, 2)
            rows.append(row)
            print(json.dumps(row), flush=True)
            del xs, ys
        torch.cuda.synchronize()
        for comms in sets.values():
            for c in comms:
                c.destroy()
    print(json.dumps({"tool": "direct_bench", "collective": "allgather" if args.allgather else "allreduce",
                      "dtype": args.dtype, "rows": rows}), flush=True)


if __name__ == "__main__":
    main()
