#!/usr/bin/env python3
"""Launch guard liveness with full-GPU grids.

A launch waiting on a communicator's guard keeps its workgroup slots.  A
fused virtual-node launch of the direct kernels takes min(co-resident slots,
CUs) workgroups, i.e. the whole GPU, so an eager launch and a graph replay of
the same comms issued together on two hardware queues could interleave their
workgroup dispatch and leave the guard's holder short of slots until the
watchdog.  This probe counts how often that happens: each rep replays a
one-shot AllReduce beside an eager one (1 MiB fp32 per rank, n ranks on
cuda:0, library default grid), with a short watchdog; a rep is exact, wrong,
or error (watchdog).

  python tools/guard_slots_probe.py [--n 4] [--reps 30] [--out profiles/r06_guard_slots.json]
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
F32 = 7


def run(orc, n, reps, order):
    import torch

    from mccs_amd import comm as C
    import vnode

    cfg = C.CommConfig(timeout_ms=4000, ll_bytes=-1, oneshot_bytes=8 << 20, direct_bytes=-1)
    out = {"exact": 0, "wrong": 0, "error": 0, "waits": 0}
    rng = np.random.default_rng(3 + n)
    count = (1 << 20) // 4
    comms = None
    for _ in range(reps):
        if comms is None:
            comms = C.init_all([0] * n, cfg)
            sa, sb = torch.cuda.Stream(priority=0), torch.cuda.Stream(priority=-1)
            sx = [vnode.to_dev(np.zeros(count, np.float32)) for _ in range(n)]
            rx = [torch.zeros_like(t) for t in sx]
            sy = [vnode.to_dev(np.zeros(count, np.float32)) for _ in range(n)]
            ry = [torch.zeros_like(t) for t in sy]
            with C.group():
                for r in range(n):
                    C.all_reduce(comms[r], sx[r], rx[r], count, F32, 0, stream=sb)
            torch.cuda.synchronize()
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=sb):
                with C.group():
                    for r in range(n):
                        C.all_reduce(comms[r], sx[r], rx[r], count, F32, 0, stream=sb)
            torch.cuda.synchronize()
        xs = [vnode.gen(F32, count, rng) for _ in range(n)]
        ys = [vnode.gen(F32, count, rng) for _ in range(n)]
        for r in range(n):
            sx[r].copy_(torch.from_numpy(xs[r].view(np.uint8).copy()))
            sy[r].copy_(torch.from_numpy(ys[r].view(np.uint8).copy()))
        torch.cuda.synchronize()
        w0 = sum(c.guard_info()["waits"] for c in comms)

        def eager():
            with C.group():
                for r in range(n):
                    C.all_reduce(comms[r], sy[r], ry[r], count, F32, 0, stream=sa)

        def replay():
            with torch.cuda.stream(sb):
                g.replay()

        for f in ((replay, eager) if order == "replay-first" else (eager, replay)):
            f()
        torch.cuda.synchronize()
        failed = False
        for c in comms:
            try:
                c.sync()
            except Exception:  # noqa: BLE001 - watchdog: the comm is dead
                failed = True
        out["waits"] += sum(c.guard_info()["waits"] for c in comms) - w0
        if failed:
            out["error"] += 1
            del g
            torch.cuda.synchronize()
            vnode.destroy(comms)
            comms = None
            continue
        ex = vnode.expected_allreduce(orc, xs, F32, 0, comms[0])
        ey = vnode.expected_allreduce(orc, ys, F32, 0, comms[0])
        ok = all(np.array_equal(vnode.from_dev(rx[r], F32).view(np.uint8), ex.view(np.uint8)) and
                 np.array_equal(vnode.from_dev(ry[r], F32).view(np.uint8), ey.view(np.uint8)) for r in range(n))
        out["exact" if ok else "wrong"] += 1
    if comms is not None:
        out["algo"] = comms[0].last_algo()
        del g
        torch.cuda.synchronize()
        vnode.destroy(comms)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, nargs="+", default=[2, 4])
    ap.add_argument("--reps", type=int, default=30)
    ap.add_argument("--out", default=os.path.join(ROOT, "profiles", "r06_guard_slots.json"))
    a = ap.parse_args()
    import torch

    from oracle import oracle as orc

    orc.lib()
    res = {"what": __doc__.strip().splitlines()[0], "device": torch.cuda.get_device_name(0), "runs": {}}
    for n in a.n:
        for order in ("eager-first", "replay-first"):
            key = f"n{n}/{order}"
            res["runs"][key] = run(orc, n, a.reps, order)
            print(key, res["runs"][key], flush=True)
    with open(a.out, "w") as f:
        json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
