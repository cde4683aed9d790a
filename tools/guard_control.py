#!/usr/bin/env python3
"""Launch guard on MI355X: what it prevents and what it costs.

  python tools/guard_control.py [--reps 6] [--out profiles/r06_launch_guard.json]

1. Control: a graph replay racing an eager launch of the
   same communicators (tests/test_gpu_launch_guard.py's scenario), with the
   guard (the default) and without it (test hook MCCS_TEST_HOOKS=1 +
   MCCS_LAUNCH_GUARD=0, read at connect).  Each rep is counted exact, wrong
   (a silent wrong sum) or error (the watchdog or a refused call); the guard's
   `waits` counter shows the overlap happened.
2. Cost: microseconds per AllReduce of graph-replayed back-to-back launches
   (50 per graph) at small sizes, guard on vs off (the guard adds one
   agent-scope CAS before a launch touches the comm's state and one
   returning add at its end, launch_guard.h; fused launches of n >= 2 rank
   slots add the leader's confirm).  n = 1 is the one-slot claim of the
   deployment shape (one rank per process and GPU).
Virtual node (every rank on cuda:0); writes one JSON file.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
os.environ["MCCS_TEST_HOOKS"] = "1"

F32, F16 = 7, 6
BIG = 8 << 20


def _streams():
    """Two streams on different hardware queues: HIP maps a process's streams
    onto a few queues (GPU_MAX_HW_QUEUES, 4 here) and runs one queue's
    kernels in order, so two streams of one priority may share a queue and
    never overlap; a queue carries one priority, so these two cannot."""
    import torch

    return torch.cuda.Stream(priority=0), torch.cuda.Stream(priority=-1)


def _cfg(C, kind, timeout_ms):
    ll = 1 << 20 if kind == "ll" else -1
    return C.CommConfig(timeout_ms=timeout_ms, lanes=2, channel_count=2, ll_bytes=ll, oneshot_bytes=-1,
                        direct_bytes=-1)


def control(orc, n, kind, guard, reps):
    import torch

    from mccs_amd import comm as C
    import vnode

    os.environ["MCCS_LAUNCH_GUARD"] = "1" if guard else "0"
    out = {"exact": 0, "wrong": 0, "error": 0, "waits": 0}
    rng = np.random.default_rng(7 + n)
    comms = None
    for rep in range(reps):
        if comms is None:
            comms = C.init_all([0] * n, _cfg(C, kind, 3000))
            sa, sb = _streams()
            cnt_x = 30001 if kind == "ll" else 1000003
            code_x = F16 if kind == "ll" else F32
            sx = [vnode.to_dev(np.zeros(cnt_x, vnode.NPDT[code_x])) for _ in range(n)]
            rx = [torch.zeros_like(t) for t in sx]
            sy = [vnode.to_dev(np.zeros(BIG, np.float32)) for _ in range(n)]
            ry = [torch.zeros_like(t) for t in sy]
            with C.group():
                for r in range(n):
                    C.all_reduce(comms[r], sx[r], rx[r], cnt_x, code_x, 0, stream=sb)
            torch.cuda.synchronize()
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=sb):
                with C.group():
                    for r in range(n):
                        C.all_reduce(comms[r], sx[r], rx[r], cnt_x, code_x, 0, stream=sb)
            torch.cuda.synchronize()
        xs = [vnode.gen(code_x, cnt_x, rng) for _ in range(n)]
        ys = [vnode.gen(F32, BIG, rng) for _ in range(n)]
        for r in range(n):
            sx[r].copy_(torch.from_numpy(xs[r].view(np.uint8).copy()))
            sy[r].copy_(torch.from_numpy(ys[r].view(np.uint8).copy()))
            rx[r].zero_()
            ry[r].zero_()
        torch.cuda.synchronize()
        w0 = sum(c.guard_info()["waits"] for c in comms)
        with C.group():
            for r in range(n):
                C.all_reduce(comms[r], sy[r], ry[r], BIG, F32, 0, stream=sa)
        with torch.cuda.stream(sb):
            g.replay()
        torch.cuda.synchronize()
        failed = False
        for c in comms:
            try:
                c.sync()
            except Exception:  # noqa: BLE001 - watchdog / abort: the comm is dead
                failed = True
        out["waits"] += sum(c.guard_info()["waits"] for c in comms) - w0
        if failed:
            out["error"] += 1
            del g
            torch.cuda.synchronize()
            vnode.destroy(comms)
            comms = None
            continue
        ex = vnode.expected_allreduce(orc, xs, code_x, 0, comms[0])
        ey = vnode.expected_allreduce(orc, ys, F32, 0, comms[0])
        ok = all(np.array_equal(vnode.from_dev(rx[r], code_x).view(np.uint8), ex.view(np.uint8)) and
                 np.array_equal(vnode.from_dev(ry[r], F32).view(np.uint8), ey.view(np.uint8)) for r in range(n))
        out["exact" if ok else "wrong"] += 1
    if comms is not None:
        del g
        torch.cuda.synchronize()
        vnode.destroy(comms)
    os.environ.pop("MCCS_LAUNCH_GUARD", None)
    return out


def cost(n, kind, nbytes, guard, iters=50, reps=20):
    import torch

    from mccs_amd import comm as C
    import vnode

    os.environ["MCCS_LAUNCH_GUARD"] = "1" if guard else "0"
    thr = dict(ll_bytes=-1, oneshot_bytes=-1, direct_bytes=-1)
    if kind == "ll":
        thr["ll_bytes"] = 1 << 20
    elif kind == "oneshot":
        thr["oneshot_bytes"] = 8 << 20
    comms = C.init_all([0] * n, C.CommConfig(timeout_ms=20000, **thr))
    count = nbytes // 2
    s = [vnode.to_dev(np.ones(count, np.float16)) for _ in range(n)]
    r_ = [torch.zeros_like(t) for t in s]
    st = torch.cuda.Stream()
    with C.group():
        for k in range(n):
            C.all_reduce(comms[k], s[k], r_[k], count, F16, 0, stream=st)
    torch.cuda.synchronize()
    algo = comms[0].last_algo()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=st):
        for _ in range(iters):
            with C.group():
                for k in range(n):
                    C.all_reduce(comms[k], s[k], r_[k], count, F16, 0, stream=st)
    torch.cuda.synchronize()
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    best = []
    for _ in range(reps):
        t0 = time.perf_counter()
        g.replay()
        torch.cuda.synchronize()
        best.append((time.perf_counter() - t0) / iters * 1e6)
    del g
    torch.cuda.synchronize()
    vnode.destroy(comms)
    os.environ.pop("MCCS_LAUNCH_GUARD", None)
    return algo, float(np.median(best)), float(np.min(best))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=6)
    ap.add_argument("--out", default=os.path.join(ROOT, "profiles", "r06_launch_guard.json"))
    a = ap.parse_args()
    import torch

    from oracle import oracle as orc

    orc.lib()
    res = {"what": "graph replay racing an eager launch of the same comms (virtual node, cuda:0); "
                   "guard on vs MCCS_LAUNCH_GUARD=0", "device": torch.cuda.get_device_name(0), "control": {},
           "cost_us_per_allreduce": {}}
    for kind in ("ring", "ll"):
        for n in (2, 4):
            for guard in (True, False):
                key = f"{kind}/n{n}/guard={'on' if guard else 'off'}"
                res["control"][key] = control(orc, n, kind, guard, a.reps)
                print(key, res["control"][key], flush=True)
    for kind, nbytes, ns in (("ring", 64 << 10, (1,)), ("ll", 32 << 10, (2, 8)), ("oneshot", 256 << 10, (2, 8)),
                             ("ring", 1 << 20, (2, 8))):
        for n in ns:
            for guard in (True, False):
                algo, med, mn = cost(n, kind, nbytes, guard)
                key = f"{kind}/n{n}/{nbytes >> 10}KiB/guard={'on' if guard else 'off'}"
                res["cost_us_per_allreduce"][key] = {"algo": algo, "median_us": round(med, 2), "min_us": round(mn, 2)}
                print(key, res["cost_us_per_allreduce"][key], flush=True)
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    with open(a.out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
