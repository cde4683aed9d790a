#!/usr/bin/env python3
"""Host cost of one eager AllReduce call (the launch path, not the kernel):
per-call wall time of C.all_reduce on a 1-rank-per-process-like comm shape,
measured while the GPU is kept busy so no call waits on the device.
  python tools/host_path.py            # 2-rank virtual node, grouped calls
Prints the median host microseconds per call for the Python face and for the
ctypes call alone."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch

    from mccs_amd import _lib
    from mccs_amd import comm as C

    n = 2
    comms = C.init_all([0] * n)
    cnt = (64 << 20) // 4  # large enough that the device stays behind the host
    xs = [torch.randn(cnt, device="cuda") for _ in range(n)]
    ys = [torch.empty_like(x) for x in xs]
    st = torch.cuda.current_stream()
    for _ in range(3):
        with C.group():
            for r in range(n):
                C.all_reduce(comms[r], xs[r], ys[r], cnt, C.AllReduceDataType.Float32, stream=st)
    torch.cuda.synchronize()
    lib = _lib.load()
    t_group, t_start, t_calls, t_end = [], [], [], []
    for _ in range(200):
        t0 = time.perf_counter()
        lib.mccsGroupStart()
        t1 = time.perf_counter()
        for r in range(n):
            C.all_reduce(comms[r], xs[r], ys[r], cnt, C.AllReduceDataType.Float32, stream=st)
        t2 = time.perf_counter()
        lib.mccsGroupEnd()
        t3 = time.perf_counter()
        t_group.append(t3 - t0)
        t_start.append(t1 - t0)
        t_calls.append((t2 - t1) / n)
        t_end.append(t3 - t2)
    torch.cuda.synchronize()
    med = lambda v: round(sorted(v)[len(v) // 2] * 1e6, 2)  # noqa: E731
    print(json.dumps({"ranks_in_group": n, "group_total_us": med(t_group), "group_start_us": med(t_start),
                      "all_reduce_enqueue_us_per_rank": med(t_calls), "group_end_launch_us": med(t_end)}))
    for c in comms:
        c.destroy()


if __name__ == "__main__":
    main()
