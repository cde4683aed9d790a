#!/usr/bin/env python3
"""Per-step time of the N = 1 chunk reduce (configs[1]: 2 x 128 MiB fp32 ->
128 MiB, 3 buffer sets rotated) launched three ways, 60 steps each, 3 reps:

  default  eager launches on torch's default (legacy null) stream
  side     eager launches on a non-blocking side stream
  graph    the 60 launches captured in one HIP graph, replayed on the side stream

  python tools/graph_reduce_probe.py   ->  one JSON line (us per step, GB/s)

Measured on MI355X: 62.6-62.9 us per step all three ways (6,400-6,430 GB/s),
so neither the stream nor graph replay is what separated bench.py's line
(63.3 us per step) from the kernel's 62.4 us: the GPU sat idle after the
timed region's start event while the host submitted the first launch.
bench.py now starts that region behind a spin kernel (torch.cuda._sleep).
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import mccs_amd  # noqa: E402
from mccs_amd import DataType  # noqa: E402

N = (128 << 20) // 4
K = 60


def main():
    dev = torch.device("cuda", 0)
    sets = [(torch.rand(N, device=dev) * 2 - 1, torch.rand(N, device=dev) * 2 - 1, torch.empty(N, device=dev))
            for _ in range(3)]
    side = torch.cuda.Stream()
    default = torch.cuda.default_stream()
    torch.cuda.synchronize()

    def step(i, s):
        a, b, c = sets[i % 3]
        mccs_amd.reduce(c, [a, b], count=N, dtype=DataType.Float32, stream=s)

    def eager(s):
        for i in range(6):
            step(i, s)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for i in range(K):
            step(i, s)
        e1.record(s)
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / K * 1e3

    def graph():
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=side):
            for i in range(K):
                step(i, side)
        g.replay()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(side)
        with torch.cuda.stream(side):
            g.replay()
        e1.record(side)
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / K * 1e3

    res = {"default": [], "side": [], "graph": []}
    for _ in range(3):
        res["default"].append(eager(default))
        res["side"].append(eager(side))
        res["graph"].append(graph())
    gbps = {k: [round(3 * N * 4 / (us * 1e-6) / 1e9, 1) for us in v] for k, v in res.items()}
    print(json.dumps({"tool": "graph_reduce_probe", "steps": K, "us_per_step": {k: [round(x, 2) for x in v]
                                                                                for k, v in res.items()},
                      "GBps": gbps}))


if __name__ == "__main__":
    main()
