#!/usr/bin/env python3
"""Per-wave start / end skew of the headline chunk reduce (one launch).

Needs a -DMCCS_REDUCE_TRACE build:
  VARIANT_SRCS=reduce tools/build_variant.sh rtrace -DMCCS_REDUCE_TRACE
  MCCS_LIB_PATH=exp/rtrace.so python tools/reduce_skew.py
Runs the bench's workload (2 x 128 MiB fp32 -> 128 MiB, three rotated buffer
sets) in bursts of back-to-back launches and reads the LAST launch's wave
timestamps (s_memrealtime, 10 ns ticks): when waves started, when they
finished, per XCC.  The gap between the median and the last wave's end is
what a perfectly balanced split could recover at most.
"""
import ctypes
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import numpy as np
    import torch

    import mccs_amd
    from mccs_amd import _lib

    lib = _lib.load()
    fn = lib.mccs_reduce_trace
    fn.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
    fn.restype = ctypes.c_int
    n = 32 << 20
    sets = [[torch.rand(n, device="cuda") for _ in range(3)] for _ in range(3)]
    W = 8192 * 3
    buf = (ctypes.c_ulonglong * W)()
    for burst in (1, 30, 30, 30, 30):
        for i in range(burst):
            a, b, c = sets[i % 3]
            mccs_amd.reduce(c, [a, b])
        torch.cuda.synchronize()
        assert fn(buf, W) == W
        t = np.ctypeslib.as_array(buf).reshape(-1, 3).astype(np.int64)
        t = t[t[:, 1] > 0]
        st, en, xcc = t[:, 0] - t[:, 0].min(), t[:, 1] - t[:, 0].min(), t[:, 2]
        per_xcc = {int(x): round(float(en[xcc == x].mean()) / 100, 2) for x in sorted(set(xcc.tolist()))}
        q = np.percentile(en, [0, 10, 50, 90, 99, 100]) / 100
        print(json.dumps({"burst": burst, "waves": int(len(t)),
                          "start_us_p50_max": [round(float(np.median(st)) / 100, 2), round(float(st.max()) / 100, 2)],
                          "end_us_p0_10_50_90_99_100": [round(float(x), 2) for x in q],
                          "tail_us_max_minus_p50": round(float(q[5] - q[2]), 2),
                          "mean_end_us_per_xcc": per_xcc}), flush=True)


if __name__ == "__main__":
    main()
