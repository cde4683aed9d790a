#!/usr/bin/env python3
"""Regenerates the committed golden fixtures (run in the build container).

abi_layout.json  sizeof/offsetof of every device-ABI struct, printed by
                 oracle/_ref/ref_layout -- a binary compiled from the
                 REFERENCE's own src/collectives/include/devcomm.h
                 (oracle/Makefile target `ref`).  Pinned to the reference.
ring_golden.npz  small ring-allreduce vectors: inputs and the expected output,
                 produced by the C oracle and accepted only if the independent
                 per-rank FIFO simulation (tests/ring_sim.py) agrees bit for
                 bit.  Regression vectors for the oracle and GPU parity tests.
                 Exact-sum cases ("verifiable") take their inputs and
                 expected sum from the nccl-tests verifiable generator the
                 reference vendors (genInOutFloatSum, verifiable.cu:466-512,
                 restated in oracle/verifiable.c): the inputs sum exactly in
                 any order, so the ring result must equal the generator's
                 own output bit for bit -- a reference-held expected value.
kat.json         allreduce_proto known answers (main.rs:111).
"""
import json
import os
import subprocess
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.dirname(HERE))

from oracle import oracle as orc  # noqa: E402
import ring_sim  # noqa: E402


def abi_layout():
    exe = os.path.join(ROOT, "oracle", "_ref", "ref_layout")
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "ref"], check=True)
    out = subprocess.run([exe], check=True, capture_output=True, text=True).stdout
    d = json.loads(out)
    d["_source"] = "oracle/_ref/ref_layout compiled from /root/reference/src/collectives/include/devcomm.h"
    with open(os.path.join(HERE, "abi_layout.json"), "w") as f:
        json.dump(d, f, indent=1, sort_keys=True)


CASES = {
    # name: (n, dtype, count, nch, nthreads, op, distribution)
    "loopback_1KiB_f32": (2, 7, 256, 1, 96, 0, "uniform"),
    "n4_f16_ragged": (4, 6, 20011, 2, 544, 0, "uniform"),
    "n8_f16_verifiable": (8, 6, 20000, 2, 544, 0, "verifiable"),
    "n4_f32_verifiable": (4, 7, 30011, 2, 544, 0, "verifiable"),
    "n8_bf16_verifiable": (8, 9, 12345, 2, 544, 0, "verifiable"),
    "n5_f16_verifiable_same_sign": (5, 6, 9999, 1, 160, 0, "verifiable_same_sign"),
    "n8_f32_uniform": (8, 7, 30011, 2, 544, 0, "uniform"),
    "n3_i32_prod": (3, 2, 5000, 1, 160, 1, "int"),
    "n4_bf16_sum": (4, 9, 10007, 2, 544, 0, "uniform"),
}


def gen_inputs(n, dtype, count, dist, seed):
    rng = np.random.default_rng(seed)
    npdt = orc.NP_DTYPE[dtype]
    out = []
    for _ in range(n):
        if dist == "int":
            out.append(rng.integers(-7, 8, count).astype(npdt))
        elif dist.startswith("verifiable"):
            return orc.verifiable_sum(dtype, n, count, seed, same_sign=dist.endswith("same_sign"))[0]
        else:
            f = rng.random(count, dtype=np.float32) * 2 - 1
            out.append((f.view(np.uint32) >> 16).astype(np.uint16) if dtype == 9 else f.astype(npdt))
    return out


def ring_golden():
    arrs = {}
    for i, (name, (n, dtype, count, nch, nthr, op, dist)) in enumerate(sorted(CASES.items())):
        inputs = gen_inputs(n, dtype, count, dist, 1000 + i)
        out = orc.ring_allreduce(dtype, op, inputs, nchannels=nch, nthreads=nthr)
        if dist.startswith("verifiable"):  # the generator's own expected sum, exact in any order
            _, want = orc.verifiable_sum(dtype, n, count, 1000 + i, same_sign=dist.endswith("same_sign"))
            assert np.array_equal(out.view(np.uint8), want.view(np.uint8)), name
        if dtype != 9:  # numpy has no bfloat16; bf16 cross-checked vs torch in tests
            sims = ring_sim.simulate(inputs, ["sum", "prod", "max", "min"][op], nch, nthr)
            for r in range(n):
                assert np.array_equal(sims[r].view(np.uint8), out.view(np.uint8)), (name, r)
        arrs[name + "__meta"] = np.array([n, dtype, nch, nthr, op], dtype=np.int64)
        for r in range(n):
            arrs[f"{name}__in{r}"] = inputs[r]
        arrs[name + "__out"] = out
    np.savez_compressed(os.path.join(HERE, "ring_golden.npz"), **arrs)


def kat():
    d = {"source": "src/mccs_examples/allreduce_proto/src/main.rs:27,111",
         "base": 2042, "expected": {str(n): 2042 * n + n * (n - 1) // 2 for n in (1, 2, 3, 4, 8)}}
    with open(os.path.join(HERE, "kat.json"), "w") as f:
        json.dump(d, f, indent=1)


if __name__ == "__main__":
    abi_layout()
    ring_golden()
    kat()
    print("golden fixtures written")
