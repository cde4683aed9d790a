"""Trace-driven AllReduce jobs: BASELINE configs[4] (two concurrent jobs).

Restates the reference trace generator's measured loop
(src/mccs_examples/traffic_gen/src/main.rs:167-228) for one job:

    for iter in 0..iters:
        for op in traces:
            spin_sleep(op.compute_interval)          # simulated compute
            all_reduce(dev_ptr, dev_ptr, size/2, Float16, Sum, stream)   # in place
            cudaStreamSynchronize(stream)
        round_time = now - start                     # per-iteration time

with the shapes of workloads/setup-2_vgg.toml (574,668,960 B, 160 ms gap, 4
ranks) and setup-2_gpt_1.toml (83,886,080 B, 6 ms gap; 2 ranks there,
widened to 4 so the two jobs cover the 8 GPUs of one node).

What is added, outside the timed op: the compute phase writes fresh
gradients (an iteration- and rank-dependent exact pattern, k/64 with |k| <=
255, so any 8-term fp16/fp32 sum is exact) and every iteration's in-place
result is checked bit for bit against the integer sum.  The reference
buffer holds 0x50 bytes and is never checked; summing it in place again
every iteration overflows fp16 after a few rounds.

A job may hold several ranks of its communicator in this process (a
virtual node: ranks sharing one GPU are issued inside one group so they run
as one launch) or exactly one (one rank per process on a real node).
"""
from __future__ import annotations

import time
from dataclasses import dataclass

from . import comm as C

# name -> (message bytes, compute interval us, ranks in the toml)
SETUP2 = {
    "setup-2_vgg": (574_668_960, 160_000, 4),
    "setup-2_gpt_1": (83_886_080, 6_000, 2),
}


def spin_sleep(seconds: float) -> None:
    """spin_sleep::sleep: OS sleep for the bulk, busy-wait the last ~1 ms."""
    end = time.perf_counter() + seconds
    if seconds > 2e-3:
        time.sleep(seconds - 1e-3)
    while time.perf_counter() < end:
        pass


def exact_pattern(torch, count: int, rank: int, it: int, dev):
    """Integer numerators k in [-255, 255] of the exact gradients (value k/64)."""
    i = torch.arange(count, device=dev, dtype=torch.int64)
    return ((i * 7 + rank * 13 + it * 101) % 511) - 255


@dataclass
class IterRecord:
    iteration: int
    iter_ms: float  # compute gap + AllReduce + stream sync (traffic_gen round time)
    op_ms: float    # the AllReduce alone (HIP events on the job's stream)
    exact: bool


class TraceJob:
    """One AllReduce trace job: in-place fp16 AllReduce of `count` elements
    after a compute gap, stream-synchronised per op, validated per iteration.

    comms / rank_ids: the communicator ranks driven from this process and
    their ranks within the job (for the input pattern); nranks: job size."""

    def __init__(self, torch, name, comms, rank_ids, nranks, count, compute_s, stream, dev, dtype=None):
        self.torch = torch
        self.name = name
        self.comms = comms
        self.rank_ids = rank_ids
        self.nranks = nranks
        self.count = count
        self.compute_s = compute_s
        self.stream = stream
        self.dev = dev
        self.tdt = dtype or torch.float16
        self.code = {torch.float16: C.AllReduceDataType.Float16, torch.float32: C.AllReduceDataType.Float32,
                     torch.bfloat16: C.AllReduceDataType.Bfloat16}[self.tdt]
        with torch.cuda.stream(stream):
            self.bufs = [torch.empty(count, dtype=self.tdt, device=dev) for _ in comms]
        self.records: list[IterRecord] = []

    def _fill(self, it):
        torch = self.torch
        with torch.cuda.stream(self.stream):
            for b, r in zip(self.bufs, self.rank_ids):
                b.copy_(exact_pattern(torch, self.count, r, it, self.dev).to(torch.float32).div_(64.0))

    def _expected(self, it):
        torch = self.torch
        with torch.cuda.stream(self.stream):
            tot = torch.zeros(self.count, dtype=torch.int64, device=self.dev)
            for r in range(self.nranks):
                tot += exact_pattern(torch, self.count, r, it, self.dev)
            return tot.to(torch.float64).div_(64.0).to(self.tdt)

    def _all_reduce(self):
        if len(self.comms) == 1:
            C.all_reduce(self.comms[0], self.bufs[0], self.bufs[0], self.count, self.code, C.AllReduceOpType.Sum,
                         self.stream)
            return
        with C.group():
            for c, b in zip(self.comms, self.bufs):
                C.all_reduce(c, b, b, self.count, self.code, C.AllReduceOpType.Sum, self.stream)

    def iteration(self, it: int, record: bool = True) -> IterRecord:
        torch = self.torch
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        # compute phase: the new gradients, then the rest of the compute gap
        self._fill(it)
        self.stream.synchronize()
        spin_sleep(max(0.0, self.compute_s - (time.perf_counter() - t0)))
        ev0.record(self.stream)
        self._all_reduce()
        ev1.record(self.stream)
        self.stream.synchronize()  # traffic_gen: cudaStreamSynchronize per op
        for c in self.comms:
            c.sync()  # raises on a device-side timeout / abort
        t1 = time.perf_counter()
        exp = self._expected(it)
        self.stream.synchronize()
        ok = all(bool(torch.equal(b, exp)) for b in self.bufs)
        del exp
        rec = IterRecord(it, (t1 - t0) * 1e3, ev0.elapsed_time(ev1), ok)
        if record:
            self.records.append(rec)
        return rec

    def summary(self) -> dict:
        recs = self.records
        nb = self.count * self.bufs[0].element_size()
        op = sum(r.op_ms for r in recs) / max(1, len(recs))
        return {"job": self.name, "ranks": self.nranks, "bytes": nb, "iterations": len(recs),
                "compute_interval_ms": round(self.compute_s * 1e3, 3),
                "iter_ms_mean": round(sum(r.iter_ms for r in recs) / max(1, len(recs)), 4),
                "ms_per_call": round(op, 4), "algbw_GBps": round(nb / (op / 1e3) / 1e9, 3) if op > 0 else None,
                "exact_every_iteration": all(r.exact for r in recs)}
