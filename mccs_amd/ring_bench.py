"""Multi-GPU leg of bench.py: ring AllReduce algbw over xGMI (configs[2..4]).

Launched by torch.distributed.run, one rank per GPU (RANK / LOCAL_RANK /
WORLD_SIZE / MASTER_*).  torch.distributed runs on gloo and is the control
plane only (connect-handle exchange, barriers, max-over-ranks timing); every
byte of the collective moves through libmccs_hip.so's ring kernels over xGMI
P2P FIFOs -- no RCCL.

One step = one AllReduce of a per-rank bucket of S bytes; value = algbw =
S / t (allreduce_bench/src/main.rs:168), busbw = algbw * 2(n-1)/n.

Correctness gates (any failure exits non-zero, no line is printed):
  * before timing: exact-sum AllReduces at 4 MiB and at the timed size and
    dtype, bit for bit on every rank, for every transport candidate;
  * after timing: the full-size exact-sum AllReduce again;
  * every extra leg (fp16 1 GiB, AllGather, size sweep, configs[4] jobs)
    validates its own results; the direct-kernel sweep (one-shot / two-shot
    beside the ring) records a failing variant instead of failing the line.
A transport candidate is skipped when its communicator cannot be created
(e.g. IPC refuses to export that memory kind) or when it fails the gate
BEFORE timing (a wrong sum or a device watchdog in the uncached-FIFO mode on
this node's xGMI): the next candidate (cached FIFOs + system-scope fences)
is tried, and the rejection is recorded in config.rejected_before_timing.
The mode that is timed must pass every gate; a failure after timing exits
non-zero.
"""
from __future__ import annotations

import os
import subprocess
import time

from ._streams import side_stream

XGMI_LINK_GBPS_PER_DIR = 76.8  # MI355X xGMI per link per direction (spec); see DESIGN.md
HBM_PEAK_GBPS = 8000.0         # MI355X_MICROARCH.md: HBM3E 8.0 TB/s
METRIC = "device-resident reduce GB/s; ring-allreduce algbw GB/s at 1/2/4/8 MI355X"


class BenchFailure(SystemExit):
    """A correctness gate failed on some rank: the bench exits non-zero."""


# Wall-clock budget of one N > 1 run (MCCS_BENCH_BUDGET_S overrides).  The
# 1-GPU rehearsals of the whole line took 27-60 s at N = 8; on a node the
# autotune connects up to 12 candidates (each with its node gate) and every
# extra leg moves more bytes, so the default leaves room for that while
# staying well inside a driver limit of 10+ minutes for the whole command
# (torchrun start, imports, first-touch of 8 GPUs included).
DEFAULT_BUDGET_S = 360.0
AUTOTUNE_SHARE = 0.35  # of the budget: later candidates are skipped past it
# Expected wall time of each extra leg on a node (s): a leg starts only if
# this much budget is left.  From the 1-GPU rehearsals' per-leg wall_s with
# margin for a node's slower first touches.
LEG_NEED_S = {"graph_replay": 5, "configs3_fp16_1GiB": 20, "allgather_16MiB_per_rank": 8, "size_sweep_fp16": 25,
              "direct_sweep_fp16": 40, "configs4_two_jobs": 45, "reference_driven": 60, "node_legs": 40,
              "cpu_ring_baseline": 8}


class Budget:
    """Wall-clock budget of one N > 1 bench run (the line ran
    about 12 legs before printing anything, bounded only by per-kernel
    watchdogs).  The headline -- the autotune's candidates up to its share,
    the timed steps and their exact-sum gates, the CPU baseline -- always
    runs.  Every other leg runs only if, when it would start, the budget left
    covers its expected time; the decision is agreed over all ranks (the legs
    are collective, so every rank must take the same branch).  `legs` records
    each leg's wall time or its skip, and goes into the line."""

    def __init__(self, dist, seconds=None, clock=time.monotonic, group=None):
        if seconds is None:
            seconds = float(os.environ.get("MCCS_BENCH_BUDGET_S", DEFAULT_BUDGET_S))
        self.dist, self.seconds, self.clock, self.group = dist, float(seconds), clock, group
        self.t0 = clock()
        self.legs: dict = {}

    def elapsed(self) -> float:
        return self.clock() - self.t0

    def allow(self, name: str, need_s: float | None = None) -> bool:
        need = LEG_NEED_S.get(name, 0.0) if need_s is None else need_s
        at = self.elapsed()
        if agree(self.dist, at + need <= self.seconds, self.group):
            return True
        self.legs[name] = {"skipped": "budget", "at_s": round(at, 2), "need_s": need}
        return False

    def run(self, name: str, fn, need_s: float | None = None):
        """fn() if the budget allows it (its wall time recorded), else None."""
        if not self.allow(name, need_s):
            return None
        t = self.clock()
        out = fn()
        self.legs[name] = {"wall_s": round(self.clock() - t, 2)}
        return out

    def note(self, name: str, t_start: float) -> None:
        """Records a leg that always runs (started at clock value t_start)."""
        self.legs[name] = {"wall_s": round(self.clock() - t_start, 2)}

    def summary(self) -> dict:
        return {"budget_s": self.seconds, "elapsed_s": round(self.elapsed(), 2), "legs": self.legs,
                "note": "a leg starts only if the budget left covers its expected time (LEG_NEED_S); "
                        "the headline timing and its gates always run"}


def _exchange_factory(dist, world, group=None):
    """Connect-handle all-gather over the control plane (replaces the
    reference's bootstrap ring + exchange engine for this path)."""
    def exchange(b: bytes):
        out = [None] * world
        dist.all_gather_object(out, b, group=group)
        return out

    return exchange


def agree(dist, ok: bool, group=None) -> bool:
    """True only if every rank passed (MIN over ranks)."""
    import torch

    t = torch.tensor([1 if ok else 0], dtype=torch.int32)
    dist.all_reduce(t, op=dist.ReduceOp.MIN, group=group)
    return bool(t.item() == 1)


def max_over_ranks(dist, x: float, group=None) -> float:
    import torch

    t = torch.tensor([float(x)], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    return float(t.item())


def require(dist, ok: bool, what: str, group=None) -> None:
    """Collective correctness gate: every rank learns whether any rank failed."""
    if not agree(dist, ok, group):
        raise BenchFailure(f"ring bench correctness gate failed: {what}")


def _exact_numerators(torch, n_elem, rank, dev):
    # k/64 with |k| <= 255: every partial sum of <= 8 ranks is exact in fp16/bf16/fp32
    i = torch.arange(n_elem, device=dev, dtype=torch.int64)
    return ((i * 7 + rank * 13) % 511) - 255


def exact_sum_ok(torch, C, comm, rank, world, n, tdt, code, dev) -> bool:
    """Size-independent property check of one AllReduce: exact inputs, so the
    result must equal the integer sum / 64 bit for bit in any order."""
    x = (_exact_numerators(torch, n, rank, dev).to(torch.float32) / 64.0).to(tdt)
    y = torch.empty_like(x)
    C.all_reduce(comm, x, y, n, code, C.AllReduceOpType.Sum)
    comm.sync()
    tot = torch.zeros(n, device=dev, dtype=torch.int64)
    for r in range(world):
        tot += _exact_numerators(torch, n, r, dev)
    ok = bool(torch.equal(y, (tot.to(torch.float64) / 64.0).to(tdt)))
    del x, y, tot
    torch.cuda.empty_cache()
    return ok


WORKLOADS = {
    ("float32", 128): "BASELINE configs[2]",
    ("float16", 1024): "BASELINE configs[3]",
}

# BASELINE configs[4]: workloads/setup-2_vgg.toml and setup-2_gpt_1.toml
# (element counts of the fp16 messages)
SETUP2_JOBS = (("setup-2_vgg", 287_334_480), ("setup-2_gpt_1", 41_943_040))

# name -> (bench dtype tag, AllReduceDataType member, kernel symbol suffix)
DTYPES = {"float32": ("f32", "Float32", "float"), "float16": ("f16", "Float16", "half"),
          "bfloat16": ("bf16", "Bfloat16", "__nv_bfloat16")}


# A rank's workgroups must all be resident at once: channels x lanes beyond
# this is never a candidate (one 576-thread ring workgroup per CU).
MAX_RING_WORKGROUPS = 256


def _candidates(C, lanes_opts, locs, chan_opts=(None,)):
    """Transport candidates in preference order.  Within one (placement,
    channels, lanes) the hand-off modes go from cheapest to safest, each tried
    only when the one before it cannot be created or fails the exact-sum gate:
      1. uncached FIFO arena, relaxed hand-offs (drain, then post);
      2. uncached FIFO arena + a system-scope release fence before every post
         (the reference's __threadfence_system before postPeer,
         prims_simple.h:120-125,211);
      3. cached (hipMalloc) arena + system-scope release/acquire."""
    out = []
    for loc in locs:
        lname = {None: "env", C.LOCALITY_RECEIVER: "receiver", C.LOCALITY_SENDER: "sender"}[loc]
        for nch in chan_opts:
            for lanes in lanes_opts:
                if nch and lanes and nch * lanes > MAX_RING_WORKGROUPS:
                    continue
                # a correct 128 MiB AllReduce takes milliseconds: a mode whose hand-off
                # fails over this node's links is caught by the watchdog within 20 s
                # the ring at every size (the library's one-shot default would take
                # the sweep's small buckets; direct_sweep times those variants)
                kw = dict(locality=loc, lanes=lanes, timeout_ms=20000, direct_bytes=-1, oneshot_bytes=-1, ll_bytes=-1)
                if nch:
                    kw["channel_count"] = nch
                tag = f"{lname}/lanes={lanes or 'auto'}" + (f"/channels={nch}" if nch else "")
                out.append((tag, [(f"{lname}-uncached-fifo", C.CommConfig(fifo_memory=C.FIFO_UNCACHED, **kw)),
                                  (f"{lname}-uncached-fifo+release-fence",
                                   C.CommConfig(fifo_memory=C.FIFO_UNCACHED_RELEASE, **kw)),
                                  (f"{lname}-cached-fifo+system-fences",
                                   C.CommConfig(fifo_memory=C.FIFO_DEVICE, **kw))]))
    return out


def channel_options(C, world: int, ranks_share_gpu: bool) -> list:
    """Channel counts the autotune times: the default (one channel per ring,
    4 at n = 2) and, on distinct GPUs, twice that (every ring twice).  A lane
    keeps one slice of its channel in flight, so a rank's bytes in flight grow
    with channels, not lanes (lanes); two channels per ring put
    two slices on each xGMI link at once.  Results stay the reference
    algorithm's for the chosen channel count (exact-sum gated)."""
    if ranks_share_gpu or world < 2 or "MCCS_CHANNELS" in os.environ:
        return [None]
    return [None, 2 * len(C.default_rings(world, 0))]


def make_validated_comm(torch, dist, C, rank, world, device, dev, exchange, modes, full, group=None,
                        rejected=None, gate=None):
    """Creates the communicator with the first mode that every rank can
    create AND that passes the exact-sum gate on every rank (4 MiB fp32, and
    the timed size and dtype).  A mode failing the gate is recorded in
    `rejected` (list of dicts; its kind is skipped by later calls sharing the
    list) and the next mode is tried.  Returns (comm, mode name), or
    (None, None) when no mode passed.  `gate(comm) -> bool` replaces the
    exact-sum gate (CPU tests of the agreement logic)."""
    rejected = [] if rejected is None else rejected
    if gate is None:
        def gate(comm):
            return (exact_sum_ok(torch, C, comm, rank, world, (4 << 20) // 4, torch.float32,
                                 C.AllReduceDataType.Float32, dev)
                    and exact_sum_ok(torch, C, comm, rank, world, full[0], full[1], full[2], dev))
    for name, cfg in modes:
        kind = name.split("-", 1)[-1]  # e.g. "uncached-fifo"
        if any(r["kind"] == kind for r in rejected):
            continue
        try:
            comm = C.init_communicator_rank(rank, world, device, exchange, cfg)
        except Exception as e:  # noqa: BLE001  (e.g. IPC refuses this memory kind: try the next mode)
            print(f"[rank {rank}] {name}: init failed: {e}", flush=True)
            comm = None
        if not agree(dist, comm is not None, group):
            if comm is not None:
                comm.destroy()
            continue
        why = ""
        try:
            ok = bool(gate(comm))
            why = "" if ok else "exact-sum mismatch"
        except Exception as e:  # noqa: BLE001  (watchdog / HIP error on this rank)
            print(f"[rank {rank}] {name}: {e}", flush=True)
            ok, why = False, str(e)[:160]
        if agree(dist, ok, group):
            return comm, name
        print(f"[rank {rank}] {name}: rejected before timing ({why or 'failed on another rank'})", flush=True)
        rejected.append({"mode": name, "kind": kind, "rank0_reason": why if rank == 0 else None})
        try:
            comm.destroy()
        except Exception as e:  # noqa: BLE001  (a comm that hit the watchdog may refuse a clean teardown)
            print(f"[rank {rank}] {name}: destroy after rejection: {e}", flush=True)
    return None, None


def autotune(torch, dist, C, rank, world, device, dev, exchange, full, step_for, warmup=2, reps=6,
             ranks_share_gpu=False, rejected=None, budget=None):
    """Transport placement chosen on the node itself: FIFO data at the
    receiver (remote writes) or at the sender (remote reads, the reference's
    SHM layout), each at the auto lane count and at 16 and 32 lanes per
    channel (a lane count equal to auto is timed once), and on distinct GPUs
    at the default and twice the default channel count (channel_options; at
    most MAX_RING_WORKGROUPS workgroups per rank).
    Every candidate passes the exact-sum gate; the fastest (max over ranks)
    is kept.  MCCS_LOCALITY / MCCS_LANES / MCCS_CHANNELS pin a dimension.
    With a `budget`, candidates after the first one that passed are tried
    only while the autotune has used less than AUTOTUNE_SHARE of it.
    Returns (comm, mode, table)."""
    locs = [None] if "MCCS_LOCALITY" in os.environ else [C.LOCALITY_RECEIVER, C.LOCALITY_SENDER]
    # lanes per channel: auto (64 / channels; 9 at n = 8), 16 and 32 -- more
    # lanes keep more bytes in flight per xGMI link, at more flag traffic
    lanes_opts = [None] if "MCCS_LANES" in os.environ else [None, 16, 32]
    if ranks_share_gpu and "MCCS_LANES" not in os.environ:
        lanes_opts = [shared_gpu_lanes(world)]
    chan_opts = channel_options(C, world, ranks_share_gpu)
    best, table, seen = None, [], set()
    for label, modes in _candidates(C, lanes_opts, locs, chan_opts):
        if best is not None and budget is not None and not budget.allow(
                f"autotune:{label}", budget.seconds * (1 - AUTOTUNE_SHARE)):
            table.append({"mode": label, "skipped": "budget"})
            continue
        comm, mode = make_validated_comm(torch, dist, C, rank, world, device, dev, exchange, modes, full,
                                         rejected=rejected)
        if comm is None:
            table.append({"mode": label, "created": False})
            continue
        key = (mode, comm.nchannels, comm.lanes)
        if key in seen:  # auto lanes already == 16
            comm.destroy()
            continue
        seen.add(key)
        el = max_over_ranks(dist, time_steps(torch, dist, comm, step_for(comm), warmup, reps))
        # fifo_memory_run: the hand-off the candidate really ran after the
        # connect-time node gate (0 uncached, 1 cached + system fences,
        # 2 uncached + release), which may be safer than its mode's name
        table.append({"mode": mode, "channels": comm.nchannels, "lanes": comm.lanes,
                      "fifo_memory_run": comm.fifo_memory, "ms_per_step": round(el / reps * 1e3, 4)})
        if best is None or el < best[0]:
            if best is not None:
                best[1].destroy()
            best = (el, comm, mode)
        else:
            comm.destroy()
    if best is None:
        raise BenchFailure("no transport candidate passed the exact-sum gate before timing")
    return best[1], best[2], table


def shared_gpu_lanes(world: int) -> int:
    """Lanes per channel when every rank is a process on ONE GPU (a 1-GPU
    rehearsal): separate processes' ring kernels must all be resident at once
    and the GPU does not guarantee that for many large grids (4 processes x
    60 workgroups timed out on MI355X; 4 lanes ran), so keep them small;
    two processes x 4 channels x 16 lanes = 128 workgroups fit."""
    return 16 if world <= 2 else 4


def graph_replay(torch, dist, comm, call_on, calls=10):
    """Per-call time of `calls` AllReduces captured in one HIP graph (max over
    ranks), after one untimed replay.  call_on(stream) issues one AllReduce."""

    torch.cuda.synchronize()
    gs = side_stream(torch, slot=1)  # one graph stream per process (mccs_amd/_streams.py)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=gs):
        for _ in range(calls):
            call_on(gs)
    g.replay()
    torch.cuda.synchronize()
    comm.sync()
    dist.barrier()
    t0 = time.perf_counter()
    g.replay()
    torch.cuda.synchronize()
    comm.sync()
    el = time.perf_counter() - t0
    dist.barrier()
    del g
    return max_over_ranks(dist, el) / calls


def extra_fp16_1gib(torch, dist, C, comm, rank, world, dev, warmup=3, K=10):
    """BASELINE configs[3] on the communicator just measured: fp16 AllReduce
    of a 1 GiB bucket per rank, exact-sum validated at full size, algbw."""
    n = (1 << 30) // 2
    g = torch.Generator(device=dev)
    g.manual_seed(3000 + rank)
    x = (torch.rand(n, device=dev, generator=g) * 2 - 1).to(torch.float16)
    y = torch.empty_like(x)
    code = C.AllReduceDataType.Float16

    def step():
        C.all_reduce(comm, x, y, n, code, C.AllReduceOpType.Sum)

    el = max_over_ranks(dist, time_steps(torch, dist, comm, step, warmup, K))
    del x, y
    torch.cuda.empty_cache()
    require(dist, exact_sum_ok(torch, C, comm, rank, world, n, torch.float16, code, dev), "configs[3] fp16 1 GiB")
    per = el / K
    return {"workload": f"{world}x ring allreduce, 1 GiB float16 buckets (BASELINE configs[3])",
            "ms_per_step": round(per * 1e3, 4), "algbw_GBps": round((1 << 30) / per / 1e9, 3),
            "busbw_GBps": round((1 << 30) / per / 1e9 * 2 * (world - 1) / world, 3), "steps": K,
            "validated_exact_sum_full_size": True}


def extra_allgather(torch, dist, C, comm, rank, world, dev, mib=16, warmup=3, K=10):
    """The other reachable collective (all_gather.h): AllGather of `mib` MiB
    per rank on the same communicator; every gathered segment checked byte
    for byte.  algbw = gathered bytes / t (nccl-tests convention)."""
    nb = mib << 20
    i = torch.arange(nb, device=dev, dtype=torch.int32)
    x = ((i * 31 + rank * 101) % 251).to(torch.uint8)
    y = torch.empty(world * nb, dtype=torch.uint8, device=dev)

    def step():
        C.all_gather(comm, x, y, nb)

    el = max_over_ranks(dist, time_steps(torch, dist, comm, step, warmup, K))
    ok = all(bool(torch.equal(y[r * nb:(r + 1) * nb], ((i * 31 + r * 101) % 251).to(torch.uint8)))
             for r in range(world))
    require(dist, ok, "AllGather 16 MiB per rank")
    per = el / K
    algbw = world * nb / per / 1e9
    del x, y, i
    torch.cuda.empty_cache()
    return {"ms_per_step": round(per * 1e3, 4), "algbw_GBps": round(algbw, 3),
            "busbw_GBps": round(algbw * (world - 1) / world, 3), "steps": K, "validated_bytes": True}


# the reference's evaluation sweep (eval/plot/single_app/allreduce_{4,8}gpu.csv:
# fp16 "half", 32 KiB ... 512 MiB)
SWEEP_BYTES = (32768, 131072, 524288, 2097152, 8388608, 33554432, 134217728, 536870912)


def size_sweep(torch, dist, C, comm, rank, world, dev, warmup=3, K=20, graph_upto=8 << 20):
    """fp16 AllReduce latency / algbw / busbw over the reference's eval sizes
    (allreduce_bench semantics: algbw = bytes / t, busbw = algbw * 2(n-1)/n),
    each size exact-sum validated.  Up to `graph_upto` bytes the same call
    is also timed captured in a HIP graph (graph_latency_us): the eager path's
    overhead over the device-side time."""
    rows = []
    for nb in SWEEP_BYTES:
        n = nb // 2
        x = torch.empty(n, dtype=torch.float16, device=dev).uniform_(-1, 1)
        y = torch.empty_like(x)

        def step():
            C.all_reduce(comm, x, y, n, C.AllReduceDataType.Float16, C.AllReduceOpType.Sum)

        el = max_over_ranks(dist, time_steps(torch, dist, comm, step, warmup, K)) / K
        gl = None
        if nb <= graph_upto:
            # 10 captured calls per size: a work-FIFO communicator (e.g. doubled
            # channels) takes graph-arena entries per captured call (2048 in all)
            try:
                gl = graph_replay(torch, dist, comm, lambda st: C.all_reduce(
                    comm, x, y, n, C.AllReduceDataType.Float16, C.AllReduceOpType.Sum, st), calls=10)
            except Exception as e:  # noqa: BLE001  (informational column only)
                print(f"[rank {rank}] sweep graph replay {nb} B: {e}", flush=True)
                gl = None
            gl = max_over_ranks(dist, gl if gl is not None else -1.0)
            gl = gl if gl > 0 else None
        del x, y
        require(dist, exact_sum_ok(torch, C, comm, rank, world, n, torch.float16, C.AllReduceDataType.Float16, dev),
                f"size sweep {nb} B")
        algbw = nb / el / 1e9
        row = {"bytes": nb, "latency_us": round(el * 1e6, 2), "algbw_GBps": round(algbw, 3),
               "busbw_GBps": round(algbw * 2 * (world - 1) / world, 3), "exact": True}
        if gl is not None:
            row["graph_latency_us"] = round(gl * 1e6, 2)
        rows.append(row)
    return rows


def direct_sweep(torch, dist, C, rank, world, device, dev, exchange, config, ring_rows, upto=32 << 20,
                 oneshot_upto=2 << 20, warmup=3, K=20):
    """The direct AllReduce variants (direct_kernel.h) beside the ring over the
    sweep's sizes up to `upto`: two-shot and one-shot communicators built with
    the measured transport's config, every size exact-sum validated, eager
    and graph-replayed latency per call (max over ranks).  ring_rows: the
    size sweep's rows of the ring.  Ends with the thresholds the table
    supports (the largest size each variant still beats the ring).

    Informational and failure-isolated: each measurement runs with no
    collective inside it, the ranks then agree on its success, and a variant
    that fails anywhere (no peer atomics, watchdog, wrong sum) is recorded
    and dropped on every rank without failing the line."""
    import dataclasses

    out = {"sizes": [nb for nb in SWEEP_BYTES if nb <= upto], "rows": []}
    ring = {r["bytes"]: r for r in ring_rows}
    comms, dead = {}, {}
    code = C.AllReduceDataType.Float16
    for algo, kw in (("direct", dict(direct_bytes=upto, oneshot_bytes=-1, ll_bytes=-1)),
                     ("oneshot", dict(direct_bytes=-1, oneshot_bytes=oneshot_upto, ll_bytes=-1)),
                     ("ll", dict(direct_bytes=-1, oneshot_bytes=-1, ll_bytes=1 << 20))):
        cfg = dataclasses.replace(config or C.CommConfig(), **kw)
        try:
            comms[algo] = C.init_communicator_rank(rank, world, device, exchange, cfg)
            # the LL one-shot needs no peer atomics (no remote atomics at all)
            ok = algo == "ll" or comms[algo].direct_enabled()
            err = None if ok else "direct kernel disabled: no peer atomics between these devices"
        except Exception as e:  # noqa: BLE001
            ok, err = False, f"{type(e).__name__}: {e}"[:200]
        if not agree(dist, ok):
            dead[algo] = err or "failed on another rank"
    out["p2p_atomics"] = "direct" not in dead or "peer atomics" not in dead.get("direct", "")
    for nb in out["sizes"]:
        n = nb // 2
        x = torch.empty(n, dtype=torch.float16, device=dev).uniform_(-1, 1)
        y = torch.empty_like(x)
        row = {"bytes": nb}
        if nb in ring:
            row["ring_us"] = ring[nb]["latency_us"]
            if "graph_latency_us" in ring[nb]:
                row["ring_graph_us"] = ring[nb]["graph_latency_us"]
        for algo, cm in comms.items():
            if algo in dead or (algo == "oneshot" and nb > oneshot_upto) or (algo == "ll" and nb > 1 << 20):
                continue
            el = gl = None
            err = None
            dist.barrier()
            try:
                for _ in range(warmup):
                    C.all_reduce(cm, x, y, n, code, C.AllReduceOpType.Sum)
                torch.cuda.synchronize()
                cm.sync()
                t0 = time.perf_counter()
                for _ in range(K):
                    C.all_reduce(cm, x, y, n, code, C.AllReduceOpType.Sum)
                torch.cuda.synchronize()
                cm.sync()
                el = (time.perf_counter() - t0) / K
                if cm.last_algo() != algo:
                    raise RuntimeError(f"took {cm.last_algo()}")
                gs = side_stream(torch, slot=1)
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g, stream=gs):
                    for _ in range(10):
                        C.all_reduce(cm, x, y, n, code, C.AllReduceOpType.Sum, gs)
                g.replay()
                torch.cuda.synchronize()
                cm.sync()
                t0 = time.perf_counter()
                g.replay()
                torch.cuda.synchronize()
                cm.sync()
                gl = (time.perf_counter() - t0) / 10
                del g
                if not exact_sum_ok(torch, C, cm, rank, world, n, torch.float16, code, dev):
                    raise RuntimeError("exact-sum check failed")
            except Exception as e:  # noqa: BLE001
                err = f"{type(e).__name__}: {e}"[:200]
            if not agree(dist, err is None):
                dead[algo] = f"{nb} B: " + (err or "failed on another rank")
                continue
            row[f"{algo}_us"] = round(max_over_ranks(dist, el) * 1e6, 2)
            row[f"{algo}_graph_us"] = round(max_over_ranks(dist, gl) * 1e6, 2)
        out["rows"].append(row)
        del x, y
    best = {}
    for algo in ("direct", "oneshot", "ll"):
        wins = [r["bytes"] for r in out["rows"] if f"{algo}_graph_us" in r and "ring_graph_us" in r
                and r[f"{algo}_graph_us"] < r["ring_graph_us"]]
        best[f"{algo}_beats_ring_upto_bytes"] = max(wins) if wins else 0
    # what the library's defaults pick at each size (thresholds of api.cpp)
    os_b, d_b = C.direct_defaults(world)
    ll_b = C.ll_default(world)
    best["default_thresholds"] = {"ll_bytes": ll_b, "oneshot_bytes": os_b, "direct_bytes": d_b}
    for r in out["rows"]:
        nb = r["bytes"]
        pick = ("ll" if 0 < nb <= ll_b else "oneshot" if 0 < nb <= os_b else "direct" if 0 < nb <= d_b else "ring")
        if not out["p2p_atomics"] or f"{pick}_graph_us" not in r and pick != "ring":
            pick = "ring"
        r["default_algo"] = pick
    out["summary"] = best
    if dead:
        out["failed"] = dead
    try:
        torch.cuda.synchronize()
    finally:
        # every rank's last kernel is done before the timing's next step
        dist.barrier()
        for cm in comms.values():
            try:
                cm.destroy()
            except Exception:  # noqa: BLE001
                pass
        dist.barrier()
    return out


def out_links(rings, rank):
    """Distinct xGMI links this rank sends on (one per distinct ring successor)."""
    nxt = set()
    for order in rings:
        p = order.index(rank)
        nxt.add(order[(p + 1) % len(order)])
    return len(nxt)


_out_links = out_links  # tools/ and older tests


def time_steps(torch, dist, comm, step, warmup, K, group=None):
    for _ in range(warmup):
        step()
    comm.sync()
    torch.cuda.synchronize()
    dist.barrier(group=group)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(K):
        step()
    torch.cuda.synchronize()
    comm.sync()
    t1 = time.perf_counter()
    dist.barrier(group=group)
    return t1 - t0


_time_steps = time_steps  # tools/ipc_ab.py


def host_record() -> dict:
    """nproc / lscpu summary of the host the CPU baseline ran on."""
    rec = {"affinity_threads": len(os.sched_getaffinity(0)), "os_cpu_count": os.cpu_count()}
    try:
        rec["nproc"] = int(subprocess.run(["nproc"], capture_output=True, text=True, timeout=10).stdout.strip())
    except Exception:  # noqa: BLE001
        rec["nproc"] = None
    try:
        out = subprocess.run(["lscpu"], capture_output=True, text=True, timeout=10).stdout
        keep = ("Model name", "Socket(s)", "Core(s) per socket", "Thread(s) per core", "CPU(s)", "NUMA node(s)")
        for line in out.splitlines():
            k, _, v = line.partition(":")
            if k.strip() in keep:
                rec["lscpu " + k.strip()] = v.strip()
    except Exception:  # noqa: BLE001
        pass
    return rec


def gpu_bus_id(device: int) -> str:
    """PCI bus id of a visible device ("ordinal:N" if the runtime will not
    say): device ordinals are local to a process, bus ids are not."""
    import ctypes

    try:
        hip = ctypes.CDLL("libamdhip64.so")
        buf = ctypes.create_string_buffer(64)
        if hip.hipDeviceGetPCIBusId(buf, 63, device) == 0 and buf.value:
            return buf.value.decode()
    except OSError:
        pass
    return f"ordinal:{device}"


def ranks_share_gpu(dist, device: int, world: int, group=None) -> bool:
    """Whether two ranks of `group` drive the same physical GPU (a 1-GPU
    rehearsal), from their PCI bus ids -- not from this process's device
    count, which per-rank device visibility (HIP_VISIBLE_DEVICES) would make
    1 on a full node."""
    ids = [None] * world
    dist.all_gather_object(ids, gpu_bus_id(device), group=group)
    return len(set(ids)) < world


def cpu_ring_baseline(world: int, nbytes: int, nchannels: int, budget_s: float = 4.0) -> dict:
    """SURVEY §8(d) configs[2]: the same ring schedule run by host threads
    over host memory (mccs_host_ring_allreduce: `world` ranks x `nchannels`
    threads, FIFOs in shared memory), on a bounded sample of the bucket.
    value = sample bytes / t (algbw, as the GPU line)."""
    import numpy as np

    from mccs_amd import comm as C

    n = nbytes // 4
    rng = np.random.default_rng(0x6D636373)
    send = [(rng.random(n, dtype=np.float32) * 2 - 1) for _ in range(world)]
    recv = [np.empty_like(x) for x in send]
    C.host_ring_allreduce(send, recv, n, C.AllReduceDataType.Float32, channels=nchannels, nthreads=544)
    reps, t0 = 0, time.perf_counter()
    while True:
        C.host_ring_allreduce(send, recv, n, C.AllReduceDataType.Float32, channels=nchannels, nthreads=544)
        reps += 1
        el = time.perf_counter() - t0
        if el >= budget_s or reps >= 200:
            break
    return {"value": round(nbytes * reps / el / 1e9, 3), "unit": "GB/s algbw (S/t)", "threads": world * nchannels,
            "kind": "port", "sample": f"{world} ranks x {nbytes >> 20} MiB fp32, {nchannels} channels, host-thread "
                                      f"ring (same schedule and FIFO protocol), {reps} AllReduces in {el:.2f}s"}


# The ring's only counter-measured traffic: the n = 2 virtual node (one GPU,
# rocprofv3 FETCH_SIZE / WRITE_SIZE with the gfx950 corrections), carried in
# the N > 1 line under its own name so nobody reads it as a node measurement.
VNODE_N2_TRAFFIC = {"traffic_over_algorithmic": 1.0042, "where": "n = 2 virtual node (both ranks on one MI355X), "
                    "128 MiB fp32, rocprofv3 PMC", "source": "profiles/r06_ring_vnode_summary.json pmc_n2 (r04: 1.0045)"}
TRAFFIC_NOT_MEASURED = ("not measured on the node: the PMC passes run on the 1-GPU box only (no 8-GPU box is "
                        "available to this repo's runs); see traffic_virtual_node_n2 for the one measured ratio")


def ring_roofline(world, nbytes, per_step_s, links, ranks_share_gpu, kernel):
    """Bound of one rank's ring AllReduce.  On a node: the xGMI links the rank
    sends on, per-rank link bytes 2(n-1)/n*S.  When every rank shares one
    GPU (a 1-GPU rehearsal) no byte crosses xGMI and the bound is that GPU's
    HBM: all n ranks' algorithmic HBM bytes, (6n-4)*S per AllReduce (per
    rank: 2 + 3(n-2) + 4 + 3(n-2) + 2 = 6n-4 chunk reads/writes of S/n)."""
    if ranks_share_gpu:
        hbm = (6 * world - 4) * nbytes
        ach = hbm / per_step_s / 1e9
        return {"bound": "hbm", "achieved": round(ach, 2), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                "frac": round(ach / HBM_PEAK_GBPS, 4), "traffic": None, "traffic_note": TRAFFIC_NOT_MEASURED,
                "traffic_virtual_node_n2": VNODE_N2_TRAFFIC, "kernel": kernel,
                "note": f"ranks share one GPU: (6n-4)*S = {hbm} algorithmic HBM bytes per AllReduce, all n ranks"}
    link_bytes = 2 * (world - 1) / world * nbytes
    ach = link_bytes / per_step_s / 1e9
    peak = links * XGMI_LINK_GBPS_PER_DIR
    return {"bound": "xgmi", "achieved": round(ach, 2), "peak": peak, "unit": "GB/s", "frac": round(ach / peak, 4),
            "traffic": None, "traffic_note": TRAFFIC_NOT_MEASURED, "traffic_virtual_node_n2": VNODE_N2_TRAFFIC,
            "kernel": kernel,
            "note": f"per-rank link bytes 2(n-1)/n*S over {links} distinct outgoing links x "
                    f"{XGMI_LINK_GBPS_PER_DIR} GB/s per direction (spec)"}


def ring_line(*, world, steps, warmup, per_step_s, nbytes, dt_name, comm_info, rings, mode, tune_table, prof,
              ranks_share_gpu, cpu_baseline, extras=None, calibration=None) -> dict:
    """The N > 1 bench line (pure: no GPU, unit-tested on CPU)."""
    algbw = nbytes / per_step_s / 1e9
    line = {
        "metric": METRIC,
        "submetric": "ring_allreduce_algbw_GBps",
        "value": round(algbw, 3),
        "unit": "GB/s",
        "n_gpus": world,
        "steps": steps,
        "warmup": warmup,
        "ms_per_step": round(per_step_s * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": DTYPES[dt_name][0],
        "data": "synthetic uniform[-1,1) per rank, device-resident buckets",
        "config": {
            "workload": f"{world}x MI355X ring allreduce over xGMI P2P, {nbytes >> 20} MiB {dt_name} "
                        f"buckets, chunked FIFO pipeline ({WORKLOADS.get((dt_name, nbytes >> 20), 'custom')})",
            "bytes_per_rank": nbytes, **comm_info, "rings": rings, "fifo_mode": mode,
            "transport_autotune": tune_table,
            "validated_exact_sum_4MiB": True, "validated_exact_sum_full_size_before_timing": True,
            "validated_exact_sum_full_size_after_timing": True,
            "busbw_GBps": round(algbw * 2 * (world - 1) / world, 3), "parallelism": f"ring{world}",
            "rank0_slice_profile": prof,
            # ranks sharing one GPU (a 1-GPU box): FIFO hand-offs stay in HBM, no xGMI link
            "ranks_share_gpu": ranks_share_gpu,
        },
        "roofline": ring_roofline(world, nbytes, per_step_s, out_links(rings, 0), ranks_share_gpu,
                                  "ring_multi_kernel<AllReduce, " + DTYPES[dt_name][2] + ", Sum>"),
        "cpu_baseline": cpu_baseline,
    }
    for k, v in (extras or {}).items():
        if v is not None:
            line["config"][k] = v
    per_dir = (calibration or {}).get("per_link_direction_GBps")
    rf = line["roofline"]
    if rf["bound"] == "xgmi" and per_dir:
        # the same links priced at the rate this node's copy kernel measured
        # with every device pushing to every peer at once (node_probe)
        links = out_links(rings, 0)
        rf["peak_calibrated"] = round(links * per_dir, 2)
        rf["frac_calibrated"] = round(rf["achieved"] / rf["peak_calibrated"], 4)
        rf["calibration"] = f"{links} links x {per_dir} GB/s per direction (all-to-all push, measured this run)"
    return line


def run(args, cpu_sum_baseline=None):
    """`cpu_sum_baseline(world, nbytes, dtype_code) -> dict`: the host-CPU
    baseline leg, supplied by bench.py (it times the oracle's threaded C sum,
    which the product package never imports)."""
    import torch
    import torch.distributed as dist

    from mccs_amd import comm as C

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", str(args.gpus)))
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    ndev = torch.cuda.device_count()
    device = local % max(1, ndev)
    torch.cuda.set_device(device)
    dev = torch.device("cuda", device)
    if not dist.is_initialized():
        import datetime

        # a rank that dies mid-collective should end the job in minutes, not gloo's default 30
        dist.init_process_group("gloo", rank=rank, world_size=world, timeout=datetime.timedelta(seconds=600))
    try:
        if getattr(args, "jobs", None) in ("setup2", "setup2-interleaved"):
            return run_setup2(args, torch, dist, C, rank, world, device, dev,
                              interleaved=args.jobs.endswith("interleaved"), cpu_sum_baseline=cpu_sum_baseline)
        return _run_ring(args, torch, dist, C, rank, world, device, dev, ndev, cpu_sum_baseline)
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


def _run_ring(args, torch, dist, C, rank, world, device, dev, ndev, cpu_sum_baseline=None):
    budget = Budget(dist)
    exchange = _exchange_factory(dist, world)
    dt_name = args.dtype
    tdt = {"float32": torch.float32, "float16": torch.float16, "bfloat16": torch.bfloat16}[dt_name]
    code = getattr(C.AllReduceDataType, DTYPES[dt_name][1])
    esize = torch.tensor([], dtype=tdt).element_size()
    nbytes = args.size_mib << 20
    n = nbytes // esize
    full = (n, tdt, code)

    # per-slice wait / stream timing on this rank's GPU: reported with the result
    os.environ.setdefault("MCCS_RING_PROFILE", "1")
    g = torch.Generator(device=dev)
    g.manual_seed(1000 + rank)
    x = (torch.rand(n, device=dev, generator=g) * 2 - 1).to(tdt)
    y = torch.empty_like(x)
    stream = torch.cuda.current_stream()

    def step_for(cm):
        return lambda: C.all_reduce(cm, x, y, n, code, C.AllReduceOpType.Sum, stream)

    tune_table = None
    share = ranks_share_gpu(dist, device, world)
    rejected = []
    t = budget.clock()
    if getattr(args, "no_autotune", False):
        lanes = shared_gpu_lanes(world) if share and "MCCS_LANES" not in os.environ else None
        comm, mode = make_validated_comm(torch, dist, C, rank, world, device, dev, exchange,
                                         _candidates(C, [lanes], [None])[0][1], full, rejected=rejected)
        if comm is None:
            raise BenchFailure("no FIFO mode passed the exact-sum gate before timing")
    else:
        comm, mode, tune_table = autotune(torch, dist, C, rank, world, device, dev, exchange, full, step_for,
                                          ranks_share_gpu=share, rejected=rejected, budget=budget)
    budget.note("autotune", t)
    t = budget.clock()
    K = args.steps
    C.ring_profile(device, reset=True)
    per_step = max_over_ranks(dist, time_steps(torch, dist, comm, step_for(comm), args.warmup, K)) / K
    prof = C.ring_profile(device, reset=True)
    ok = exact_sum_ok(torch, C, comm, rank, world, n, tdt, code, dev)
    if os.environ.get("MCCS_BENCH_INJECT_MISMATCH") == "1":
        ok = False  # fault injection: the bench must exit non-zero
    require(dist, ok, "full-size exact-sum AllReduce after timing")
    budget.note("headline", t)
    extras = {"rejected_before_timing": [{k: v for k, v in r.items() if v is not None} for r in rejected]}
    # connect (+ node gate) time of the timed communicator on every rank
    timings = [None] * world
    dist.all_gather_object(timings, getattr(comm, "connect_timing", None))
    extras["connect_timing_per_rank"] = timings
    extra = not getattr(args, "no_extra", False)
    if extra:
        def _graph():
            gr = graph_replay(torch, dist, comm,
                              lambda st: C.all_reduce(comm, x, y, n, code, C.AllReduceOpType.Sum, st))
            return {"ms_per_step": round(gr * 1e3, 4), "algbw_GBps": round(nbytes / gr / 1e9, 3),
                    "note": "the same AllReduce captured 10x in one HIP graph and replayed (no host path per "
                            "call); value above is the eager path"}
        extras["graph_replay"] = budget.run("graph_replay", _graph)
    del x, y
    torch.cuda.empty_cache()
    if extra and (dt_name, args.size_mib) == ("float32", 128):
        extras["configs3_fp16_1GiB"] = budget.run(
            "configs3_fp16_1GiB", lambda: extra_fp16_1gib(torch, dist, C, comm, rank, world, dev))
        extras["allgather_16MiB_per_rank"] = budget.run(
            "allgather_16MiB_per_rank", lambda: extra_allgather(torch, dist, C, comm, rank, world, dev))
        extras["size_sweep_fp16"] = budget.run(
            "size_sweep_fp16", lambda: size_sweep(torch, dist, C, comm, rank, world, dev))
    info = {"channels": comm.nchannels, "lanes": comm.lanes, "block_threads": comm.block_threads}
    # the connect-time node gate of the timed communicator (csrc/host/gate.cpp):
    # whether it ran, the hand-off it left (MCCS_FIFO_* code: what the line
    # really ran), the paths it found wrong and the direct variants it disabled
    gi = comm.gate_info()
    extras["node_gate"] = {"ran": gi["ran"], "fifo_memory_run": gi["fifo_mode"], "failed_bits": gi["failed"],
                           "disabled_bits": gi["disabled"],
                           "bits": "0x1 ring uncached, 0x2 ring release, 0x4 ring system, 0x8 LL, 0x10 one-shot, "
                                   "0x20 two-shot, 0x40 no peer atomics",
                           "fifo_memory_codes": "0 uncached (relaxed), 1 cached + system fences, 2 uncached + release"}
    if extra and extras.get("size_sweep_fp16") and 2 <= world <= 8:
        extras["direct_sweep_fp16"] = budget.run(
            "direct_sweep_fp16", lambda: direct_sweep(torch, dist, C, rank, world, device, dev, exchange,
                                                      mode_config(C, mode, info), extras["size_sweep_fp16"]))
    rings = comm.rings()
    comm.destroy()
    if extra and world % 2 == 0 and world >= int(os.environ.get("MCCS_BENCH_SETUP2_MIN_WORLD", "8")):
        # BASELINE configs[4] on a full node: the two trace jobs on disjoint halves
        extras["configs4_two_jobs"] = budget.run(
            "configs4_two_jobs", lambda: setup2_measure(torch, dist, C, rank, world, device, dev, False, warmup=1,
                                                        iters=int(os.environ.get("MCCS_SETUP2_ITERS", "10"))))
    dist.barrier()
    if extra and os.environ.get("MCCS_BENCH_NO_REFDRV") != "1":
        extras["reference_driven"] = budget.run(
            "reference_driven", lambda: reference_driven_leg(torch, dist, rank, world, device, nbytes, share))
    calib = None
    if extra and budget.allow("node_legs"):
        # rank 0 alone drives every GPU; ranks 1..N-1 wait at the barrier below
        t = budget.clock()
        if rank == 0:
            extras["in_process_multi_device"], calib = node_legs(torch, C, world, ndev, nbytes,
                                                                 mode_config(C, mode, info))
            extras["xgmi_calibration"] = calib
        dist.barrier()
        budget.note("node_legs", t)
    # every rank decides the CPU ring leg alike (rank 0 runs it; the others wait)
    cpu_ring = extra and budget.allow("cpu_ring_baseline")
    if rank != 0:
        dist.barrier()  # rank 0 times the host baseline
        return None
    cpu = None
    if not getattr(args, "no_cpu_baseline", False) and cpu_sum_baseline is not None:
        t = budget.clock()
        cpu = cpu_sum_baseline(world, nbytes, 7)
        budget.note("cpu_baseline", t)
        if cpu_ring:
            # host threads = world x channels: at most the default channel count
            # (a doubled-channel transport would double the spinning threads)
            host_ch = min(info["channels"], len(C.default_rings(world, 0)))
            t = budget.clock()
            extras["cpu_ring_baseline"] = cpu_ring_baseline(world, min(nbytes, 16 << 20), host_ch)
            budget.note("cpu_ring_baseline", t)
    dist.barrier()
    extras["budget"] = budget.summary()
    prof = {k: (round(v, 3) if isinstance(v, float) else v) for k, v in prof.items()}
    return ring_line(world=world, steps=K, warmup=args.warmup, per_step_s=per_step, nbytes=nbytes, dt_name=dt_name,
                     comm_info=info, rings=rings, mode=mode, tune_table=tune_table, prof=prof,
                     ranks_share_gpu=share, cpu_baseline=cpu, extras=extras, calibration=calib)


def reference_driven_leg(torch, dist, rank, world, device, nbytes, share=None) -> dict:
    """The depth-A drop-in timed on this node (mccs_amd/refdrive.py): the
    reference-named kernels driven exactly as plan.rs drives them, for the
    configurations an unchanged Rust service selects by configuration alone.
    Never fails the line (errors are recorded per variant)."""
    from . import comm as C
    from . import refdrive

    t0 = time.perf_counter()
    # ranks sharing one GPU (a rehearsal): every rank's one-workgroup-per-
    # channel kernel must be resident at once, so keep them to half the CUs
    if share is None:
        share = ranks_share_gpu(dist, device, world)
    max_ch = max(2, 128 // world) if share else 32
    try:
        # a hang on a bad node ends in 20 s, not the kernels' 10 min default
        rows = refdrive.time_reference_driven(torch, dist, rank, world, device, nbytes,
                                              refdrive.default_variants(world, C.default_rings, max_ch),
                                              watchdog_ms=20000)
    except Exception as e:  # noqa: BLE001
        rows = [{"error": f"{type(e).__name__}: {e}"[:300]}]
    torch.cuda.empty_cache()
    return {"what": "reference-named kernels launched as plan.rs:602-669 does (grid = channels, block = "
                    "get_task_schema threads, SHM-meta connector layout in IPC-shared device memory, "
                    "host-mapped work ring, reference hand-off policy); fp32 exact-sum gated",
            "bytes_per_rank": nbytes, "variants": rows, "wall_s": round(time.perf_counter() - t0, 2)}


def mode_config(C, mode: str, info: dict):
    """The CommConfig of the transport the line timed (its mode name, e.g.
    "sender-uncached-fifo+release-fence", plus its channels and lanes), so a
    leg can rerun the same transport through another deployment path."""
    loc = C.LOCALITY_SENDER if (mode or "").startswith("sender") else C.LOCALITY_RECEIVER
    kind = (mode or "").split("-", 1)[-1]
    fifo = {"uncached-fifo": C.FIFO_UNCACHED, "uncached-fifo+release-fence": C.FIFO_UNCACHED_RELEASE,
            "cached-fifo+system-fences": C.FIFO_DEVICE}.get(kind, C.FIFO_UNCACHED)
    return C.CommConfig(channel_count=info.get("channels"), lanes=info.get("lanes"), locality=loc, fifo_memory=fifo,
                        timeout_ms=20000, direct_bytes=-1, oneshot_bytes=-1, ll_bytes=-1)


def node_legs(torch, C, world, ndev, nbytes, config=None):
    """Rank 0 only: the one-process multi-device AllReduce (the reference's
    service model) with the transport the line timed (`config`), and the
    xGMI calibration, when this process sees `world` distinct GPUs.  Returns
    (in_process dict, calibration dict)."""
    from . import node_probe

    if ndev < world:
        na = {"n/a": f"this process sees {ndev} GPU(s) for {world} ranks (ranks share a GPU: no xGMI link)"}
        return na, dict(na)
    t0 = time.perf_counter()
    try:
        inproc = node_probe.in_process_multi_device(torch, C, world, nbytes, config=config)
    except Exception as e:  # noqa: BLE001
        inproc = {"error": f"{type(e).__name__}: {e}"[:300]}
    inproc["wall_s"] = round(time.perf_counter() - t0, 2)
    t0 = time.perf_counter()
    try:
        calib = node_probe.xgmi_calibration(torch, list(range(world)))
    except Exception as e:  # noqa: BLE001
        calib = {"error": f"{type(e).__name__}: {e}"[:300]}
    calib["wall_s"] = round(time.perf_counter() - t0, 2)
    torch.cuda.set_device(0)
    return inproc, calib


def setup2_jobs(world: int, interleaved: bool) -> list[list[int]]:
    """Global ranks of the two jobs: halves {0..n/2-1}/{n/2..n-1} (disjoint
    GPU sets, no shared links) or even/odd ranks (rings share links)."""
    if world < 4 or world % 2:
        raise ValueError("two concurrent jobs need an even world size >= 4")
    if interleaved:
        return [list(range(0, world, 2)), list(range(1, world, 2))]
    return [list(range(0, world // 2)), list(range(world // 2, world))]


def setup2_measure(torch, dist, C, rank, world, device, dev, interleaved, warmup, iters, compute_scale=1.0):
    """Both setup-2 trace jobs at once, one communicator per job on its half
    of the node, run like traffic_gen (mccs_amd/traffic.py: compute gap,
    in-place fp16 AllReduce, stream sync per op, per-iteration exact check).
    Returns the per-job summaries (identical on every rank)."""
    from mccs_amd import traffic

    members = setup2_jobs(world, interleaved)
    groups = [dist.new_group(m) for m in members]
    job = 0 if rank in members[0] else 1
    jrank = members[job].index(rank)
    half = len(members[job])
    grp = groups[job]
    name, count = SETUP2_JOBS[job]
    nbytes, compute_us, _ = traffic.SETUP2[name]
    assert nbytes == 2 * count
    share = ranks_share_gpu(dist, device, world)  # a 1-GPU rehearsal: every process on one GPU
    modes = _candidates(C, [shared_gpu_lanes(world) if share and "MCCS_LANES" not in os.environ else None],
                        [None])[0][1]
    comm, mode = make_validated_comm(torch, dist, C, jrank, half, device, dev, _exchange_factory(dist, half, grp),
                                     modes, (count, torch.float16, C.AllReduceDataType.Float16), grp)
    if comm is None:
        raise BenchFailure(f"{name}: communicator creation failed")

    stream = side_stream(torch, device, slot=1)
    tj = traffic.TraceJob(torch, name, [comm], [jrank], half, count, compute_us * 1e-6 * compute_scale, stream, dev)
    dist.barrier()  # both jobs start together
    for w in range(warmup):
        tj.iteration(-1 - w, record=False)
    for it in range(iters):
        tj.iteration(it)
    ok = all(r.exact for r in tj.records)
    try:
        # the all-rank agreement doubles as the barrier mccsCommDestroy needs
        require(dist, ok, f"{name}: in-place exact-sum check of every iteration")
    finally:
        comm.destroy()
    mine = tj.summary()
    mine["fifo_mode"] = mode
    # per-job numbers as the max over the job's ranks (the slowest rank ends the op)
    vals = torch.zeros(2, 2, dtype=torch.float64)
    vals[job, 0] = mine["iter_ms_mean"]
    vals[job, 1] = mine["ms_per_call"]
    dist.all_reduce(vals, op=dist.ReduceOp.MAX)
    out = []
    for j, (nm, cnt) in enumerate(SETUP2_JOBS):
        it_ms, op_ms = float(vals[j, 0]), float(vals[j, 1])
        out.append({"job": nm, "ranks": len(members[j]), "global_ranks": members[j], "bytes": cnt * 2,
                    "compute_interval_ms": round(traffic.SETUP2[nm][1] * 1e-3 * compute_scale, 3),
                    "iterations": iters, "iter_ms_mean": round(it_ms, 4), "ms_per_call": round(op_ms, 4),
                    "algbw_GBps": round(cnt * 2 / (op_ms / 1e3) / 1e9, 3), "exact_every_iteration": True})
    dist.barrier()
    del tj
    torch.cuda.empty_cache()
    return {"workload": "2 concurrent allreduce jobs, setup-2 traces (BASELINE configs[4]), "
                        + ("interleaved ranks sharing links" if interleaved else "disjoint GPU halves"),
            "semantics": "traffic_gen/src/main.rs:167-200: compute gap, in-place fp16 AllReduce, stream sync "
                         "per op; fresh exact gradients each iteration, checked bit for bit",
            "jobs": out}


def setup2_roofline(jobs, ranks_share_gpu: bool) -> dict:
    """Roofline of the two-job line (value = the sum of the jobs' algbw).
    Each job's per-rank link bytes 2(n-1)/n*S per call over its rings'
    distinct outgoing links (n = 4: 3 links) at the spec rate; the line sums
    achieved and peak over the jobs.  Ranks sharing one GPU (a rehearsal):
    all jobs' (6n-4)*S algorithmic HBM bytes per call against that one HBM."""
    from . import comm as C

    per, ach, peak = [], 0.0, 0.0
    for j in jobs:
        n, s, t = j["ranks"], j["bytes"], j["ms_per_call"] / 1e3
        if ranks_share_gpu:
            a = (6 * n - 4) * s / t / 1e9
            per.append({"job": j["job"], "bound": "hbm", "achieved": round(a, 2)})
            ach += a
            continue
        links = out_links(C.default_rings(n), 0)
        a = 2 * (n - 1) / n * s / t / 1e9
        p = links * XGMI_LINK_GBPS_PER_DIR
        per.append({"job": j["job"], "bound": "xgmi", "achieved": round(a, 2), "peak": round(p, 2),
                    "frac": round(a / p, 4), "links": links})
        ach += a
        peak += p
    if ranks_share_gpu:
        peak = HBM_PEAK_GBPS
    return {"bound": "hbm" if ranks_share_gpu else "xgmi", "achieved": round(ach, 2), "peak": round(peak, 2),
            "unit": "GB/s", "frac": round(ach / peak, 4), "traffic": None, "traffic_note": TRAFFIC_NOT_MEASURED,
            "traffic_virtual_node_n2": VNODE_N2_TRAFFIC,
            "kernel": "ring_multi_kernel<AllReduce, half, Sum>", "per_job": per,
            "note": ("ranks share one GPU: all jobs' (6n-4)*S algorithmic HBM bytes per call" if ranks_share_gpu
                     else "per job: per-rank link bytes 2(n-1)/n*S per call over its distinct outgoing links x "
                          f"{XGMI_LINK_GBPS_PER_DIR} GB/s per direction (spec); summed over the jobs")}


def setup2_line(res, world, steps, warmup, scale, ranks_share_gpu, cpu_baseline) -> dict:
    """The configs[4] line (pure: no GPU, unit-tested on CPU)."""
    jobs = res["jobs"]
    return {
        "metric": METRIC,
        "submetric": "concurrent_jobs_algbw_GBps",
        "value": round(sum(j["algbw_GBps"] for j in jobs), 3),
        "unit": "GB/s",
        "n_gpus": world,
        "steps": steps,
        "warmup": warmup,
        "ms_per_step": max(j["iter_ms_mean"] for j in jobs),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f16",
        "data": "synthetic exact fp16 gradients per rank and iteration, device-resident buckets",
        "config": {**res, "compute_scale": scale, "ranks_share_gpu": ranks_share_gpu},
        "roofline": setup2_roofline(jobs, ranks_share_gpu),
        "cpu_baseline": cpu_baseline,
    }


def run_setup2(args, torch, dist, C, rank, world, device, dev, interleaved=False, cpu_sum_baseline=None):
    """BASELINE configs[4] alone: two concurrent trace jobs on the node.
    value = sum of the jobs' algbw; ms_per_step = the slower job's mean
    iteration time (compute gap + AllReduce + sync, traffic_gen's round
    time, traffic_gen/src/main.rs:167-228).  MCCS_SETUP2_COMPUTE_SCALE
    scales the compute gaps (rehearsals).  cpu_baseline: the host sum of the
    larger job's buckets (4 x setup-2_vgg fp16, sampled)."""
    scale = float(os.environ.get("MCCS_SETUP2_COMPUTE_SCALE", "1.0"))
    res = setup2_measure(torch, dist, C, rank, world, device, dev, interleaved, args.warmup, args.steps, scale)
    share = ranks_share_gpu(dist, device, world)
    if rank != 0:
        dist.barrier()
        return None
    cpu = None
    if not getattr(args, "no_cpu_baseline", False) and cpu_sum_baseline is not None:
        name, count = SETUP2_JOBS[0]
        cpu = cpu_sum_baseline(len(setup2_jobs(world, interleaved)[0]), 2 * count, 6)
    dist.barrier()
    return setup2_line(res, world, args.steps, args.warmup, scale, share, cpu)
