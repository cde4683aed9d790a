"""Multi-GPU leg of bench.py: ring AllReduce algbw over xGMI (configs[2..3]).

Launched by torch.distributed.run, one rank per GPU (RANK / LOCAL_RANK /
WORLD_SIZE / MASTER_*).  torch.distributed runs on gloo and is the control
plane only (connect-handle exchange, barriers, max-over-ranks timing); every
byte of the collective moves through libmccs_hip.so's ring kernels over xGMI
P2P FIFOs -- no RCCL.

One step = one AllReduce of a per-rank bucket of S bytes; value = algbw =
S / t (allreduce_bench/src/main.rs:168), busbw = algbw * 2(n-1)/n.
Before timing, an exact-sum fp32 AllReduce on the timed buffers is checked
bit for bit on every rank; a communicator whose FIFO hand-off fails that
check is rebuilt with cached FIFO memory + system-scope fences and checked
again (the result says which ran).
"""
from __future__ import annotations

import os
import time

XGMI_LINK_GBPS_PER_DIR = 76.8  # MI355X xGMI per link per direction (spec); see DESIGN.md


def _exchange_factory(dist, world):
    """Connect-handle all-gather over the control plane (replaces the
    reference's bootstrap ring + exchange engine for this path)."""
    def exchange(b: bytes):
        out = [None] * world
        dist.all_gather_object(out, b)
        return out

    return exchange


def agree(dist, ok: bool, group=None) -> bool:
    """True only if every rank passed (MIN over ranks)."""
    import torch

    t = torch.tensor([1 if ok else 0], dtype=torch.int32)
    dist.all_reduce(t, op=dist.ReduceOp.MIN, group=group)
    return bool(t.item() == 1)


def max_over_ranks(dist, x: float) -> float:
    import torch

    t = torch.tensor([float(x)], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def _exact_inputs(torch, n_elem, rank, dev):
    # k/64 with |k| <= 255: every partial sum of <= 8 ranks is exact in fp32
    i = torch.arange(n_elem, device=dev, dtype=torch.int64)
    k = ((i * 7 + rank * 13) % 511) - 255
    return k.to(torch.float32) / 64.0


def _expected_exact(torch, n_elem, world, dev):
    i = torch.arange(n_elem, device=dev, dtype=torch.int64)
    tot = torch.zeros(n_elem, device=dev, dtype=torch.int64)
    for r in range(world):
        tot += ((i * 7 + r * 13) % 511) - 255
    return tot.to(torch.float64).div(64.0).to(torch.float32)


WORKLOADS = {
    ("float32", 128): "BASELINE configs[2]",
    ("float16", 1024): "BASELINE configs[3]",
}

# BASELINE configs[4]: workloads/setup-2_vgg.toml (fp16, 574,668,960 B) and
# setup-2_gpt_1.toml (fp16, 83,886,080 B), one job per half of the node.
SETUP2_JOBS = (("setup-2_vgg", 287_334_480), ("setup-2_gpt_1", 41_943_040))

# name -> (bench dtype tag, AllReduceDataType member, kernel symbol suffix)
DTYPES = {"float32": ("f32", "Float32", "float"), "float16": ("f16", "Float16", "half"),
          "bfloat16": ("bf16", "Bfloat16", "bfloat16")}


def _subgroup_exchange(dist, group, n):
    def exchange(b: bytes):
        out = [None] * n
        dist.all_gather_object(out, b, group=group)
        return out

    return exchange


def _default_modes(C):
    return [("uncached-fifo", C.CommConfig(timeout_ms=60000)),
            ("cached-fifo+system-fences", C.CommConfig(fifo_memory=C.FIFO_DEVICE, timeout_ms=60000)),
            ("sender-side-uncached-fifo", C.CommConfig(locality=C.LOCALITY_SENDER, timeout_ms=60000)),
            ("sender-side-cached-fifo", C.CommConfig(locality=C.LOCALITY_SENDER, fifo_memory=C.FIFO_DEVICE,
                                                     timeout_ms=60000))]


def _make_validated_comm(torch, dist, C, rank, world, device, dev, exchange, group=None, full=None, modes=None,
                         required=True):
    """Build the communicator; check an exact-sum fp32 AllReduce bit for bit
    on every rank (and, with full=(n, torch dtype, AllReduceDataType), one at
    the timed size and dtype); on failure rebuild with the next FIFO mode.
    Returns (comm, mode name), or (None, None) when no mode passes and not
    required."""
    for name, cfg in (modes or _default_modes(C)):
        try:
            comm = C.init_communicator_rank(rank, world, device, exchange, cfg)
        except Exception as e:  # noqa: BLE001  (e.g. IPC refuses this memory kind: try the next mode)
            print(f"[rank {rank}] {name}: init failed: {e}", flush=True)
            comm = None
        if not agree(dist, comm is not None, group):
            if comm is not None:
                comm.destroy()
            continue
        nv = (4 << 20) // 4  # 4 MiB exact-sum fp32 check (multi-loop, ragged chunks)
        xv = _exact_inputs(torch, nv, rank, dev)
        yv = torch.empty_like(xv)
        ok = True
        try:
            C.all_reduce(comm, xv, yv, nv, C.AllReduceDataType.Float32)
            comm.sync()
            torch.cuda.synchronize()
            ok = bool(torch.equal(yv, _expected_exact(torch, nv, world, dev)))
            del xv, yv
            if ok and full is not None:
                ok = _full_size_exact(torch, C, comm, rank, world, full[0], full[1], full[2], dev)
        except Exception as e:  # noqa: BLE001  (watchdog / HIP error: try the next mode)
            print(f"[rank {rank}] {name}: {e}", flush=True)
            ok = False
        if agree(dist, ok, group):
            return comm, name
        comm.destroy()
    if required:
        raise SystemExit("ring allreduce failed validation in every FIFO mode")
    return None, None


def _autotune(torch, dist, C, rank, world, device, dev, exchange, full, step_for, warmup=2, reps=6):
    """Transport placement chosen on the node itself: FIFO data at the
    receiver (remote writes) or at the sender (remote reads, the reference's
    SHM layout), each at the auto lane count and at 16 lanes per channel.
    Every candidate is validated exactly like the timed communicator; the
    fastest (max over ranks) is kept.  MCCS_LOCALITY / MCCS_LANES pin a
    dimension.  Returns (comm, mode, table)."""
    locs = [None] if "MCCS_LOCALITY" in os.environ else [C.LOCALITY_RECEIVER, C.LOCALITY_SENDER]
    lanes_opts = [None] if "MCCS_LANES" in os.environ else [None, 16]
    best, table, seen = None, [], set()
    for loc in locs:
        lname = {None: "env", C.LOCALITY_RECEIVER: "receiver", C.LOCALITY_SENDER: "sender"}[loc]
        for lanes in lanes_opts:
            modes = [(f"{lname}-uncached-fifo", C.CommConfig(locality=loc, lanes=lanes, timeout_ms=60000)),
                     (f"{lname}-cached-fifo+system-fences",
                      C.CommConfig(locality=loc, lanes=lanes, fifo_memory=C.FIFO_DEVICE, timeout_ms=60000))]
            comm, mode = _make_validated_comm(torch, dist, C, rank, world, device, dev, exchange, full=full,
                                              modes=modes, required=False)
            if comm is None:
                table.append({"mode": f"{lname}/lanes={lanes or 'auto'}", "ok": False})
                continue
            key = (mode, comm.lanes)
            if key in seen:  # auto lanes already == 16
                comm.destroy()
                continue
            seen.add(key)
            el = max_over_ranks(dist, _time_steps(torch, dist, comm, step_for(comm), warmup, reps))
            table.append({"mode": mode, "lanes": comm.lanes, "ms_per_step": round(el / reps * 1e3, 4)})
            if best is None or el < best[0]:
                if best is not None:
                    best[1].destroy()
                best = (el, comm, mode)
            else:
                comm.destroy()
    if best is None:
        raise SystemExit("ring allreduce failed validation in every transport mode")
    return best[1], best[2], table


def _full_size_exact(torch, C, comm, rank, world, n, tdt, code, dev) -> bool:
    """BASELINE-size check through a size-independent property: k/64 inputs
    (|k| <= 255) sum exactly in fp16/bf16/fp32 for <= 8 ranks, so the
    AllReduce must equal the integer sum bit for bit in any order."""
    i = torch.arange(n, device=dev, dtype=torch.int64)
    k = ((i * 7 + rank * 13) % 511) - 255
    x = (k.to(torch.float32) / 64.0).to(tdt)
    del k
    y = torch.empty_like(x)
    C.all_reduce(comm, x, y, n, code, C.AllReduceOpType.Sum)
    comm.sync()
    tot = torch.zeros(n, device=dev, dtype=torch.int64)
    for r in range(world):
        tot += ((i * 7 + r * 13) % 511) - 255
    exp = (tot.to(torch.float64) / 64.0).to(tdt)
    ok = bool(torch.equal(y, exp)) if world <= 8 else True
    del x, y, tot, exp, i
    torch.cuda.empty_cache()
    return ok


def _graph_replay(torch, dist, comm, call_on, calls=10):
    """Per-call time of `calls` AllReduces captured in one HIP graph (max over
    ranks), after one untimed replay.  call_on(stream) issues one AllReduce."""
    torch.cuda.synchronize()
    gs = torch.cuda.Stream()
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


def _extra_fp16_1gib(torch, dist, C, comm, rank, world, dev, warmup=3, K=10):
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

    el = max_over_ranks(dist, _time_steps(torch, dist, comm, step, warmup, K))
    del x, y
    torch.cuda.empty_cache()
    ok = agree(dist, _full_size_exact(torch, C, comm, rank, world, n, torch.float16, code, dev))
    per = el / K
    return {"workload": f"{world}x ring allreduce, 1 GiB float16 buckets (BASELINE configs[3])",
            "ms_per_step": round(per * 1e3, 4), "algbw_GBps": round((1 << 30) / per / 1e9, 3),
            "busbw_GBps": round((1 << 30) / per / 1e9 * 2 * (world - 1) / world, 3), "steps": K,
            "validated_exact_sum_full_size": ok}


def _extra_allgather(torch, dist, C, comm, rank, world, dev, mib=16, warmup=3, K=10):
    """The other reachable collective (all_gather.h): AllGather of `mib` MiB
    per rank on the same communicator; every gathered segment checked byte
    for byte.  algbw = gathered bytes / t (nccl-tests convention)."""
    nb = mib << 20
    i = torch.arange(nb, device=dev, dtype=torch.int32)
    x = ((i * 31 + rank * 101) % 251).to(torch.uint8)
    y = torch.empty(world * nb, dtype=torch.uint8, device=dev)

    def step():
        C.all_gather(comm, x, y, nb)

    el = max_over_ranks(dist, _time_steps(torch, dist, comm, step, warmup, K))
    ok = all(bool(torch.equal(y[r * nb:(r + 1) * nb], ((i * 31 + r * 101) % 251).to(torch.uint8)))
             for r in range(world))
    ok = agree(dist, ok)
    per = el / K
    algbw = world * nb / per / 1e9
    del x, y, i
    torch.cuda.empty_cache()
    return {"ms_per_step": round(per * 1e3, 4), "algbw_GBps": round(algbw, 3),
            "busbw_GBps": round(algbw * (world - 1) / world, 3), "steps": K, "validated_bytes": ok}


# the reference's evaluation sweep (eval/plot/single_app/allreduce_{4,8}gpu.csv:
# fp16 "half", 32 KiB ... 512 MiB)
SWEEP_BYTES = (32768, 131072, 524288, 2097152, 8388608, 33554432, 134217728, 536870912)


def _size_sweep(torch, dist, C, comm, rank, world, dev, warmup=3, K=20):
    """fp16 AllReduce latency / algbw / busbw over the reference's eval sizes
    (allreduce_bench semantics: algbw = bytes / t, busbw = algbw * 2(n-1)/n),
    each size exact-sum validated."""
    rows = []
    for nb in SWEEP_BYTES:
        n = nb // 2
        x = torch.empty(n, dtype=torch.float16, device=dev).uniform_(-1, 1)
        y = torch.empty_like(x)

        def step():
            C.all_reduce(comm, x, y, n, C.AllReduceDataType.Float16, C.AllReduceOpType.Sum)

        el = max_over_ranks(dist, _time_steps(torch, dist, comm, step, warmup, K)) / K
        del x, y
        ok = agree(dist, _full_size_exact(torch, C, comm, rank, world, n, torch.float16,
                                          C.AllReduceDataType.Float16, dev))
        algbw = nb / el / 1e9
        rows.append({"bytes": nb, "latency_us": round(el * 1e6, 2), "algbw_GBps": round(algbw, 3),
                     "busbw_GBps": round(algbw * 2 * (world - 1) / world, 3), "exact": ok})
    return rows


def _out_links(rings, rank):
    """Distinct xGMI links this rank sends on (one per distinct ring successor)."""
    nxt = set()
    for order in rings:
        p = order.index(rank)
        nxt.add(order[(p + 1) % len(order)])
    return len(nxt)


def _time_steps(torch, dist, comm, step, warmup, K, group=None):
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


def cpu_ring_baseline(C, world: int, budget_s: float = 3.0) -> dict:
    """The same ring schedule on host threads (mccs_host_ring_allreduce, the
    configs[0] plumbing) over a bounded fp32 sample, for scale."""
    import numpy as np

    n = (16 << 20) // 4
    rng = np.random.default_rng(0)
    send = [(rng.random(n, dtype=np.float32) * 2 - 1) for _ in range(world)]
    recv = [np.empty_like(x) for x in send]
    t0 = time.perf_counter()
    reps = 0
    while True:
        C.host_ring_allreduce(send, recv, n, C.AllReduceDataType.Float32, channels=2, nthreads=544)
        reps += 1
        if time.perf_counter() - t0 > budget_s:
            break
    dt = (time.perf_counter() - t0) / reps
    return {"value": round(n * 4 / dt / 1e9, 3), "unit": "GB/s algbw", "cores": 2 * world, "kind": "port",
            "sample": f"{world} ranks x 16 MiB fp32, host-thread ring (2 channels), {reps} reps"}


def run(args):
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

        # a rank that dies mid-collective should end the job in minutes, not
        # gloo's default 30
        dist.init_process_group("gloo", rank=rank, world_size=world, timeout=datetime.timedelta(seconds=600))
    if getattr(args, "jobs", None) in ("setup2", "setup2-interleaved"):
        return run_setup2(args, torch, dist, C, rank, world, device, dev, interleaved=args.jobs.endswith("interleaved"))
    exchange = _exchange_factory(dist, world)

    dt_name = args.dtype
    tdt = {"float32": torch.float32, "float16": torch.float16, "bfloat16": torch.bfloat16}[dt_name]
    code = getattr(C.AllReduceDataType, DTYPES[dt_name][1])
    esize = torch.tensor([], dtype=tdt).element_size()
    nbytes = args.size_mib << 20
    n = nbytes // esize

    # per-slice wait / stream timing on this rank's GPU (3 atomics per slice
    # per workgroup): reported with the result to show where ring time goes
    os.environ.setdefault("MCCS_RING_PROFILE", "1")
    g = torch.Generator(device=dev)
    g.manual_seed(1000 + rank)
    x = (torch.rand(n, device=dev, generator=g) * 2 - 1).to(tdt)
    y = torch.empty_like(x)
    stream = torch.cuda.current_stream()

    def step_for(cm):
        return lambda: C.all_reduce(cm, x, y, n, code, C.AllReduceOpType.Sum, stream)

    tune_table = None
    if getattr(args, "no_autotune", False):
        comm, mode = _make_validated_comm(torch, dist, C, rank, world, device, dev, exchange, full=(n, tdt, code))
    else:
        comm, mode, tune_table = _autotune(torch, dist, C, rank, world, device, dev, exchange, (n, tdt, code),
                                           step_for)
    K = args.steps
    failed_after_timing = []
    while True:
        step = step_for(comm)
        C.ring_profile(device, reset=True)
        elapsed = max_over_ranks(dist, _time_steps(torch, dist, comm, step, args.warmup, K))
        prof = C.ring_profile(device, reset=True)
        per_step = elapsed / K
        full_ok = _full_size_exact(torch, C, comm, rank, world, n, tdt, code, dev)
        if os.environ.get("MCCS_BENCH_INJECT_MISMATCH") == "1" and not failed_after_timing:
            full_ok = False  # fault injection: exercises the re-timing path below
        full_ok = agree(dist, full_ok)
        if full_ok or failed_after_timing:
            break
        # the timed mode passed validation but a later sum was wrong: re-time
        # with the most conservative hand-off (release/acquire fences on cached
        # FIFOs), or with uncached FIFOs if that was the failing mode
        failed_after_timing.append(mode)
        print(f"[rank {rank}] {mode}: full-size exact-sum mismatch after timing; re-timing", flush=True)
        comm.destroy()
        cached = "uncached" not in mode
        fallback = [m for m in _default_modes(C) if ("uncached" in m[0]) == bool(cached)]
        comm, mode = _make_validated_comm(torch, dist, C, rank, world, device, dev, exchange, full=(n, tdt, code),
                                          modes=fallback)
    graph = None
    if not getattr(args, "no_extra", False):
        graph = _graph_replay(torch, dist, comm,
                              lambda st: C.all_reduce(comm, x, y, n, code, C.AllReduceOpType.Sum, st))
    del x, y
    extra = gather = sweep = None
    if not getattr(args, "no_extra", False) and (dt_name, args.size_mib) == ("float32", 128):
        extra = _extra_fp16_1gib(torch, dist, C, comm, rank, world, dev)
        gather = _extra_allgather(torch, dist, C, comm, rank, world, dev)
        sweep = _size_sweep(torch, dist, C, comm, rank, world, dev)
    setup2 = None
    if (not getattr(args, "no_extra", False) and world % 2 == 0
            and world >= int(os.environ.get("MCCS_BENCH_SETUP2_MIN_WORLD", "8"))):
        # BASELINE configs[4] on a full node: the two jobs on disjoint halves
        _, jobs2, _ = _setup2_measure(torch, dist, C, rank, world, device, dev, False, 3, 10)
        setup2 = {"workload": "2 concurrent allreduce jobs, setup-2 shapes (BASELINE configs[4]), disjoint halves",
                  "jobs": jobs2, "steps": 10}
    algbw = nbytes / per_step / 1e9
    busbw = algbw * 2 * (world - 1) / world
    link_bytes = 2 * (world - 1) / world * nbytes
    out = None
    if rank == 0:
        rings = comm.rings()
        links = _out_links(rings, 0)
        link_gbps = link_bytes / per_step / 1e9
        peak = links * XGMI_LINK_GBPS_PER_DIR
        out = {
            "metric": "device-resident reduce GB/s; ring-allreduce algbw GB/s at 1/2/4/8 MI355X",
            "submetric": "ring_allreduce_algbw_GBps",
            "value": round(algbw, 3),
            "unit": "GB/s",
            "n_gpus": world,
            "steps": K,
            "warmup": args.warmup,
            "ms_per_step": round(per_step * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": DTYPES[dt_name][0],
            "data": "synthetic uniform[-1,1) per rank, device-resident buckets",
            "config": {
                "workload": f"{world}x MI355X ring allreduce over xGMI P2P, {args.size_mib} MiB {dt_name} "
                            f"buckets, chunked FIFO pipeline ({WORKLOADS.get((dt_name, args.size_mib), 'custom')})",
                "bytes_per_rank": nbytes, "channels": comm.nchannels, "lanes": comm.lanes,
                "block_threads": comm.block_threads, "rings": rings, "fifo_mode": mode,
                "transport_autotune": tune_table,
                "validated_exact_sum_4MiB": True, "validated_exact_sum_full_size_before_timing": True,
                "validated_exact_sum_full_size_after_timing": full_ok,
                "failed_after_timing": failed_after_timing,
                "busbw_GBps": round(busbw, 3), "parallelism": f"ring{world}",
                "rank0_slice_profile": {k: (round(v, 3) if isinstance(v, float) else v) for k, v in prof.items()},
                # ranks sharing one GPU (a 1-GPU box): FIFO hand-offs stay in HBM, no xGMI link
                "ranks_share_gpu": ndev < world,
            },
            # the ring's bound is the xGMI links it sends on, not HBM
            "roofline": {
                "bound": "xgmi",
                "achieved": round(link_gbps, 2),
                "peak": peak,
                "unit": "GB/s",
                "frac": round(link_gbps / peak, 4),
                "traffic": None,
                "kernel": "mccsKernel_AllReduce_RING_SIMPLE_Sum_" + DTYPES[dt_name][2],
                "note": f"per-rank link bytes 2(n-1)/n*S over {links} distinct outgoing links x "
                        f"{XGMI_LINK_GBPS_PER_DIR} GB/s per direction (spec)",
            },
            "cpu_baseline": None,
        }
        if extra is not None:
            out["config"]["configs3_fp16_1GiB"] = extra
        if gather is not None:
            out["config"]["allgather_16MiB_per_rank"] = gather
        if sweep is not None:
            out["config"]["size_sweep_fp16"] = sweep
        if setup2 is not None:
            out["config"]["configs4_two_jobs"] = setup2
        if graph is not None:
            out["config"]["graph_replay"] = {
                "ms_per_step": round(graph * 1e3, 4), "algbw_GBps": round(nbytes / graph / 1e9, 3),
                "note": "the same AllReduce captured 10x in one HIP graph and replayed (no host path per call); "
                        "value above is the eager path"}
        if not getattr(args, "no_cpu_baseline", False):
            out["cpu_ring_baseline"] = cpu_ring_baseline(C, world)
    comm.destroy()
    dist.barrier()
    dist.destroy_process_group()
    if not full_ok:
        raise SystemExit("full-size exact-sum AllReduce mismatch")
    return out


def setup2_jobs(world: int, interleaved: bool) -> list[list[int]]:
    """Global ranks of the two jobs: halves {0..n/2-1}/{n/2..n-1} (disjoint
    GPU sets, no shared links) or even/odd ranks (rings share links)."""
    if world < 4 or world % 2:
        raise ValueError("two concurrent jobs need an even world size >= 4")
    if interleaved:
        return [list(range(0, world, 2)), list(range(1, world, 2))]
    return [list(range(0, world // 2)), list(range(world // 2, world))]


def _setup2_measure(torch, dist, C, rank, world, device, dev, interleaved, warmup, steps):
    """Both setup-2 jobs at once (one communicator per job on its half of the
    node); returns (members, per-job dicts, fifo mode) on every rank."""
    members = setup2_jobs(world, interleaved)
    groups = [dist.new_group(m) for m in members]
    job = 0 if rank in members[0] else 1
    jrank = members[job].index(rank)
    half = len(members[job])
    grp = groups[job]
    exchange = _subgroup_exchange(dist, grp, half)
    name, n = SETUP2_JOBS[job]
    comm, mode = _make_validated_comm(torch, dist, C, jrank, half, device, dev, exchange, grp,
                                      full=(n, torch.float16, C.AllReduceDataType.Float16))
    g = torch.Generator(device=dev)
    g.manual_seed(2000 + rank)
    x = (torch.rand(n, device=dev, generator=g) * 2 - 1).to(torch.float16)
    y = torch.empty_like(x)

    def step():
        C.all_reduce(comm, x, y, n, C.AllReduceDataType.Float16, C.AllReduceOpType.Sum)

    dist.barrier()  # both jobs start together
    el = _time_steps(torch, dist, comm, step, warmup, steps, grp)
    t = torch.tensor([el], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=grp)
    per_job = torch.zeros(2, dtype=torch.float64)
    per_job[job] = t[0] / steps
    dist.all_reduce(per_job, op=dist.ReduceOp.MAX)
    comm.destroy()
    del x, y
    torch.cuda.empty_cache()
    dist.barrier()
    jobs = []
    for j, (nm, cnt) in enumerate(SETUP2_JOBS):
        ps = float(per_job[j])
        jobs.append({"job": nm, "ranks": half, "bytes": cnt * 2, "ms_per_call": round(ps * 1e3, 4),
                     "algbw_GBps": round(cnt * 2 / ps / 1e9, 3)})
    return members, jobs, mode


def run_setup2(args, torch, dist, C, rank, world, device, dev, interleaved=False):
    """BASELINE configs[4]: two concurrent AllReduce jobs on the node, shapes
    from workloads/setup-2_{vgg,gpt_1}.toml.  Each job times its own K calls;
    both run at the same time (traffic_gen/src/main.rs:167-228 reports each
    job's per-iteration time the same way)."""
    members, jobs, mode = _setup2_measure(torch, dist, C, rank, world, device, dev, interleaved, args.warmup,
                                          args.steps)
    dist.destroy_process_group()
    if rank != 0:
        return None
    return {
        "metric": "device-resident reduce GB/s; ring-allreduce algbw GB/s at 1/2/4/8 MI355X",
        "submetric": "concurrent_jobs_algbw_GBps",
        "value": round(sum(j["algbw_GBps"] for j in jobs), 3),
        "unit": "GB/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f16",
        "data": "synthetic uniform[-1,1) per rank, device-resident buckets",
        "config": {"workload": "2 concurrent allreduce jobs, setup-2 shapes (BASELINE configs[4]), "
                               + ("interleaved ranks sharing links" if interleaved else "disjoint GPU halves"),
                   "job_ranks": members, "jobs": jobs, "fifo_mode": mode},
    }
