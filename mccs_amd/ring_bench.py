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


def agree(dist, ok: bool) -> bool:
    """True only if every rank passed (MIN over ranks)."""
    import torch

    t = torch.tensor([1 if ok else 0], dtype=torch.int32)
    dist.all_reduce(t, op=dist.ReduceOp.MIN)
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
        dist.init_process_group("gloo", rank=rank, world_size=world)
    exchange = _exchange_factory(dist, world)

    dt_name = args.dtype
    tdt = {"float32": torch.float32, "float16": torch.float16, "bfloat16": torch.bfloat16}[dt_name]
    code = {"float32": C.AllReduceDataType.Float32, "float16": C.AllReduceDataType.Float16,
            "bfloat16": C.AllReduceDataType.Bfloat16}[dt_name]
    esize = torch.tensor([], dtype=tdt).element_size()
    nbytes = args.size_mib << 20
    n = nbytes // esize

    attempts = [("uncached-fifo", C.CommConfig(timeout_ms=60000)),
                ("cached-fifo+system-fences", C.CommConfig(fifo_memory=C.FIFO_DEVICE, timeout_ms=60000))]
    comm = None
    mode = None
    validated = False
    for name, cfg in attempts:
        comm = C.init_communicator_rank(rank, world, device, exchange, cfg)
        nv = (4 << 20) // 4  # 4 MiB exact-sum fp32 check (multi-loop, ragged chunks)
        xv = _exact_inputs(torch, nv, rank, dev)
        yv = torch.empty_like(xv)
        ok = True
        try:
            C.all_reduce(comm, xv, yv, nv, C.AllReduceDataType.Float32)
            comm.sync()
            torch.cuda.synchronize()
            ok = bool(torch.equal(yv, _expected_exact(torch, nv, world, dev)))
        except Exception as e:  # noqa: BLE001  (watchdog / HIP error: try the next mode)
            print(f"[rank {rank}] {name}: {e}", flush=True)
            ok = False
        if agree(dist, ok):
            mode, validated = name, True
            break
        comm.destroy()
        comm = None
    if comm is None:
        raise SystemExit("ring allreduce failed validation in every FIFO mode")

    g = torch.Generator(device=dev)
    g.manual_seed(1000 + rank)
    x = (torch.rand(n, device=dev, generator=g) * 2 - 1).to(tdt)
    y = torch.empty_like(x)
    stream = torch.cuda.current_stream()

    def step():
        C.all_reduce(comm, x, y, n, code, C.AllReduceOpType.Sum, stream)

    for _ in range(args.warmup):
        step()
    comm.sync()
    torch.cuda.synchronize()
    dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    K = args.steps
    for _ in range(K):
        step()
    torch.cuda.synchronize()
    comm.sync()
    t1 = time.perf_counter()
    dist.barrier()
    elapsed = max_over_ranks(dist, t1 - t0)
    per_step = elapsed / K
    algbw = nbytes / per_step / 1e9
    busbw = algbw * 2 * (world - 1) / world
    # per-rank HBM bytes the ring moves (local reads/writes of user buffers and
    # FIFO slots): send input S/n, (n-2) x [read input + FIFO, write FIFO],
    # final [read input + FIFO, write output + FIFO], (n-2) x [read FIFO,
    # write output + FIFO], last [read FIFO, write output]
    s = nbytes
    hbm_bytes = s / world * (1 + 1 + (world - 2) * 3 + 4 + (world - 2) * 3 + 2)
    link_bytes = 2 * (world - 1) / world * s
    out = None
    if rank == 0:
        nch = comm.nchannels
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
            "dtype": {"float32": "f32", "float16": "f16", "bfloat16": "bf16"}[dt_name],
            "data": "synthetic uniform[-1,1) per rank, device-resident buckets",
            "config": {
                "workload": f"{world}x MI355X ring allreduce over xGMI P2P, {args.size_mib} MiB {dt_name} "
                            f"buckets, chunked FIFO pipeline (BASELINE configs[2])",
                "bytes_per_rank": nbytes, "channels": nch, "lanes": comm.lanes,
                "block_threads": comm.block_threads, "rings": comm.rings(), "fifo_mode": mode,
                "validated_exact_sum": validated, "busbw_GBps": round(busbw, 3),
                "parallelism": f"ring{world}",
            },
            "roofline": {
                "bound": "hbm",
                "achieved": round(hbm_bytes / per_step / 1e9, 2),
                "peak": 8000.0,
                "unit": "GB/s",
                "frac": round(hbm_bytes / per_step / 1e9 / 8000.0, 5),
                "traffic": None,
                "kernel": "mccsKernel_AllReduce_RING_SIMPLE_Sum",
                "note": "ring is xGMI-link bound; see xgmi",
            },
            "xgmi": {
                "link_bytes_per_rank": int(link_bytes),
                "achieved_GBps_per_rank": round(link_bytes / per_step / 1e9, 2),
                "rings_per_rank_out_links": nch,
                "assumed_link_GBps_per_direction": XGMI_LINK_GBPS_PER_DIR,
            },
            "cpu_baseline": None,
        }
    comm.destroy()
    dist.barrier()
    dist.destroy_process_group()
    return out
