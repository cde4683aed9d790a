#!/usr/bin/env python3
"""bench.py — headline benchmark of the MI355X mCCS allreduce path.

  python bench.py [--gpus N] [--steps K] [--warmup W]

N == 1 (BASELINE.json configs[1]): device-resident chunk reduce, two 128 MiB
fp32 buffers -> elementwise sum kernel (mccs_hip_reduce).  One step = one
kernel pass over the 2 x 128 MiB inputs (algorithmic bytes 3 x 128 MiB).

N > 1 (configs[2]; launched by torch.distributed.run, one rank per GPU):
ring allreduce of a 128 MiB fp32 bucket per rank over xGMI P2P FIFOs
(mccs_hip allreduce, no RCCL).  One step = one allreduce; value = algbw =
S / t (reference definition, allreduce_bench/src/main.rs:168).

Prints ONE JSON line on rank 0.  cpu_baseline: the oracle's threaded C
elementwise sum (oracle/mccs_oracle.c, kind "port") timed on this host.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "device-resident reduce GB/s; ring-allreduce algbw GB/s at 1/2/4/8 MI355X"
HBM_PEAK_GBPS = 8000.0  # MI355X_MICROARCH.md chip table: HBM3E 8.0 TB/s spec


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--size-mib", type=int, default=128)
    ap.add_argument("--dtype", default="float32", choices=["float32", "float16", "bfloat16"])
    ap.add_argument("--jobs", default=None, choices=["setup2", "setup2-interleaved"],
                    help="N>1: two concurrent allreduce jobs on the two halves of the node (BASELINE configs[4])")
    ap.add_argument("--variant", type=int, default=0, help="reduce main loop: 0 default, 1 REG, 2 LDS")
    ap.add_argument("--unroll", type=int, default=0)
    ap.add_argument("--policy", type=int, default=-1)
    ap.add_argument("--blocks-per-cu", type=int, default=0)
    ap.add_argument("--stages", type=int, default=0)
    ap.add_argument("--waves", type=int, default=0)
    ap.add_argument("--rotate-mib", type=int, default=1152,
                    help="rotate over buffer sets totalling >= this many MiB so no step's inputs are "
                         "resident in the 256 MiB Infinity Cache (0 = reuse one set)")
    ap.add_argument("--cpu-seconds", type=float, default=8.0, help="bounded CPU baseline budget")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--sweep", action="store_true", help="interleaved A/B of reduce variants (stderr)")
    ap.add_argument("--sweep-reg", action="store_true", help="interleaved A/B of the REG loop's map/policy/grid")
    ap.add_argument("--sweep-cfgs", default=None,
                    help="interleaved A/B of explicit configs 'v,u,pol,bpc,s,w;...' (stderr)")
    ap.add_argument("--sweep-rounds", type=int, default=5)
    ap.add_argument("--sweep-launches", type=int, default=12, help="timed back-to-back launches per sweep sample")
    ap.add_argument("--no-autotune", action="store_true",
                    help="N>1: skip the on-node choice of FIFO placement / lanes (library defaults + fallbacks)")
    ap.add_argument("--no-extra", action="store_true",
                    help="N>1: skip the extra BASELINE configs[3] line (fp16 1 GiB) reported in config")
    ap.add_argument("--no-hot", action="store_true", help="skip the same-buffer measurement (profiling)")
    return ap.parse_args()


def cpu_threads() -> int:
    """Threads of the host-CPU baseline: this process's CPU share.  The GPU
    box exposes every hardware thread of the host (256) to each job but
    grants a share of 16 (OMP_NUM_THREADS, which `nproc` also honours);
    the baseline runs on that share, not on CPUs other jobs own."""
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    share = os.environ.get("OMP_NUM_THREADS", "")
    if share.isdigit() and int(share) > 0:
        n = min(n, int(share))
    return max(1, n)


def cpu_baseline(dtype_code: int, nelem: int, budget_s: float) -> dict:
    """Times the oracle's threaded C elementwise sum on the same workload shape."""
    import numpy as np

    from oracle import oracle as orc

    npdt = orc.NP_DTYPE[dtype_code]
    rng = np.random.default_rng(0x6D636373)
    def gen():
        f = rng.random(nelem, dtype=np.float32) * 2 - 1
        if dtype_code == 9:  # bfloat16 stored as raw bits
            return (f.view(np.uint32) >> 16).astype(np.uint16)
        return f.astype(npdt)

    a, b = gen(), gen()
    c = np.empty_like(a)
    bytes_per = 3 * a.nbytes
    res = {}
    for label, nthr, share in (("mt", cpu_threads(), 0.7), ("st", 1, 0.3)):
        orc.reduce_mt(dtype_code, orc.SUM, [a, b], c, nthr)  # warm (page faults)
        reps, t0 = 0, time.perf_counter()
        while True:
            orc.reduce_mt(dtype_code, orc.SUM, [a, b], c, nthr)
            reps += 1
            el = time.perf_counter() - t0
            if el >= budget_s * share and reps >= 2:
                break
        res[label] = (bytes_per * reps / el / 1e9, nthr, reps, el)
    gbps, nthr, reps, el = res["mt"]
    return {
        "value": round(gbps, 3),
        "unit": "GB/s",
        "cores": nthr,
        "kind": "port",
        "sample": f"full workload: {nelem} elems x 2 srcs -> 1 dst, {reps} passes in {el:.2f}s "
                  f"on {nthr} threads; 1-thread {res['st'][0]:.3f} GB/s ({res['st'][2]} passes)",
        "single_thread_value": round(res["st"][0], 3),
    }


def ring_cpu_baseline(world: int, nbytes: int, dtype_code: int = 7, budget_s: float = 6.0) -> dict:
    """N > 1 lines: the host computes the AllReduce result itself -- the
    elementwise sum of `world` buckets of `nbytes` (oracle_reduce_mt, C,
    pthreads) on this process's CPU share (cpu_threads), plus one
    thread.  value = S / t, comparable with algbw; the host moved (n+1)*S
    bytes per pass.  A bucket larger than 256 MiB is sampled (its first
    256 MiB), so the leg stays within budget_s."""
    import numpy as np

    from mccs_amd import ring_bench as rb
    from oracle import oracle as orc

    npdt = orc.NP_DTYPE[dtype_code]
    esz = np.dtype(npdt).itemsize
    sample = min(nbytes, 256 << 20)
    n = sample // esz
    rng = np.random.default_rng(0x6D636373)
    srcs = [(rng.random(n, dtype=np.float32) * 2 - 1).astype(npdt) for _ in range(world)]
    dst = np.empty_like(srcs[0])
    threads = cpu_threads()
    res = {}
    for label, nthr, share in (("mt", threads, 0.8), ("st", 1, 0.2)):
        orc.reduce_mt(dtype_code, orc.SUM, srcs, dst, nthr)  # page in
        reps, t0 = 0, time.perf_counter()
        while True:
            orc.reduce_mt(dtype_code, orc.SUM, srcs, dst, nthr)
            reps += 1
            el = time.perf_counter() - t0
            if el >= budget_s * share or (label == "st" and reps >= 1):
                break
        res[label] = (sample * reps / el / 1e9, nthr, reps, el)
    gbps, nthr, reps, el = res["mt"]
    tname = {6: "fp16", 7: "fp32", 9: "bf16"}.get(dtype_code, str(dtype_code))
    return {"value": round(gbps, 3), "unit": "GB/s of bucket (S/t, as algbw)", "cores": nthr, "kind": "port",
            "sample": f"{world} x {sample >> 20} MiB {tname} -> 1 sum (oracle_reduce_mt)"
                      + (f", first {sample >> 20} MiB of the {nbytes >> 20} MiB bucket" if sample < nbytes else "")
                      + f", {reps} passes in {el:.2f}s on {nthr} threads = {gbps * (world + 1):.1f} GB/s of host "
                        f"memory traffic; 1-thread {res['st'][0]:.3f} GB/s",
            "single_thread_value": round(res["st"][0], 3), "host": rb.host_record()}


def host_loopback_latency(calls: int = 200) -> dict:
    """BASELINE configs[0]: 2-rank loopback AllReduce of 1 KiB fp32 on host
    threads (mccs_host_ring_allreduce: the ring protocol over host memory,
    reference schema 1 channel x 96 threads).  Median wall time per call over
    `calls` calls, timed at the C ABI with the pointer arrays built once (as a
    Rust caller holds its raw pointers), and through the Python wrapper
    (which rebuilds them per call); every result is checked against a + b
    (n = 2: exact)."""
    import numpy as np

    from mccs_amd import _lib
    from mccs_amd import comm as C

    rng = np.random.default_rng(0x6D636373)
    send = [(rng.random(256, dtype=np.float32) * 2 - 1) for _ in range(2)]
    exp = send[0] + send[1]
    fn = _lib.load().mccs_host_ring_allreduce
    f32 = int(C.AllReduceDataType.Float32)

    def timed(call):
        recv = [np.empty_like(x) for x in send]
        ts = []
        for i in range(calls + 10):
            for r in recv:
                r.fill(np.nan)
            t0 = time.perf_counter()
            call(recv)
            if i >= 10:
                ts.append(time.perf_counter() - t0)
            if not all(np.array_equal(r, exp) for r in recv):
                raise SystemExit("configs[0] host loopback: result mismatch")
        ts.sort()
        return ts

    sp = _lib.ptr_array([x.ctypes.data for x in send])
    arrays = {}

    def c_abi(recv):
        rp = arrays.get(id(recv[0]))
        if rp is None:
            rp = arrays[id(recv[0])] = _lib.ptr_array([x.ctypes.data for x in recv])
        _lib.check(fn(2, sp, rp, 256, f32, 0, 1, 96, 1 << 22, None), "mccs_host_ring_allreduce")

    ts = timed(c_abi)
    tw = timed(lambda recv: C.host_ring_allreduce(send, recv, 256, C.AllReduceDataType.Float32, channels=1,
                                                  nthreads=96))
    return {"workload": "2-rank loopback allreduce, 1 KiB fp32, host-side sum (BASELINE configs[0])",
            "median_us": round(ts[len(ts) // 2] * 1e6, 2), "p10_us": round(ts[len(ts) // 10] * 1e6, 2),
            "p90_us": round(ts[9 * len(ts) // 10] * 1e6, 2), "timed_at": "C ABI (ctypes call, pointer arrays built once)",
            "python_wrapper_median_us": round(tw[len(tw) // 2] * 1e6, 2), "calls": calls, "exact": True}


def load_pmc_traffic(tag: str):
    """HBM bytes per launch from the committed rocprofv3 --pmc summary, if any."""
    p = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if not os.path.exists(p):
        return None
    try:
        with open(p) as f:
            d = json.load(f)
        v = d.get(tag)
        return int(v["hbm_bytes_per_launch"]) if v else None
    except Exception:
        return None


def bench_reduce(args) -> dict:
    import torch

    import mccs_amd
    from mccs_amd import DataType

    dt = {"float32": (torch.float32, DataType.Float32), "float16": (torch.float16, DataType.Float16),
          "bfloat16": (torch.bfloat16, DataType.Bfloat16)}[args.dtype]
    tdt, code = dt
    esize = torch.tensor([], dtype=tdt).element_size()
    nbytes = args.size_mib << 20
    n = nbytes // esize
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    g = torch.Generator(device=dev)
    g.manual_seed(1)
    set_bytes = 3 * n * esize
    nsets = max(1, -(-(args.rotate_mib << 20) // set_bytes)) if args.rotate_mib > 0 else 1
    sets = []
    for i in range(nsets):
        g.manual_seed(2 * i + 1)
        a_i = (torch.rand(n, device=dev, generator=g) * 2 - 1).to(tdt)
        g.manual_seed(2 * i + 2)
        b_i = (torch.rand(n, device=dev, generator=g) * 2 - 1).to(tdt)
        sets.append((a_i, b_i, torch.empty_like(a_i)))
    a, b, c = sets[0]
    if args.variant or args.unroll or args.policy >= 0 or args.blocks_per_cu or args.stages or args.waves:
        mccs_amd.tune(args.variant, args.unroll, args.policy, args.blocks_per_cu, args.stages, args.waves)
    # The timed launches go to a non-blocking side stream of their own (a
    # collective library's kernels run on the caller's or its own stream, not
    # the legacy null stream); the events are recorded on that stream.
    from mccs_amd._streams import side_stream

    stream = side_stream(torch, 0, slot=0)
    stream.wait_stream(torch.cuda.current_stream())  # the inputs were generated on the default stream
    torch.cuda.set_stream(stream)
    cur = [0]

    def step():
        a_, b_, c_ = sets[cur[0] % nsets]
        cur[0] += 1
        mccs_amd.reduce(c_, [a_, b_], count=n, dtype=code, stream=stream)

    # correctness gate on the exact timed buffers: fp32/fp16/bf16 a+b is one
    # correctly rounded add, so the torch result is bit-identical
    for _ in range(nsets):
        step()
    torch.cuda.synchronize()
    for a_, b_, c_ in sets:
        ref = (a_.float() + b_.float()).to(tdt) if tdt != torch.float32 else a_ + b_
        if not torch.equal(c_, ref):
            raise SystemExit("bench_reduce: result mismatch vs a+b")
        del ref

    if args.sweep or args.sweep_reg or args.sweep_cfgs:
        # 'v,u,pol,bpc,s,w[,grid]' (grid: LDS grid cap, 0 = default)
        cfgs = [tuple(int(x) for x in c.split(",")) for c in args.sweep_cfgs.split(";")] if args.sweep_cfgs else None
        sweep_variants(sets, n, code, stream, reg_only=args.sweep_reg, cfgs=cfgs, rounds=args.sweep_rounds,
                       launches=args.sweep_launches)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    K = args.steps
    t_start, t_end = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    # A spin kernel ahead of the start event (outside the timed region) keeps
    # the GPU busy while the host enqueues the K launches, so the timed
    # region is K back-to-back steps and not the host's latency to submit the
    # first one after the synchronize (~5 us, 0.25 us per step at K = 20).
    torch.cuda._sleep(1_000_000)
    t_start.record(stream)
    for _ in range(K):
        step()
    t_end.record(stream)
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    total_ms = t_start.elapsed_time(t_end)
    alg_bytes = 3 * n * esize
    avg_launch_s = total_ms / K / 1e3  # kernel + same-stream launch boundary
    achieved = alg_bytes / avg_launch_s / 1e9
    value = alg_bytes * K / (total_ms / 1e3) / 1e9

    # same-buffer ("hot") rate for reference: inputs may partly stay in the MALL
    hot_gbps = None
    if not args.no_hot:
        for _ in range(3):
            mccs_amd.reduce(c, [a, b], count=n, dtype=code, stream=stream)
        hs, he = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        hs.record(stream)
        for _ in range(20):
            mccs_amd.reduce(c, [a, b], count=n, dtype=code, stream=stream)
        he.record(stream)
        torch.cuda.synchronize()
        hot_gbps = round(20 * 3 * n * esize / (hs.elapsed_time(he) / 1e3) / 1e9, 2)
    calib = None if args.no_hot else hbm_calibration(sets, n, code, stream)
    tune = mccs_amd.get_tune()
    kernel_name = "reduce_lds_kernel" if tune["variant"] == 2 else "reduce_reg_kernel"
    tag = f"reduce_{args.dtype}_{args.size_mib}MiB_{kernel_name}"
    traffic = load_pmc_traffic(tag)
    out = {
        "metric": METRIC,
        "submetric": "device_resident_reduce_GBps",
        "value": round(value, 2),
        "unit": "GB/s",
        "n_gpus": 1,
        "steps": K,
        "warmup": args.warmup,
        "ms_per_step": round(total_ms / K, 5),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": {"float32": "f32", "float16": "f16", "bfloat16": "bf16"}[args.dtype],
        "data": "synthetic uniform[-1,1) seeds 1,2, device-resident",
        "config": {"workload": f"1-GPU device-resident reduce: two {args.size_mib} MiB {args.dtype} "
                               f"buffers -> elementwise sum kernel (BASELINE configs[1])",
                   "elements": n, "bytes_per_step": alg_bytes,
                   "buffer_sets_rotated": nsets,
                   "same_buffer_GBps": hot_gbps,
                   "hbm_calibration": calib,
                   "reduce_tune": tune},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBPS,
                     "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBPS, 4),
                     "traffic": traffic, "kernel": kernel_name,
                     "avg_launch_us": round(avg_launch_s * 1e6, 3)},
        "wall_s": round(wall, 4),
    }
    return out


def hbm_calibration(sets, n, code, stream) -> dict:
    """What the same chip streams on simpler mixes, same buffers and rotation:
    a 1:1 copy through the same kernel (1 source -> 1 destination).  Context
    for roofline.frac (the reduce's 2:1 read/write mix streams at the copy's
    rate), not a measurement of the reduce."""
    import torch

    import mccs_amd

    def timed(fn, reps=20):
        for i in range(3):
            fn(i)
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record(stream)
        for i in range(reps):
            fn(i)
        e.record(stream)
        torch.cuda.synchronize()
        return s.elapsed_time(e) / reps / 1e3

    nb = sets[0][0].numel() * sets[0][0].element_size()
    t_copy = timed(lambda i: mccs_amd.reduce(sets[i % len(sets)][2], [sets[i % len(sets)][0]], count=n, dtype=code,
                                             stream=stream))
    return {"copy_1to1_GBps": round(2 * nb / t_copy / 1e9, 1)}


def sweep_variants(sets, n, code, stream, reg_only=False, cfgs=None, rounds=5, launches=12):
    """Interleaved rounds of reduce variants in one process, rotating buffer
    sets like the timed loop (stderr)."""
    import torch

    import mccs_amd

    if cfgs:
        pass
    elif reg_only:  # REG: grid-strided (1) / per-block contiguous (3) tiles / wave rows (4), policy, grid
        cfgs = []
        for v in (1, 3, 4):
            for u in (2, 4, 8):
                for pol in (1, 2, 3):
                    for bpc in (8, 16, 32):
                        cfgs.append((v, u, pol, bpc, 0, 0))
    else:
        cfgs = []
        for u, bpc in ((4, 32), (4, 16), (8, 16)):  # REG
            cfgs.append((1, u, 1, bpc, 0, 0))
        for u, s, w in ((1, 3, 4), (2, 2, 4), (2, 3, 4), (4, 2, 4), (4, 3, 4), (4, 4, 4), (8, 2, 4),
                        (4, 3, 5), (2, 3, 6), (4, 2, 6), (4, 3, 6), (1, 2, 8), (2, 2, 8), (4, 2, 8)):  # LDS
            for bpc in (1, 2):
                if w * s * 2 * u * bpc <= 160:
                    cfgs.append((2, u, 1, bpc, s, w))
        cfgs.append((2, 4, 2, 1, 3, 4))  # plain LDS-DMA reads
        for pol in (3, 4, 5):  # write-through stores: nt+sc1, sc1, sc0+sc1+nt
            cfgs.append((2, 4, pol, 1, 3, 4))
        cfgs.append((1, 4, 0, 8, 0, 0))
    c0 = sets[0][2]
    alg = 3 * c0.numel() * c0.element_size()
    times = {cfg: [] for cfg in cfgs}
    k = 0
    for _ in range(rounds):
        for cfg in cfgs:
            mccs_amd.tune(*cfg[:6])
            mccs_amd.tune_grid(cfg[6] if len(cfg) > 6 else 0)
            for _ in range(2):
                a_, b_, c_ = sets[k % len(sets)]
                k += 1
                mccs_amd.reduce(c_, [a_, b_], count=n, dtype=code, stream=stream)
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record(stream)
            for _ in range(launches):
                a_, b_, c_ = sets[k % len(sets)]
                k += 1
                mccs_amd.reduce(c_, [a_, b_], count=n, dtype=code, stream=stream)
            e.record(stream)
            torch.cuda.synchronize()
            times[cfg].append(s.elapsed_time(e) / launches)
    rows = sorted(((sorted(v)[len(v) // 2], min(v), cfg) for cfg, v in times.items()))
    for med, mn, cfg in rows:
        print(f"[sweep] variant={cfg[0]} unroll={cfg[1]} policy={cfg[2]} bpc={cfg[3]} stages={cfg[4]} "
              f"waves={cfg[5]} grid={cfg[6] if len(cfg) > 6 else 0} median {med*1e3:.2f} us  {alg/med/1e6:.1f} GB/s  (best {alg/mn/1e6:.1f})",
              file=sys.stderr)
    mccs_amd.tune()
    mccs_amd.tune_grid(0)


def relaunch_under_torchrun(args) -> int:
    """`python bench.py --gpus N` outside torchrun: start N ranks as children
    (this process has not touched the GPU) and return their exit code."""
    import socket
    import subprocess

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__), *sys.argv[1:]]
    return subprocess.call(cmd)


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(relaunch_under_torchrun(args))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world > 1 or args.gpus > 1:
        from mccs_amd import ring_bench

        out = ring_bench.run(args, cpu_sum_baseline=ring_cpu_baseline)
        if out is None:  # non-zero rank
            return
    else:
        out = bench_reduce(args)
        if not args.no_cpu_baseline:
            from mccs_amd import DataType

            code = {"float32": DataType.Float32, "float16": DataType.Float16,
                    "bfloat16": DataType.Bfloat16}[args.dtype]
            esz = 2 if args.dtype != "float32" else 4
            out["cpu_baseline"] = cpu_baseline(int(code), (args.size_mib << 20) // esz, args.cpu_seconds)
            out["config"]["configs0_host_loopback_1KiB"] = host_loopback_latency()
        else:
            out["cpu_baseline"] = None
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
