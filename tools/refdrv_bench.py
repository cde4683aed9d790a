#!/usr/bin/env python3
"""Times the depth-A drop-in: the reference-named kernels driven exactly as
the reference's plan.rs drives them (mccs_amd/refdrive.py), one rank per
process, at 128 MiB fp32 per rank, for the configurations an unchanged Rust
service can select by configuration alone (refdrive.default_variants).

  python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
      --master-addr 127.0.0.1 --master-port 29531 tools/refdrv_bench.py [--mib 128]

Prints one JSON line (rank 0).  On a one-GPU box the ranks share the GPU, so
no byte crosses xGMI: the numbers then price the kernels and the FIFO
protocol, not the link.
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mib", type=int, default=128)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--rotate-mib", type=int, default=1152,
                    help="send/recv pairs rotated per rank (>= this many MiB; 0 = one pair reused)")
    ap.add_argument("--variants", default=None, help="comma-separated variant names (default: all)")
    a = ap.parse_args()
    import torch
    import torch.distributed as dist

    from mccs_amd import comm as C
    from mccs_amd import refdrive

    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    ndev = torch.cuda.device_count()
    dev = int(os.environ.get("LOCAL_RANK", rank)) % ndev
    torch.cuda.set_device(dev)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    max_ch = max(2, 128 // world) if ndev < world else 32  # ranks sharing a GPU: half the CUs
    variants = refdrive.default_variants(world, C.default_rings, max_ch)
    if a.variants:
        keep = set(a.variants.split(","))
        variants = [v for v in variants if v["name"] in keep]
    res = refdrive.time_reference_driven(torch, dist, rank, world, dev, a.mib << 20, variants,
                                         warmup=a.warmup, steps=a.steps, rotate_bytes=a.rotate_mib << 20)
    if rank == 0:
        print(json.dumps({"tool": "refdrv_bench", "world": world, "ranks_share_gpu": ndev < world,
                          "bytes_per_rank": a.mib << 20, "dtype": "f32", "rotate_mib": a.rotate_mib,
                          "library": os.environ.get("MCCS_LIB_PATH", "mccs_amd/libmccs_hip.so"),
                          "variants": res}), flush=True)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
