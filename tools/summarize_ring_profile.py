#!/usr/bin/env python3
"""Per-configuration durations of the fused virtual-node ring kernel from a
rocprofv3 kernel trace (tools/profile_ring.sh), grouped by grid shape.

  python tools/summarize_ring_profile.py <round_tag>

Grid_Size_Y = ranks sharing the GPU, Grid_Size_X / Workgroup_Size_X =
workgroups per rank (channels x lanes).  Writes profiles/<tag>_ring_vnode_*.
"""
import csv
import json
import os
import shutil
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "gpurun_out", "prof_ring_trace")
PROF = os.path.join(ROOT, "profiles")


def main():
    tag = sys.argv[1]
    bucket = 128 << 20
    groups = defaultdict(list)
    for r in csv.DictReader(open(os.path.join(OUT, "trace_kernel_trace.csv"))):
        if "ring" not in r["Kernel_Name"]:
            continue
        ranks = int(r["Grid_Size_Y"])
        wgs = int(r["Grid_Size_X"]) // int(r["Workgroup_Size_X"])
        groups[(ranks, wgs)].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    rows = []
    for (ranks, wgs), d in sorted(groups.items()):
        if ranks < 2 or len(d) < 5:  # validation / warm-up launches of other shapes
            continue
        d = d[2:]  # first launches of a shape include first-touch of the FIFO arenas
        avg = sum(d) / len(d)
        rows.append({"ranks": ranks, "workgroups_per_rank": wgs, "launches": len(d), "avg_us": round(avg, 1),
                     "min_us": round(min(d), 1), "bucket_MiB": 128,
                     "kernel_algbw_GBps": round(bucket / (avg * 1e-6) / 1e9, 1)})
    for r in rows:  # algorithmic HBM bytes of all ranks per launch: (6n-4)*S
        n = r["ranks"]
        r["algorithmic_hbm_bytes"] = (6 * n - 4) * bucket
        r["algorithmic_hbm_GBps"] = round((6 * n - 4) * bucket / (r["avg_us"] * 1e-6) / 1e9, 1)
        r["hbm_frac_of_8TBps"] = round(r["algorithmic_hbm_GBps"] / 8000.0, 4)
    out = {"source": "rocprofv3 --kernel-trace --stats, tools/profile_ring.sh (virtual node, one MI355X)",
           "per_config": rows}
    # PMC passes at n = 2 (FETCH_SIZE x2 gfx950 wide-read correction, WRITE_SIZE exact; KiB per launch)
    pmc = {}
    for c in ("FETCH_SIZE", "WRITE_SIZE"):
        f = os.path.join(ROOT, "gpurun_out", f"prof_ring_{c}", "pmc_counter_collection.csv")
        if not os.path.exists(f):
            continue
        vals = [float(r["Counter_Value"]) for r in csv.DictReader(open(f))
                if "ring_multi" in r["Kernel_Name"]]  # the PMC passes run n = 2 only
        vals = vals[2:]
        if vals:
            pmc[c] = sum(vals) / len(vals) * 1024 * (2 if c == "FETCH_SIZE" else 1)
            shutil.copy(f, os.path.join(PROF, f"{tag}_ring_vnode_pmc_{c}.csv"))
    if len(pmc) == 2:
        alg = (6 * 2 - 4) * bucket
        out["pmc_n2"] = {"read_bytes": int(pmc["FETCH_SIZE"]), "write_bytes": int(pmc["WRITE_SIZE"]),
                         "traffic_bytes": int(pmc["FETCH_SIZE"] + pmc["WRITE_SIZE"]), "algorithmic_bytes": alg,
                         "traffic_over_algorithmic": round((pmc["FETCH_SIZE"] + pmc["WRITE_SIZE"]) / alg, 4)}
    json.dump(out, open(os.path.join(PROF, f"{tag}_ring_vnode_summary.json"), "w"), indent=1)
    shutil.copy(os.path.join(OUT, "trace_kernel_stats.csv"), os.path.join(PROF, f"{tag}_ring_vnode_kernel_stats.csv"))
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
