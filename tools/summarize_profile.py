#!/usr/bin/env python3
"""Copies rocprofv3 summaries from gpurun_out/ into profiles/ and derives the
per-launch HBM traffic of the reduce kernel from the PMC passes.

  python tools/summarize_profile.py <round_tag> [prof_tag] [bench_tag]

gfx950 correction (MI355X_MICROARCH.md §HBM): FETCH_SIZE reports half the
bytes of a wide (16 B/lane) coalesced read stream -> multiply by 2;
WRITE_SIZE is exact for 16 B/lane streaming stores.  Both are in KiB.
"""
import csv
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "gpurun_out")
PROF = os.path.join(ROOT, "profiles")


def mean_counter(path, kernel_sub):
    rows = list(csv.DictReader(open(path)))
    vals = [float(r["Counter_Value"]) for r in rows if kernel_sub in r["Kernel_Name"]]
    return (sum(vals) / len(vals), len(vals)) if vals else (None, 0)


def main():
    rtag = sys.argv[1]
    ptag = sys.argv[2] if len(sys.argv) > 2 else "reduce"
    btag = sys.argv[3] if len(sys.argv) > 3 else "reduce_float32_128MiB_reduce_lds_kernel"
    os.makedirs(PROF, exist_ok=True)
    stats = os.path.join(OUT, f"prof_{ptag}_trace", "trace_kernel_stats.csv")
    dst = os.path.join(PROF, f"{rtag}_{ptag}_kernel_stats.csv")
    shutil.copy(stats, dst)
    kname = btag.split("MiB_")[-1]
    fetch, nf = mean_counter(os.path.join(OUT, f"prof_{ptag}_FETCH_SIZE", "pmc_counter_collection.csv"), kname)
    write, nw = mean_counter(os.path.join(OUT, f"prof_{ptag}_WRITE_SIZE", "pmc_counter_collection.csv"), kname)
    tj = os.path.join(PROF, "pmc_traffic.json")
    d = json.load(open(tj)) if os.path.exists(tj) else {}
    if fetch is not None and write is not None:
        read_b = 2 * fetch * 1024
        write_b = write * 1024
        d[btag] = {
            "hbm_bytes_per_launch": int(read_b + write_b),
            "read_bytes_corrected": int(read_b),
            "write_bytes": int(write_b),
            "FETCH_SIZE_KiB_mean": fetch,
            "WRITE_SIZE_KiB_mean": write,
            "launches": [nf, nw],
            "correction": "FETCH_SIZE x2 (gfx950 wide-stream undercount), KiB -> bytes",
            "source": f"profiles/{rtag}_{ptag}_* (rocprofv3 --pmc separate passes)",
        }
        json.dump(d, open(tj, "w"), indent=1, sort_keys=True)
    for c in ("FETCH_SIZE", "WRITE_SIZE"):
        src = os.path.join(OUT, f"prof_{ptag}_{c}", "pmc_counter_collection.csv")
        if os.path.exists(src):
            shutil.copy(src, os.path.join(PROF, f"{rtag}_{ptag}_pmc_{c}.csv"))
    # the bench's timed region = the last `steps` launches of the kernel
    steps = int(os.environ.get("PROF_STEPS", "50"))
    trace = os.path.join(OUT, f"prof_{ptag}_trace", "trace_kernel_trace.csv")
    if os.path.exists(trace):
        durs = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
                for r in csv.DictReader(open(trace)) if kname in r["Kernel_Name"]]
        timed = durs[-steps:]
        if timed and btag in d:
            d[btag]["timed_region_avg_us"] = round(sum(timed) / len(timed), 3)
            d[btag]["timed_region_launches"] = len(timed)
            d[btag]["all_launches_avg_us"] = round(sum(durs) / len(durs), 3)
            json.dump(d, open(tj, "w"), indent=1, sort_keys=True)
    print(open(dst).read())
    print(json.dumps(d.get(btag), indent=1))


if __name__ == "__main__":
    main()
