#!/usr/bin/env python3
"""Register, scratch and LDS use of the shipped ring and direct kernels (gfx950).

Compiles the ring translation units (ring.hip, ring_ar_*.hip) with
--save-temps into a scratch directory and reads each kernel's AMDGPU
metadata from the generated assembly: .vgpr_count, .agpr_count,
.sgpr_count, .private_segment_fixed_size (scratch bytes per lane) and
.group_segment_fixed_size (LDS bytes).  Extra arguments are passed to hipcc
(e.g. -DMCCS_PLAIN_INPUT_GRID=0), so two builds can be compared:

  python tools/kernel_resources.py > /tmp/a.json
  python tools/kernel_resources.py --diff /tmp/a.json
"""
import glob
import json
import os
import re
import subprocess
import sys
import tempfile
from concurrent.futures import ThreadPoolExecutor

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "mccs_amd", "csrc")
KEYS = (".vgpr_count", ".agpr_count", ".sgpr_count", ".private_segment_fixed_size", ".group_segment_fixed_size",
        ".vgpr_spill_count", ".sgpr_spill_count")


def compile_tu(src, extra, tmp):
    d = os.path.join(tmp, os.path.basename(src))
    os.makedirs(d, exist_ok=True)
    cmd = ["hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", f"-I{ROOT}/include", f"-I{CSRC}",
           "--save-temps", "-c", src, "-o", os.path.join(d, "x.o"), *extra]
    subprocess.run(cmd, check=True, cwd=d, capture_output=True)
    out = {}
    for s in glob.glob(os.path.join(d, "*gfx950*.s")):
        text = open(s).read()
        # metadata: one "- .args: ..." map per kernel, keys in any order
        for block in re.split(r"\n  - ", text.split("amdhsa.kernels:")[-1])[1:]:
            name = re.search(r"\.name:\s+(\S+)", block)
            if not name:
                continue
            rec = {}
            for k in KEYS:
                m = re.search(re.escape(k) + r":\s+(\d+)", block)
                if m:
                    rec[k.lstrip(".")] = int(m.group(1))
            out[name.group(1)] = rec
    return out


def main():
    args = sys.argv[1:]
    diff = None
    if args[:1] == ["--diff"]:
        diff = json.load(open(args[1]))
        args = args[2:]
    srcs = sorted(glob.glob(os.path.join(CSRC, "ring*.hip"))) + [os.path.join(CSRC, "direct.hip")]
    with tempfile.TemporaryDirectory() as tmp, ThreadPoolExecutor(8) as ex:
        res = {}
        for r in ex.map(lambda s: compile_tu(s, args, tmp), srcs):
            res.update(r)
    if diff is None:
        print(json.dumps(res, indent=1, sort_keys=True))
        return
    changed = {k: {"before": diff.get(k), "after": v} for k, v in res.items() if diff.get(k) != v}
    gone = sorted(set(diff) - set(res))
    print(json.dumps({"kernels": len(res), "changed": changed, "missing": gone}, indent=1))
    sys.exit(1 if changed or gone else 0)


if __name__ == "__main__":
    main()
