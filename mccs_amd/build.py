"""In-tree build of libmccs_hip.so (gfx950) and the CPU oracle.

``python -m mccs_amd.build`` or ``__graft_entry__.build()``.  Sources are compiled
one object per file with hipcc (parallel), then linked into
``mccs_amd/libmccs_hip.so`` so the library travels with the repo snapshot to the
GPU box.  Objects are cached under ``build/`` keyed on source mtimes.
"""
from __future__ import annotations

import concurrent.futures as cf
import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "mccs_amd")
CSRC = os.path.join(PKG, "csrc")
INCLUDE = os.path.join(ROOT, "include")
BUILD = os.path.join(ROOT, "build", "obj")
LIB = os.path.join(PKG, "libmccs_hip.so")
ARCH = os.environ.get("MCCS_OFFLOAD_ARCH", "gfx950")

HIPCC = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
CFLAGS = [
    f"--offload-arch={ARCH}",
    "-O3",
    "-std=c++17",
    "-fPIC",
    "-Wall",
    "-Wno-unused-function",
    "-Wno-unused-variable",
    f"-I{INCLUDE}",
    f"-I{CSRC}",
]


def _sources() -> list[str]:
    out = []
    for d in (CSRC, os.path.join(CSRC, "host")):
        if not os.path.isdir(d):
            continue
        for f in sorted(os.listdir(d)):
            if f.endswith((".hip", ".cpp")):
                out.append(os.path.join(d, f))
    return out


def _headers_mtime() -> float:
    m = 0.0
    for d in (CSRC, os.path.join(CSRC, "host"), INCLUDE):
        if os.path.isdir(d):
            for f in os.listdir(d):
                if f.endswith((".h", ".hpp", ".inc")):
                    m = max(m, os.path.getmtime(os.path.join(d, f)))
    return m


def _obj_for(src: str) -> str:
    rel = os.path.relpath(src, CSRC).replace(os.sep, "_")
    return os.path.join(BUILD, rel + ".o")


def _compile(src: str, hdr_mtime: float, verbose: bool) -> str:
    obj = _obj_for(src)
    if os.path.exists(obj):
        om = os.path.getmtime(obj)
        if om >= os.path.getmtime(src) and om >= hdr_mtime:
            return obj
    cmd = [HIPCC, *CFLAGS, "-c", src, "-o", obj]
    if verbose:
        print(" ".join(cmd), flush=True)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed for {src}:\n{r.stdout}\n{r.stderr}")
    return obj


# Reference kernel names (collectives.h:43-49 MCCS_KERN_NAME, common.h:182-188)
REF_OPS = ("Sum", "Prod", "Max", "Min")
REF_TYPES = ("int8_t", "uint8_t", "int32_t", "uint32_t", "int64_t", "uint64_t", "half", "float", "double",
             "bfloat16")


def kernel_names() -> list[str]:
    """The extern "C" kernel handles ring.hip defines."""
    out = ["mccsKernel_AllGather_RING_SIMPLE_Sum_int8_t"]
    for op in REF_OPS:
        out += [f"mccsKernel_AllReduce_RING_SIMPLE_{op}_{t}" for t in REF_TYPES]
    return out


def cxx_mangled(name: str) -> str:
    """Itanium mangling of the reference declaration (collectives.h:49):
    void name(struct mccsDevComm*, uint64_t, struct mccsDevWork*)."""
    return f"_Z{len(name)}{name}P11mccsDevCommmP11mccsDevWork"


def reference_aliases() -> list[tuple[str, str]]:
    """(alias, target) symbol pairs the link adds so the reference's own
    collectives.h binds unchanged: the reference declares the kernels with
    C++ linkage (no extern "C"; collectives-sys/build.rs runs bindgen with
    -x c++), and names bf16 after CUDA's type, ..._<Op>___nv_bfloat16."""
    pairs = []
    for k in kernel_names():
        names = [k]
        if k.endswith("_bfloat16"):
            nv = k[: -len("bfloat16")] + "__nv_bfloat16"
            pairs.append((nv, k))
            names.append(nv)
        pairs += [(cxx_mangled(n), k) for n in names]
    return pairs


def build_lib(verbose: bool = False, jobs: int | None = None) -> str:
    os.makedirs(BUILD, exist_ok=True)
    srcs = _sources()
    hm = _headers_mtime()
    jobs = jobs or min(8, max(1, (os.cpu_count() or 2)))
    with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
        objs = list(ex.map(lambda s: _compile(s, hm, verbose), srcs))
    newest = max(os.path.getmtime(o) for o in objs)
    if not os.path.exists(LIB) or os.path.getmtime(LIB) < newest:
        tmp = LIB + ".tmp"
        aliases = [f"-Wl,--defsym={a}={t}" for a, t in reference_aliases()]
        cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", tmp, *objs, "-lpthread", *aliases]
        if verbose:
            print(" ".join(cmd), flush=True)
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n{r.stdout}\n{r.stderr}")
        os.replace(tmp, LIB)
    return LIB


CAPI_SRC = os.path.join(ROOT, "tests", "capi", "capi_allreduce.c")
CAPI_BIN = os.path.join(ROOT, "tests", "capi", "capi_allreduce")


def capi_cmd(src: str, out: str, syntax_only: bool = False) -> list[str]:
    """gcc (C11) against include/mccs_hip.h: the C-ABI as a non-C++ binding sees it."""
    cmd = ["gcc", "-std=c11", "-O2", "-Wall", "-Werror", f"-I{INCLUDE}", "-I/opt/rocm/include",
           "-D__HIP_PLATFORM_AMD__", src]
    if syntax_only:
        return cmd + ["-fsyntax-only"]
    return cmd + [f"-L{PKG}", "-lmccs_hip", "-L/opt/rocm/lib", "-lamdhip64",
                  "-Wl,-rpath,$ORIGIN/../../mccs_amd", "-Wl,-rpath,/opt/rocm/lib", "-o", out]


def build_capi(verbose: bool = False) -> str:
    """tests/capi/capi_allreduce: plain-C driver of the C-ABI (run on the GPU by tests/test_gpu_capi.py)."""
    build_lib(verbose=verbose)
    if os.path.exists(CAPI_BIN) and os.path.getmtime(CAPI_BIN) >= max(os.path.getmtime(CAPI_SRC),
                                                                        os.path.getmtime(LIB)):
        return CAPI_BIN
    cmd = capi_cmd(CAPI_SRC, CAPI_BIN)
    if verbose:
        print(" ".join(cmd), flush=True)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"C-ABI driver build failed:\n{r.stdout}\n{r.stderr}")
    return CAPI_BIN


def build_oracle(verbose: bool = False) -> None:
    """Builds oracle/libmccs_oracle.so (+ oracle/_ref when the reference tree exists)."""
    cmd = ["make", "-s", "-C", os.path.join(ROOT, "oracle")]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if verbose or r.returncode != 0:
        print(r.stdout, r.stderr, file=sys.stderr)
    if r.returncode != 0:
        raise RuntimeError("oracle build failed")


def main() -> None:
    verbose = "-v" in sys.argv
    print(build_lib(verbose=verbose))
    build_capi(verbose=verbose)
    build_oracle(verbose=verbose)


if __name__ == "__main__":
    main()
