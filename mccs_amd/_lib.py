"""ctypes binding of libmccs_hip.so (the C-ABI in include/mccs_hip.h).

The product path has exactly one implementation: the in-tree HIP library.
If it is missing or fails to load, every call raises -- there is no CPU or
PyTorch fallback.
"""
from __future__ import annotations

import ctypes
import enum
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("MCCS_LIB_PATH") or os.path.join(_HERE, "libmccs_hip.so")  # override: A/B builds


class DataType(enum.IntEnum):
    """mccsDevDataType_t (reference src/collectives/include/collectives.h:177-192)."""

    Int8 = 0
    Uint8 = 1
    Int32 = 2
    Uint32 = 3
    Int64 = 4
    Uint64 = 5
    Float16 = 6
    Float32 = 7
    Float64 = 8
    Bfloat16 = 9


class RedOp(enum.IntEnum):
    """mccsDevRedOp_t (collectives.h:194-198)."""

    Sum = 0
    Prod = 1
    Max = 2
    Min = 3
    PreMulSum = 4
    SumPostDiv = 5


ELEM_BYTES = {
    DataType.Int8: 1, DataType.Uint8: 1, DataType.Int32: 4, DataType.Uint32: 4,
    DataType.Int64: 8, DataType.Uint64: 8, DataType.Float16: 2, DataType.Float32: 4,
    DataType.Float64: 8, DataType.Bfloat16: 2,
}

RESULT_NAMES = {
    0: "mccsSuccess", 1: "mccsUnhandledCudaError", 2: "mccsSystemError", 3: "mccsInternalError",
    4: "mccsInvalidArgument", 5: "mccsInvalidUsage", 6: "mccsRemoteError", 7: "mccsInProgress",
    8: "mccsTimeout",
}


class MccsError(RuntimeError):
    """A failed C-ABI call: the result code, plus the library's own diagnosis
    of where it failed (mccsGetLastErrorString: step, runtime call, hipError_t)."""

    def __init__(self, code: int, what: str, detail: str = ""):
        self.code = code
        self.detail = detail
        super().__init__(f"{what}: {RESULT_NAMES.get(code, code)} ({code})" + (f" [{detail}]" if detail else ""))


_c_void_p = ctypes.c_void_p
_c_int = ctypes.c_int
_c_size_t = ctypes.c_size_t
_P = ctypes.POINTER

class _CommConfig(ctypes.Structure):
    """mccsCommConfig (include/mccs_hip.h)."""

    _fields_ = [("channel_count", _c_int), ("buffer_size", _c_int), ("lanes", _c_int),
                ("block_threads", _c_int), ("locality", _c_int), ("fifo_memory", _c_int),
                ("timeout_ms", _c_int), ("work_fifo_depth", _c_int), ("bridge_streams", _c_int),
                ("rings", _P(_c_int)), ("fifo_slots", _c_int), ("direct_bytes", _c_int),
                ("oneshot_bytes", _c_int), ("ll_bytes", _c_int), ("reserved", _c_int * 16)]


# name -> (restype, argtypes); every symbol declared in include/mccs_hip.h
SIGNATURES: dict[str, tuple] = {
    "mccs_hip_version": (ctypes.c_char_p, []),
    "mccs_hip_reduce": (_c_int, [_c_void_p, _P(_c_void_p), _c_int, _c_size_t, _c_int, _c_int, _c_void_p]),
    "mccs_hip_reduce_copy": (
        _c_int,
        [_P(_c_void_p), _c_int, _P(_c_void_p), _c_int, _c_size_t, _c_int, _c_int, _c_void_p],
    ),
    "mccs_hip_reduce_tune": (_c_int, [_c_int] * 6),
    "mccs_hip_reduce_get_tune": (None, [_P(_c_int)] * 6),
    "mccs_hip_reduce_tune_grid": (_c_int, [_c_int]),
    # ring kernels + communicator runtime
    "mccs_hip_coll_kernel": (_c_void_p, [_c_int, _c_int, _c_int]),
    "mccs_hip_launch_coll": (
        _c_int, [_c_int, _c_int, _c_int, _c_void_p, ctypes.c_uint64, _c_void_p, ctypes.c_uint, ctypes.c_uint,
                 _c_void_p]),
    "mccs_hip_set_ref_watchdog": (_c_int, [_c_int]),
    "mccsCommConfigDefault": (None, [_P(_CommConfig)]),
    "mccsCommConfigSize": (_c_size_t, []),
    "mccsCommConfigDefaultSized": (_c_int, [_P(_CommConfig), _c_size_t]),
    "mccsCommInitAll": (_c_int, [_P(_c_void_p), _c_int, _P(_c_int), _P(_CommConfig)]),
    "mccsConnectHandleSize": (_c_size_t, []),
    "mccsCommSetupRank": (_c_int, [_P(_c_void_p), _c_int, _c_int, _c_int, _P(_CommConfig), _c_void_p]),
    "mccsCommConnect": (_c_int, [_c_void_p, _c_void_p]),
    "mccsAllReduce": (_c_int, [_c_void_p, _c_void_p, _c_size_t, _c_int, _c_int, _c_void_p, _c_void_p]),
    "mccsAllGather": (_c_int, [_c_void_p, _c_void_p, _c_size_t, _c_void_p, _c_void_p]),
    "mccsGroupStart": (_c_int, []),
    "mccsGroupEnd": (_c_int, []),
    "mccsCommSync": (_c_int, [_c_void_p]),
    "mccsCommAbort": (_c_int, [_c_void_p]),
    "mccsCommDestroy": (_c_int, [_c_void_p]),
    "mccsCommInfo": (_c_int, [_c_void_p, _P(_c_int)]),
    "mccsCommRing": (_c_int, [_c_void_p, _c_int, _P(_c_int)]),
    "mccsCommDevComm": (_c_int, [_c_void_p, _P(_c_void_p)]),
    "mccsCommLastAlgo": (_c_int, [_c_void_p]),
    "mccs_ll_default": (_c_int, [_c_int]),
    "mccsCommDirectEnabled": (_c_int, [_c_void_p]),
    "mccsCommGateInfo": (_c_int, [_c_void_p, _P(_c_int)]),
    "mccsCommGuardInfo": (_c_int, [_c_void_p, _P(ctypes.c_uint64)]),
    "mccs_stream_id_native": (_c_int, []),
    "mccs_ring_profile": (_c_int, [_c_int, _P(ctypes.c_ulonglong), _c_int]),
    "mccsMemAllocShared": (_c_int, [_c_int, _c_size_t, _P(_c_void_p), _c_void_p]),
    "mccsMemFreeShared": (_c_int, [_c_int, _c_void_p]),
    "mccsMemOpenShared": (_c_int, [_c_int, _c_void_p, _P(_c_void_p)]),
    "mccsMemCloseShared": (_c_int, [_c_int, _c_void_p]),
    "mccsEventCreateShared": (_c_int, [_c_int, _P(_c_void_p), _c_void_p]),
    "mccsEventOpenShared": (_c_int, [_c_int, _c_void_p, _P(_c_void_p)]),
    "mccsEventDestroyShared": (_c_int, [_c_void_p]),
    "mccsCommEventHandle": (_c_int, [_c_void_p, _c_void_p]),
    "mccsCommStream": (_c_int, [_c_void_p, _P(_c_void_p)]),
    "mccsCommWaitEvent": (_c_int, [_c_void_p, _c_void_p]),
    "mccsEventRecordShared": (_c_int, [_c_void_p, _c_void_p]),
    "mccsStreamWaitShared": (_c_int, [_c_void_p, _c_void_p]),
    "mccsGetErrorString": (ctypes.c_char_p, [_c_int]),
    "mccsGetLastErrorString": (ctypes.c_char_p, []),
    "mccsGetLastHipError": (_c_int, []),
    "mccs_default_rings": (_c_int, [_c_int, _c_int, _P(_c_int), _c_int]),
    "mccs_task_schema": (None, [_c_size_t, _c_int, _P(_c_int), _P(_c_int)]),
    "mccs_direct_defaults": (None, [_c_int, _P(_c_int), _P(_c_int)]),
    "mccs_host_ring_allreduce": (
        _c_int, [_c_int, _P(_c_void_p), _P(_c_void_p), _c_size_t, _c_int, _c_int, _c_int, _c_int, _c_int,
                 _P(_c_int)]),
}

# Symbols appended after round 4: an older build (an A/B library under abvar/,
# MCCS_LIB_PATH) loads without them; the in-tree build must export them
# (tests/test_lib_exports.py).
_ADDED_R5 = {"mccsGetLastErrorString", "mccsGetLastHipError", "mccs_hip_set_ref_watchdog"}

_lib = None


def load(path: str | None = None) -> ctypes.CDLL:
    """Loads libmccs_hip.so once; raises if absent (no fallback exists)."""
    global _lib
    if _lib is not None:
        return _lib
    p = path or LIB_PATH
    if not os.path.exists(p):
        raise RuntimeError(
            f"{p} not found: build it with `python -m mccs_amd.build` (hipcc --offload-arch=gfx950)"
        )
    lib = ctypes.CDLL(p, mode=ctypes.RTLD_GLOBAL)
    for name, (res, args) in SIGNATURES.items():
        if name in _ADDED_R5 and not hasattr(lib, name):
            continue
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if lib.mccsCommConfigSize() != ctypes.sizeof(_CommConfig):  # the struct grew in 0.3 (mccs_hip.h ABI note)
        raise RuntimeError(f"{p}: mccsCommConfig is {lib.mccsCommConfigSize()} bytes, this binding "
                           f"{ctypes.sizeof(_CommConfig)}: rebuild or update mccs_amd/_lib.py")
    _lib = lib
    return lib


def last_error() -> str:
    """The calling thread's diagnosis of its latest failed library call ("" if none)."""
    if _lib is None or not hasattr(_lib, "mccsGetLastErrorString"):
        return ""
    return _lib.mccsGetLastErrorString().decode(errors="replace")


def check(code: int, what: str) -> None:
    """Raises MccsError for a nonzero result; call it right after the failed
    call, on the same thread (the diagnosis is per thread)."""
    if code != 0:
        raise MccsError(code, what, last_error())


def ptr_array(ptrs) -> ctypes.Array:
    arr = (ctypes.c_void_p * max(1, len(ptrs)))()
    for i, p in enumerate(ptrs):
        arr[i] = ctypes.c_void_p(int(p))
    return arr
