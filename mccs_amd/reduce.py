"""Device-resident chunk reduce / reduce-copy (mccs_hip_reduce*, include/mccs_hip.h).

Python face of the reference's per-chunk ReduceOrCopyMulti
(src/collectives/src/common_kernel.h:624-685) run as a standalone full-chip
gfx950 kernel.  Inputs are device pointers (ints) or torch CUDA tensors.
"""
from __future__ import annotations

from . import _lib
from ._lib import DataType, RedOp

_TORCH_DT = None


def _torch_dtype_map():
    global _TORCH_DT
    if _TORCH_DT is None:
        import torch

        _TORCH_DT = {
            torch.int8: DataType.Int8, torch.uint8: DataType.Uint8, torch.int32: DataType.Int32,
            torch.int64: DataType.Int64, torch.float16: DataType.Float16,
            torch.float32: DataType.Float32, torch.float64: DataType.Float64,
            torch.bfloat16: DataType.Bfloat16,
        }
        for name, dt in (("uint32", DataType.Uint32), ("uint64", DataType.Uint64)):
            if hasattr(torch, name):
                _TORCH_DT[getattr(torch, name)] = dt
    return _TORCH_DT


def dtype_of(t) -> DataType:
    return _torch_dtype_map()[t.dtype]


def _ptr(x) -> int:
    return x.data_ptr() if hasattr(x, "data_ptr") else int(x)


def _stream_handle(stream) -> int:
    if stream is None:
        import torch

        return torch.cuda.current_stream().cuda_stream
    return stream.cuda_stream if hasattr(stream, "cuda_stream") else int(stream)


def reduce_copy(dsts, srcs, count: int | None = None, dtype=None, op=RedOp.Sum, stream=None) -> None:
    """dsts[j][i] = srcs[0][i] (op) srcs[1][i] (op) ... for i < count."""
    if not srcs or not dsts:
        raise ValueError("need at least one source and one destination")
    if dtype is None:
        dtype = dtype_of(srcs[0])
    if count is None:
        count = min(min(s.numel() for s in srcs), min(d.numel() for d in dsts))
    lib = _lib.load()
    rc = lib.mccs_hip_reduce_copy(
        _lib.ptr_array([_ptr(d) for d in dsts]), len(dsts),
        _lib.ptr_array([_ptr(s) for s in srcs]), len(srcs),
        int(count), int(dtype), int(op), _stream_handle(stream),
    )
    _lib.check(rc, "mccs_hip_reduce_copy")


def reduce(dst, srcs, count: int | None = None, dtype=None, op=RedOp.Sum, stream=None) -> None:
    """dst[i] = srcs[0][i] (op) srcs[1][i] (op) ...; dst may alias srcs[0]."""
    reduce_copy([dst], srcs, count=count, dtype=dtype, op=op, stream=stream)


def tune(variant: int = 0, unroll: int = 0, policy: int = -1, blocks_per_cu: int = 0,
         stages: int = 0, waves: int = 0) -> None:
    """Process-wide main-loop selection (0 / -1 = default for each field)."""
    _lib.check(_lib.load().mccs_hip_reduce_tune(variant, unroll, policy, blocks_per_cu, stages, waves),
               "mccs_hip_reduce_tune")


def tune_grid(blocks: int = 0) -> None:
    """Caps the LDS main loop's grid (0 = default: blocks_per_cu x CUs)."""
    _lib.check(_lib.load().mccs_hip_reduce_tune_grid(int(blocks)), "mccs_hip_reduce_tune_grid")


def get_tune() -> dict:
    import ctypes

    vals = [ctypes.c_int() for _ in range(6)]
    _lib.load().mccs_hip_reduce_get_tune(*(ctypes.byref(v) for v in vals))
    keys = ("variant", "unroll", "policy", "blocks_per_cu", "stages", "waves")
    return {k: v.value for k, v in zip(keys, vals)}
