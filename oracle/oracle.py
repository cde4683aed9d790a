"""TEST INFRASTRUCTURE: numpy-facing wrapper of the C oracle (mccs_oracle.c).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import
this module, and only as the checker / CPU baseline.  The product path
(mccs_amd) never imports it.  See mccs_oracle.c for the reference file:line
each function restates.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_SO = os.path.join(_HERE, "libmccs_oracle.so")

# mccsDevDataType_t codes -> numpy storage dtype (bf16 as raw uint16 bits)
NP_DTYPE = {
    0: np.int8, 1: np.uint8, 2: np.int32, 3: np.uint32, 4: np.int64, 5: np.uint64,
    6: np.float16, 7: np.float32, 8: np.float64, 9: np.uint16,
}
SUM, PROD, MAX, MIN = 0, 1, 2, 3

_lib = None


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(_SO):
            subprocess.run(["make", "-s", "-C", _HERE], check=True)
        L = ctypes.CDLL(_SO)
        vp, sz, ci = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int
        P = ctypes.POINTER
        L.oracle_apply.argtypes = [ci, ci, vp, vp, vp, sz]
        L.oracle_reduce_copy.argtypes = [ci, ci, P(vp), ci, P(vp), ci, sz]
        L.oracle_reduce_mt.argtypes = [ci, ci, P(vp), ci, vp, sz, ci]
        L.oracle_task_schema.argtypes = [sz, ci, P(ci), P(ci)]
        L.oracle_task_schema.restype = None
        L.oracle_ring_allreduce.argtypes = [ci, ci, ci, P(vp), P(vp), sz, ci, ci, ci, P(ci), P(ci)]
        L.oracle_ring_allgather.argtypes = [ci, P(vp), P(vp), sz]
        L.oracle_ring_allreduce_mt.argtypes = [ci, ci, ci, P(vp), vp, sz, ci, ci, ci, P(ci),
                                               ctypes.c_longlong, ctypes.c_longlong, ci]
        L.oracle_half_to_float.argtypes = [ctypes.c_uint16]
        L.oracle_half_to_float.restype = ctypes.c_float
        L.oracle_float_to_half.argtypes = [ctypes.c_float]
        L.oracle_float_to_half.restype = ctypes.c_uint16
        L.oracle_float_to_bf16.argtypes = [ctypes.c_float]
        L.oracle_float_to_bf16.restype = ctypes.c_uint16
        L.oracle_verifiable_float_sum.argtypes = [ci, ci, ci, ci, ctypes.c_uint64, ctypes.c_int64, sz, ci, vp]
        L.oracle_sum_float_tolerance.argtypes = [ci, ci]
        L.oracle_sum_float_tolerance.restype = ctypes.c_uint
        _lib = L
    return _lib


def _pa(arrs):
    a = (ctypes.c_void_p * len(arrs))()
    for i, x in enumerate(arrs):
        a[i] = x.ctypes.data
    return a


def apply(dtype: int, op: int, x: np.ndarray, y: np.ndarray) -> np.ndarray:
    """fn(x, y) elementwise (reduce_kernel.h functor semantics)."""
    out = np.empty_like(x)
    rc = lib().oracle_apply(dtype, op, out.ctypes.data, x.ctypes.data, y.ctypes.data, x.size)
    assert rc == 0
    return out


def reduce_copy(dtype: int, op: int, srcs: list[np.ndarray], ndsts: int = 1) -> list[np.ndarray]:
    srcs = [np.ascontiguousarray(s) for s in srcs]
    dsts = [np.empty_like(srcs[0]) for _ in range(ndsts)]
    rc = lib().oracle_reduce_copy(dtype, op, _pa(srcs), len(srcs), _pa(dsts), ndsts, srcs[0].size)
    assert rc == 0
    return dsts


def reduce_mt(dtype: int, op: int, srcs: list[np.ndarray], dst: np.ndarray, nthreads: int) -> None:
    rc = lib().oracle_reduce_mt(dtype, op, _pa(srcs), len(srcs), dst.ctypes.data, dst.size, nthreads)
    assert rc == 0


def task_schema(total_bytes: int, nchannels_cfg: int) -> tuple[int, int]:
    a, b = ctypes.c_int(), ctypes.c_int()
    lib().oracle_task_schema(total_bytes, nchannels_cfg, ctypes.byref(a), ctypes.byref(b))
    return a.value, b.value


def ring_allreduce(dtype: int, op: int, inputs: list[np.ndarray], nchannels: int, nthreads: int,
                   buff_size: int = 1 << 22, ring_orders=None, want_owner: bool = False):
    """Result of the reference ring kernel on every rank (all ranks identical)."""
    n = len(inputs)
    inputs = [np.ascontiguousarray(x) for x in inputs]
    out = [np.empty_like(inputs[0])]
    outs = (ctypes.c_void_p * n)()
    for r in range(n):
        outs[r] = out[0].ctypes.data  # every rank's result is identical
    ro = None
    if ring_orders is not None:
        flat = np.ascontiguousarray(np.asarray(ring_orders, dtype=np.int32).reshape(-1))
        ro = flat.ctypes.data_as(ctypes.POINTER(ctypes.c_int))
    owner = np.empty(inputs[0].size, dtype=np.int32) if want_owner else None
    rc = lib().oracle_ring_allreduce(
        dtype, op, n, _pa(inputs), outs, inputs[0].size, nchannels, nthreads, buff_size, ro,
        owner.ctypes.data_as(ctypes.POINTER(ctypes.c_int)) if owner is not None else None,
    )
    assert rc == 0, rc
    return (out[0], owner) if want_owner else out[0]


def ring_allreduce_mt(dtype: int, op: int, inputs, nchannels: int, nthreads: int, buff_size: int = 1 << 22,
                      ring_orders=None, workers: int = 16, out: np.ndarray | None = None) -> np.ndarray:
    """ring_allreduce's result, chunks evaluated on `workers` threads (same
    walk, same per-chunk order; for the BASELINE sizes).  `inputs` are
    C-contiguous numpy arrays (not copied); `out` must not alias them."""
    n = len(inputs)
    for x in inputs:
        assert x.flags.c_contiguous and x.size == inputs[0].size and x.dtype == inputs[0].dtype
    if out is None:
        out = np.empty_like(inputs[0])
    ro = None
    if ring_orders is not None:
        flat = np.ascontiguousarray(np.asarray(ring_orders, dtype=np.int32).reshape(-1))
        ro = flat.ctypes.data_as(ctypes.POINTER(ctypes.c_int))
    rc = lib().oracle_ring_allreduce_mt(dtype, op, n, _pa(inputs), out.ctypes.data, inputs[0].size, nchannels,
                                        nthreads, buff_size, ro, 0, 0, workers)
    assert rc == 0, rc
    return out


def ring_allgather(inputs: list[np.ndarray]) -> np.ndarray:
    n = len(inputs)
    inputs = [np.ascontiguousarray(x).view(np.uint8) for x in inputs]
    out = np.empty(n * inputs[0].size, dtype=np.uint8)
    outs = (ctypes.c_void_p * n)(*([out.ctypes.data] * n))
    assert lib().oracle_ring_allgather(n, _pa(inputs), outs, inputs[0].size) == 0
    return out


def verifiable_sum(dtype: int, nranks: int, count: int, seed: int, index0: int = 0, same_sign: bool = False):
    """nccl-tests verifiable float-sum vectors (verifiable.c restates
    verifiable.cu:466-512, 664-676): returns (inputs per rank, expected sum);
    the inputs sum exactly to the expected value in any order."""
    npdt = NP_DTYPE[dtype]
    ins = []
    for r in range(nranks):
        x = np.empty(count, dtype=npdt)
        rc = lib().oracle_verifiable_float_sum(dtype, 1, nranks, r, seed, index0, count, int(same_sign),
                                               x.ctypes.data)
        assert rc == 0, rc
        ins.append(x)
    y = np.empty(count, dtype=npdt)
    rc = lib().oracle_verifiable_float_sum(dtype, 0, nranks, 0, seed, index0, count, int(same_sign), y.ctypes.data)
    assert rc == 0, rc
    return ins, y


def sum_float_tolerance(nranks: int, dtype: int) -> int:
    """calcSumFloatTolerance (verifiable.cu:981-1004): max bit distance of an
    inexact n-term float sum from the correctly rounded one."""
    return int(lib().oracle_sum_float_tolerance(nranks, dtype))
