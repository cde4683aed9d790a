"""ctypes mirror of include/mccs_devcomm.h (reference devcomm.h:36-163).

Used to inspect device-ABI structures copied back to the host (tests, tools)
and as the template of the reference-side binding shown in INTEGRATION.md.
Offsets are pinned by tests/test_abi_layout.py against the reference header.
"""
from __future__ import annotations

import ctypes as C

MCCS_NUM_PROTOCOLS = 1
MCCS_MAX_CONNS = 2
MCCS_MAX_NCHANNELS = 32
MCCS_WORK_SIZE = 512
MCCS_MAX_WORK_ELEMENTS = 10
MCCS_BUFFER_SLOTS = 8


class mccsDevConnInfo(C.Structure):
    _fields_ = [("buffs", C.c_void_p * MCCS_NUM_PROTOCOLS), ("tail", C.c_void_p), ("head", C.c_void_p),
                ("sizesFifo", C.c_void_p), ("offsFifo", C.c_void_p), ("step", C.c_uint64)]


class mccsDevRing(C.Structure):
    _fields_ = [("prev", C.c_int), ("next", C.c_int), ("userRanks", C.c_void_p), ("index", C.c_int)]


class _HdrUnion(C.Union):
    _fields_ = [("workNext", C.c_int32), ("doneAcks", C.c_uint32)]


class mccsDevWorkHeader(C.Structure):
    _anonymous_ = ("u",)
    _fields_ = [("u", _HdrUnion), ("funcIndex", C.c_uint16), ("isLast", C.c_uint8, 1),
                ("inFifo", C.c_uint8, 1), ("type", C.c_uint8)]


class mccsDevWorkElem(C.Structure):
    _fields_ = [("isUsed", C.c_uint8, 1), ("nWarps", C.c_uint8), ("sendbuff", C.c_void_p),
                ("recvbuff", C.c_void_p), ("count", C.c_size_t), ("root", C.c_uint32), ("bid", C.c_uint8),
                ("nChannels", C.c_uint8), ("redOpArg", C.c_uint64)]


class _WorkUnion(C.Union):
    _fields_ = [("pad", C.c_char * (MCCS_WORK_SIZE - 8)), ("elems", mccsDevWorkElem * MCCS_MAX_WORK_ELEMENTS)]


class mccsDevWork(C.Structure):
    _anonymous_ = ("u",)
    _fields_ = [("header", mccsDevWorkHeader), ("u", _WorkUnion)]


class mccsDevChannelPeer(C.Structure):
    _fields_ = [("send", mccsDevConnInfo * MCCS_MAX_CONNS), ("recv", mccsDevConnInfo * MCCS_MAX_CONNS)]


class mccsDevChannel(C.Structure):
    _fields_ = [("peers", C.c_void_p), ("ring", mccsDevRing), ("workFifoDone", C.c_void_p),
                ("_pad", C.c_uint8 * 8)]  # alignas(16) tail padding


class mccsDevComm(C.Structure):
    _fields_ = [("rank", C.c_int), ("nRanks", C.c_int), ("buffSizes", C.c_int * MCCS_NUM_PROTOCOLS),
                ("abortFlag", C.c_void_p)]


class mccsDevCommAndChannels(C.Structure):
    _fields_ = [("comm", mccsDevComm), ("_pad", C.c_uint8 * 8),
                ("channels", mccsDevChannel * MCCS_MAX_NCHANNELS)]


_STRUCTS = [mccsDevConnInfo, mccsDevRing, mccsDevWorkHeader, mccsDevWorkElem, mccsDevWork,
            mccsDevChannelPeer, mccsDevChannel, mccsDevComm, mccsDevCommAndChannels]

SIZES = {s.__name__: C.sizeof(s) for s in _STRUCTS}

OFFSETS = {
    ("mccsDevConnInfo", f): getattr(mccsDevConnInfo, f).offset
    for f in ("tail", "head", "sizesFifo", "offsFifo", "step")
}
OFFSETS.update({("mccsDevRing", f): getattr(mccsDevRing, f).offset for f in ("prev", "next", "userRanks", "index")})
OFFSETS.update({("mccsDevWorkElem", f): getattr(mccsDevWorkElem, f).offset
                for f in ("nWarps", "sendbuff", "recvbuff", "count", "root", "bid", "nChannels", "redOpArg")})
OFFSETS.update({("mccsDevWorkHeader", f): getattr(mccsDevWorkHeader, f).offset for f in ("funcIndex", "type")})
OFFSETS.update({("mccsDevChannel", f): getattr(mccsDevChannel, f).offset for f in ("peers", "ring", "workFifoDone")})
OFFSETS.update({("mccsDevComm", f): getattr(mccsDevComm, f).offset for f in ("rank", "nRanks", "buffSizes", "abortFlag")})
OFFSETS[("mccsDevCommAndChannels", "channels")] = mccsDevCommAndChannels.channels.offset
OFFSETS[("mccsDevWork", "elems")] = 8
