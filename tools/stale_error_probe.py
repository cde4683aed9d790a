#!/usr/bin/env python3
"""Does a stale HIP error on the calling thread fail communicator setup?

HIP keeps a per-thread "last error" that a failed runtime call sets and only
hipGetLastError() clears.  This probe leaves one there on purpose (a
hipSetDevice on a device that does not exist), then runs mccsCommSetupRank and
mccsCommInitAll of the library named by MCCS_LIB_PATH (default: the in-tree
build) and reports what they returned; then checks whether hipErrorNotReady
from hipEventQuery on a busy event sticks the same way.  Raw ctypes only, so
an older build (abvar/libmccs_r04.so) loads too.  One JSON line on stdout.

  MCCS_LIB_PATH=abvar/libmccs_r04.so python tools/stale_error_probe.py
"""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch

    from mccs_amd._lib import _CommConfig

    path = os.environ.get("MCCS_LIB_PATH") or os.path.join(ROOT, "mccs_amd", "libmccs_hip.so")
    torch.cuda.set_device(0)
    torch.zeros(1, device="cuda")
    torch.cuda.synchronize()
    hip = ctypes.CDLL("libamdhip64.so", mode=ctypes.RTLD_GLOBAL)
    lib = ctypes.CDLL(path, mode=ctypes.RTLD_GLOBAL)
    lib.mccsConnectHandleSize.restype = ctypes.c_size_t
    lib.mccsCommSetupRank.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                      ctypes.POINTER(_CommConfig), ctypes.c_void_p]
    lib.mccsCommInitAll.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_int, ctypes.POINTER(ctypes.c_int),
                                    ctypes.POINTER(_CommConfig)]
    lib.mccsCommDestroy.argtypes = [ctypes.c_void_p]
    out = {"library": os.path.relpath(path, ROOT)}

    def cfg():
        c = _CommConfig()
        lib.mccsCommConfigDefault(ctypes.byref(c))
        return c

    def setup_rc():
        buf = (ctypes.c_char * lib.mccsConnectHandleSize())()
        h = ctypes.c_void_p()
        c = cfg()
        rc = lib.mccsCommSetupRank(ctypes.byref(h), 0, 1, 0, ctypes.byref(c), buf)
        if rc == 0:
            lib.mccsCommDestroy(h)
        return rc

    def init_all_rc():
        hs = (ctypes.c_void_p * 2)()
        devs = (ctypes.c_int * 2)(0, 0)
        c = cfg()
        rc = lib.mccsCommInitAll(hs, 2, devs, ctypes.byref(c))
        if rc == 0:
            for h in hs:
                lib.mccsCommDestroy(h)
        return rc

    out["setup_rc_clean"] = setup_rc()
    out["init_all_rc_clean"] = init_all_rc()
    out["hipSetDevice_9999_rc"] = hip.hipSetDevice(9999)
    out["setup_rc_with_stale_error"] = setup_rc()
    hip.hipGetLastError()
    hip.hipSetDevice(9999)
    out["init_all_rc_with_stale_error"] = init_all_rc()
    out["stale_error_left_after"] = hip.hipGetLastError()  # clears

    # hipEventQuery on a busy event: does hipErrorNotReady stick?
    ev = ctypes.c_void_p()
    hip.hipEventCreateWithFlags(ctypes.byref(ev), 2)
    torch.cuda._sleep(200_000_000)  # a long kernel on torch's stream
    hip.hipEventRecord(ev, ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
    out["event_query_rc"] = hip.hipEventQuery(ev)
    out["peek_after_not_ready"] = hip.hipPeekAtLastError()
    torch.cuda.synchronize()
    hip.hipGetLastError()
    hip.hipEventDestroy(ev)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
