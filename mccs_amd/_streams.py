"""Side streams of the bench legs, created once per (device, slot) and reused.

Every HIP stream a process uses is mapped onto one of its hardware queues
(GPU_MAX_HW_QUEUES = 4 per process on the GPU box).  Ranks that share one
GPU as processes (the 1-GPU rehearsals) each bring their own queues; once
they outnumber what the GPU schedules at once, the firmware time-slices the
queues and ring kernels that spin on each other's flags wait for their
peer's queue to be scheduled: the N = 8 rehearsal went from ~0.1 ms to
75-100 ms per AllReduce after its size sweep created a fresh graph stream
per size in each of the 8 processes.  So the legs reuse a few streams.
"""
from __future__ import annotations

_cache: dict = {}


def side_stream(torch, device: int | None = None, slot: int = 0):
    """A torch stream on `device` (default: the current one), the same object
    for the same (device, slot) for the life of the process."""
    if device is None:
        device = torch.cuda.current_device()
    key = (int(device), int(slot))
    st = _cache.get(key)
    if st is None:
        st = torch.cuda.Stream(device=torch.device("cuda", int(device)))
        _cache[key] = st
    return st
