"""CPU: host-side planner pieces of libmccs_hip.so (no GPU calls).

* task schema of the C++ planner == the oracle's restatement of
  get_task_schema (plan.rs:602-635);
* default ring patterns are valid rings (engine.rs:274-279 asserts a
  permutation) and, for n >= 5, edge-disjoint Hamiltonian cycles used in both
  directions (each directed xGMI link carries at most one ring);
* the ctypes mirror of mccsCommConfig matches the C layout used by the lib.
"""
import ctypes
from collections import Counter

import pytest

from mccs_amd import comm


@pytest.mark.parametrize("nbytes", [0, 1, 1024, 4095, 65536, 1 << 20, 3 << 20, 128 << 20, 1 << 30])
@pytest.mark.parametrize("nch", [1, 2, 6, 14, 32])
def test_schema_matches_oracle(orc, nbytes, nch):
    assert comm.task_schema(nbytes, nch) == orc.task_schema(nbytes, nch)


@pytest.mark.parametrize("n", [1, 2, 3, 4, 5, 6, 7, 8, 12, 16])
def test_default_rings_are_rings(n):
    rings = comm.default_rings(n)
    assert rings
    for r in rings:
        assert sorted(r) == list(range(n))
        assert r[0] == 0


@pytest.mark.parametrize("n", [5, 6, 7, 8, 12, 16])
def test_default_rings_edge_disjoint(n):
    rings = comm.default_rings(n)
    use = Counter((r[i], r[(i + 1) % n]) for r in rings for i in range(n))
    assert max(use.values()) == 1
    # every rank drives as many distinct out-links as there are rings
    outs = {b for (a, b) in use if a == 0}
    assert len(outs) == len(rings)
    assert len(rings) >= n - 2  # K_n: floor((n-1)/2) Hamiltonian cycles x 2 directions


def test_n8_uses_all_seven_links_both_ways():
    """n = 8: 7 arc-disjoint directed Hamiltonian cycles cover all 56 arcs of
    the complete digraph, so every GPU sends and receives on all 7 xGMI links,
    one ring per link and direction."""
    rings = comm.default_rings(8)
    assert len(rings) == 7
    use = Counter((r[i], r[(i + 1) % 8]) for r in rings for i in range(8))
    assert len(use) == 56 and set(use.values()) == {1}
    for g in range(8):
        assert {b for (a, b) in use if a == g} == set(range(8)) - {g}
        assert {a for (a, b) in use if b == g} == set(range(8)) - {g}


def test_n4_balanced_overlap():
    rings = comm.default_rings(4)
    use = Counter((r[i], r[(i + 1) % 4]) for r in rings for i in range(4))
    assert len(rings) == 6 and set(use.values()) == {2} and len(use) == 12


def test_requested_channel_count():
    assert len(comm.default_rings(8, 2)) == 2
    assert len(comm.default_rings(8, 32)) == 32
    assert len(comm.default_rings(2, 5)) == 5


def test_config_struct_matches_header():
    from mccs_amd._lib import _CommConfig

    # 9 ints, pad, pointer, fifo_slots, direct_bytes, oneshot_bytes, ll_bytes, 16 reserved words
    assert ctypes.sizeof(_CommConfig) == 9 * 4 + 4 + 8 + 4 * 4 + 16 * 4
    assert _CommConfig.fifo_slots.offset == 48
    assert _CommConfig.direct_bytes.offset == 52 and _CommConfig.oneshot_bytes.offset == 56
    assert _CommConfig.ll_bytes.offset == 60 and _CommConfig.reserved.offset == 64
    assert comm._sig().mccsCommConfigSize() == ctypes.sizeof(_CommConfig)
    lib = comm._sig()
    c = _CommConfig()
    lib.mccsCommConfigDefault(ctypes.byref(c))
    assert c.buffer_size == 1 << 22 and c.block_threads == 576 and c.work_fifo_depth == 4096
    assert c.locality == comm.LOCALITY_RECEIVER and c.fifo_memory == comm.FIFO_UNCACHED


def test_error_strings():
    lib = comm._sig()
    assert lib.mccsGetErrorString(8) == b"FIFO watchdog timeout"
    assert lib.mccsGetErrorString(0) == b"no error"
