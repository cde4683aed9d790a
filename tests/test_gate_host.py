"""The node gate's decisions on CPU (csrc/host/gate.cpp).

When a communicator spans two or more GPUs, connecting it runs one exact-sum
AllReduce through the ring in its configured hand-off and through each
enabled direct variant; a wrong ring sum steps every rank down uncached ->
uncached + release -> cached, a wrong direct sum disables that variant, and
every rank applies the same verdict.  Here the recording fake runtime
(csrc/host/rt.cpp: host memory, no kernel runs) stands in for the GPUs:
MCCS_GATE_ASSUME_PASS takes every sum as exact and MCCS_GATE_INJECT marks
chosen paths as wrong, on every rank or on one (MCCS_GATE_INJECT_RANK), so
the step-down, the disabling and the agreement are checked from the launches
the library issues.  tests/test_gpu_gate.py runs the same injections on the
GPU across processes, where the verdicts travel through the ring vote.
"""
import ctypes

import pytest

from mccs_amd import _lib
from mccs_amd import comm as C

F32, SUM = 7, 0
G_RING_UC, G_RING_REL, G_RING_SYS, G_LL, G_ONE, G_TWO = 0x1, 0x2, 0x4, 0x8, 0x10, 0x20
FIFO_UNCACHED, FIFO_DEVICE, FIFO_RELEASE = 0, 1, 2
FENCE = {FIFO_DEVICE: "0", FIFO_UNCACHED: "1", FIFO_RELEASE: "2"}  # MCCS_FENCE_* the launches carry


def _parse(line):
    kind, *kv = line.split()
    return kind, dict(x.split("=", 1) for x in kv)


def _log():
    lib = _lib.load()
    n = lib.mccs_test_fake_log(None, 0, 0)
    assert n >= 0
    buf = ctypes.create_string_buffer(n + 1)
    lib.mccs_test_fake_log(buf, n + 1, 1)
    return [_parse(x) for x in buf.value.decode().splitlines() if x]


@pytest.fixture
def gate(monkeypatch):
    lib = _lib.load()
    monkeypatch.setenv("MCCS_TEST_HOOKS", "1")
    monkeypatch.setenv("MCCS_GATE_ASSUME_PASS", "1")
    for v in ("MCCS_GATE", "MCCS_GATE_INJECT", "MCCS_GATE_SKIP", "MCCS_GATE_INJECT_RANK", "MCCS_ONESHOT_BYTES",
              "MCCS_DIRECT_BYTES",
              "MCCS_LL_BYTES", "MCCS_FIFO_MEMORY"):
        monkeypatch.delenv(v, raising=False)
    made = []

    def init(n, inject=None, rank=None, **cfg):
        assert lib.mccs_test_fake_runtime(n) == 0
        if inject is not None:
            monkeypatch.setenv("MCCS_GATE_INJECT", hex(inject))
        if rank is not None:
            monkeypatch.setenv("MCCS_GATE_INJECT_RANK", str(rank))
        comms = C.init_all(list(range(n)), C.CommConfig(buffer_size=1 << 20, **cfg))
        made.extend(comms)
        return comms

    yield init
    for c in made:
        c.destroy()
    lib.mccs_test_fake_runtime(0)


def _gate_launches(ev):
    return [kv for k, kv in ev if k == "launch"]


def test_gate_runs_every_default_path_once_per_repetition(gate):
    comms = gate(2)
    ev = _log()
    ls = _gate_launches(ev)
    # n = 2 defaults: ring (3 reps), LL (2), one-shot (2); two-shot is off at 2 ranks
    assert [kv["kind"] for kv in ls].count("ring") == 3 * 2  # one launch per device
    assert sorted(kv.get("mode") for kv in ls if kv["kind"] == "direct") == ["ll"] * 4 + ["oneshot"] * 4
    # the gate waits for every launch (it checks the sums)
    assert any(k == "host_wait" for k, _ in ev)
    for c in comms:
        gi = c.gate_info()
        assert gi == {"ran": True, "fifo_mode": FIFO_UNCACHED, "failed": 0, "disabled": 0}
        assert c.fifo_memory == FIFO_UNCACHED


def test_gate_two_shot_at_four_ranks(gate):
    gate(4)
    ls = _gate_launches(_log())
    modes = [kv.get("mode") for kv in ls if kv["kind"] == "direct"]
    assert modes.count("twoshot") == 2 * 4 and modes.count("oneshot") == 2 * 4 and modes.count("ll") == 2 * 4


@pytest.mark.parametrize("inject,mode,failed", [
    (G_RING_UC, FIFO_RELEASE, G_RING_UC),
    (G_RING_UC | G_RING_REL, FIFO_DEVICE, G_RING_UC | G_RING_REL),
])
def test_wrong_ring_sums_step_the_hand_off_down(gate, inject, mode, failed):
    comms = gate(2, inject=inject)
    for c in comms:
        gi = c.gate_info()
        assert gi["ran"] and gi["fifo_mode"] == mode and gi["failed"] & 0x7 == failed
        assert c.fifo_memory == mode
    gate_ls = _gate_launches(_log())
    # the ring's re-test ran in the new mode(s)
    assert {kv["fence"] for kv in gate_ls if kv["kind"] == "ring"} >= {"1", FENCE[mode]}
    # ... and so does every later launch
    with C.group():
        for r, c in enumerate(comms):
            C.all_reduce(c, 0x10000000 * (r + 1), 0x10000000 * (r + 1) + 0x8000000, 8 << 20, F32, SUM, stream=0)
    ls = _gate_launches(_log())
    assert ls and all(kv["kind"] == "ring" and kv["fence"] == FENCE[mode] for kv in ls)


def test_cached_mode_turns_the_ll_path_off(gate):
    """After stepping down to system-scope fences the LL one-shot (which needs
    uncached lines) is no longer taken: a 32 KiB bucket goes one-shot."""
    comms = gate(2, inject=G_RING_UC | G_RING_REL)
    _log()
    with C.group():
        for r, c in enumerate(comms):
            C.all_reduce(c, 0x10000000 * (r + 1), 0x10000000 * (r + 1) + 0x8000000, 8192, F32, SUM, stream=0)
    ls = _gate_launches(_log())
    assert [kv["mode"] for kv in ls] == ["oneshot", "oneshot"] and all(kv["fence"] == "0" for kv in ls)
    assert [c.last_algo() for c in comms] == ["oneshot", "oneshot"]


def test_wrong_in_every_mode_refuses_the_communicator(gate):
    with pytest.raises(RuntimeError, match="mccsCommInitAll"):
        gate(2, inject=G_RING_UC | G_RING_REL | G_RING_SYS)


@pytest.mark.parametrize("rank", [0, 1])
def test_one_ranks_wrong_direct_sum_disables_it_everywhere(gate, rank):
    comms = gate(2, inject=G_ONE, rank=rank)
    for c in comms:
        gi = c.gate_info()
        assert gi["disabled"] == G_ONE and gi["failed"] == G_ONE and gi["fifo_mode"] == FIFO_UNCACHED
    _log()
    # 512 KiB: one-shot by default at n = 2; with it off (two-shot is off at
    # n = 2) the bucket takes the ring on both ranks
    with C.group():
        for r, c in enumerate(comms):
            C.all_reduce(c, 0x10000000 * (r + 1), 0x10000000 * (r + 1) + 0x8000000, 131072, F32, SUM, stream=0)
    assert [kv["kind"] for kv in _gate_launches(_log())] == ["ring", "ring"]
    # LL is untouched: 32 KiB still takes it
    with C.group():
        for r, c in enumerate(comms):
            C.all_reduce(c, 0x10000000 * (r + 1), 0x10000000 * (r + 1) + 0x8000000, 8192, F32, SUM, stream=0)
    assert [kv.get("mode") for kv in _gate_launches(_log())] == ["ll", "ll"]


def test_two_shot_disabled_falls_back_to_the_ring(gate):
    comms = gate(4, inject=G_TWO | G_LL)
    for c in comms:
        assert c.gate_info()["disabled"] == G_TWO | G_LL
    _log()
    with C.group():
        for r, c in enumerate(comms):
            C.all_reduce(c, 0x10000000 * (r + 1), 0x10000000 * (r + 1) + 0x8000000, 1 << 20, F32, SUM, stream=0)
    assert {kv["kind"] for kv in _gate_launches(_log())} == {"ring"}


def test_gate_off_or_one_gpu(gate, monkeypatch):
    monkeypatch.setenv("MCCS_GATE", "0")
    comms = gate(2, inject=G_RING_UC)
    assert not any(k == "launch" for k, _ in _log())
    assert all(c.gate_info()["ran"] is False and c.fifo_memory == FIFO_UNCACHED for c in comms)


def test_gate_skipped_when_every_rank_shares_one_gpu(monkeypatch):
    lib = _lib.load()
    monkeypatch.setenv("MCCS_TEST_HOOKS", "1")
    monkeypatch.delenv("MCCS_GATE", raising=False)
    assert lib.mccs_test_fake_runtime(1) == 0
    try:
        comms = C.init_all([0, 0], C.CommConfig(buffer_size=1 << 20, lanes=1))
        try:
            assert not any(k == "launch" for k, _ in _log())
            assert all(not c.gate_info()["ran"] for c in comms)
        finally:
            for c in comms:
                c.destroy()
    finally:
        lib.mccs_test_fake_runtime(0)


def test_config_reserved_words_and_sized_default():
    lib = _lib.load()
    cfg = _lib._CommConfig()
    assert lib.mccsCommConfigSize() == ctypes.sizeof(cfg)
    assert lib.mccsCommConfigDefaultSized(ctypes.byref(cfg), ctypes.sizeof(cfg)) == 0
    assert cfg.buffer_size == 1 << 22 and list(cfg.reserved) == [0] * 16
    assert lib.mccsCommConfigDefaultSized(ctypes.byref(cfg), ctypes.sizeof(cfg) - 64) == 4  # mccsInvalidArgument


def test_nonzero_reserved_word_is_refused(monkeypatch):
    lib = _lib.load()
    monkeypatch.setenv("MCCS_TEST_HOOKS", "1")
    assert lib.mccs_test_fake_runtime(2) == 0
    try:
        cfg = _lib._CommConfig()
        lib.mccsCommConfigDefault(ctypes.byref(cfg))
        cfg.reserved[3] = 1
        comms = (ctypes.c_void_p * 2)()
        devs = (ctypes.c_int * 2)(0, 1)
        assert lib.mccsCommInitAll(comms, 2, devs, ctypes.byref(cfg)) == 4
    finally:
        lib.mccs_test_fake_runtime(0)


def test_a_hung_direct_path_turns_every_direct_variant_off(gate, monkeypatch):
    """A direct launch that hangs (here: never launched, MCCS_GATE_SKIP) is a
    vote against every direct variant -- they share one control block -- and
    the gate launches no further direct test; the ring stays."""
    monkeypatch.setenv("MCCS_GATE_SKIP", hex(G_LL))
    comms = gate(4)
    ls = _gate_launches(_log())
    assert {kv["kind"] for kv in ls} == {"ring"}  # no direct test launched after the LL one was skipped
    for c in comms:
        gi = c.gate_info()
        assert gi["disabled"] == G_LL | G_ONE | G_TWO and gi["fifo_mode"] == FIFO_UNCACHED
    with C.group():
        for r, c in enumerate(comms):
            C.all_reduce(c, 0x10000000 * (r + 1), 0x10000000 * (r + 1) + 0x8000000, 8192, F32, SUM, stream=0)
    assert {kv["kind"] for kv in _gate_launches(_log())} == {"ring"}
