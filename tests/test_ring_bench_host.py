"""CPU: host-side helpers of the multi-GPU bench leg (mccs_amd/ring_bench.py)."""
import json

import pytest

import bench
from mccs_amd import comm as C
from mccs_amd import ring_bench as rb


@pytest.mark.parametrize("n", [2, 3, 4, 5, 8])
def test_default_rings_use_distinct_links(n):
    """Each default ring sends on a different outgoing link where the node has
    enough (2 x floor((n-1)/2) edge-disjoint directed cycles)."""
    rings = C.default_rings(n)
    for r in range(n):
        links = rb._out_links(rings, r)
        assert links == min(n - 1, len(rings)) or (n == 2 and links == 1), (n, r, links, rings)


def test_setup2_job_split():
    assert rb.setup2_jobs(8, False) == [[0, 1, 2, 3], [4, 5, 6, 7]]
    assert rb.setup2_jobs(8, True) == [[0, 2, 4, 6], [1, 3, 5, 7]]
    with pytest.raises(ValueError):
        rb.setup2_jobs(3, False)


def test_setup2_shapes_match_workload_files():
    # workloads/setup-2_vgg.toml: 574,668,960 B fp16; setup-2_gpt_1.toml: 83,886,080 B fp16
    assert [c * 2 for _, c in rb.SETUP2_JOBS] == [574_668_960, 83_886_080]


def test_workload_labels():
    assert rb.WORKLOADS[("float32", 128)].endswith("configs[2]")
    assert rb.WORKLOADS[("float16", 1024)].endswith("configs[3]")


def _line(share, cpu=True):
    return rb.ring_line(world=8, steps=20, warmup=5, per_step_s=1.2e-3, nbytes=128 << 20, dt_name="float32",
                        comm_info={"channels": 7, "lanes": 9, "block_threads": 576},
                        rings=C.default_rings(8), mode="receiver-uncached-fifo", tune_table=[], prof={},
                        ranks_share_gpu=share,
                        cpu_baseline=bench.ring_cpu_baseline(2, 1 << 20, budget_s=0.2) if cpu else None)


@pytest.mark.parametrize("share", [False, True])
def test_ring_line_schema(share):
    """The N > 1 line carries the contract keys, a roofline whose frac is
    achieved/peak <= 1 (HBM-bound when the ranks share one GPU) and a
    non-null host baseline with its core count and host record."""
    d = _line(share)
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
              "scaling", "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline"):
        assert k in d, k
    assert d["n_gpus"] == 8 and d["dtype"] == "f32" and d["scaling"] == "weak"
    assert abs(d["value"] - (128 << 20) / 1.2e-3 / 1e9) < 1e-3
    assert d["config"]["workload"].endswith("(BASELINE configs[2])")
    rf = d["roofline"]
    assert rf["bound"] == ("hbm" if share else "xgmi")
    # no counter traffic from a node: labelled as such, the one measured
    # ratio (virtual node) under its own name
    assert rf["traffic"] is None and rf["traffic_note"].startswith("not measured on the node")
    tv = rf["traffic_virtual_node_n2"]
    assert tv["traffic_over_algorithmic"] == 1.0042 and "virtual node" in tv["where"]
    assert tv["source"].startswith("profiles/r06_ring_vnode_summary.json")
    assert abs(rf["frac"] - rf["achieved"] / rf["peak"]) < 1e-3 and 0 < rf["frac"] <= 1
    if share:
        assert rf["peak"] == 8000.0 and abs(rf["achieved"] - 44 * (128 << 20) / 1.2e-3 / 1e9) < 0.01
    else:
        assert rf["peak"] == 7 * rb.XGMI_LINK_GBPS_PER_DIR  # all 7 links (7 directed rings)
    cb = d["cpu_baseline"]
    assert cb["value"] > 0 and cb["cores"] >= 1 and cb["kind"] == "port"
    assert cb["host"]["affinity_threads"] >= 1 and "nproc" in cb["host"]
    json.dumps(d)


def test_rehearsal_roofline_never_above_one():
    # the round-1 rehearsal (n = 2 on one GPU, 128 MiB in 0.43 ms) priced
    # against xGMI gave frac 4; against the shared HBM it is below 1
    rf = rb.ring_roofline(2, 128 << 20, 0.43e-3, 1, True, "k")
    assert rf["bound"] == "hbm" and rf["frac"] < 1


def test_bench_failure_is_nonzero_exit():
    e = rb.BenchFailure("x")
    assert isinstance(e, SystemExit) and e.code == "x"  # a non-int code exits with status 1


def test_channel_options_double_the_rings_on_distinct_gpus(monkeypatch):
    """Distinct GPUs: the autotune times the default channel count and twice
    it (bytes in flight per link grow with channels, not lanes); ranks
    sharing one GPU keep the default (co-residency)."""
    monkeypatch.delenv("MCCS_CHANNELS", raising=False)
    assert rb.channel_options(C, 2, False) == [None, 8]
    assert rb.channel_options(C, 4, False) == [None, 12]
    assert rb.channel_options(C, 8, False) == [None, 14]
    assert rb.channel_options(C, 8, True) == [None]
    monkeypatch.setenv("MCCS_CHANNELS", "7")
    assert rb.channel_options(C, 8, False) == [None]


def test_handoff_modes_go_from_relaxed_to_release_fence_to_cached():
    """Gate order within every candidate: relaxed uncached hand-offs, then the
    uncached arena with a release fence before each post, then the cached
    arena with system-scope fences; each is a distinct rejectable kind."""
    for tag, modes in rb._candidates(C, [None], [C.LOCALITY_RECEIVER, C.LOCALITY_SENDER]):
        names = [n for n, _ in modes]
        loc = tag.split("/")[0]
        assert names == [f"{loc}-uncached-fifo", f"{loc}-uncached-fifo+release-fence",
                         f"{loc}-cached-fifo+system-fences"]
        assert [cfg.fifo_memory for _, cfg in modes] == [C.FIFO_UNCACHED, C.FIFO_UNCACHED_RELEASE, C.FIFO_DEVICE]
        kinds = [n.split("-", 1)[-1] for n in names]
        assert len(set(kinds)) == 3


def test_candidates_stay_within_coresident_workgroups():
    cands = rb._candidates(C, [None, 16, 32], [C.LOCALITY_RECEIVER], [None, 14])
    tags = [t for t, _ in cands]
    assert tags == ["receiver/lanes=auto", "receiver/lanes=16", "receiver/lanes=32",
                    "receiver/lanes=auto/channels=14", "receiver/lanes=16/channels=14"]
    for _, modes in cands:
        for _, cfg in modes:
            if cfg.channel_count and cfg.lanes:
                assert cfg.channel_count * cfg.lanes <= rb.MAX_RING_WORKGROUPS


def _setup2_res():
    return {"workload": "w", "semantics": "s", "jobs": [
        {"job": "setup-2_vgg", "ranks": 4, "global_ranks": [0, 1, 2, 3], "bytes": 574_668_960, "iterations": 10,
         "iter_ms_mean": 170.0, "ms_per_call": 9.0, "algbw_GBps": 574_668_960 / 9e-3 / 1e9},
        {"job": "setup-2_gpt_1", "ranks": 4, "global_ranks": [4, 5, 6, 7], "bytes": 83_886_080, "iterations": 10,
         "iter_ms_mean": 8.0, "ms_per_call": 1.5, "algbw_GBps": 83_886_080 / 1.5e-3 / 1e9}]}


@pytest.mark.parametrize("share", [False, True])
def test_setup2_line_is_self_standing(share):
    """configs[4] alone: value = the jobs' summed algbw, ms_per_step = the
    slower job's round, an xGMI roofline summed over the jobs (HBM when the
    ranks share one GPU) and a host cpu_baseline."""
    cpu = bench.ring_cpu_baseline(2, 1 << 20, 6, budget_s=0.2)
    d = rb.setup2_line(_setup2_res(), 8, 10, 1, 1.0, share, cpu)
    for k in ("metric", "value", "unit", "n_gpus", "ms_per_step", "roofline", "cpu_baseline", "dtype", "config"):
        assert d[k] is not None, k
    assert d["ms_per_step"] == 170.0 and d["dtype"] == "f16"
    rf = d["roofline"]
    assert abs(rf["frac"] - rf["achieved"] / rf["peak"]) < 1e-3 and 0 < rf["frac"] <= 1
    if share:
        assert rf["bound"] == "hbm" and rf["peak"] == 8000.0
    else:
        assert rf["bound"] == "xgmi" and abs(rf["peak"] - 2 * 3 * rb.XGMI_LINK_GBPS_PER_DIR) < 1e-6  # 3 links per job rank
        want = sum(2 * 3 / 4 * j["bytes"] / (j["ms_per_call"] / 1e3) / 1e9 for j in _setup2_res()["jobs"])
        assert abs(rf["achieved"] - want) < 0.05
    assert d["cpu_baseline"]["kind"] == "port" and d["cpu_baseline"]["cores"] >= 1
    json.dumps(d)


def test_ring_line_carries_the_calibrated_peak_beside_the_spec():
    calib = {"per_link_direction_GBps": 50.0}
    d = rb.ring_line(world=8, steps=20, warmup=5, per_step_s=1.2e-3, nbytes=128 << 20, dt_name="float32",
                     comm_info={}, rings=C.default_rings(8), mode="m", tune_table=[], prof={}, ranks_share_gpu=False,
                     cpu_baseline=None, calibration=calib)
    rf = d["roofline"]
    assert rf["peak"] == 7 * rb.XGMI_LINK_GBPS_PER_DIR and rf["peak_calibrated"] == 350.0
    assert abs(rf["frac_calibrated"] - rf["achieved"] / 350.0) < 1e-3
    # sharing one GPU: no calibration fields (HBM-bound line)
    d2 = rb.ring_line(world=8, steps=20, warmup=5, per_step_s=1.2e-3, nbytes=128 << 20, dt_name="float32",
                      comm_info={}, rings=C.default_rings(8), mode="m", tune_table=[], prof={}, ranks_share_gpu=True,
                      cpu_baseline=None, calibration=calib)
    assert "peak_calibrated" not in d2["roofline"]


@pytest.mark.parametrize("mode,loc,fifo", [
    ("receiver-uncached-fifo", "LOCALITY_RECEIVER", "FIFO_UNCACHED"),
    ("sender-uncached-fifo+release-fence", "LOCALITY_SENDER", "FIFO_UNCACHED_RELEASE"),
    ("sender-cached-fifo+system-fences", "LOCALITY_SENDER", "FIFO_DEVICE")])
def test_mode_config_reproduces_the_timed_transport(mode, loc, fifo):
    cfg = rb.mode_config(C, mode, {"channels": 14, "lanes": 16})
    assert cfg.locality == getattr(C, loc) and cfg.fifo_memory == getattr(C, fifo)
    assert cfg.channel_count == 14 and cfg.lanes == 16
    # every candidate mode name maps back to its own config
    for _, modes in rb._candidates(C, [None], [C.LOCALITY_RECEIVER, C.LOCALITY_SENDER]):
        for name, want in modes:
            got = rb.mode_config(C, name, {})
            assert (got.locality, got.fifo_memory) == (want.locality, want.fifo_memory), name


def test_node_legs_report_na_when_ranks_share_a_gpu():
    inproc, calib = rb.node_legs(None, C, world=8, ndev=1, nbytes=128 << 20)
    assert "n/a" in inproc and "n/a" in calib
    # an n/a calibration leaves the spec-priced roofline alone
    d = rb.ring_line(world=8, steps=20, warmup=5, per_step_s=1.2e-3, nbytes=128 << 20, dt_name="float32",
                     comm_info={}, rings=C.default_rings(8), mode="m", tune_table=[], prof={}, ranks_share_gpu=False,
                     cpu_baseline=None, extras={"xgmi_calibration": calib}, calibration=calib)
    assert "peak_calibrated" not in d["roofline"] and "n/a" in d["config"]["xgmi_calibration"]


def test_ring_cpu_baseline_samples_large_buckets():
    cb = bench.ring_cpu_baseline(2, 1 << 30, 6, budget_s=0.2)
    assert "first 256 MiB of the 1024 MiB bucket" in cb["sample"] and cb["value"] > 0


class _OneRankDist:
    """torch.distributed stand-in for a world of one (agree() reduces over it)."""

    class ReduceOp:
        MIN, MAX = "min", "max"

    @staticmethod
    def all_reduce(t, op=None, group=None):
        return None


def test_budget_skips_late_legs_and_the_line_keeps_its_headline():
    """the N > 1 line must survive a slow node.  With a clock
    that jumps 100 s per leg and a 210 s budget, the first two legs run, the
    rest are recorded as skipped, and the line still carries value, roofline
    and cpu_baseline, plus every leg's wall time or skip."""
    now = [0.0]

    def clock():
        return now[0]

    b = rb.Budget(_OneRankDist, seconds=210, clock=clock)
    ran = []
    for name in ("graph_replay", "configs3_fp16_1GiB", "size_sweep_fp16", "reference_driven", "node_legs"):
        def leg(name=name):
            ran.append(name)
            now[0] += 100.0
            return {"ok": True}
        b.run(name, leg)
    assert ran == ["graph_replay", "configs3_fp16_1GiB"]
    legs = b.summary()["legs"]
    assert legs["graph_replay"]["wall_s"] == 100.0
    for name in ("size_sweep_fp16", "reference_driven", "node_legs"):
        assert legs[name]["skipped"] == "budget" and legs[name]["at_s"] == 200.0
    d = rb.ring_line(world=8, steps=20, warmup=5, per_step_s=1.2e-3, nbytes=128 << 20, dt_name="float32",
                     comm_info={"channels": 7, "lanes": 9, "block_threads": 576}, rings=C.default_rings(8),
                     mode="receiver-uncached-fifo", tune_table=[], prof={}, ranks_share_gpu=False,
                     cpu_baseline=bench.ring_cpu_baseline(2, 1 << 20, budget_s=0.2),
                     extras={"budget": b.summary(), "size_sweep_fp16": None})
    assert d["value"] > 0 and d["roofline"]["frac"] > 0 and d["cpu_baseline"]["value"] > 0
    assert d["config"]["budget"]["legs"]["node_legs"]["skipped"] == "budget"
    assert "size_sweep_fp16" not in d["config"]
    json.dumps(d)


def test_budget_default_and_override(monkeypatch):
    monkeypatch.delenv("MCCS_BENCH_BUDGET_S", raising=False)
    assert rb.Budget(_OneRankDist).seconds == rb.DEFAULT_BUDGET_S
    monkeypatch.setenv("MCCS_BENCH_BUDGET_S", "42")
    assert rb.Budget(_OneRankDist).seconds == 42.0
    # every leg the N > 1 run can skip has an expected time
    for name in ("graph_replay", "configs3_fp16_1GiB", "allgather_16MiB_per_rank", "size_sweep_fp16",
                 "direct_sweep_fp16", "configs4_two_jobs", "reference_driven", "node_legs", "cpu_ring_baseline"):
        assert rb.LEG_NEED_S[name] > 0


def test_scale_report_reads_a_node_line(tmp_path):
    """tools/scale_report.py (the round-6 reading of the first SCALE record)
    finds N > 1 lines at any nesting and reports gate, roofline, autotune,
    depth A and budget."""
    import importlib.util
    import os

    spec = importlib.util.spec_from_file_location(
        "scale_report", os.path.join(os.path.dirname(os.path.dirname(__file__)), "tools", "scale_report.py"))
    sr = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(sr)
    b = rb.Budget(_OneRankDist, seconds=10, clock=lambda: 0.0)
    b.legs = {"headline": {"wall_s": 1.5}, "size_sweep_fp16": {"skipped": "budget", "at_s": 9.0, "need_s": 25}}
    d = rb.ring_line(world=8, steps=20, warmup=5, per_step_s=1.2e-3, nbytes=128 << 20, dt_name="float32",
                     comm_info={"channels": 7, "lanes": 9, "block_threads": 576}, rings=C.default_rings(8),
                     mode="receiver-uncached-fifo",
                     tune_table=[{"mode": "receiver-uncached-fifo", "channels": 7, "lanes": 9, "ms_per_step": 1.2}],
                     prof={}, ranks_share_gpu=False, cpu_baseline=None,
                     extras={"budget": b.summary(),
                             "node_gate": {"ran": True, "fifo_memory_run": 2, "failed_bits": 0x1, "disabled_bits": 0x8},
                             "rejected_before_timing": [{"mode": "sender-uncached-fifo", "rank0_reason": "exact-sum mismatch"}],
                             "connect_timing_per_rank": [{"setup_s": 0.1, "exchange_s": 0.2, "connect_s": 1.5}]})
    p = tmp_path / "scale.json"
    p.write_text(json.dumps({"runs": {"8": d}, "1": {"metric": "x", "n_gpus": 1, "config": {}}}))
    lines = [l for line in sr.load(str(p)) for l in sr.report(line)]
    text = "\n".join(lines)
    assert "N = 8" in text and "N = 1" not in text
    assert "hand-off=uncached + release" in text and "failed=[ring uncached]" in text and "disabled=[LL]" in text
    assert "stepped down" in text and "rejected before timing: sender-uncached-fifo (exact-sum mismatch)" in text
    assert "skipped ['size_sweep_fp16']" in text and "slowest connect (+ gate): 1.5 s" in text
