"""GPU smoke of the bench's in-process multi-device legs (mccs_amd/node_probe.py)
on the one-GPU box: the same code with repeated devices -- the in-process
AllReduce as a fused virtual node, the xGMI calibration as HBM copies -- so
the code the 8-GPU node runs has run on hardware.  (The reference-driven
leg needs one rank per process; tests/test_gpu_reference_driver.py and
tools/refdrv_bench.py run it.)"""
import pytest

from mccs_amd import comm as C
from mccs_amd import node_probe

pytestmark = pytest.mark.gpu


def test_in_process_multi_device_code_path():
    import torch

    r = node_probe.in_process_multi_device(torch, C, 2, 16 << 20, warmup=1, steps=3, devices=[0, 0])
    assert r["exact_sum_full_size"] is True and r["algbw_GBps"] > 0, r


def test_xgmi_calibration_code_path():
    import torch

    import importlib

    R = importlib.import_module("mccs_amd.reduce")

    before = R.get_tune()
    r = node_probe.xgmi_calibration(torch, [0, 0, 0], nbytes=4 << 20, reps=2)
    assert "error" not in r, r
    assert r["peers_distinct_gpus"] is False
    assert r["one_link"]["pull_GBps"] > 0 and r["one_link"]["push_GBps"] > 0
    assert len(r["per_peer"]) == 2 and r["all_to_all_push"]["directed_links"] == 6
    assert r["all_links_of_dev0"]["pull_GBps_total"] > 0 and r["all_links_of_dev0"]["push_GBps_total"] > 0
    assert r["per_link_direction_GBps"] > 0
    assert R.get_tune() == before  # the reduce tuning is restored
