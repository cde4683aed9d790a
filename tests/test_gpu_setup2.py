"""BASELINE configs[4] on one MI355X: two concurrent AllReduce jobs with the
setup-2 trace shapes, run the way the reference trace generator runs them
(traffic_gen/src/main.rs:167-200: compute gap, in-place fp16 AllReduce,
stream sync per op), every iteration's result checked bit for bit.

Each job is a 4-rank virtual node on cuda:0 (two communicators, 8 ranks in
all, as on the 8-GPU node), on its own stream and host thread, so both
jobs' ring kernels are in flight at the same time.  Lanes are pinned so the
two fused launches fit on the GPU together (each job's blocks spin on each
other's flags only within the job).  Compute gaps are scaled down 10x.
"""
import threading

import pytest

from mccs_amd import comm as C
from mccs_amd import traffic

pytestmark = pytest.mark.gpu

SCALE = 0.1  # compute gaps: 160 ms -> 16 ms, 6 ms -> 0.6 ms


def _run_jobs(iters):
    import torch

    dev = torch.device("cuda", 0)
    jobs, comms_all = [], []
    try:
        for name, (nbytes, compute_us, _) in traffic.SETUP2.items():
            comms = C.init_all([0] * 4, C.CommConfig(lanes=4, timeout_ms=60000))
            comms_all.append(comms)
            jobs.append(traffic.TraceJob(torch, name, comms, [0, 1, 2, 3], 4, nbytes // 2, compute_us * 1e-6 * SCALE,
                                         torch.cuda.Stream(dev), dev))
        errors = []

        def drive(job, n):
            try:
                torch.cuda.set_device(dev)
                job.iteration(-1, record=False)  # warm-up (traffic_gen: 5 warm-up ops)
                for it in range(n):
                    job.iteration(it)
            except Exception as e:  # noqa: BLE001  (re-raised in the main thread)
                errors.append((job.name, e))

        threads = [threading.Thread(target=drive, args=(j, n)) for j, n in zip(jobs, iters)]
        for t in threads:
            t.start()
        for t in threads:
            t.join(timeout=110)
        assert not any(t.is_alive() for t in threads), "a job did not finish"
        assert not errors, errors
        return [j.summary() for j in jobs], jobs
    finally:
        torch.cuda.synchronize()
        for comms in comms_all:
            for c in comms:
                c.destroy()


def test_setup2_two_concurrent_jobs_exact_every_iteration():
    summaries, jobs = _run_jobs((3, 12))
    for s, j in zip(summaries, jobs):
        assert s["iterations"] == len(j.records) > 0
        assert s["exact_every_iteration"], s
        assert all(r.op_ms > 0 for r in j.records)
        # the iteration contains the compute gap
        assert s["iter_ms_mean"] >= s["compute_interval_ms"]
    vgg = summaries[0]
    assert vgg["bytes"] == 574_668_960 and summaries[1]["bytes"] == 83_886_080
    print(summaries)
