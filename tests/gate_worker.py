#!/usr/bin/env python3
"""The node gate across processes (a worker of tests/test_gpu_gate.py).

  python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 \
      --master-port 29541 tests/gate_worker.py

One rank per process, all on cuda:0 of the one-GPU box, MCCS_GATE=1 (the
gate runs although no pair of ranks is on distinct GPUs).  Cases, each on a
fresh communicator:
  clean      nothing injected: the gate passes every path, the comm keeps the
             relaxed uncached hand-off and every default path;
  ring       rank 1 alone reports a wrong ring sum (MCCS_GATE_INJECT): the
             ring vote carries it to every rank, all step down to the
             release mode together;
  oneshot    rank 0 alone reports a wrong one-shot sum: every rank disables
             the one-shot, its buckets take the ring on every rank;
  hang       rank 1 does not launch the LL test (MCCS_GATE_SKIP), so rank 0's
             LL kernel waits for lines that never come until the 5 s watchdog:
             a hang in a direct variant is a vote against every direct
             variant (they share one control block), not a dead communicator;
             both ranks keep the ring, exact;
  mismatch   ranks resolve different one-shot thresholds that round to the
             same arena: Connect refuses on every rank;
  late       rank 1 enters Connect 8 s after rank 0 (the gate's
             first launch used to time out after 5 s on the early rank); the
             connect-time barrier waits under the configured 20 s watchdog,
             and the gate then passes as in "clean".
After each connect, exact-sum AllReduces at LL / one-shot / ring sizes check
the results and which kernel ran.
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

G_RING_UC, G_LL, G_ONE, G_TWO = 0x1, 0x8, 0x10, 0x20


def main():
    import torch
    import torch.distributed as dist

    from mccs_amd import comm as C
    from mccs_amd import refdrive

    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dev = int(os.environ.get("LOCAL_RANK", rank)) % torch.cuda.device_count()
    torch.cuda.set_device(dev)
    dist.init_process_group("gloo", rank=rank, world_size=world)

    def exchange(b):
        out = [None] * world
        dist.all_gather_object(out, b)
        return out

    os.environ["MCCS_GATE"] = "1"
    os.environ["MCCS_TEST_HOOKS"] = "1"
    cases = {"clean": {}, "ring": {"MCCS_GATE_INJECT": hex(G_RING_UC), "MCCS_GATE_INJECT_RANK": "1"},
             "oneshot": {"MCCS_GATE_INJECT": hex(G_ONE), "MCCS_GATE_INJECT_RANK": "0"},
             "hang": {"MCCS_GATE_SKIP": hex(G_LL), "MCCS_GATE_INJECT_RANK": "1"},
             "mismatch": {"MCCS_ONESHOT_BYTES": "1000000" if rank == 0 else "1048576"},
             "late": {}}

    def late_exchange(b):
        out = exchange(b)
        if rank == 1:
            time.sleep(8.0)
        return out
    results = {}
    dv = torch.device("cuda", dev)
    for name, env in cases.items():
        for k in ("MCCS_GATE_INJECT", "MCCS_GATE_SKIP", "MCCS_GATE_INJECT_RANK", "MCCS_ONESHOT_BYTES",
                  "MCCS_DIRECT_BYTES", "MCCS_LL_BYTES"):
            os.environ.pop(k, None)
        os.environ.update(env)
        dist.barrier()
        try:
            comm = C.init_communicator_rank(rank, world, dev, late_exchange if name == "late" else exchange,
                                            C.CommConfig(timeout_ms=20000))
        except RuntimeError as e:
            results[f"{name}/connect"] = {"ok": name == "mismatch" and "mccsCommConnect" in str(e), "err": str(e)[:200]}
            continue
        if name == "mismatch":
            results["mismatch/connect"] = {"ok": False, "err": "connected"}
            comm.destroy()
            continue
        gi = comm.gate_info()
        want_mode = 2 if name == "ring" else 0  # MCCS_FIFO_UNCACHED_RELEASE / MCCS_FIFO_UNCACHED
        ok = gi["ran"] and gi["fifo_mode"] == want_mode and comm.fifo_memory == want_mode
        want_off = {"oneshot": G_ONE, "hang": G_LL | G_ONE | G_TWO}.get(name, 0)
        ok = ok and gi["disabled"] == want_off
        ok = ok and (gi["failed"] & G_RING_UC) == (G_RING_UC if name == "ring" else 0)
        results[f"{name}/gate"] = {"ok": bool(ok), "info": gi}
        # LL-sized, one-shot-sized and ring-sized buckets (defaults at n = 2:
        # LL <= 128 KiB, one-shot <= 2 MiB, two-shot off)
        for nbytes, algo in ((32 << 10, "ring" if name == "hang" else "ll"),
                             (512 << 10, "ring" if name in ("oneshot", "hang") else "oneshot"), (8 << 20, "ring")):
            count = nbytes // 4
            send = refdrive.exact_inputs(torch, count, rank, torch.float32, dv)
            want = refdrive.expected_exact(torch, count, world, torch.float32, dv)
            recv = torch.empty_like(send)
            C.all_reduce(comm, send, recv, count, 7, 0)
            comm.sync()
            results[f"{name}/{nbytes}"] = {"ok": bool(torch.equal(recv, want)) and comm.last_algo() == algo,
                                           "algo": comm.last_algo()}
        dist.barrier()  # every rank's last kernel is done before any arena returns to the pool
        comm.destroy()
    allres = [None] * world
    dist.all_gather_object(allres, results)
    if rank == 0:
        merged = {k: all(r[k]["ok"] for r in allres) for k in results}
        print(json.dumps({"world": world, "cases": merged, "all_ok": all(merged.values()),
                          "detail": {k: [r[k] for r in allres] for k in results if not merged[k]}}), flush=True)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
