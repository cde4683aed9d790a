#!/usr/bin/env python3
"""The reference-named kernels driven the way the reference host drives them,
one rank per process (a worker of tests/test_gpu_reference_driver.py).

  python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 \
      --master-port 29513 tests/refdrv_worker.py

No communicator of this library is involved.  Each rank restates the Rust
service's host side in Python:

* transport/shm/transporter.rs:49-183 + transport/meta.rs:7-67 (SHM
  connector): per channel, a 4096-byte SendBufMeta (head at offset 0), a
  4096-byte RecvBufMeta (tail at offset 0) and the FIFO data of this rank's
  outgoing edge (Locality::Sender), zeroed, shared with the peers over IPC
  (the reference shares host memory inside one service process);
* comm/device.rs:35-183 (CommDevResources::new, conn_info_to_dev): the
  mccsDevCommAndChannels, per-channel peers arrays, userRanks, ring
  prev/next/index, abortFlag, workFifoDone;
* plan.rs:424-600 (upload_work / work_elem_conversion): one mccsDevWork per
  channel with isLast / inFifo / doneAcks and the reference nWarps;
* plan.rs:638-669 (launch_plan): grid = #channels, block = get_task_schema's
  nthreads (544 = 8.5 waves), through mccs_hip_launch_coll.

Each case runs three times on the same structures (conn->step persists across
launches, prims_simple.h:318-319,461); results are compared bit for bit with
the oracle, workFifoDone with doneAcks, and conn->step across ranks.
"""
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

FUNC_ALLREDUCE = 4  # mccsFuncAllReduce (mccs_devcomm.h)
BUFF_SIZE = 1 << 22  # mccs.toml buffer_sizes = [4194304]
META = 4096
BLOCK = 2 * META + BUFF_SIZE  # [SendBufMeta][RecvBufMeta][FIFO data] per channel


def main():
    import torch
    import torch.distributed as dist

    from mccs_amd import _lib as L
    from mccs_amd import abi
    from oracle import oracle as orc
    import vnode

    rank, n = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dev = int(os.environ.get("LOCAL_RANK", rank)) % torch.cuda.device_count()
    torch.cuda.set_device(dev)
    dist.init_process_group("gloo", rank=rank, world_size=n)
    lib = L.load()
    hip = ctypes.CDLL("libamdhip64.so")
    keep = []

    def upload(b: bytes) -> int:
        t = torch.frombuffer(bytearray(b), dtype=torch.uint8).cuda()
        keep.append(t)
        return t.data_ptr()

    def download(ptr, nbytes) -> bytes:
        buf = (ctypes.c_char * nbytes)()
        assert hip.hipMemcpy(buf, ctypes.c_void_p(ptr), ctypes.c_size_t(nbytes), 2) == 0  # DeviceToHost
        return bytes(buf)

    nch = 2  # mccs.toml channel_count; every case below is large enough for 2
    ring = list(range(n))
    # this rank's side of every channel, exported to the peers
    mine, handles = [], []
    for c in range(nch):
        p = ctypes.c_void_p()
        h = (ctypes.c_char * 64)()
        L.check(lib.mccsMemAllocShared(dev, BLOCK, ctypes.byref(p), h), "mccsMemAllocShared")
        assert hip.hipMemset(p, 0, ctypes.c_size_t(BLOCK)) == 0
        mine.append(p.value)
        handles.append(bytes(h))
    allh = [None] * n
    dist.all_gather_object(allh, handles)
    blocks = [[None] * n for _ in range(nch)]  # blocks[c][r]: rank r's block, as mapped here
    for c in range(nch):
        for r in range(n):
            if r == rank:
                blocks[c][r] = mine[c]
            else:
                p = ctypes.c_void_p()
                L.check(lib.mccsMemOpenShared(dev, allh[r][c], ctypes.byref(p)), "mccsMemOpenShared")
                blocks[c][r] = p.value
    assert hip.hipDeviceSynchronize() == 0
    dist.barrier()

    def send_meta(c, r):
        return blocks[c][r]

    def recv_meta(c, r):
        return blocks[c][r] + META

    def fifo(c, r):
        return blocks[c][r] + 2 * META

    done = torch.zeros(32, dtype=torch.int32, device="cuda")  # workFifoDone per channel
    abort = torch.zeros(16, dtype=torch.int32, device="cuda")
    hc = abi.mccsDevCommAndChannels()
    hc.comm.rank = rank
    hc.comm.nRanks = n
    hc.comm.buffSizes[0] = BUFF_SIZE
    hc.comm.abortFlag = abort.data_ptr()
    peer_ptrs = []
    for c in range(nch):
        pos = ring.index(rank)
        user_ranks = [ring[(pos + i) % n] for i in range(n)]
        prev, nxt = user_ranks[n - 1], user_ranks[1]
        peers = (abi.mccsDevChannelPeer * n)()
        s = peers[nxt].send[0]
        s.buffs[0] = fifo(c, rank)  # Locality::Sender: the edge's data lives with its sender
        s.head = send_meta(c, rank)
        s.tail = recv_meta(c, nxt)
        rc = peers[prev].recv[0]
        rc.buffs[0] = fifo(c, prev)
        rc.tail = recv_meta(c, rank)
        rc.head = send_meta(c, prev)
        ch = hc.channels[c]
        ch.peers = upload(bytes(peers))
        peer_ptrs.append(ch.peers)
        ch.ring.prev, ch.ring.next = prev, nxt
        ch.ring.userRanks = upload(np.asarray(user_ranks, np.int32).tobytes())
        ch.ring.index = (pos - ring.index(0)) % n
        ch.workFifoDone = done.data_ptr() + 4 * c
    comm_ptr = upload(bytes(hc))
    stream = torch.cuda.Stream()

    results, acks = {}, 0
    for code, count in ((6, 1 << 20), (7, (1 << 21) + 3), (2, 300007), (6, 777777)):
        sched_nch, nthr = orc.task_schema(count * vnode.ESIZE[code], nch)
        assert sched_nch == nch, (count, sched_nch)
        rng = np.random.default_rng(count + rank)
        for rep in range(3):
            x = np.full(count, 2042 + rank, np.int32) if code == 2 else vnode.gen(code, count, rng)
            xs = [None] * n
            dist.all_gather_object(xs, x)
            send, recv = vnode.to_dev(x), vnode.to_dev(np.zeros_like(x))
            acks += 1
            works = (abi.mccsDevWork * nch)()
            for c in range(nch):
                w = works[c]
                e = w.elems[0]
                e.isUsed, e.nWarps = 1, nthr // 32
                e.sendbuff, e.recvbuff, e.count = send.data_ptr(), recv.data_ptr(), count
                e.bid, e.nChannels = c, nch
                w.header.type = 1  # mccsDevWorkTypeColl
                w.header.isLast, w.header.inFifo, w.header.doneAcks = 1, 1, acks
            wptr = upload(bytes(works))
            torch.cuda.synchronize()
            dist.barrier()
            rc_ = lib.mccs_hip_launch_coll(FUNC_ALLREDUCE, code, 0, comm_ptr, (1 << nch) - 1, wptr, nch, nthr,
                                           stream.cuda_stream)
            stream.synchronize()
            exp = orc.ring_allreduce(code, 0, xs, nchannels=nch, nthreads=nthr, buff_size=BUFF_SIZE,
                                     ring_orders=[ring] * nch)
            got = vnode.from_dev(recv, code)
            ok = rc_ == 0 and bool(np.array_equal(got.view(np.uint8), exp.view(np.uint8)))
            ok = ok and int(abort[0].item()) == 0 and bool((done[:nch].cpu().numpy() == acks).all())
            if code == 2:
                ok = ok and int(exp[0]) == 2042 * n + n * (n - 1) // 2
            steps = []
            for c in range(nch):
                pr = (abi.mccsDevChannelPeer * n).from_buffer_copy(
                    download(peer_ptrs[c], ctypes.sizeof(abi.mccsDevChannelPeer) * n))
                pos = ring.index(rank)
                steps += [pr[ring[(pos + 1) % n]].send[0].step, pr[ring[(pos - 1) % n]].recv[0].step]
            results[f"dtype{code}/n{count}/rep{rep}"] = {"ok": ok, "steps": [int(v) for v in steps]}
            del send, recv
    allres = [None] * n
    dist.all_gather_object(allres, results)
    if rank == 0:
        merged = {}
        for k in results:
            steps = [r[k]["steps"] for r in allres]
            merged[k] = all(r[k]["ok"] for r in allres) and all(s == steps[0] for s in steps)
        print(json.dumps({"world": n, "cases": merged, "all_ok": all(merged.values()),
                          "final_steps": allres[0][k]["steps"]}), flush=True)
    dist.barrier()
    for c in range(nch):
        for r in range(n):
            if r != rank:
                lib.mccsMemCloseShared(dev, ctypes.c_void_p(blocks[c][r]))
    dist.barrier()
    for c in range(nch):
        lib.mccsMemFreeShared(dev, ctypes.c_void_p(mine[c]))
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
