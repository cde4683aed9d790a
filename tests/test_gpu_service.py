"""GPU: the application <-> backend split of libmccs across two processes.

The backend process owns a 2-rank virtual-node communicator and allocates
the buckets (mccsMemAllocShared); the application (this process) opens them
over IPC, fills them on its own stream, and issues the AllReduce through the
backend with only interprocess events ordering the two processes' streams
(libmccs memory.rs / communicator.rs / collectives.rs).  No host
synchronisation sits between fill, AllReduce and read-back.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def test_app_backend_allreduce_stream_ordered():
    import multiprocessing as mp

    import torch

    import mccs_amd
    from mccs_amd import DataType
    from mccs_amd import service as S
    import vnode

    ctx = mp.get_context("spawn")
    app_conn, be_conn = ctx.Pipe()
    proc = ctx.Process(target=S.backend_main, args=(be_conn,))
    proc.start()
    client = S.Client(app_conn)
    ptrs = []
    try:
        n, count = 2, 300007
        ranks = client.init_all([0] * n)
        stream = torch.cuda.current_stream()
        sid = stream.cuda_stream
        for r in ranks:
            client.register_stream(r, sid)
        send = [client.cuda_malloc(0, count * 4) for _ in ranks]
        recv = [client.cuda_malloc(0, count * 4) for _ in ranks]
        ptrs = send + recv
        rng = np.random.default_rng(3)
        inputs = [vnode.gen(7, count, rng) for _ in ranks]
        src = [torch.from_numpy(x).to("cuda") for x in inputs]
        out = [torch.empty_like(x) for x in src]
        for _ in range(3):  # repeated: stream order must hold every time
            for r in ranks:  # fill the backend-owned buckets on the app stream (1-source reduce = copy)
                mccs_amd.reduce(send[r].ptr, [src[r]], count=count, dtype=DataType.Float32, stream=stream)
            client.all_reduce([(r, send[r], recv[r], count, 7, 0, sid) for r in ranks])
            for r in ranks:  # read back on the same stream, ordered after the backend's launch
                mccs_amd.reduce(out[r], [recv[r].ptr], count=count, dtype=DataType.Float32, stream=stream)
            torch.cuda.synchronize()
            got = [o.cpu().numpy() for o in out]
            assert np.array_equal(got[0].view(np.uint32), got[1].view(np.uint32))
            # n = 2: x0 + x1 in fp32 is order-independent
            assert np.array_equal(got[0], (inputs[0] + inputs[1]).astype(np.float32))
            for o in out:
                o.zero_()
    finally:
        client.close(ptrs)
        proc.join(timeout=60)
        assert proc.exitcode == 0
