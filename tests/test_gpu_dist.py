"""The multi-GPU data path composed end to end on the one GPU of the box:
two (or three) rank processes, each running the HIP segment compressor
(dist.hip_segment_compressor -> lz4r_compress_segment_async) on its static
whole-block shard, then dist.compress_sharded's length all_gather and P2P
gatherv.  RCCL refuses two ranks on one device, so the
transport here is gloo and each rank hands its segment over on the host; the
framed result on rank 0 must equal the single-GPU stream and the oracle's.
The decomposition is the reference's thread-per-block split
(Algorithms/parallel/LZ4/LZ4.c:742) lifted to processes."""
import os
import socket
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, data, q):
    sys.path.insert(0, HERE)
    sys.path.insert(0, os.path.join(os.path.dirname(HERE), "lz4-jpeg_amd"))
    import torch
    import torch.distributed as dist
    from lz4jpeg import dist as d
    from lz4jpeg import lz4
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank,
                            world_size=world)
    try:
        n = len(data)
        lo, hi = d.shard_bytes(n, world, rank)
        local = torch.from_numpy(np.frombuffer(data[lo:hi], dtype=np.uint8).copy()).cuda()
        comp = lz4.Compressor()
        hip = d.hip_segment_compressor(comp, final_shard=(hi == n))

        def seg_to_host(t):                  # gloo's P2P moves host tensors
            out, ln = hip(t)
            return out[:max(ln, 1)].cpu(), ln

        got = d.compress_sharded(local, n, seg_to_host, dst=0)
        if rank == 0:
            single = lz4.Compressor().compress(data)          # the one-GPU stream
            q.put((bytes(got.numpy().tobytes()), single))
        comp.close()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,n", [(2, 300 * 4001 + 123), (3, 300 * 999), (2, 1 << 22)])
def test_hip_sharded_stream_equals_single_gpu(oracle, world, n):
    import torch.multiprocessing as mp
    from lz4jpeg import synth
    data = synth.random_passages(n, length=30000, seed=1).tobytes()
    expect = oracle.lz4_compress(data)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, data, q)) for r in range(world)]
    for p in procs:
        p.start()
    got, single = q.get(timeout=180)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert single == expect
    assert got == expect
