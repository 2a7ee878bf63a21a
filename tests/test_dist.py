"""The N>1 path on CPU: gloo, world_size 2 (and 3), static whole-block shards,
length all_gather + P2P gatherv.  The per-rank compressor here is the CPU
oracle (a test checker standing in for the GPU); on the GPU box the same
dist.compress_sharded runs with lz4jpeg.dist.hip_segment_compressor."""
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from lz4jpeg import dist as ldist

HERE = os.path.dirname(os.path.abspath(__file__))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, data, expect, q, chunk=ldist.GATHER_CHUNK):
    sys.path.insert(0, HERE)
    sys.path.insert(0, os.path.join(os.path.dirname(HERE), "lz4-jpeg_amd"))
    import oracle_api
    from lz4jpeg import dist as d
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank,
                            world_size=world)
    try:
        o = oracle_api.load()
        n = len(data)
        lo, hi = d.shard_bytes(n, world, rank)
        local = torch.from_numpy(np.frombuffer(data[lo:hi], dtype=np.uint8).copy())

        def seg(t):
            b = t.numpy()
            nb = (b.size + 299) // 300
            out = o.lz4_blocks(b, 0, nb)
            return torch.from_numpy(np.frombuffer(out, dtype=np.uint8).copy()), len(out)

        got = d.compress_sharded(local, n, seg, dst=0, chunk=chunk)
        if rank == 0:
            q.put(bytes(got.numpy().tobytes()) == expect)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,n,chunk", [
    (2, 300 * 41 + 17, ldist.GATHER_CHUNK), (2, 300 * 40, ldist.GATHER_CHUNK),
    (3, 300 * 7 + 1, ldist.GATHER_CHUNK), (2, 300 * 3, ldist.GATHER_CHUNK),
    # config 4's world size: uneven segments (41 or 42 blocks of differing
    # compressibility), gathered in 1 KiB pieces, i.e. 3-4 rounds per sender
    (8, 300 * 333 + 17, 1024),
    # more ranks than blocks: ranks 0 (the destination) and 4 hold empty shards
    # (no rounds) while the others send two pieces each
    (8, 300 * 5 + 1, 256),
    # a chunk that divides a segment exactly is one more edge of the rounds
    (8, 300 * 64, 100)])
def test_sharded_stream_equals_single(oracle, world, n, chunk):
    import golden_inputs
    data = golden_inputs.lz4_input("metamorphosis_spaces")[:n]
    expect = oracle.lz4_compress(data)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, data, expect, q, chunk))
             for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert q.get(timeout=5) is True


def _corrupt_worker(rank, world, port, bad_rank, q):
    sys.path.insert(0, os.path.join(os.path.dirname(HERE), "lz4-jpeg_amd"))
    from lz4jpeg import dist as d
    from lz4jpeg.lz4 import Lz4Error
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank,
                            world_size=world)
    try:
        def seg(t):
            # what hip_segment_compressor returns: the raw signed length, bit 63
            # set (negative as int64) on the rank whose call flagged a corrupt
            # LDS index
            n = 1000 + rank
            return torch.zeros(n, dtype=torch.uint8), (n | (1 << 63)) - (1 << 64) \
                if rank == bad_rank else n

        try:
            d.compress_sharded(torch.zeros(600, dtype=torch.uint8), 600 * world, seg, dst=0)
            q.put((rank, "no error"))
        except Lz4Error as e:
            q.put((rank, e.code))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("bad_rank", [0, 1])
def test_corrupt_segment_raises_on_every_rank(bad_rank):
    """One rank's segment carries LZ4R_LEN_CORRUPT: every rank raises
    Lz4Error(-6) after the length all_gather -- none hangs in the collective,
    none reaches the gatherv (a rank raising before the
    all_gather deadlocked the others)."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_corrupt_worker, args=(r, world, port, bad_rank, q))
             for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0, "a rank hung or crashed"
    got = dict(q.get(timeout=5) for _ in range(world))
    assert got == {0: -6, 1: -6}


def test_shards_are_block_aligned_and_cover():
    for n in [300, 301, 12345, 10 ** 6 + 7, 1 << 30]:
        for world in [1, 2, 3, 4, 8]:
            prev = 0
            for r in range(world):
                lo, hi = ldist.shard_bytes(n, world, r)
                assert lo == prev and lo % 300 == 0
                assert hi == n or hi % 300 == 0
                prev = hi
            assert prev == n


def test_chunk_ranges():
    assert ldist.chunk_ranges(0, 4) == []
    assert ldist.chunk_ranges(8, 4) == [(0, 4), (4, 8)]
    assert ldist.chunk_ranges(9, 4) == [(0, 4), (4, 8), (8, 9)]
    big = 9_000_000_000                    # an 8-GPU config-4 segment
    r = ldist.chunk_ranges(big)
    assert len(r) == 9 and r[-1][1] == big
    assert all(hi - lo <= 1 << 30 for lo, hi in r)
    with pytest.raises(ValueError):
        ldist.chunk_ranges(10, 0)
