"""Multi-GPU sharding of the LZ4 path: one process per GPU, static split of
whole 300-byte blocks, one exchange (RCCL over xGMI with backend "nccl";
gloo on CPU for tests).

Blocks are independent (the match window is the block prefix: p < 300 <
WINDOW_SIZE, LZ4.c:295), so rank r compresses blocks [b0, b1) with no data-path
communication -- the reference's thread-per-block decomposition
(Algorithms/parallel/LZ4/LZ4.c:742) lifted to GPUs.  The only collective is the
assembly of the framed stream:
  1. all_gather of one int64 segment length per rank -> exclusive offsets
     (every rank then knows where its segment lands in the global stream);
  2. gatherv of the segments to the destination rank as batched P2P
     send/recv in rounds of <= 1 GiB pieces (segment sizes differ, so no
     padded gather), which writes the frame header byte u8(total_blocks) in
     front (write_output, LZ4.c:429).
Concatenation is exact because a block's bytes depend only on that block.

The JPEG path shards images (or tile rows) with no exchange at all.
"""
import torch
import torch.distributed as dist

BLOCK = 300


def nblocks(n):
    return (n + BLOCK - 1) // BLOCK


def shard_blocks(nb, world, rank):
    """Contiguous, balanced range of whole blocks [b0, b1) for `rank`."""
    return (nb * rank) // world, (nb * (rank + 1)) // world


def shard_bytes(n, world, rank):
    """Byte range [lo, hi) of rank's shard of an n-byte input: block aligned,
    only the globally last shard may end in a short block."""
    b0, b1 = shard_blocks(nblocks(n), world, rank)
    return b0 * BLOCK, min(b1 * BLOCK, n)


def exchange_lengths(seg_len, device, group=None):
    """all_gather of every rank's segment length -> (lengths list, offsets list)."""
    world = dist.get_world_size(group)
    mine = torch.tensor([seg_len], dtype=torch.int64, device=device)
    allv = torch.empty(world, dtype=torch.int64, device=device)
    dist.all_gather_into_tensor(allv, mine, group=group)
    lens = [int(x) for x in allv.cpu().tolist()]
    if any(L < 0 for L in lens):
        # a rank's HIP compressor flagged a corrupt LDS index (bit 63 of its
        # length): every rank raises, none gathers a wrong stream
        from .lz4 import Lz4Error
        from ._lib import LZ4R_ERR_CORRUPT
        bad = [r for r, L in enumerate(lens) if L < 0]
        raise Lz4Error(LZ4R_ERR_CORRUPT, f"exchange_lengths: corrupt segment on rank(s) {bad}")
    offs, acc = [], 0
    for L in lens:
        offs.append(acc)
        acc += L
    return lens, offs


# Largest single P2P message of the gatherv.  An 8-GPU config-4 segment is
# ~8.9 GB; one isend of that size has never run on RCCL, so every segment
# moves as a sequence of <= 1 GiB send/recv pairs.
GATHER_CHUNK = 1 << 30


def chunk_ranges(length, chunk=GATHER_CHUNK):
    """[(lo, hi), ...] cutting [0, length) into pieces of at most `chunk` bytes."""
    if chunk <= 0:
        raise ValueError("chunk must be positive")
    return [(lo, min(lo + chunk, length)) for lo in range(0, length, chunk)]


def gather_stream(segment, seg_len, nb_total, lens, offs, dst=0, group=None,
                  chunk=GATHER_CHUNK):
    """Assemble [u8 nb_total] + seg_0 + ... + seg_{W-1} on rank `dst`.
    `segment` is this rank's uint8 tensor (at least seg_len bytes) on the
    backend's device.  Returns the framed stream tensor on dst, None elsewhere.

    The gatherv runs in rounds: round k moves the k-th <= `chunk`-byte piece
    of every segment that has one, as one batched P2P group, and waits for it
    before the next round -- so no message exceeds `chunk` bytes and at most
    one piece per sender is in flight.  Every rank derives the same round
    count from `lens` (the all_gather'ed lengths), so sends and receives pair
    up round by round; empty segments take part in no round."""
    rank = dist.get_rank(group)
    world = dist.get_world_size(group)
    pieces = [chunk_ranges(L, chunk) for L in lens]
    rounds = max((len(p) for r, p in enumerate(pieces) if r != dst), default=0)
    out = None
    if rank == dst:
        total = 1 + sum(lens)
        out = torch.empty(total, dtype=torch.uint8, device=segment.device)
        out[0] = nb_total & 0xFF
        out[1 + offs[rank]:1 + offs[rank] + seg_len].copy_(segment[:seg_len])
    for k in range(rounds):
        ops = []
        if rank == dst:
            for r in range(world):
                if r == dst or k >= len(pieces[r]):
                    continue
                lo, hi = pieces[r][k]
                view = out[1 + offs[r] + lo:1 + offs[r] + hi]
                ops.append(dist.P2POp(dist.irecv, view, r, group=group))
        elif k < len(pieces[rank]):
            lo, hi = pieces[rank][k]
            ops.append(dist.P2POp(dist.isend, segment[lo:hi].contiguous(), dst, group=group))
        if ops:
            for req in dist.batch_isend_irecv(ops):
                req.wait()
    return out


def compress_sharded(local, n_total, compress_segment, dst=0, group=None, chunk=GATHER_CHUNK):
    """Full sharded job on this rank's slice `local` (uint8 tensor of
    shard_bytes(n_total, W, rank)).  `compress_segment(tensor) -> (out, len)`
    is the per-rank compressor (the HIP path in production; tests may pass a
    CPU checker).  Returns the framed stream on dst, None elsewhere."""
    seg, seg_len = compress_segment(local)
    lens, offs = exchange_lengths(seg_len, seg.device, group)
    return gather_stream(seg, seg_len, nblocks(n_total), lens, offs, dst, group, chunk)


def hip_segment_compressor(compressor, final_shard, stream=None):
    """compress_segment callable over the HIP path (lz4r_compress_segment_async).
    `final_shard`: this rank holds the globally last block (the only shard
    that may end short).  An empty shard (more ranks than blocks) gives
    length 0 without a launch."""
    from .lz4 import compress_bound

    def run(local):
        n = local.numel()
        if n == 0:
            return torch.empty(1, dtype=torch.uint8, device=local.device), 0
        out = torch.empty(compress_bound(n), dtype=torch.uint8, device=local.device)
        d_len = torch.zeros(1, dtype=torch.int64, device=local.device)
        compressor.compress_async(local, n, out, d_len, stream=stream, segment=True,
                                  final_shard=final_shard)
        if stream is not None:
            stream.synchronize()      # .item() below waits only for torch's current stream
        # the raw signed length: negative when the call flagged a corrupt LDS
        # index (bit 63).  It is NOT raised here -- a rank that raised before
        # the collective would leave the healthy ranks waiting in
        # all_gather_into_tensor forever; exchange_lengths runs the gather
        # first and then raises on every rank, so no segment reaches the
        # gatherv
        return out, int(d_len.item())
    return run
