"""BASELINE configs 4 and 5 as one rank of the 8-GPU job sees them, on one GPU.

Config 4: 64 GiB of random_extract-style text, static whole-block shards over
8 ranks.  Rank 7's 8 GiB shard holds the globally last (short) block, crosses
the compressor's 2^24-block launch chunk, and is synthesised in HBM
(csrc/synth_dev.hip).  Every byte of its segment is compared with the
oracle's md5 (tests/golden/fullsize.json), every device block offset is
checked against the segment length, and the whole segment decodes back to the
shard on the GPU.

Config 5: 1024 4K images from one continuous rand() stream; rank 7 encodes
images 896..1023.  Every coefficient of the 128 images is compared with the
oracle's md5, and image 0 of the stream is the reference's single-image md5.
"""
import hashlib
import json
import os

import numpy as np
import pytest

import golden_inputs

pytestmark = pytest.mark.gpu

GOLDEN = json.load(open(os.path.join(golden_inputs.GOLDEN, "golden.json")))
FULLSIZE = json.load(open(os.path.join(golden_inputs.GOLDEN, "fullsize.json")))
W4K, H4K = 3840, 2160


def test_device_synthesis_equals_host(gpu):
    import torch
    from lz4jpeg import synth
    for first, npix in [(0, 1), (0, 7936 * 3 + 5), (12345, 40000), (3 * W4K * H4K - 7, 100)]:
        d = torch.empty(4 * npix, dtype=torch.uint8, device=gpu)
        synth.rand_rgba_device(d, first, npix, seed=1)
        assert (d.cpu().numpy().reshape(-1, 4) == synth.rand_rgba_stream(first, npix, 1)).all()
    for first, total in [(0, 17), (0, 100_000), (29_990, 61_234), (7 * (1 << 33) + 5, 300_001)]:
        d = torch.empty(total + 16, dtype=torch.uint8, device=gpu)
        synth.random_passages_device(d, total, length=30000, seed=1, first=first)
        assert (d[:total].cpu().numpy() ==
                synth.random_passages(total, length=30000, seed=1, first=first)).all()


@pytest.mark.slow
def test_config4_rank7_shard(gpu, oracle):
    import torch
    from lz4jpeg import dist as ldist
    from lz4jpeg import lz4, synth
    n_total, world, rank = 64 << 30, 8, 7
    lo, hi = ldist.shard_bytes(n_total, world, rank)
    n = hi - lo
    nb = ldist.nblocks(n)
    assert nb > (1 << 24)                        # crosses the launch chunk
    assert n % 300 != 0                          # holds the short global last block
    d_in = torch.empty(n + 16, dtype=torch.uint8, device=gpu)
    synth.random_passages_device(d_in, n, length=30000, seed=1, first=lo)
    comp = lz4.Compressor()
    # the segment lands after one spare byte, so buffer[0:] is a framed stream
    buf = torch.empty(1 + lz4.compress_bound(n), dtype=torch.uint8, device=gpu)
    d_len = torch.zeros(1, dtype=torch.int64, device=gpu)
    comp.compress_async(d_in, n, buf[1:], d_len, segment=True, final_shard=True)
    torch.cuda.synchronize()
    seg = int(d_len.item())
    assert 0 < seg < lz4.compress_bound(n)
    offs = comp.block_offsets(nb).astype(np.int64)
    assert offs[0] == 0 and (np.diff(offs) >= 3).all() and offs[-1] < seg
    # EVERY byte of the segment against the oracle's md5 (fullsize.json), plus
    # spot blocks byte for byte on both sides of the launch chunk
    ref = FULLSIZE["config4_r7"]
    assert (lo, hi) == (ref["lo"], ref["hi"])
    ck = 1 << 24
    for b in (0, ck - 1, ck, nb - 1):
        blen = min(300, n - 300 * b)
        src = synth.random_passages(blen, length=30000, seed=1, first=lo + 300 * b)
        a = 1 + int(offs[b])
        e = 1 + (int(offs[b + 1]) if b + 1 < nb else seg)
        assert buf[a:e].cpu().numpy().tobytes() == oracle.lz4_blocks(src, 0, 1), b
    assert seg == ref["seg_len"]
    h = hashlib.md5()
    step = 1 << 30
    for a in range(1, 1 + seg, step):                 # host copies of <= 1 GiB at a time
        h.update(buf[a:min(1 + seg, a + step)].cpu().numpy().tobytes())
    assert h.hexdigest() == ref["md5"]
    # the whole segment decodes back to the shard (device offsets, no host hop)
    buf[0] = nb & 0xFF
    optr, cnt = comp.block_offsets_device()
    assert cnt == nb
    d_dec = torch.empty(n + 300, dtype=torch.uint8, device=gpu)
    _, got = lz4.decompress_device(buf, 1 + seg, optr, nb, n + 300, d_out=d_dec)
    assert got == n
    assert torch.equal(d_dec[:n], d_in[:n])
    comp.close()


def test_config5_stream_image0_is_the_reference_image(gpu):
    import torch
    from lz4jpeg import jpeg, synth
    e = [g for g in GOLDEN["jpeg"] if (g["w"], g["h"]) == (W4K, H4K)][0]
    d = torch.empty(4 * W4K * H4K, dtype=torch.uint8, device=gpu)
    synth.rand_rgba_device(d, 0, W4K * H4K, seed=1)
    out = jpeg.encode_device(d, W4K, H4K, 1)
    torch.cuda.synchronize()
    assert hashlib.md5(out.cpu().numpy().tobytes()).hexdigest() == e["md5"]


@pytest.mark.slow
def test_config5_rank7_images(gpu, oracle):
    """Images 896..1023 of the stream (rank 7 of 8) in one launch."""
    import torch
    from lz4jpeg import jpeg, synth
    first, count = 896, 128
    px = W4K * H4K
    d = torch.empty(4 * px * count, dtype=torch.uint8, device=gpu)
    synth.rand_rgba_device(d, first * px, px * count, seed=1)
    out = jpeg.encode_device(d, W4K, H4K, count)
    torch.cuda.synchronize()
    per = jpeg.coef_count(W4K, H4K)
    # EVERY coefficient of the 128 images against the oracle's md5 (fullsize.json)
    ref = FULLSIZE["config5_r7"]
    assert (ref["first_image"], ref["count"]) == (first, count)
    assert out.numel() * 2 == ref["bytes"]
    assert hashlib.md5(out.cpu().numpy().tobytes()).hexdigest() == ref["md5"]
    for k in (0, 127):
        img = synth.rand_rgba_stream((first + k) * px, px, 1).reshape(H4K, W4K, 4)
        got = out[k * per:(k + 1) * per]
        band = img[:32]                               # tile rows 0..3 byte for byte
        r = oracle.jpeg_encode(band)
        assert (got[:r.size].cpu().numpy() == r).all(), k
        # and the device-built image equals the host stream
        dimg = d[4 * px * k:4 * px * (k + 1)].view(H4K, W4K, 4)
        assert torch.equal(dimg[::97].cpu(), torch.from_numpy(img[::97].copy()))
