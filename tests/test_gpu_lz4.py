"""HIP LZ4 path vs the pinned CPU oracle: bit-exact on golden vectors, edge
cases and seeded fuzz; at BASELINE.json's full size (1 GiB) every byte of
the stream against the oracle's md5 (tests/golden/fullsize.json) and a
decode round trip.  All calls go through the C ABI."""
import hashlib
import json
import os

import numpy as np
import pytest

import golden_inputs

pytestmark = pytest.mark.gpu

GOLDEN = json.load(open(os.path.join(golden_inputs.GOLDEN, "golden.json")))


@pytest.fixture(scope="module")
def comp(gpu):
    from lz4jpeg.lz4 import Compressor
    c = Compressor()
    yield c
    c.close()


def _gpu_compress(comp, data):
    import torch
    d_in = torch.from_numpy(np.frombuffer(bytes(data), dtype=np.uint8).copy()).cuda()
    d_out, n = comp.compress_device(d_in)
    torch.cuda.synchronize()
    return d_out[:n].cpu().numpy().tobytes()


@pytest.mark.parametrize("e", GOLDEN["lz4"], ids=lambda e: e["name"])
def test_golden(comp, e):
    data = golden_inputs.lz4_input(e["input"])
    got = _gpu_compress(comp, data)
    assert len(got) == e["out_len"]
    assert hashlib.md5(got).hexdigest() == e["md5"]


def test_committed_compressed_bin(comp):
    data = golden_inputs.lz4_input("file:lz4_input.txt")
    ref = open(os.path.join(golden_inputs.GOLDEN, "lz4_input.compressed.bin"), "rb").read()
    assert _gpu_compress(comp, data) == ref


def test_host_api_matches(comp, oracle):
    from lz4jpeg import lz4
    data = golden_inputs.lz4_input("text_10000")
    assert lz4.compress(data) == oracle.lz4_compress(data)
    assert comp.compress(data) == oracle.lz4_compress(data)


def test_too_small_raises(comp):
    from lz4jpeg import lz4
    with pytest.raises(lz4.InputTooSmall):
        lz4.compress(b"x" * 299)


def _fuzz_inputs():
    rng = np.random.default_rng(1234)
    text = golden_inputs.lz4_input("metamorphosis_spaces")
    cases = []
    for k in range(40):
        n = int(rng.integers(300, 40_000))
        kind = k % 5
        if kind == 0:
            s = int(rng.integers(0, len(text) - n))
            b = text[s:s + n]
        elif kind == 1:
            b = rng.integers(0, int(rng.integers(2, 8)), n, dtype=np.uint8).tobytes()
        elif kind == 2:
            b = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        elif kind == 3:  # repeated short motifs with noise
            motif = rng.integers(0, 256, int(rng.integers(1, 40)), dtype=np.uint8)
            b = np.resize(motif, n)
            flips = rng.integers(0, n, n // 50)
            b[flips] = rng.integers(0, 256, flips.size, dtype=np.uint8)
            b = b.tobytes()
        else:  # runs of one byte of random lengths (uint8 truncation region)
            out = bytearray()
            while len(out) < n:
                out += bytes([int(rng.integers(0, 4))]) * int(rng.integers(1, 400))
            b = bytes(out[:n])
        cases.append(b)
    return cases


@pytest.mark.parametrize("idx", range(40))
def test_fuzz_vs_oracle(comp, oracle, idx):
    data = _fuzz_inputs()[idx]
    assert _gpu_compress(comp, data) == oracle.lz4_compress(data)


@pytest.mark.parametrize("n", [301, 308, 300 * 2 + 4, 300 * 77 + 20, 300 * 5 + 24])
def test_input_ending_at_allocation_end(comp, oracle, n):
    """A last block of 1..23 bytes: the block before it must not read its
    24 bytes past its own end (the unstaged 4-gram loads) beyond the input.
    The input sits at the very end of its own hipMalloc allocation (raw, not
    torch's caching allocator), 4-byte aligned when n is (the unstaged path);
    with the over-read those loads would leave the allocation."""
    import ctypes
    import torch
    from lz4jpeg import _lib
    from lz4jpeg.lz4 import compress_bound
    torch.cuda.init()
    hip = ctypes.CDLL("libamdhip64.so")
    text = golden_inputs.lz4_input("metamorphosis_spaces")
    data = bytes(text[1000:1000 + n])
    size = 64 << 10                                 # a page multiple
    p = ctypes.c_void_p()
    assert hip.hipMalloc(ctypes.byref(p), ctypes.c_size_t(size)) == 0
    try:
        src = ctypes.c_void_p(p.value + size - n)   # the input ends at the allocation end
        assert hip.hipMemcpy(src, data, ctypes.c_size_t(n), 1) == 0   # host -> device
        d_out = torch.empty(compress_bound(n), dtype=torch.uint8, device="cuda")
        got = ctypes.c_size_t(0)
        torch.cuda.synchronize()
        rc = _lib.lib().lz4r_compress_device(comp._h, src, n, ctypes.c_void_p(d_out.data_ptr()),
                                             d_out.numel(), ctypes.byref(got), None)
        assert rc == 0
        assert d_out[:got.value].cpu().numpy().tobytes() == oracle.lz4_compress(data)
    finally:
        hip.hipFree(p)


def test_check_reads_the_contexts_own_verdict(comp):
    """lz4r_check after an async call whose length buffer is already freed:
    it reads a word the context owns, not the caller's buffer,
    and an empty segment (no launch) reports OK."""
    import torch
    from lz4jpeg.lz4 import compress_bound
    data = golden_inputs.lz4_input("text_10000")
    d_in = torch.from_numpy(np.frombuffer(bytes(data), dtype=np.uint8).copy()).cuda()
    d_out = torch.empty(compress_bound(len(data)), dtype=torch.uint8, device="cuda")
    d_len = torch.zeros(1, dtype=torch.int64, device="cuda")
    comp.compress_async(d_in, len(data), d_out, d_len)
    del d_len
    torch.cuda.empty_cache()
    junk = torch.full((1 << 20,), -1, dtype=torch.int64, device="cuda")   # reuse the memory
    comp.check()
    del junk
    d_len = torch.zeros(1, dtype=torch.int64, device="cuda")
    comp.compress_async(d_in, 0, d_out, d_len, segment=True, final_shard=True)
    comp.check()
    assert comp.async_length(d_len) == 0


def test_timed_back_to_back_async_calls(comp, oracle):
    """Timing of stream-ordered async calls (the bench's N = 1 step): every
    call has its own events, read after the last one; an empty segment is a
    timed call of no launches; the last call's output equals the oracle's."""
    import torch
    from lz4jpeg.lz4 import compress_bound
    data = golden_inputs.lz4_input("metamorphosis_spaces") * 40
    d_in = torch.from_numpy(np.frombuffer(bytes(data), dtype=np.uint8).copy()).cuda()
    d_out = torch.empty(compress_bound(len(data)), dtype=torch.uint8, device="cuda")
    d_len = torch.zeros(1, dtype=torch.int64, device="cuda")
    comp.set_timing(True)
    try:
        for _ in range(7):
            comp.compress_async(d_in, len(data), d_out, d_len)
        calls, tiles = comp.timed_calls()
        assert len(calls) == 7 and all(0 < t <= c for c, t in zip(calls, tiles))
        assert comp.timed_calls(3)[0] == calls[-3:]
        comp.compress_async(d_in, 0, d_out, d_len, segment=True, final_shard=True)
        calls, tiles = comp.timed_calls()
        assert len(calls) == 8 and tiles[-1] == 0.0
        comp.set_timing(True)                       # a new record
        comp.compress_async(d_in, len(data), d_out, d_len)
        assert len(comp.timed_calls()[0]) == 1
        n = comp.async_length(d_len)
    finally:
        comp.set_timing(False)
    assert d_out[:n].cpu().numpy().tobytes() == oracle.lz4_compress(bytes(data))


def test_segments_concatenate_to_stream(comp, oracle):
    """Shard outputs (lz4r_compress_segment_async) + header byte == framed stream."""
    import torch
    from lz4jpeg import dist as ldist
    data = golden_inputs.lz4_input("metamorphosis_spaces")
    n = len(data)
    nb = ldist.nblocks(n)
    parts = []
    for r in range(3):
        lo, hi = ldist.shard_bytes(n, 3, r)
        d_in = torch.from_numpy(np.frombuffer(data[lo:hi], dtype=np.uint8).copy()).cuda()
        out = torch.empty(1 + ldist.nblocks(hi - lo) * 1152, dtype=torch.uint8, device="cuda")
        d_len = torch.zeros(1, dtype=torch.int64, device="cuda")
        comp.compress_async(d_in, hi - lo, out, d_len, segment=True, final_shard=(r == 2))
        torch.cuda.synchronize()
        parts.append(out[:int(d_len.item())].cpu().numpy().tobytes())
    assert bytes([nb & 0xFF]) + b"".join(parts) == oracle.lz4_compress(data)


def test_segment_contract_rejects_misaligned_nonfinal_shard(comp):
    """Only the globally last shard may end in a short block (lz4r.h)."""
    import torch
    from lz4jpeg import lz4
    d_in = torch.zeros(1000, dtype=torch.uint8, device="cuda")
    out = torch.empty(4096, dtype=torch.uint8, device="cuda")
    d_len = torch.zeros(1, dtype=torch.int64, device="cuda")
    with pytest.raises(lz4.Lz4Error) as ei:
        comp.compress_async(d_in, 1000, out, d_len, segment=True, final_shard=False)
    assert ei.value.code == -1
    comp.compress_async(d_in, 900, out, d_len, segment=True, final_shard=False)
    comp.compress_async(d_in, 1000, out, d_len, segment=True, final_shard=True)
    d_len.fill_(123)
    comp.compress_async(d_in, 0, out, d_len, segment=True, final_shard=True)   # empty shard
    torch.cuda.synchronize()
    assert int(d_len.item()) == 0


def test_device_block_offsets_delimit_every_block(comp, oracle):
    """The placement kernel's device offsets (lz4r_block_offsets_device) cut
    the stream into exactly the oracle's per-block bytes."""
    import torch
    data = golden_inputs.lz4_input("metamorphosis_spaces")
    d_in = torch.from_numpy(np.frombuffer(data, dtype=np.uint8).copy()).cuda()
    d_out, length = comp.compress_device(d_in)
    nb = (len(data) + 299) // 300
    ptr, cnt = comp.block_offsets_device()
    assert cnt == nb and ptr
    offs = comp.block_offsets(nb).astype(np.int64)
    stream = d_out[:length].cpu().numpy().tobytes()
    ends = list(offs[1:]) + [length - 1]
    buf = np.frombuffer(data, dtype=np.uint8)
    for b in range(nb):
        assert stream[1 + offs[b]:1 + ends[b]] == oracle.lz4_blocks(buf, b, b + 1), b


def test_capacity_error_reports_need(comp):
    import torch
    from lz4jpeg import lz4
    data = golden_inputs.lz4_input("text_10000")
    d_in = torch.from_numpy(np.frombuffer(data, dtype=np.uint8).copy()).cuda()
    small = torch.zeros(100, dtype=torch.uint8, device="cuda")
    with pytest.raises(lz4.Lz4Error) as ei:
        comp.compress_device(d_in, d_out=small)
    assert ei.value.code == -3
    assert small.cpu().numpy().any()            # bytes up to cap were written


@pytest.mark.slow
def test_full_size_1gib_whole_stream_md5_and_roundtrip(comp, oracle):
    """BASELINE.json config 2: 1 GiB random_extract-style text.  EVERY byte of
    the framed stream (the reference's block loop LZ4.c:707-721 over all
    3,579,140 blocks + write_output) against the oracle's md5
    (tests/golden/fullsize.json, make_fullsize.py), spot blocks compared
    byte for byte for a readable failure, and the whole stream decodes back
    to the input."""
    import hashlib
    import json
    import torch
    from lz4jpeg import synth
    ref = json.load(open(os.path.join(golden_inputs.GOLDEN, "fullsize.json")))["config2"]
    n = ref["n"]
    data = synth.random_passages(n, length=ref["passage"], seed=ref["seed"])
    d_in = torch.from_numpy(data).cuda()
    d_out, length = comp.compress_device(d_in)
    torch.cuda.synchronize()
    nb = (n + 299) // 300
    stream = d_out[:length].cpu().numpy()
    assert stream[0] == nb & 0xFF
    offs = comp.block_offsets(nb)
    for b in (0, 1, nb // 2, nb - 1):
        lo = 1 + int(offs[b])
        hi = 1 + int(offs[b + 1]) if b + 1 < nb else length
        assert stream[lo:hi].tobytes() == oracle.lz4_blocks(data, b, b + 1), b
    assert length == ref["out_len"]
    assert hashlib.md5(stream.tobytes()).hexdigest() == ref["md5"]
    dec = oracle.lz4_decompress(stream.tobytes(), nb, n + 300)
    assert len(dec) == n
    assert dec == data.tobytes()
