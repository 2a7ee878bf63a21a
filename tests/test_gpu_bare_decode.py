"""GPU decode of a bare framed stream (lz4r_decompress_stream[_device]): the
block boundaries are found on the device from the stream alone, as the
reference's LZ4_decode (Algorithms/sequential/LZ4/LZ4.c:1038) takes only the
file.  Every stream here is decoded with no side information and compared
with the input byte for byte: the pinned oracle's streams (== the reference's
compressed.bin format) including the truncated-match blocks whose size
fields over-count (LZ4.c:569-575, the exact second pass), seeded fuzz through
the GPU compressor across many 4 KiB chunk boundaries, >= 256 blocks, and the
1 GiB bench corpus.  Structural corruption is an error, never a fault."""
import numpy as np
import pytest

import golden_inputs

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def comp(gpu):
    from lz4jpeg.lz4 import Compressor
    c = Compressor()
    yield c
    c.close()


@pytest.mark.parametrize("name", golden_inputs.LZ4_EDGE_CASES + [
    "file:lz4_input.txt", "metamorphosis_spaces", "file:Metamorphosis.txt"])
def test_bare_roundtrip_oracle_streams(gpu, oracle, name):
    from lz4jpeg import lz4
    data = golden_inputs.lz4_input(name)
    stream = oracle.lz4_compress(data)
    assert lz4.decompress_stream(stream) == data


def test_bare_committed_compressed_bin(gpu):
    """The reference's own Output-Input/out/compressed.bin (committed fixture)."""
    from lz4jpeg import lz4
    stream = golden_inputs.lz4_input("file:lz4_input.compressed.bin")
    assert lz4.decompress_stream(stream) == golden_inputs.lz4_input("file:lz4_input.txt")


def test_bare_truncated_match_streams(gpu, oracle):
    """Blocks holding M = 1..3 (tokens 0xFD..0xFF read as truncated matches),
    concatenated with text so that their over-counting size fields sit in the
    middle of a long chain of chunks."""
    from lz4jpeg import lz4
    text = golden_inputs.lz4_input("metamorphosis_spaces")[:60_000]
    for name in ("m_eq_1", "m_eq_2", "m_eq_3"):
        mid = golden_inputs.lz4_input(name)
        pad = (-len(text)) % 300
        data = text + b" " * pad + mid + text
        stream = oracle.lz4_compress(data)
        assert lz4.decompress_stream(stream) == data, name


def test_bare_seeded_fuzz_via_gpu_compressor(comp):
    import torch
    from lz4jpeg import lz4
    rng = np.random.default_rng(77)
    for k in range(40):
        n = int(rng.integers(300, 400_000))
        kind = k % 5
        if kind == 0:
            b = rng.integers(0, 3, n, dtype=np.uint8)
        elif kind == 1:
            motif = rng.integers(0, 256, int(rng.integers(1, 12)), dtype=np.uint8)
            b = np.resize(motif, n)
        elif kind == 2:
            out = bytearray()
            while len(out) < n:
                out += bytes([int(rng.integers(0, 3))]) * int(rng.integers(1, 420))
            b = np.frombuffer(bytes(out[:n]), dtype=np.uint8)
        elif kind == 3:
            b = rng.integers(0, 256, n, dtype=np.uint8)
        else:
            t = np.frombuffer(golden_inputs.lz4_input("metamorphosis_spaces"), dtype=np.uint8)
            o = int(rng.integers(0, t.size - 1))
            b = np.resize(np.roll(t, -o), n)
        d_in = torch.from_numpy(b.copy()).cuda()
        d_stream, length = comp.compress_device(d_in)
        d_out, got = lz4.decompress_stream_device(d_stream, length, n + 300)
        torch.cuda.synchronize()
        assert got == n, k
        assert torch.equal(d_out[:n], d_in), k


def test_bare_many_blocks_and_tight_capacity(comp):
    """> 256 blocks (the frame byte wraps) and an output buffer of exactly the
    decoded length; one byte less is a capacity error naming the need."""
    import torch
    from lz4jpeg import lz4
    data = golden_inputs.lz4_input("file:Metamorphosis.txt")
    b = np.frombuffer(data, dtype=np.uint8)
    d_in = torch.from_numpy(b.copy()).cuda()
    d_stream, length = comp.compress_device(d_in)
    d_out, got = lz4.decompress_stream_device(d_stream, length, b.size)
    assert got == b.size and torch.equal(d_out[:b.size], d_in)
    with pytest.raises(lz4.Lz4Error) as ei:
        lz4.decompress_stream_device(d_stream, length, b.size - 1)
    assert ei.value.code == -3


def test_bare_output_capacity_paths(comp):
    """An output buffer that cannot hold the stream's block count is a
    capacity error before anything is decoded (the device-side gate); one far
    larger than the stream could decode to takes the path that reads the
    block count back first, and decodes the same bytes."""
    import torch
    from lz4jpeg import lz4
    data = golden_inputs.lz4_input("file:Metamorphosis.txt")
    b = np.frombuffer(data, dtype=np.uint8)
    d_in = torch.from_numpy(b.copy()).cuda()
    d_stream, length = comp.compress_device(d_in)
    for cap in (1, 299, 301, 3000):
        with pytest.raises(lz4.Lz4Error) as ei:
            lz4.decompress_stream_device(d_stream, length, cap)
        assert ei.value.code == -3, cap
    big = 300 * (length // 8 + 8)
    d_out, got = lz4.decompress_stream_device(d_stream, length, big)
    assert got == b.size and torch.equal(d_out[:b.size], d_in)


def test_bare_structural_corruption_reported(gpu, oracle):
    from lz4jpeg import lz4
    data = golden_inputs.lz4_input("metamorphosis_spaces")[:50_000]
    stream = oracle.lz4_compress(data)
    cases = {
        "truncated": stream[:-2],
        "frame byte": bytes([stream[0] ^ 1]) + stream[1:],
        "short": stream[:5],
    }
    bad = bytearray(stream)
    bad[1 + 1] ^= 0x40                         # block 0's u16 size field
    cases["block 0 size"] = bytes(bad)
    bad = bytearray(stream)
    bad[len(stream) // 2] = 0xFF               # a byte in the middle (structure or literal)
    for what, s in cases.items():
        with pytest.raises(lz4.Lz4Error) as ei:
            lz4.decompress_stream(s)
        assert ei.value.code == -6, what
    # a mid-stream byte change either decodes (a literal) or is reported
    try:
        out = lz4.decompress_stream(bytes(bad))
        assert len(out) == len(data)
    except lz4.Lz4Error as e:
        assert e.code == -6


@pytest.mark.slow
def test_bare_full_size_1gib_roundtrip(comp):
    """BASELINE.json config 2: 1 GiB of text compressed on the GPU and decoded
    from the stream alone on the GPU."""
    import torch
    from lz4jpeg import lz4, synth
    n = 1 << 30
    d_in = torch.empty(n + 16, dtype=torch.uint8, device="cuda")
    synth.random_passages_device(d_in, n, length=30000, seed=1)
    d_stream, length = comp.compress_device(d_in[:n])
    d_out, got = lz4.decompress_stream_device(d_stream, length, n + 300)
    torch.cuda.synchronize()
    assert got == n
    assert torch.equal(d_out[:n], d_in[:n])
