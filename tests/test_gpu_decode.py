"""GPU block-parallel LZ4 decoder (lz4r_decompress_device):
every stream the compressor writes -- golden, edge cases including the
ambiguous truncated-match tokens 0xFD..0xFF, literal runs >= 271 and > 256
blocks -- decodes back to the input byte for byte; at BASELINE.json's full
size (1 GiB) as a whole-stream round trip.  Malformed blocks are reported by
index.  Streams are the pinned oracle's (== the reference's compressed.bin),
so the decoder is checked independently of the GPU compressor too."""
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


def _offsets_of(oracle, data):
    """Per-block offsets (relative to the first block byte) from the oracle's
    per-block encodings, independent of the GPU compressor."""
    nb = (len(data) + 299) // 300
    sizes = [len(oracle.lz4_blocks(data, b, b + 1)) for b in range(nb)]
    return np.concatenate([[0], np.cumsum(sizes)[:-1]]).astype(np.int64)


def _gpu_decode(stream, offs, n_expected):
    import torch
    from lz4jpeg import lz4
    d_stream = torch.from_numpy(np.frombuffer(stream, dtype=np.uint8).copy()).cuda()
    d_offs = torch.from_numpy(np.asarray(offs, dtype=np.int64)).cuda()
    d_out, n = lz4.decompress_device(d_stream, len(stream), d_offs, len(offs),
                                     n_expected + 300)
    torch.cuda.synchronize()
    return d_out[:n].cpu().numpy().tobytes()


@pytest.mark.parametrize("name", golden_inputs.LZ4_EDGE_CASES + [
    "file:lz4_input.txt", "metamorphosis_spaces", "file:Metamorphosis.txt"])
def test_roundtrip_oracle_streams(gpu, oracle, name):
    data = golden_inputs.lz4_input(name)
    stream = oracle.lz4_compress(data)
    assert _gpu_decode(stream, _offsets_of(oracle, data), len(data)) == data


def test_ambiguous_tokens(gpu, oracle):
    for name, tok in (("m_eq_1", 0xFD), ("m_eq_2", 0xFE), ("m_eq_3", 0xFF)):
        data = golden_inputs.lz4_input(name)
        stream = oracle.lz4_compress(data)
        assert bytes([tok]) in stream
        assert _gpu_decode(stream, _offsets_of(oracle, data), len(data)) == data


def test_seeded_fuzz_via_gpu_compressor(comp):
    """Compressor offsets (lz4r_copy_block_offsets) feed the decoder directly."""
    import torch
    from lz4jpeg import lz4
    rng = np.random.default_rng(2024)
    for k in range(48):
        n = int(rng.integers(300, 30_000))
        kind = k % 4
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
        else:
            b = rng.integers(0, 256, n, dtype=np.uint8)
        d_in = torch.from_numpy(b.copy()).cuda()
        d_stream, length = comp.compress_device(d_in)
        nb = (n + 299) // 300
        d_offs = torch.from_numpy(comp.block_offsets(nb).astype(np.int64)).cuda()
        d_out, got = lz4.decompress_device(d_stream, length, d_offs, nb, n + 300)
        torch.cuda.synchronize()
        assert got == n, k
        assert torch.equal(d_out[:n], d_in), k


def test_corrupt_block_reported(gpu, oracle):
    from lz4jpeg import lz4
    data = golden_inputs.lz4_input("text_10000")
    stream = bytearray(oracle.lz4_compress(data))
    offs = _offsets_of(oracle, data)
    bad_block = 7
    p = 1 + int(offs[bad_block])
    stream[p + 1] ^= 0x40                      # first sequence's u16 size field
    with pytest.raises(lz4.Lz4Error) as ei:
        _gpu_decode(bytes(stream), offs, len(data))
    assert ei.value.code == -6
    assert f"block {bad_block}" in str(ei.value)


def test_truncated_stream_reported(gpu, oracle):
    from lz4jpeg import lz4
    data = golden_inputs.lz4_input("text_10000")
    stream = oracle.lz4_compress(data)
    with pytest.raises(lz4.Lz4Error):
        _gpu_decode(stream[:-2], _offsets_of(oracle, data), len(data))


@pytest.mark.slow
def test_full_size_1gib_roundtrip(comp):
    """BASELINE.json config 2 (1 GiB text): compress on the GPU, decode on the
    GPU, compare in HBM."""
    import torch
    from lz4jpeg import lz4, synth
    n = 1 << 30
    d_in = torch.from_numpy(synth.random_passages(n, length=30000, seed=1)).cuda()
    d_stream, length = comp.compress_device(d_in)
    nb = (n + 299) // 300
    d_offs = torch.from_numpy(comp.block_offsets(nb).astype(np.int64)).cuda()
    d_out, got = lz4.decompress_device(d_stream, length, d_offs, nb, n + 300)
    torch.cuda.synchronize()
    assert got == n
    assert torch.equal(d_out[:n], d_in)


def test_tight_capacity_and_mixed_inputs(comp):
    """Output buffers sized exactly to the decoded length (the last slot's
    8-byte accesses stay inside the capacity) over mixed inputs."""
    import torch
    from lz4jpeg import lz4
    rng = np.random.default_rng(5)
    parts = [golden_inputs.lz4_input("metamorphosis_spaces"),
             rng.integers(0, 256, 50_000, dtype=np.uint8).tobytes(),
             golden_inputs.lz4_input("m_eq_2"), golden_inputs.lz4_input("lit_270")]
    for data in parts:
        b = np.frombuffer(data, dtype=np.uint8)
        d_in = torch.from_numpy(b.copy()).cuda()
        d_stream, length = comp.compress_device(d_in)
        nb = (b.size + 299) // 300
        d_offs = torch.from_numpy(comp.block_offsets(nb).astype(np.int64)).cuda()
        d_out, got = lz4.decompress_device(d_stream, length, d_offs, nb, b.size)
        torch.cuda.synchronize()
        assert got == b.size
        assert torch.equal(d_out[:b.size], d_in)


def test_capacity_too_small_reported(comp):
    import torch
    from lz4jpeg import lz4
    data = golden_inputs.lz4_input("text_10000")
    b = np.frombuffer(data, dtype=np.uint8)
    d_in = torch.from_numpy(b.copy()).cuda()
    d_stream, length = comp.compress_device(d_in)
    nb = (b.size + 299) // 300
    d_offs = torch.from_numpy(comp.block_offsets(nb).astype(np.int64)).cuda()
    with pytest.raises(lz4.Lz4Error) as ei:
        lz4.decompress_device(d_stream, length, d_offs, nb, b.size - 1)
    assert ei.value.code == -3
