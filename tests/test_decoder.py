"""The product's host decoder (lz4r_decompress, host C in liblz4jpeg.so)
inverts every stream the reference format produces -- including the cases
the reference's own LZ4_decode gets wrong (>= 256 blocks, literal runs
>= 271, truncated match lengths 257..259 whose tokens are ambiguous).
Streams come from the pinned oracle, so this runs without a GPU."""
import numpy as np
import pytest

import golden_inputs
from lz4jpeg import lz4
from lz4jpeg._lib import Lz4Error


@pytest.mark.parametrize("name", golden_inputs.LZ4_EDGE_CASES + [
    "file:lz4_input.txt", "metamorphosis_spaces:76500", "file:Metamorphosis.txt"])
def test_roundtrip_named(oracle, name):
    data = golden_inputs.lz4_input(name)
    assert lz4.decompress(oracle.lz4_compress(data)) == data


def test_roundtrip_many_blocks_header_wraps(oracle):
    """> 256 blocks: the frame byte is nblocks & 0xFF (LZ4.c:429)."""
    data = golden_inputs.lz4_input("metamorphosis_spaces")     # 395 blocks
    comp = oracle.lz4_compress(data)
    assert comp[0] == 395 & 0xFF
    assert lz4.decompress(comp) == data


def test_roundtrip_seeded_fuzz(oracle):
    rng = np.random.default_rng(99)
    for k in range(60):
        n = int(rng.integers(300, 6000))
        kind = k % 4
        if kind == 0:
            b = rng.integers(0, 3, n, dtype=np.uint8).tobytes()
        elif kind == 1:
            motif = rng.integers(0, 256, int(rng.integers(1, 12)), dtype=np.uint8)
            b = np.resize(motif, n).tobytes()
        elif kind == 2:
            out = bytearray()
            while len(out) < n:
                out += bytes([int(rng.integers(0, 3))]) * int(rng.integers(1, 420))
            b = bytes(out[:n])
        else:
            b = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        assert lz4.decompress(oracle.lz4_compress(b)) == b, k


def test_ambiguous_tokens_present_and_resolved(oracle):
    """m_eq_1..3: a match of 257..259 is stored as M = 1..3 and its token
    reads 0xFD..0xFF, the same byte as (L >= 15, M = 17 / 18 / >= 19)."""
    for name, tok in (("m_eq_1", 0xFD), ("m_eq_2", 0xFE), ("m_eq_3", 0xFF)):
        data = golden_inputs.lz4_input(name)
        comp = oracle.lz4_compress(data)
        assert bytes([tok]) in comp
        assert lz4.decompress(comp) == data


def test_corrupt_streams_rejected(oracle):
    data = golden_inputs.lz4_input("text_10000")
    comp = bytearray(oracle.lz4_compress(data))
    with pytest.raises(Lz4Error):
        lz4.decompress(bytes(comp[:-3]))                # truncated
    bad = bytearray(comp)
    bad[0] ^= 0x01                                      # wrong block count byte
    with pytest.raises(Lz4Error):
        lz4.decompress(bytes(bad))
    with pytest.raises(Lz4Error):
        lz4.decompress(b"")


def test_block_size_field_checked(oracle):
    """The block header's u16 size (3 + sum of sequence size fields,
    LZ4.c:617) is validated."""
    data = golden_inputs.lz4_input("text_10000")
    comp = bytearray(oracle.lz4_compress(data))
    comp[2] ^= 0x40                                     # block 0's size field
    with pytest.raises(Lz4Error):
        lz4.decompress(bytes(comp))
