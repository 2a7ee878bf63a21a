"""The CPU oracle (oracle/liboracle.so) against every known answer the
reference provides, before any GPU result is trusted against it."""
import hashlib
import json
import os

import numpy as np
import pytest

import golden_inputs
import oracle_api

GOLDEN = json.load(open(os.path.join(golden_inputs.GOLDEN, "golden.json")))


def md5(b):
    return hashlib.md5(b).hexdigest()


@pytest.mark.parametrize("e", GOLDEN["lz4"], ids=lambda e: e["name"])
def test_lz4_oracle_golden(oracle, e):
    data = golden_inputs.lz4_input(e["input"])
    assert len(data) == e["in_len"]
    got = oracle.lz4_compress(data)
    assert len(got) == e["out_len"]
    assert md5(got) == e["md5"]


def test_lz4_committed_compressed_bin_bytes(oracle):
    """Byte-for-byte equal to the reference's committed Output-Input/out/compressed.bin."""
    data = golden_inputs.lz4_input("file:lz4_input.txt")
    ref = open(os.path.join(golden_inputs.GOLDEN, "lz4_input.compressed.bin"), "rb").read()
    assert oracle.lz4_compress(data) == ref


def test_lz4_committed_hex_dump(oracle):
    """The reference's committed Output-Input/out/compressed.txt is the "%02X "
    dump (LZ4.c:75-107) of its compressed.bin: pins the hex-dump format the
    executables write, byte for byte, to a file the reference itself produced."""
    data = open(os.path.join(golden_inputs.GOLDEN, "lz4_input.txt"), "rb").read()
    ref = open(os.path.join(golden_inputs.GOLDEN, "lz4_input.compressed.txt"), "rb").read()
    assert ref == "".join("%02X " % b for b in oracle.lz4_compress(data)).encode()


def test_lz4_too_small(oracle):
    with pytest.raises(ValueError):
        oracle.lz4_compress(b"x" * 299)


@pytest.mark.parametrize("name", ["metamorphosis_spaces", "text_10000", "random_bytes_3000",
                                  "alphabet2_3000", "lit_270", "lit_300", "a_x_600"])
def test_lz4_oracle_roundtrip(oracle, name):
    """decode(encode(x)) == x where the format is lossless (no uint8-truncated
    matches of length 257..259, whose token nibble overflows)."""
    data = golden_inputs.lz4_input(name)
    comp = oracle.lz4_compress(data)
    nb = (len(data) + 299) // 300
    assert oracle.lz4_decompress(comp, nb, nb * 300) == data


@pytest.mark.parametrize("e", [e for e in GOLDEN["jpeg"] if e["w"] * e["h"] <= 1920 * 1080],
                         ids=lambda e: f'{e["w"]}x{e["h"]}')
def test_jpeg_oracle_golden(oracle, e):
    img = oracle.rand_image(e["w"], e["h"], e["seed"])
    got = oracle.jpeg_encode(img, threads=8).tobytes()
    assert len(got) == e["bytes"]
    assert md5(got) == e["md5"]


def test_jpeg_oracle_kat_8x8(oracle):
    got = oracle.jpeg_encode(oracle.rand_image(8, 8, 1))
    kat = GOLDEN["jpeg_kat_8x8"]
    assert list(got[:64]) == kat["Y"]
    assert list(got[64:96]) == kat["Cr"]
    assert list(got[96:]) == kat["Cb"]


def test_jpeg_oracle_vs_reference_build(oracle):
    """Against the reference's own JPEG.c compiled from /root/reference
    (oracle/_ref, built only where the reference tree exists)."""
    ref = oracle_api.ref_jpeg()
    if ref is None:
        pytest.skip("oracle/_ref not built (no reference tree)")
    rng = np.random.default_rng(5)
    for (w, h) in [(8, 8), (16, 24), (40, 8), (64, 48), (120, 72), (200, 136)]:
        img = rng.integers(0, 256, (h, w, 4), dtype=np.uint8)
        mine = oracle.jpeg_encode(img)
        theirs = np.empty_like(mine)
        ref.ref_jpeg_encode_image(img.ctypes.data, w, h, theirs.ctypes.data)
        assert (mine == theirs).all(), (w, h)
        raw = oracle.jpeg_dct_raw(img)
        rraw = np.empty_like(raw)
        ref.ref_jpeg_dct_raw(img.ctypes.data, w, h, rraw.ctypes.data)
        assert raw.tobytes() == rraw.tobytes(), (w, h)


@pytest.mark.parametrize("w,h,seed", [(8, 8, 1), (64, 48, 2), (38, 21, 3), (2, 1, 4), (4, 4, 5),
                                      (120, 63, 6), (256, 256, 7), (1200, 630, 8)])
def test_reconstruction_oracle_matches_reference(oracle, w, h, seed):
    """jo_reconstruct_image == the reference's whole pipeline (JPEG.c main:
    DCT, Quantize, zigzag, RLE, Huffman round trip, inverse RLE, reverse
    zigzag, Inverse_quantize, IDCT, assemble_image), compiled from its
    sources.  Sizes that are not tile multiples exercise the ceil(W*H/64)
    block-count quirk (38x21: 15 tiles, 13 transformed).  Widths are even:
    for odd widths divide_image reads Cs[row][W/2], one past the
    malloc(W/2) row (JPEG.c:541-544, :316) -- undefined; we define it as 0."""
    ref = oracle_api.ref_reconstruct(oracle.rand_image(w, h, seed=seed))
    if ref is None:
        pytest.skip("reference not built")
    got = oracle_api.reconstruct(oracle, oracle.rand_image(w, h, seed=seed))
    assert np.array_equal(got, ref)


def test_many_sequences_input_covers_the_multi_round_path(oracle):
    """The edge case 'many_sequences' holds blocks of 64 and of more than 64
    sequences (the compressor's sequence rounds are 64 wide), checked here so
    the GPU golden test keeps covering that path."""
    import golden_inputs
    d = golden_inputs.lz4_input("many_sequences")
    counts = [oracle.lz4_blocks(d[300 * b:300 * b + 300], 0, 1)[0] for b in range(len(d) // 300)]
    assert 64 in counts and max(counts) > 64
