"""The reference-named functions of include/lz4jpeg_compat.h (GPU-backed)
give the reference's results: discrete_cosine_transform / Quantize /
zigzag_pattern against the oracle's per-tile values, lz4_encode / LZ4_decode
against the file contract."""
import ctypes
import os

import numpy as np
import pytest

import golden_inputs
from lz4jpeg import _lib

pytestmark = pytest.mark.gpu

ZZ8 = [0, 1, 8, 16, 9, 2, 3, 10, 17, 24, 32, 25, 18, 11, 4, 5, 12, 19, 26, 33, 40, 48, 41, 34,
       27, 20, 13, 6, 7, 14, 21, 28, 35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23, 30, 37,
       44, 51, 58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63]
ZZ4 = [0, 1, 4, 8, 5, 2, 3, 6, 9, 12, 16, 13, 10, 7, 11, 14, 17, 20, 24, 21, 18, 15, 19, 22,
       25, 28, 29, 26, 23, 27, 30, 31]
LUMA_Q = [8, 6, 6, 8, 10, 14, 18, 22, 6, 6, 7, 9, 12, 20, 22, 20, 6, 7, 8, 10, 14, 22, 25, 22,
          8, 9, 10, 14, 18, 28, 27, 22, 10, 12, 14, 18, 22, 35, 33, 26, 14, 18, 22, 22, 27, 33,
          36, 30, 18, 22, 26, 28, 33, 40, 40, 34, 22, 26, 28, 30, 36, 34, 35, 33]


def _dct(block_u8, width):
    L = _lib.lib()
    buf = np.ascontiguousarray(block_u8, dtype=np.uint8)
    out = ctypes.POINTER(ctypes.c_double)()
    L.discrete_cosine_transform(buf.ctypes.data_as(ctypes.c_void_p), width, 8, ctypes.byref(out))
    res = np.array([out[i] for i in range(8 * width)])
    ctypes.CDLL(None).free(out)
    return res


def test_dct_quant_zigzag_match_oracle(gpu, oracle):
    w, h = 16, 8
    img = oracle.rand_image(w, h, seed=11)
    raw = oracle.jpeg_dct_raw(img).reshape(-1, 128)          # per tile [Y64][Cr32][Cb32]
    coef = oracle.jpeg_encode(img).reshape(-1, 128)
    y = np.empty((h, w), np.uint8)
    cr = np.empty((h, w), np.uint8)
    cb = np.empty((h, w), np.uint8)
    oracle.L.jo_planes(np.ascontiguousarray(img).ctypes.data_as(ctypes.c_void_p), w, h,
                       y.ctypes.data_as(ctypes.c_void_p), cr.ctypes.data_as(ctypes.c_void_p),
                       cb.ctypes.data_as(ctypes.c_void_p))
    L = _lib.lib()
    for t in range(2):
        yblk = y[:, 8 * t:8 * t + 8]
        d = _dct(yblk, 8)
        assert np.array_equal(d.view(np.uint64), raw[t, :64].view(np.uint64))   # bit-exact
        crs = cr[:, 1::2][:, 4 * t:4 * t + 4]                 # odd columns (JPEG.c:329)
        dc = _dct(crs, 4)
        assert np.array_equal(dc.view(np.uint64), raw[t, 64:96].view(np.uint64))
        # Quantize (JPEG.c:621) then zigzag (JPEG.c:693) == the fused kernel's tile
        q = d.copy()
        qp = ctypes.cast(q.ctypes.data, ctypes.POINTER(ctypes.c_double))
        tab = np.array(LUMA_Q, dtype=np.uint64)
        L.Quantize(ctypes.byref(qp), tab.ctypes.data_as(ctypes.c_void_p), 64)
        assert np.array_equal(q, np.trunc(d / np.array(LUMA_Q, dtype=np.float64)))
        zz = np.empty(64)
        L.zigzag_pattern(8, 8, q.ctypes.data_as(ctypes.c_void_p), zz.ctypes.data_as(ctypes.c_void_p))
        assert np.array_equal(zz, q[ZZ8])
        assert np.array_equal(zz.astype(np.int16), coef[t, :64])
        z4 = np.empty(32)
        L.zigzag_pattern(4, 8, dc.ctypes.data_as(ctypes.c_void_p), z4.ctypes.data_as(ctypes.c_void_p))
        assert np.array_equal(z4, dc[ZZ4])


def test_lz4_encode_decode_file_contract(gpu, oracle, tmp_path, monkeypatch):
    for d in ("Experiment", "Output-Input/input", "Output-Input/out", "Output-Input/log"):
        os.makedirs(tmp_path / d, exist_ok=True)
    data = golden_inputs.lz4_input("text_10000")
    (tmp_path / "Output-Input/input/input.txt").write_bytes(data)
    monkeypatch.chdir(tmp_path / "Experiment")
    L = _lib.lib()
    L.lz4_encode()
    comp = (tmp_path / "Output-Input/out/compressed.bin").read_bytes()
    assert comp == oracle.lz4_compress(data)
    L.LZ4_decode(b"../Output-Input/out/compressed.bin", b"../Output-Input/log/encoding_log.txt")
    assert (tmp_path / "Output-Input/out/uncompressed.txt").read_bytes() == data


# ---- LZ4 per-block API: find_longest_match / block_encode / write_output ----
class LZ4Sequence(ctypes.Structure):          # LZ4.c:30-38
    _fields_ = [("token", ctypes.c_uint8), ("byte_size", ctypes.c_size_t),
                ("literals", ctypes.c_void_p), ("literals_count", ctypes.c_size_t),
                ("match_offset", ctypes.c_uint16), ("match_length", ctypes.c_size_t)]


class LZ4Block(ctypes.Structure):             # LZ4.c:40-46
    _fields_ = [("token", ctypes.c_uint8), ("byte_size", ctypes.c_size_t),
                ("sequences_count", ctypes.c_size_t),
                ("sequences", ctypes.POINTER(LZ4Sequence))]


class LZ4Frame(ctypes.Structure):             # LZ4.c:48-52
    _fields_ = [("blocks", ctypes.c_size_t), ("frame_blocks", ctypes.POINTER(LZ4Block))]


def _libc():
    c = ctypes.CDLL(None)
    c.fopen.restype = ctypes.c_void_p
    c.fopen.argtypes = [ctypes.c_char_p, ctypes.c_char_p]
    c.fclose.argtypes = [ctypes.c_void_p]
    return c


def _reference_loop(data, path):
    """lz4_encode's block loop (LZ4.c:707-721) + write_output (:427-441),
    through the C ABI."""
    L = _lib.lib()
    buf = ctypes.create_string_buffer(bytes(data), len(data))
    frame = LZ4Frame(0, None)
    nb = (len(data) + 299) // 300
    blocks = []
    for i in range(nb):
        blk = LZ4Block()
        n = min(300, len(data) - 300 * i)
        L.block_encode(ctypes.addressof(buf) + 300 * i, n, ctypes.byref(blk), None, None,
                       ctypes.byref(frame))
        blocks.append((blk.token, blk.byte_size, blk.sequences_count))
    assert frame.blocks == nb
    c = _libc()
    f = c.fopen(str(path).encode(), b"wb")
    L.write_output(ctypes.byref(frame), f)
    c.fclose(f)
    assert frame.blocks == 0
    return open(path, "rb").read(), blocks


@pytest.mark.parametrize("name", ["file:lz4_input.txt", "text_10000", "metamorphosis_spaces",
                                  "m_eq_1", "m_eq_2", "m_eq_3", "len_256", "lit_270", "lit_300",
                                  "text_last_block_1", "zeros_900", "alphabet2_3000"])
def test_block_encode_and_write_output_equal_the_oracle(gpu, oracle, tmp_path, name):
    data = golden_inputs.lz4_input(name)
    got, blocks = _reference_loop(data, tmp_path / "c.bin")
    assert got == oracle.lz4_compress(data)
    # the committed golden pair, byte for byte
    if name == "file:lz4_input.txt":
        ref = open(os.path.join(golden_inputs.GOLDEN, "lz4_input.compressed.bin"), "rb").read()
        assert got == ref


def test_find_longest_match_every_position(gpu, oracle):
    """find_longest_match at every position of a 300-B block (the standalone
    form: the 300 bytes at `input`) against a direct restatement of
    LZ4.c:290-323 with the block-end clamp."""
    L = _lib.lib()
    rng = np.random.default_rng(5)
    text = golden_inputs.lz4_input("metamorphosis_spaces")
    for trial in range(4):
        if trial < 2:
            blk = text[300 * (7 + trial):300 * (8 + trial)]
        else:
            blk = bytes(rng.integers(97, 100, 300, dtype=np.uint8))   # {a,b,c}: long matches
        buf = ctypes.create_string_buffer(blk, 300)
        for p in range(300):
            best, bd = 0, 0
            for i in range(p):
                l = 0
                while p + l < 300 and l < 1024 and blk[i + l] == blk[p + l]:
                    l += 1
                if l > best:
                    best, bd = l, p - i
            d = ctypes.c_uint16(0)
            m = L.find_longest_match(ctypes.addressof(buf), p, ctypes.byref(d))
            if best >= 4:
                assert (m, d.value) == (best & 0xFF, bd), (trial, p)
            else:
                assert m == 0, (trial, p)


def _oracle_block(oracle, data):
    """[u8 1] + the oracle's block_encode/write_block bytes of one block of
    any length (lz4o_encode_block: the 65535-byte window, MAX_MATCH 1024)."""
    out = ctypes.create_string_buffer(3 * len(data) + 64)
    n = oracle.L.lz4o_encode_block(bytes(data), len(data), out)
    return b"\x01" + out.raw[:n]


@pytest.mark.parametrize("n", [301, 1000, 5000, 70000])
def test_block_encode_longer_than_300(gpu, oracle, tmp_path, n):
    """block_encode accepts any block_length (LZ4.c:506; the reference's
    window is 65535 bytes, LZ4.c:22/295): blocks past 300 B take the
    whole-window GPU match finder; 70,000 B crosses the window."""
    text = golden_inputs.lz4_input("metamorphosis_spaces")
    data = (text * (n // len(text) + 1))[:n]      # repeats the book: long matches
    L = _lib.lib()
    buf = ctypes.create_string_buffer(bytes(data), n)
    frame = LZ4Frame(0, None)
    blk = LZ4Block()
    L.block_encode(ctypes.addressof(buf), n, ctypes.byref(blk), None, None, ctypes.byref(frame))
    c = _libc()
    path = tmp_path / "long.bin"
    f = c.fopen(str(path).encode(), b"wb")
    L.write_output(ctypes.byref(frame), f)
    c.fclose(f)
    assert path.read_bytes() == _oracle_block(oracle, data)


def test_find_longest_match_standalone_short_block_then_long(gpu, oracle):
    """The per-thread cache grows: a 300-B standalone call, then a 2,000-B
    block_encode, then a 300-B block again (each answered for its own
    bytes)."""
    L = _lib.lib()
    text = golden_inputs.lz4_input("metamorphosis_spaces")
    a = ctypes.create_string_buffer(text[:300], 300)
    d = ctypes.c_uint16(0)
    first = [(L.find_longest_match(ctypes.addressof(a), p, ctypes.byref(d)), d.value)
             for p in range(300)]
    long_ = (text * 2)[:2000]
    b = ctypes.create_string_buffer(long_, 2000)
    frame = LZ4Frame(0, None)
    blk = LZ4Block()
    L.block_encode(ctypes.addressof(b), 2000, ctypes.byref(blk), None, None, ctypes.byref(frame))
    assert frame.blocks == 1
    again = [(L.find_longest_match(ctypes.addressof(a), p, ctypes.byref(d)), d.value)
             for p in range(300)]
    assert [m for m, _ in again] == [m for m, _ in first]
    assert [dd for m, dd in again if m] == [dd for m, dd in first if m]
