"""Synthetic-input generators follow the reference generators' semantics."""
import numpy as np

from lz4jpeg import synth


def test_rand_rgba_matches_oracle_stream(oracle):
    a = synth.rand_rgba(33, 17, seed=1)
    b = oracle.rand_image(33, 17, 1)
    assert (a == b).all()
    assert (a[..., 3] == 255).all()


def test_rand_rgba_seed1_first_pixel():
    # glibc: srand(1); rand() -> 1804289383, 846930886, 1681692777
    a = synth.rand_rgba(1, 1, seed=1)
    assert list(a[0, 0]) == [1804289383 % 256, 846930886 % 256, 1681692777 % 256, 255]


def test_random_passages_slices_are_consistent():
    whole = synth.random_passages(100_000, length=3000, seed=4)
    part = synth.random_passages(30_000, length=3000, seed=4, first=41_234)
    assert (whole[41_234:71_234] == part).all()
    assert not np.isin(whole, [10, 13]).any()      # newlines -> spaces


def test_random_passages_are_corpus_passages():
    src = synth.corpus().replace(b"\n", b" ").replace(b"\r", b" ")
    out = synth.random_passages(9000, length=3000, seed=2).tobytes()
    for k in range(3):
        assert out[3000 * k:3000 * (k + 1)] in src


def _libc():
    import ctypes
    libc = ctypes.CDLL(None)
    libc.srand.argtypes = [ctypes.c_uint]
    libc.rand.restype = ctypes.c_int
    return libc


def _libc_rand(seed, count, skip=0):
    libc = _libc()
    libc.srand(seed)
    for _ in range(skip):
        libc.rand()
    return [libc.rand() for _ in range(count)]


def test_restated_generator_equals_libc_rand():
    """host/synth.c restates glibc's TYPE_3 rand(); compare with libc itself."""
    for seed in (1, 2, 12345):
        r = _libc_rand(seed, 3 * 500)
        px = synth.rand_rgba(500, 1, seed=seed).reshape(-1, 4)
        assert [int(v) for v in px[:, :3].reshape(-1)] == [v % 256 for v in r]


def test_stream_entry_points_agree():
    """Jump-ahead (companion-matrix powers) == running the generator."""
    whole = synth.rand_rgba(700, 3, seed=1).reshape(-1, 4)
    for first in (0, 1, 30, 31, 100, 1033):
        part = synth.rand_rgba_stream(first, 64, seed=1)
        assert (part == whole[first:first + 64]).all()
    # far entry: check against libc at rand() index 3 * 20011
    r = _libc_rand(1, 6, skip=3 * 20011)
    part = synth.rand_rgba_stream(20011, 2, seed=1)
    assert [int(v) for v in part[:, :3].reshape(-1)] == [v % 256 for v in r]


def test_rand_states_match_stepping():
    import ctypes
    from lz4jpeg import _lib
    st = np.empty((3, 31), dtype=np.uint32)
    _lib.lib().lz4jpeg_rand_states(1, 5, 40, 3, st.ctypes.data_as(ctypes.c_void_p))
    # state before output k holds r[k+313 .. k+343]; its last word >> 1 is output k-1
    r = _libc_rand(1, 100)
    for c in range(3):
        k = 5 + 40 * c
        assert int(st[c, 30]) >> 1 == r[k - 1]
        assert [int(x) >> 1 for x in st[c, 28:31]] == r[k - 3:k]


def test_passage_starts_equal_libc():
    import ctypes
    from lz4jpeg import _lib
    src_len, length = 118489, 30000
    got = np.empty(7, dtype=np.uint32)
    _lib.lib().lz4jpeg_passage_starts(src_len, 1, length, 3, 7, got.ctypes.data_as(ctypes.c_void_p))
    r = _libc_rand(1, 10)
    assert [int(x) for x in got] == [v % (src_len - length) for v in r[3:10]]
