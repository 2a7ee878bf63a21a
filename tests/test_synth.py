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
