"""Seeded synthetic inputs with the reference generators' semantics.

rand_rgba        <- generate_noise_image  (Experiment/random_image.c:58-74)
random_passages  <- extract_random_passage(Experiment/random_extract.c:8-71),
                    repeated to any total size.
The corpus source text (Output-Input/input/Metamorphosis.txt, 118,489 B) is
committed as data under tests/golden/ so the GPU box never reads the
reference tree.
"""
import ctypes
import os

import numpy as np

from . import _lib

_REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
CORPUS_PATH = os.path.join(_REPO, "tests", "golden", "Metamorphosis.txt")


def corpus():
    with open(CORPUS_PATH, "rb") as f:
        return f.read()


def rand_rgba(w, h, seed=1):
    """(h, w, 4) uint8 from glibc rand() after srand(seed)."""
    out = np.empty((h, w, 4), dtype=np.uint8)
    _lib.lib().lz4jpeg_rand_rgba(seed, w, h, out.ctypes.data_as(ctypes.c_void_p))
    return out


def random_passages(total, length=30000, seed=1, first=0, src=None):
    """Bytes [first, first+total) of the seeded stream of random `length`-byte
    passages of the corpus (a rank can synthesise just its shard)."""
    src = corpus() if src is None else src
    s = np.frombuffer(src, dtype=np.uint8)
    out = np.empty(total, dtype=np.uint8)
    got = _lib.lib().lz4jpeg_random_passages(s.ctypes.data_as(ctypes.c_void_p), s.size, seed,
                                             length, first, total,
                                             out.ctypes.data_as(ctypes.c_void_p))
    if got != total:
        raise ValueError("random_passages: bad arguments")
    return out
