"""Seeded synthetic inputs with the reference generators' semantics.

rand_rgba        <- generate_noise_image  (Experiment/random_image.c:58-74)
rand_rgba_stream    the same rand() stream entered at any pixel: a batch of
                    images drawn from one continuous stream (config 5)
random_passages  <- extract_random_passage(Experiment/random_extract.c:8-71),
                    repeated to any total size.
*_device            the same bytes synthesised in HBM (csrc/synth_dev.hip), for
                    inputs too large to build on the host (configs 4 and 5).
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


def rand_rgba_stream(first_pixel, npix, seed=1):
    """(npix, 4) uint8: pixels [first_pixel, first_pixel + npix) of the
    rand() stream after srand(seed) (pixel i = outputs 3i, 3i+1, 3i+2)."""
    out = np.empty((npix, 4), dtype=np.uint8)
    _lib.lib().lz4jpeg_rand_rgba_stream(seed, first_pixel, npix,
                                        out.ctypes.data_as(ctypes.c_void_p))
    return out


def _stream_ptr(stream):
    import torch
    s = stream if stream is not None else torch.cuda.current_stream()
    return ctypes.c_void_p(s.cuda_stream)


def rand_rgba_device(d_out, first_pixel, npix, seed=1, stream=None):
    """Fill the uint8 CUDA tensor d_out (>= 4*npix bytes) with the pixels
    rand_rgba_stream(first_pixel, npix, seed) returns."""
    if d_out.numel() * d_out.element_size() < 4 * npix:
        raise ValueError("rand_rgba_device: output too small")
    rc = _lib.lib().lz4jpeg_rand_rgba_device(seed, first_pixel, npix,
                                             ctypes.c_void_p(d_out.data_ptr()),
                                             _stream_ptr(stream))
    if rc != 0:
        raise RuntimeError(f"lz4jpeg_rand_rgba_device: error {rc}")
    return d_out


def random_passages_device(d_out, total, length=30000, seed=1, first=0, src=None, stream=None):
    """Fill the first `total` bytes of the uint8 CUDA tensor d_out with
    random_passages(total, length, seed, first)."""
    src = corpus() if src is None else src
    s = np.frombuffer(src, dtype=np.uint8)
    if d_out.numel() < total:
        raise ValueError("random_passages_device: output too small")
    rc = _lib.lib().lz4jpeg_random_passages_device(s.ctypes.data_as(ctypes.c_void_p), s.size,
                                                   seed, length, first, total,
                                                   ctypes.c_void_p(d_out.data_ptr()),
                                                   _stream_ptr(stream))
    if rc != 0:
        raise RuntimeError(f"lz4jpeg_random_passages_device: error {rc}")
    return d_out
