"""lz4jpeg -- MI355X-native LZ4 / JPEG hot paths of CyrilMorel42/LZ4-JPEG.

Python host mirror over the C ABI in include/ (liblz4jpeg.so, hand-written
HIP kernels for gfx950).  Import path: add `lz4-jpeg_amd/` to sys.path (the
repository's package directory name is not a Python identifier).

  lz4jpeg.lz4    compress / Compressor      (LZ4.c lz4_encode, block_encode)
  lz4jpeg.jpeg   encode / encode_device     (JPEG.c DCT + Quantize + zigzag)
  lz4jpeg.dist   shard_blocks / compress_sharded (one process per GPU, RCCL)
  lz4jpeg.synth  rand_rgba / random_passages (random_image.c, random_extract.c)
"""
from . import _lib  # noqa: F401
from ._lib import LIB_PATH, LibraryMissing, lib  # noqa: F401

__all__ = ["lz4", "jpeg", "synth", "dist", "lib", "LIB_PATH", "LibraryMissing"]
