"""ctypes view of oracle/liboracle.so (the CPU checker; tests only) and of the
reference's own JPEG.c built into oracle/_ref (present only where the
reference tree was available at build time)."""
import ctypes
import os

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE = os.path.join(REPO, "oracle", "liboracle.so")
REF_JPEG = os.path.join(REPO, "oracle", "_ref", "libref_jpeg.so")

_vp = ctypes.c_void_p
_sz = ctypes.c_size_t


class Oracle:
    def __init__(self, path=ORACLE):
        L = ctypes.CDLL(path)
        L.lz4o_compress.restype = _sz
        L.lz4o_compress.argtypes = [_vp, _sz, _vp]
        L.lz4o_encode_block.restype = _sz
        L.lz4o_encode_block.argtypes = [_vp, _sz, _vp]
        L.lz4o_encode_blocks.restype = _sz
        L.lz4o_encode_blocks.argtypes = [_vp, _sz, _sz, _sz, _vp]
        L.lz4o_encode_parallel.restype = _sz
        L.lz4o_encode_parallel.argtypes = [_vp, _sz, ctypes.c_int, _vp]
        L.lz4o_decompress.restype = _sz
        L.lz4o_decompress.argtypes = [_vp, _sz, _vp, _sz, _sz]
        L.lz4o_block_bound.restype = _sz
        for f in ("jo_encode_image", "jo_dct_raw_image"):
            getattr(L, f).argtypes = [_vp, ctypes.c_int, ctypes.c_int, _vp]
        L.jo_encode_image_parallel.argtypes = [_vp, ctypes.c_int, ctypes.c_int, ctypes.c_int, _vp]
        L.jo_rand_image.argtypes = [ctypes.c_uint, ctypes.c_int, ctypes.c_int, _vp]
        L.jo_planes.argtypes = [_vp, ctypes.c_int, ctypes.c_int, _vp, _vp, _vp]
        self.L = L

    # ---- LZ4 -------------------------------------------------------------
    def lz4_compress(self, data):
        b = np.frombuffer(bytes(data), dtype=np.uint8)
        out = np.empty(1 + ((b.size + 299) // 300) * self.L.lz4o_block_bound(), np.uint8)
        n = self.L.lz4o_compress(b.ctypes.data_as(_vp), b.size, out.ctypes.data_as(_vp))
        if n == ctypes.c_size_t(-1).value:
            raise ValueError("input shorter than one block")
        return out[:n].tobytes()

    def lz4_blocks(self, data, b0, b1):
        """Concatenated encoding of whole blocks [b0, b1) of `data` (no header)."""
        b = np.frombuffer(bytes(data), dtype=np.uint8) if not isinstance(data, np.ndarray) else data
        out = np.empty((b1 - b0) * self.L.lz4o_block_bound() + 16, np.uint8)
        n = self.L.lz4o_encode_blocks(b.ctypes.data_as(_vp), b.size, b0, b1,
                                      out.ctypes.data_as(_vp))
        return out[:n].tobytes()

    def lz4_decompress(self, comp, nblocks, cap):
        c = np.frombuffer(bytes(comp), dtype=np.uint8)
        out = np.empty(cap, np.uint8)
        n = self.L.lz4o_decompress(c.ctypes.data_as(_vp), c.size, out.ctypes.data_as(_vp),
                                   cap, nblocks)
        if n == ctypes.c_size_t(-1).value:
            raise ValueError("malformed stream")
        return out[:n].tobytes()

    # ---- JPEG ------------------------------------------------------------
    def jpeg_encode(self, rgba, threads=1):
        h, w = rgba.shape[:2]
        a = np.ascontiguousarray(rgba, dtype=np.uint8)
        out = np.empty(((w + 7) // 8) * ((h + 7) // 8) * 128, np.int16)
        if threads > 1:
            self.L.jo_encode_image_parallel(a.ctypes.data_as(_vp), w, h, threads,
                                            out.ctypes.data_as(_vp))
        else:
            self.L.jo_encode_image(a.ctypes.data_as(_vp), w, h, out.ctypes.data_as(_vp))
        return out

    def jpeg_dct_raw(self, rgba):
        h, w = rgba.shape[:2]
        a = np.ascontiguousarray(rgba, dtype=np.uint8)
        out = np.empty(((w + 7) // 8) * ((h + 7) // 8) * 128, np.float64)
        self.L.jo_dct_raw_image(a.ctypes.data_as(_vp), w, h, out.ctypes.data_as(_vp))
        return out

    def rand_image(self, w, h, seed=1):
        out = np.empty((h, w, 4), np.uint8)
        self.L.jo_rand_image(seed, w, h, out.ctypes.data_as(_vp))
        return out


def load():
    return Oracle()


def ref_jpeg():
    """The reference's own JPEG.c (compiled by oracle/Makefile), or None."""
    if not os.path.exists(REF_JPEG):
        return None
    L = ctypes.CDLL(REF_JPEG)
    L.ref_jpeg_encode_image.argtypes = [_vp, ctypes.c_int, ctypes.c_int, _vp]
    L.ref_jpeg_dct_raw.argtypes = [_vp, ctypes.c_int, ctypes.c_int, _vp]
    return L


def reconstruct(oracle, rgba):
    """Oracle restatement of reconstructed.png's pixels."""
    h, w = rgba.shape[:2]
    a = np.ascontiguousarray(rgba, dtype=np.uint8)
    out = np.empty((h, w, 4), np.uint8)
    oracle.L.jo_reconstruct_image.argtypes = [_vp, ctypes.c_int, ctypes.c_int, _vp]
    oracle.L.jo_reconstruct_image(a.ctypes.data_as(_vp), w, h, out.ctypes.data_as(_vp))
    return out


def ref_reconstruct(rgba):
    """The reference's own pipeline (JPEG.c main, via oracle/_ref), or None."""
    L = ref_jpeg()
    if L is None:
        return None
    h, w = rgba.shape[:2]
    a = np.ascontiguousarray(rgba, dtype=np.uint8)
    out = np.empty((h, w, 4), np.uint8)
    L.ref_jpeg_reconstruct.argtypes = [_vp, ctypes.c_int, ctypes.c_int, _vp]
    L.ref_jpeg_reconstruct(a.ctypes.data_as(_vp), w, h, out.ctypes.data_as(_vp))
    return out
