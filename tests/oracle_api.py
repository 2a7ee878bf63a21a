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


def _entropy_call(fn, zz, with_decoded):
    """Shared marshalling of jo_entropy_stream / ref_jpeg_entropy."""
    zz = np.ascontiguousarray(zz, dtype=np.int16)
    n = zz.size
    rle = np.zeros(256, np.int32)
    rle_len, ncodes, nbits = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
    tv = np.zeros(256, np.int16)
    tl = np.zeros(256, np.uint8)
    tc = np.zeros(256, np.uint64)
    bits = np.zeros(2048, np.uint8)
    dec = np.zeros(64, np.int16)
    args = [zz.ctypes.data_as(_vp), n, rle.ctypes.data_as(_vp), ctypes.byref(rle_len),
            ctypes.byref(ncodes), tv.ctypes.data_as(_vp), tl.ctypes.data_as(_vp),
            tc.ctypes.data_as(_vp), bits.ctypes.data_as(_vp)]
    if with_decoded:
        rc = fn(*args, ctypes.byref(nbits), dec.ctypes.data_as(_vp))
    else:
        rc = fn(*args, 16384, ctypes.byref(nbits))
    k = ncodes.value
    out = {"rc": rc, "rle": rle[:rle_len.value].tolist(),
           "table": list(zip(tv[:k].tolist(), tl[:k].tolist(), tc[:k].tolist())),
           "nbits": nbits.value, "bits": bits[:(nbits.value + 7) // 8].tobytes()}
    if with_decoded:
        out["decoded"] = dec[:n].tolist()
    return out


def entropy(oracle, zz):
    """Oracle restatement of the entropy stage for one stream."""
    fn = oracle.L.jo_entropy_stream
    fn.argtypes = [_vp, ctypes.c_int, _vp, _vp, _vp, _vp, _vp, _vp, _vp, ctypes.c_int, _vp]
    return _entropy_call(fn, zz, False)


def entropy_decode(oracle, e, n):
    """Oracle decode of an entropy record back to n ints."""
    fn = oracle.L.jo_entropy_decode
    fn.argtypes = [_vp, ctypes.c_int, ctypes.c_int, ctypes.c_int, _vp, _vp, _vp, ctypes.c_int, _vp]
    k = len(e["table"])
    tv = np.array([t[0] for t in e["table"]] or [0], np.int16)
    tl = np.array([t[1] for t in e["table"]] or [0], np.uint8)
    tc = np.array([t[2] for t in e["table"]] or [0], np.uint64)
    bits = np.frombuffer(e["bits"] + b"\0" * 8, np.uint8).copy()
    out = np.zeros(n, np.int16)
    rc = fn(bits.ctypes.data_as(_vp), e["nbits"], len(e["rle"]), k, tv.ctypes.data_as(_vp),
            tl.ctypes.data_as(_vp), tc.ctypes.data_as(_vp), n, out.ctypes.data_as(_vp))
    assert rc == 0
    return out.tolist()


def ref_entropy(zz):
    """The reference's own entropy stage on one stream (oracle/_ref), or None."""
    L = ref_jpeg()
    if L is None:
        return None
    fn = L.ref_jpeg_entropy
    fn.argtypes = [_vp, ctypes.c_int, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp]
    return _entropy_call(fn, zz, True)
