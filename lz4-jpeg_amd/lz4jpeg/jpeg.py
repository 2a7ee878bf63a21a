"""Host-side mirror of the reference's JPEG encode hot path over the HIP path.

Reference (Algorithms/sequential/JPEG/JPEG.c main, :1110-1178): colour
matrices -> chroma_subsample -> divide_image -> discrete_cosine_transform ->
Quantize -> zigzag_pattern, per 8x8 tile.  Here one call covers a whole image
(or a batch); output int16 per tile [Y 64 zz][Cr 32 zz][Cb 32 zz], raster tiles.
"""
import ctypes

import numpy as np

from . import _lib
from ._lib import JpegError


def coef_count(w, h):
    return int(_lib.lib().jpegr_coef_count(w, h))


def tiles(w, h):
    return ((w + 7) // 8) * ((h + 7) // 8)


def _stream_handle(stream=None):
    import torch
    s = stream if stream is not None else torch.cuda.current_stream()
    return ctypes.c_void_p(s.cuda_stream)


def encode_device(d_rgba, w, h, nimg=1, d_out=None, stream=None):
    """d_rgba: uint8 CUDA tensor of nimg*h*w*4 bytes.  Returns int16 tensor of
    nimg*coef_count(w, h) coefficients."""
    import torch
    if d_rgba.numel() < nimg * w * h * 4:
        raise ValueError("d_rgba smaller than nimg*h*w*4")
    if d_out is None:
        d_out = torch.empty(nimg * coef_count(w, h), dtype=torch.int16, device=d_rgba.device)
    rc = _lib.lib().jpegr_encode_device(ctypes.c_void_p(d_rgba.data_ptr()), w, h, nimg,
                                        ctypes.c_void_p(d_out.data_ptr()), _stream_handle(stream))
    if rc != 0:
        raise JpegError(rc, "jpegr_encode_device")
    return d_out


def dct_raw_device(d_rgba, w, h, nimg=1, stream=None):
    """Un-quantised fp64 DCT coefficients, row-major per plane, 128 per tile."""
    import torch
    d_out = torch.empty(nimg * coef_count(w, h), dtype=torch.float64, device=d_rgba.device)
    rc = _lib.lib().jpegr_dct_raw_device(ctypes.c_void_p(d_rgba.data_ptr()), w, h, nimg,
                                         ctypes.c_void_p(d_out.data_ptr()), _stream_handle(stream))
    if rc != 0:
        raise JpegError(rc, "jpegr_dct_raw_device")
    return d_out


def time_device(d_rgba, w, h, nimg, d_out, iters, stream=None):
    ms = ctypes.c_float(0)
    rc = _lib.lib().jpegr_time_device(ctypes.c_void_p(d_rgba.data_ptr()), w, h, nimg,
                                      ctypes.c_void_p(d_out.data_ptr()), iters,
                                      _stream_handle(stream), ctypes.byref(ms))
    if rc != 0:
        raise JpegError(rc, "jpegr_time_device")
    return ms.value


def encode(rgba):
    """Host API: rgba uint8 array (h, w, 4) -> int16 array (tiles, 128)."""
    a = np.ascontiguousarray(rgba, dtype=np.uint8)
    if a.ndim != 3 or a.shape[2] != 4:
        raise ValueError("rgba must be (h, w, 4) uint8")
    h, w = a.shape[:2]
    out = np.empty(coef_count(w, h), dtype=np.int16)
    rc = _lib.lib().jpegr_encode(a.ctypes.data_as(ctypes.c_void_p), w, h,
                                 out.ctypes.data_as(ctypes.c_void_p))
    if rc != 0:
        raise JpegError(rc, "jpegr_encode")
    return out.reshape(-1, 128)


def reconstruct_device(d_coef, w, h, nimg=1, d_orig=None, stream=None):
    """Reconstructed RGBA8 (uint8 tensor nimg*h*w*4) from encode_device's
    coefficients: reverse zigzag, dequantisation, fp64 IDCT, YCbCr->RGB
    (JPEG.c:1408-1425).  d_orig reproduces the reference's untransformed
    trailing tiles (see jpegr.h)."""
    import torch
    out = torch.empty(nimg * w * h * 4, dtype=torch.uint8, device=d_coef.device)
    rc = _lib.lib().jpegr_reconstruct_device(
        ctypes.c_void_p(d_coef.data_ptr()),
        ctypes.c_void_p(d_orig.data_ptr() if d_orig is not None else 0), w, h, nimg,
        ctypes.c_void_p(out.data_ptr()), _stream_handle(stream))
    if rc != 0:
        raise JpegError(rc, "jpegr_reconstruct_device")
    return out


class Entropy:
    """Device buffers of the entropy stage for `ntiles` tiles (all images):
    bits (256 B/tile), meta (3 u32/tile), table (256 u32/tile), scratch and
    the status words (see jpegr.h: [0] encode, [1] decode, [2] the decoder's
    call tag)."""

    def __init__(self, ntiles, device="cuda"):
        import torch
        self.ntiles = ntiles
        self.bits = torch.zeros(ntiles * 256, dtype=torch.uint8, device=device)
        self.meta = torch.zeros(ntiles * 3, dtype=torch.int32, device=device)
        self.table = torch.zeros(ntiles * 256, dtype=torch.int32, device=device)
        nscr = _lib.lib().jpegr_entropy_scratch_bytes(ntiles)
        self.scratch = torch.empty(nscr, dtype=torch.uint8, device=device)
        self.status = torch.zeros(4, dtype=torch.int32, device=device)

    def encode(self, d_coef, stream=None):
        """RLE + per-stream Huffman + encoded bits of every stream
        (JPEG.c:767-1097) from encode_device's coefficients."""
        rc = _lib.lib().jpegr_entropy_encode_device(
            ctypes.c_void_p(d_coef.data_ptr()), self.ntiles, ctypes.c_void_p(self.bits.data_ptr()),
            ctypes.c_void_p(self.meta.data_ptr()), ctypes.c_void_p(self.table.data_ptr()),
            ctypes.c_void_p(self.scratch.data_ptr()), ctypes.c_void_p(self.status.data_ptr()),
            _stream_handle(stream))
        if rc != 0:
            raise JpegError(rc, "jpegr_entropy_encode_device")

    def decode(self, d_coef_out, stream=None):
        """bits + tables -> coefficients (decode_huffman + inverse_RLE)."""
        rc = _lib.lib().jpegr_entropy_decode_device(
            ctypes.c_void_p(self.bits.data_ptr()), ctypes.c_void_p(self.meta.data_ptr()),
            ctypes.c_void_p(self.table.data_ptr()), self.ntiles,
            ctypes.c_void_p(d_coef_out.data_ptr()), ctypes.c_void_p(self.status.data_ptr()),
            _stream_handle(stream))
        if rc != 0:
            raise JpegError(rc, "jpegr_entropy_decode_device")

    def stream(self, tile, c):
        """Host view of one stream: dict(rle_len, table [(value, len)], nbits, bits)."""
        m = int(self.meta[tile * 3 + c].item()) & 0xFFFFFFFF
        nbits, rle_len, ncodes = m & 0xFFFF, (m >> 16) & 255, m >> 24
        off = (0, 128, 192)[c]
        tab = self.table[tile * 256 + off: tile * 256 + off + ncodes].cpu().numpy()
        table = [(int((e & 0xFFFF) ^ 0x8000) - 0x8000, int((e >> 16) & 255)) for e in tab.tolist()]
        raw = self.bits[tile * 256 + off: tile * 256 + off + (nbits + 7) // 8].cpu().numpy()
        return {"rle_len": rle_len, "table": table, "nbits": nbits, "bits": raw.tobytes()}
