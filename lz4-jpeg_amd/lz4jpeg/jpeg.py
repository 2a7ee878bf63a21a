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
