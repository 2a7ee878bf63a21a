"""Host-side mirror of the reference's LZ4 encoder interface over the HIP path.

Reference (Algorithms/sequential/LZ4/LZ4.c):
  lz4_encode()         :670-742  file in -> compressed.bin  ==  compress(bytes)
  divide_input()       :123-177  300-byte blocks            ==  nblocks()/shard_blocks()
  block_encode() + find_longest_match()  run inside the HIP kernels.

Errors follow the reference's exit paths as exceptions: an input shorter than
300 bytes raises InputTooSmall (the reference prints and exit(1)s, :632-637).
Device memory and streams come from torch (plumbing only); the compute is the
C ABI in include/lz4r.h.
"""
import ctypes

import numpy as np

from . import _lib
from ._lib import Lz4Error, LZ4R_BLOCK, LZ4R_BLOCK_BOUND  # noqa: F401

BLOCK = LZ4R_BLOCK


class InputTooSmall(Lz4Error):
    pass


def _raise(code, where):
    if code == _lib.LZ4R_ERR_TOO_SMALL:
        raise InputTooSmall(code, where)
    raise Lz4Error(code, where)


def nblocks(n):
    return (n + BLOCK - 1) // BLOCK


def compress_bound(n):
    return int(_lib.lib().lz4r_compress_bound(n))


def _stream_handle(stream=None):
    import torch
    s = stream if stream is not None else torch.cuda.current_stream()
    return ctypes.c_void_p(s.cuda_stream)


class Compressor:
    """Owns an lz4r context (device scratch) on the current device."""

    def __init__(self):
        L = _lib.lib()
        h = ctypes.c_void_p()
        rc = L.lz4r_ctx_create(ctypes.byref(h))
        if rc != 0:
            _raise(rc, "lz4r_ctx_create")
        self._h = h

    def close(self):
        if getattr(self, "_h", None):
            _lib.lib().lz4r_ctx_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # -- device API -------------------------------------------------------
    def compress_device(self, d_in, n=None, d_out=None, stream=None):
        """Compress the uint8 CUDA tensor d_in (first n bytes).  Returns
        (d_out, length): the framed stream is d_out[:length]."""
        import torch
        n = d_in.numel() if n is None else n
        if d_out is None:
            d_out = torch.empty(compress_bound(n), dtype=torch.uint8, device=d_in.device)
        got = ctypes.c_size_t(0)
        rc = _lib.lib().lz4r_compress_device(self._h, ctypes.c_void_p(d_in.data_ptr()), n,
                                             ctypes.c_void_p(d_out.data_ptr()), d_out.numel(),
                                             ctypes.byref(got), _stream_handle(stream))
        if rc != 0:
            _raise(rc, "lz4r_compress_device")
        return d_out, got.value

    def compress_async(self, d_in, n, d_out, d_len, stream=None, segment=False,
                       final_shard=None):
        """Enqueue only; the uint64 length lands in d_len (1-element int64 tensor),
        with bit 63 set if the call met a corrupt LDS index: read it with
        async_length(d_len), which raises then.
        segment=True: whole blocks without the frame header (one shard);
        final_shard must then be given: only the globally last shard may end
        in a short block, a non-final shard (final_shard=False) must be a
        multiple of 300 bytes (else the concatenated stream would differ from
        the single-GPU one)."""
        if segment and final_shard is None:
            raise ValueError("compress_async(segment=True) needs final_shard=True/False")
        L = _lib.lib()
        args = (self._h, ctypes.c_void_p(d_in.data_ptr()), n, ctypes.c_void_p(d_out.data_ptr()),
                d_out.numel(), ctypes.c_void_p(d_len.data_ptr()))
        if segment:
            rc = L.lz4r_compress_segment_async(*args, 1 if final_shard else 0,
                                               _stream_handle(stream))
        else:
            rc = L.lz4r_compress_async(*args, _stream_handle(stream))
        if rc != 0:
            _raise(rc, "lz4r_compress_segment_async" if segment else "lz4r_compress_async")

    @staticmethod
    def async_length(d_len):
        """The length an async call stored in the int64 tensor d_len (reads it
        back: waits for torch's current stream).  Raises Lz4Error(-6) when the
        call flagged a corrupt LDS index (LZ4R_LEN_CORRUPT, bit 63: the int64
        is negative) -- the stream must not be used then."""
        v = int(d_len.item())
        if v < 0:
            raise Lz4Error(_lib.LZ4R_ERR_CORRUPT,
                           "lz4r_compress_*_async: corrupt LDS index (LZ4R_LEN_CORRUPT)")
        return v

    def block_offsets(self, count, stream=None):
        """numpy uint64 array: the last call's first `count` per-block output
        offsets (relative to the first block byte)."""
        out = np.empty(count, dtype=np.uint64)
        rc = _lib.lib().lz4r_copy_block_offsets(self._h, out.ctypes.data_as(ctypes.c_void_p),
                                                count, _stream_handle(stream))
        if rc != 0:
            _raise(rc, "lz4r_copy_block_offsets")
        return out

    def block_offsets_device(self):
        """(device pointer, count) of the last call's per-block offsets, as the
        placement kernel wrote them (valid until the next call on this
        context); lz4r_block_offsets_device."""
        ptr, cnt = ctypes.c_void_p(), ctypes.c_size_t(0)
        rc = _lib.lib().lz4r_block_offsets_device(self._h, ctypes.byref(ptr), ctypes.byref(cnt))
        if rc != 0:
            _raise(rc, "lz4r_block_offsets_device")
        return ptr.value, cnt.value

    def check(self, stream=None):
        """lz4r_check: synchronise and raise Lz4Error(-6) if the last call met
        a corrupt bucket head (compress_device and async_length check by
        themselves)."""
        rc = _lib.lib().lz4r_check(self._h, _stream_handle(stream))
        if rc != 0:
            _raise(rc, "lz4r_check")

    def set_timing(self, enable=True):
        """Record HIP events on the launch stream around each call and its
        match-finder/parse kernel (see last_timing)."""
        _lib.lib().lz4r_set_timing(self._h, 1 if enable else 0)

    def last_timing(self):
        """(ms of the whole last call, ms of its lz4_analyze kernel)."""
        a, b = ctypes.c_float(0), ctypes.c_float(0)
        rc = _lib.lib().lz4r_last_timing(self._h, ctypes.byref(a), ctypes.byref(b))
        if rc != 0:
            _raise(rc, "lz4r_last_timing")
        return a.value, b.value

    def timed_calls(self, max_calls=4096):
        """(ms of each call, ms of its lz4_tiles launches): two lists over the
        newest calls timed since set_timing(True), oldest first (waits for
        the newest; lz4r_timed_calls)."""
        a = (ctypes.c_float * max_calls)()
        b = (ctypes.c_float * max_calls)()
        cnt = ctypes.c_size_t(0)
        rc = _lib.lib().lz4r_timed_calls(self._h, max_calls, a, b, ctypes.byref(cnt))
        if rc != 0:
            _raise(rc, "lz4r_timed_calls")
        return list(a[:cnt.value]), list(b[:cnt.value])

    # -- host convenience -------------------------------------------------
    def compress(self, data):
        """bytes -> framed compressed bytes (== the reference's compressed.bin)."""
        import torch
        buf = np.frombuffer(bytes(data), dtype=np.uint8)
        if buf.size < BLOCK:
            raise InputTooSmall(_lib.LZ4R_ERR_TOO_SMALL, "compress")
        d_in = torch.from_numpy(buf.copy()).cuda()
        d_out, length = self.compress_device(d_in)
        torch.cuda.synchronize()
        return d_out[:length].cpu().numpy().tobytes()


def compress(data):
    """One-shot host API: compressed bytes of `data` (a bytes-like object)."""
    buf = np.frombuffer(bytes(data), dtype=np.uint8)
    n = buf.size
    if n < BLOCK:
        raise InputTooSmall(_lib.LZ4R_ERR_TOO_SMALL, "lz4r_compress")
    cap = 1 + nblocks(n) * LZ4R_BLOCK_BOUND
    out = np.empty(cap, dtype=np.uint8)
    got = ctypes.c_size_t(0)
    rc = _lib.lib().lz4r_compress(buf.ctypes.data_as(ctypes.c_void_p), n,
                                  out.ctypes.data_as(ctypes.c_void_p), cap, ctypes.byref(got))
    if rc != 0:
        _raise(rc, "lz4r_compress")
    return out[:got.value].tobytes()


def decompress(stream, cap=None):
    """Exact host decoder (lz4r_decompress): framed stream bytes -> original
    bytes.  Replaces LZ4_decode (LZ4.c:1038-1121); raises Lz4Error(-6) on a
    malformed stream."""
    buf = np.frombuffer(bytes(stream), dtype=np.uint8)
    if cap is None:
        cap = (buf.size // 5 + 1) * BLOCK
    out = np.empty(max(cap, 1), dtype=np.uint8)
    got = ctypes.c_size_t(0)
    rc = _lib.lib().lz4r_decompress(buf.ctypes.data_as(ctypes.c_void_p), buf.size,
                                    out.ctypes.data_as(ctypes.c_void_p), cap, ctypes.byref(got))
    if rc != 0:
        _raise(rc, "lz4r_decompress")
    return out[:got.value].tobytes()


def decompress_device(d_stream, length, d_offsets, nb, out_cap, d_out=None, stream=None,
                      check=True):
    """Block-parallel GPU decode (lz4r_decompress_device).  d_stream: uint8
    tensor holding the framed stream (first `length` bytes); d_offsets: int64
    tensor of nb per-block offsets (Compressor.block_offsets), or the raw
    device pointer Compressor.block_offsets_device() returns.  Returns
    (d_out, decoded_length); raises Lz4Error(-6) naming the first malformed
    block.  check=False skips the result read-back (no host sync) and
    returns (d_out, None)."""
    import torch
    if d_out is None:
        d_out = torch.empty(max(out_cap, 1), dtype=torch.uint8, device=d_stream.device)
    res = torch.empty(2, dtype=torch.int64, device=d_stream.device)
    offs = d_offsets if isinstance(d_offsets, int) else d_offsets.data_ptr()
    rc = _lib.lib().lz4r_decompress_device(
        ctypes.c_void_p(d_stream.data_ptr()), length, ctypes.c_void_p(offs), nb,
        ctypes.c_void_p(d_out.data_ptr()), out_cap, ctypes.c_void_p(res.data_ptr()),
        _stream_handle(stream))
    if rc != 0:
        _raise(rc, "lz4r_decompress_device")
    if not check:
        return d_out, None
    if stream is not None:
        stream.synchronize()          # the result is written on `stream`, not torch's current one
    n, bad = (int(x) for x in res.cpu().tolist())
    if bad != -1:
        raise Lz4Error(_lib.LZ4R_ERR_CORRUPT, f"lz4r_decompress_device: block {bad - 1}")
    if n > out_cap:
        raise Lz4Error(_lib.LZ4R_ERR_CAPACITY,
                       f"lz4r_decompress_device: needs {n} bytes, capacity {out_cap}")
    return d_out, n


def decompress_stream_device(d_stream, length, out_cap, d_out=None, stream=None):
    """GPU decode of a bare framed stream (lz4r_decompress_stream_device):
    the block boundaries are found on the device, as LZ4_decode (LZ4.c:1038)
    needs only the stream.  Returns (d_out, decoded_length); raises
    Lz4Error(-6) on a malformed stream."""
    import torch
    if d_out is None:
        d_out = torch.empty(max(out_cap, 1), dtype=torch.uint8, device=d_stream.device)
    got = ctypes.c_size_t(0)
    rc = _lib.lib().lz4r_decompress_stream_device(
        ctypes.c_void_p(d_stream.data_ptr()), length, ctypes.c_void_p(d_out.data_ptr()), out_cap,
        ctypes.byref(got), _stream_handle(stream))
    if rc != 0:
        _raise(rc, "lz4r_decompress_stream_device")
    return d_out, got.value


def decompress_stream(stream_bytes, cap=None):
    """Host-buffer form of decompress_stream_device (lz4r_decompress_stream)."""
    buf = np.frombuffer(bytes(stream_bytes), dtype=np.uint8)
    if cap is None:
        cap = (buf.size // 8 + 1) * BLOCK
    out = np.empty(max(cap, 1), dtype=np.uint8)
    got = ctypes.c_size_t(0)
    rc = _lib.lib().lz4r_decompress_stream(buf.ctypes.data_as(ctypes.c_void_p), buf.size,
                                           out.ctypes.data_as(ctypes.c_void_p), cap,
                                           ctypes.byref(got))
    if rc != 0:
        _raise(rc, "lz4r_decompress_stream")
    return out[:got.value].tobytes()
