"""ctypes binding of liblz4jpeg.so (the C ABI declared in include/*.h).

The HIP path is the only compute path: if the shared library is missing or
fails to load, every entry point raises -- there is no CPU fallback.
"""
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("LZ4JPEG_LIB") or os.path.join(_HERE, "liblz4jpeg.so")

_c_size = ctypes.c_size_t
_vp = ctypes.c_void_p
_i = ctypes.c_int

# (name, restype, argtypes) for every symbol in include/lz4r.h, jpegr.h,
# lz4jpeg_synth.h.  tests/test_abi.py checks this list against the headers.
SIGNATURES = [
    # lz4r.h
    ("lz4r_ctx_create", _i, [ctypes.POINTER(_vp)]),
    ("lz4r_ctx_destroy", None, [_vp]),
    ("lz4r_compress_bound", _c_size, [_c_size]),
    ("lz4r_nblocks", _c_size, [_c_size]),
    ("lz4r_compress_device", _i, [_vp, _vp, _c_size, _vp, _c_size, ctypes.POINTER(_c_size), _vp]),
    ("lz4r_compress_async", _i, [_vp, _vp, _c_size, _vp, _c_size, _vp, _vp]),
    ("lz4r_compress_segment_async", _i, [_vp, _vp, _c_size, _vp, _c_size, _vp, _i, _vp]),
    ("lz4r_copy_block_sizes", _i, [_vp, _vp, _c_size, _vp]),
    ("lz4r_copy_block_offsets", _i, [_vp, _vp, _c_size, _vp]),
    ("lz4r_block_offsets_device", _i, [_vp, ctypes.POINTER(_vp), ctypes.POINTER(_c_size)]),
    ("lz4r_block_matches_device", _i, [_vp, _c_size, _vp, _vp]),
    ("lz4r_window_matches_device", _i, [_vp, _c_size, _vp, _vp]),
    ("lz4r_compress", _i, [_vp, _c_size, _vp, _c_size, ctypes.POINTER(_c_size)]),
    ("lz4r_decompress", _i, [_vp, _c_size, _vp, _c_size, ctypes.POINTER(_c_size)]),
    ("lz4r_decompress_device", _i, [_vp, _c_size, _vp, _c_size, _vp, _c_size, _vp, _vp]),
    ("lz4r_decompress_stream_device", _i, [_vp, _c_size, _vp, _c_size, ctypes.POINTER(_c_size),
                                           _vp]),
    ("lz4r_decompress_stream", _i, [_vp, _c_size, _vp, _c_size, ctypes.POINTER(_c_size)]),
    ("lz4r_check", _i, [_vp, _vp]),
    ("lz4r_set_timing", _i, [_vp, _i]),
    ("lz4r_last_timing", _i, [_vp, ctypes.POINTER(ctypes.c_float), ctypes.POINTER(ctypes.c_float)]),
    ("lz4r_timed_calls", _i, [_vp, _c_size, ctypes.POINTER(ctypes.c_float),
                              ctypes.POINTER(ctypes.c_float), ctypes.POINTER(_c_size)]),
    ("lz4r_strerror", ctypes.c_char_p, [_i]),
    # jpegr.h
    ("jpegr_coef_count", _c_size, [_i, _i]),
    ("jpegr_encode_device", _i, [_vp, _i, _i, _i, _vp, _vp]),
    ("jpegr_dct_raw_device", _i, [_vp, _i, _i, _i, _vp, _vp]),
    ("jpegr_encode", _i, [_vp, _i, _i, _vp]),
    ("jpegr_time_device", _i, [_vp, _i, _i, _i, _vp, _i, _vp, ctypes.POINTER(ctypes.c_float)]),
    ("jpegr_reconstruct_device", _i, [_vp, _vp, _i, _i, _i, _vp, _vp]),
    ("jpegr_entropy_scratch_bytes", _c_size, [_c_size]),
    ("jpegr_entropy_encode_device", _i, [_vp, _c_size, _vp, _vp, _vp, _vp, _vp, _vp]),
    ("jpegr_entropy_decode_device", _i, [_vp, _vp, _vp, _c_size, _vp, _vp, _vp]),
    ("jpegr_planes_device", _i, [_vp, _i, _i, _vp, _vp, _vp, _vp]),
    ("jpegr_dct_blocks_device", _i, [_vp, _i, _i, _i, _vp, _vp]),
    ("jpegr_quantize_device", _i, [_vp, _vp, _i, _c_size, _vp]),
    ("jpegr_permute_device", _i, [_vp, _vp, _vp, _i, _c_size, _vp]),
    ("jpegr_strerror", ctypes.c_char_p, [_i]),
    # lz4jpeg_synth.h
    ("lz4jpeg_rand_rgba", None, [ctypes.c_uint, _i, _i, _vp]),
    ("lz4jpeg_random_passages", _c_size, [_vp, _c_size, ctypes.c_uint, _c_size, _c_size, _c_size,
                                         _vp]),
    ("lz4jpeg_rand_rgba_stream", None, [ctypes.c_uint, ctypes.c_uint64, _c_size, _vp]),
    ("lz4jpeg_rand_states", None, [ctypes.c_uint, ctypes.c_uint64, ctypes.c_uint64, _c_size,
                                   _vp]),
    ("lz4jpeg_passage_starts", _c_size, [_c_size, ctypes.c_uint, _c_size, ctypes.c_uint64,
                                         _c_size, _vp]),
    ("lz4jpeg_rand_rgba_device", _i, [ctypes.c_uint, ctypes.c_uint64, _c_size, _vp, _vp]),
    ("lz4jpeg_random_passages_device", _i, [_vp, _c_size, ctypes.c_uint, _c_size,
                                            ctypes.c_uint64, _c_size, _vp, _vp]),
    # lz4jpeg_compat.h (the reference's own function names, on the GPU path)
    ("lz4_encode", None, []),
    ("find_longest_match", ctypes.c_uint8, [_vp, _c_size, ctypes.POINTER(ctypes.c_uint16)]),
    ("block_encode", None, [_vp, _c_size, _vp, _vp, _vp, _vp]),
    ("write_output", None, [_vp, _vp]),
    ("LZ4_decode", None, [ctypes.c_char_p, ctypes.c_char_p]),
    ("discrete_cosine_transform", None, [_vp, _c_size, _c_size, ctypes.POINTER(ctypes.POINTER(
        ctypes.c_double))]),
    ("Quantize", None, [ctypes.POINTER(ctypes.POINTER(ctypes.c_double)), _vp, _c_size]),
    ("zigzag_pattern", None, [_c_size, _c_size, _vp, _vp]),
]

_lib = None


class LibraryMissing(RuntimeError):
    pass


def lib():
    """Load liblz4jpeg.so once; raise loudly if it is not built."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise LibraryMissing(
            f"{LIB_PATH} not built: run `make -C {os.path.dirname(os.path.dirname(_HERE))}` "
            "(the HIP path is the only compute path; there is no CPU fallback)")
    handle = ctypes.CDLL(LIB_PATH)
    for name, res, args in SIGNATURES:
        fn = getattr(handle, name)
        fn.restype = res
        fn.argtypes = args
    _lib = handle
    return _lib


class Lz4Error(RuntimeError):
    def __init__(self, code, where=""):
        msg = lib().lz4r_strerror(code).decode()
        super().__init__(f"{where}: lz4r error {code} ({msg})")
        self.code = code


class JpegError(RuntimeError):
    def __init__(self, code, where=""):
        msg = lib().jpegr_strerror(code).decode()
        super().__init__(f"{where}: jpegr error {code} ({msg})")
        self.code = code


# error codes (include/lz4r.h)
LZ4R_OK = 0
LZ4R_ERR_ARG = -1
LZ4R_ERR_TOO_SMALL = -2
LZ4R_ERR_CAPACITY = -3
LZ4R_ERR_HIP = -4
LZ4R_ERR_NOMEM = -5
LZ4R_ERR_CORRUPT = -6
LZ4R_BLOCK = 300
LZ4R_BLOCK_BOUND = 1152
