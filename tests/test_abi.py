"""The C-ABI library loads and exports exactly what include/*.h declares
(no compute calls: this runs without a GPU)."""
import ctypes
import os
import re
import subprocess

import pytest

from lz4jpeg import _lib

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADERS = [os.path.join(REPO, "include", h)
           for h in ("lz4r.h", "jpegr.h", "lz4jpeg_synth.h", "lz4jpeg_compat.h")]


def declared_functions():
    names = set()
    for h in HEADERS:
        src = open(h).read()
        src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
        for m in re.finditer(r"^[A-Za-z_][\w \*]*?\b(\w+)\s*\(", src, flags=re.M):
            name = m.group(1)
            if name not in ("defined",):
                names.add(name)
    return names


def test_headers_declare_functions():
    names = declared_functions()
    assert {"lz4r_compress", "lz4r_compress_device", "jpegr_encode_device",
            "lz4jpeg_rand_rgba"} <= names


def test_library_exports_every_declared_symbol():
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True,
                         text=True, check=True).stdout
    exported = {line.split()[-1] for line in out.splitlines() if " T " in line}
    missing = declared_functions() - exported
    assert not missing, missing


def test_bindings_cover_headers():
    assert {n for n, _, _ in _lib.SIGNATURES} == declared_functions()


def test_library_loads_and_binds():
    L = _lib.lib()
    for name, _, _ in _lib.SIGNATURES:
        assert getattr(L, name) is not None


def test_host_only_entry_points():
    L = _lib.lib()
    assert L.lz4r_nblocks(300) == 1 and L.lz4r_nblocks(301) == 2
    assert L.lz4r_compress_bound(600) == 1 + 2 * _lib.LZ4R_BLOCK_BOUND
    assert L.jpegr_coef_count(3840, 2160) == 480 * 270 * 128
    assert L.jpegr_coef_count(9, 9) == 4 * 128
    assert L.jpegr_coef_count(0, 8) == 0
    assert L.lz4r_strerror(-2).decode().startswith("input shorter")
    assert L.jpegr_strerror(-1).decode() == "invalid argument"


def test_too_small_fails_before_device():
    """The reference exit(1)s below 300 bytes (LZ4.c:632); we return an error
    code -- without touching a device, so this runs anywhere."""
    L = _lib.lib()
    buf = ctypes.create_string_buffer(299)
    out = ctypes.create_string_buffer(4096)
    got = ctypes.c_size_t(0)
    rc = L.lz4r_compress(buf, 299, out, 4096, ctypes.byref(got))
    assert rc == _lib.LZ4R_ERR_TOO_SMALL


def test_missing_library_fails_loudly(monkeypatch, tmp_path):
    monkeypatch.setattr(_lib, "_lib", None)
    monkeypatch.setattr(_lib, "LIB_PATH", str(tmp_path / "nope.so"))
    with pytest.raises(_lib.LibraryMissing):
        _lib.lib()


def test_match_finders_reject_bad_arguments_before_device():
    """lz4r_block_matches_device launches in chunks of 2^24 blocks (HIP's
    2^32 work-item grid limit); what it cannot take -- NULL, empty, above the
    2^40-byte call limit -- is an argument error, found before any HIP call."""
    L = _lib.lib()
    p = ctypes.c_void_p(16)          # never dereferenced: every case fails first
    assert L.lz4r_block_matches_device(None, 300, p, None) == _lib.LZ4R_ERR_ARG
    assert L.lz4r_block_matches_device(p, 0, p, None) == _lib.LZ4R_ERR_ARG
    assert L.lz4r_block_matches_device(p, (1 << 40) + 1, p, None) == _lib.LZ4R_ERR_ARG
    assert L.lz4r_window_matches_device(p, 0, p, None) == _lib.LZ4R_ERR_ARG
    assert L.lz4r_window_matches_device(p, 1 << 32, p, None) == _lib.LZ4R_ERR_ARG
