"""The compressor never reads past its input: the input ends exactly at the
end of the only mapped page range, and the address range after it is
reserved but NOT mapped, so any read past the input faults (VERDICT r05 item
7).

Why the hipMalloc form of this test (test_gpu_lz4.py::
test_input_ending_at_allocation_end) cannot fail: a hipMalloc allocation's
end is not the end of mapped memory -- the allocator's next allocation, or
the rest of its 2 MiB fragment, is usually mapped right behind it, so a
24-byte over-read would read some other buffer's bytes and the output would
still match whenever those bytes do not extend a match.  Here the range is
built with the virtual-memory API: hipMemAddressReserve of the mapped
range plus one more granule, hipMemCreate + hipMemMap + hipMemSetAccess of
the mapped range only (whole granules, at least n bytes).

The bug this pins: lz4_tiles' unstaged 4-gram loads read 24
bytes past a block's end (row 4 of the index, lz4r.hip), which is safe only
when those bytes belong to the input: the guard is
`t + 2 < nb || (t + 2 == nb && last_n >= 24)`.  With the pre-fix guard
(`t + 1 < nb`) every 4-byte-aligned n below whose last block holds fewer
than 24 bytes (308: 8 B, 604: 4 B, 23120: 20 B) had block nb - 2 read up
to 24 - last_n bytes into the unmapped granule -> a GPU page fault.  n = 1524
(last block 24 B) is the boundary case that must stay on the fast path;
301 and 1525 (input not 4-byte aligned) take the staged path; 2700 ends on
a whole block.

The compress runs in a child process, so a regression kills that process
(a memory-access fault aborts it) and fails this one test, not the session.
The reference's own over-read (LZ4.c:302 reads past the block) is what the
block clamp replaces."""
import hashlib
import os
import subprocess
import sys

import pytest

import golden_inputs

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(os.path.dirname(HERE), "lz4-jpeg_amd")

CHILD = r"""
import ctypes, hashlib, sys
import torch
sys.path.insert(0, sys.argv[1])
from lz4jpeg import _lib, lz4
from lz4jpeg.lz4 import compress_bound

hip = ctypes.CDLL("libamdhip64.so")


class Loc(ctypes.Structure):
    _fields_ = [("type", ctypes.c_int), ("id", ctypes.c_int)]


class Flags(ctypes.Structure):
    _fields_ = [("compressionType", ctypes.c_ubyte), ("gpuDirectRDMACapable", ctypes.c_ubyte),
                ("usage", ctypes.c_ushort)]


class Prop(ctypes.Structure):        # hipMemAllocationProp
    _fields_ = [("type", ctypes.c_int), ("requestedHandleType", ctypes.c_int),
                ("location", Loc), ("win32HandleMetaData", ctypes.c_void_p),
                ("allocFlags", Flags)]


class Access(ctypes.Structure):      # hipMemAccessDesc
    _fields_ = [("location", Loc), ("flags", ctypes.c_int)]


def ok(rc, what):
    if rc != 0:
        raise SystemExit(f"{what}: hip error {rc}")


torch.cuda.init()
dev = torch.cuda.current_device()
data = open(sys.argv[2], "rb").read()
n = len(data)
prop = Prop(type=1, requestedHandleType=0, location=Loc(1, dev))     # pinned, on the device
gran = ctypes.c_size_t(0)
ok(hip.hipMemGetAllocationGranularity(ctypes.byref(gran), ctypes.byref(prop), 0), "granularity")
g0 = gran.value
g = -(-n // g0) * g0                             # the mapped range: whole granules >= n
base = ctypes.c_void_p()
ok(hip.hipMemAddressReserve(ctypes.byref(base), ctypes.c_size_t(g + g0), ctypes.c_size_t(0),
                            None, ctypes.c_ulonglong(0)), "reserve")
h = ctypes.c_uint64(0)
ok(hip.hipMemCreate(ctypes.byref(h), ctypes.c_size_t(g), ctypes.byref(prop), ctypes.c_ulonglong(0)),
   "create")
ok(hip.hipMemMap(base, ctypes.c_size_t(g), ctypes.c_size_t(0), h, ctypes.c_ulonglong(0)), "map")
acc = Access(location=Loc(1, dev), flags=3)                              # read-write
ok(hip.hipMemSetAccess(base, ctypes.c_size_t(g), ctypes.byref(acc), ctypes.c_size_t(1)), "access")
src = ctypes.c_void_p(base.value + g - n)        # the input ends at the last mapped byte
ok(hip.hipMemcpy(src, data, ctypes.c_size_t(n), 1), "copy")             # host -> device
comp = lz4.Compressor()
d_out = torch.empty(compress_bound(n), dtype=torch.uint8, device="cuda")
got = ctypes.c_size_t(0)
torch.cuda.synchronize()
rc = _lib.lib().lz4r_compress_device(comp._h, src, n, ctypes.c_void_p(d_out.data_ptr()),
                                     d_out.numel(), ctypes.byref(got), None)
torch.cuda.synchronize()
assert rc == 0, rc
out = d_out[:got.value].cpu().numpy().tobytes()
comp.close()
ok(hip.hipMemUnmap(base, ctypes.c_size_t(g)), "unmap")
ok(hip.hipMemRelease(h), "release")
ok(hip.hipMemAddressFree(base, ctypes.c_size_t(g + g0)), "free")
print("granule", g0, "mapped", g, "src_mod4", src.value % 4, "md5", hashlib.md5(out).hexdigest(), flush=True)
"""


@pytest.mark.parametrize("n", [301, 308, 300 * 2 + 4, 300 * 77 + 20, 300 * 5 + 24, 300 * 5 + 25,
                               300 * 9])
def test_input_ending_at_unmapped_range(oracle, tmp_path, n):
    text = golden_inputs.lz4_input("metamorphosis_spaces")
    data = bytes(text[1000:1000 + n])
    f = tmp_path / "in.bin"
    f.write_bytes(data)
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    r = subprocess.run([sys.executable, "-c", CHILD, PKG, str(f)], capture_output=True, text=True,
                       timeout=180, env=env)
    assert r.returncode == 0, (r.returncode, r.stdout[-2000:], r.stderr[-3000:])
    line = r.stdout.strip().splitlines()[-1]
    assert line.endswith("md5 " + hashlib.md5(oracle.lz4_compress(data)).hexdigest()), line
