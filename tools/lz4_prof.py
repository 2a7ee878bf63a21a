"""Diagnostic: per-phase s_memtime totals of a LZ4R_PROF build (tools/build_variants.sh)."""
import ctypes
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["LZ4JPEG_LIB"] = os.path.join(REPO, "tools", "variants",
                                         sys.argv[1] if len(sys.argv) > 1 else "liblz4_p0.so")
sys.path[:0] = [os.path.join(REPO, "lz4-jpeg_amd")]
import torch  # noqa: E402
from lz4jpeg import _lib, lz4, synth  # noqa: E402

n = 1 << 28
host = synth.random_passages(n, length=30000, seed=1)
d_in = torch.from_numpy(host).cuda()
c = lz4.Compressor()
d_out = torch.empty(lz4.compress_bound(n), dtype=torch.uint8, device="cuda")
_, got = c.compress_device(d_in, n, d_out)
buf = (ctypes.c_ulonglong * 16)()
_lib.lib().lz4r_debug_prof(buf)
names = ["index (sort)", "candidates+lcp", "sync", "best+nm+succ", "walk+visit", "sequences",
         "literals", "block start", "bsizes", "store"]
tot = sum(buf[:10])
for i, nm in enumerate(names):
    print(f"{nm:14s} {buf[i] / 1e9:8.3f} Gcyc  {100 * buf[i] / tot:5.1f}%")
