"""Per-phase cycle shares of lz4_tiles from an LZ4R_PROF build
(tools/build_variants.sh with PROF=0): run the 1 GiB corpus once to warm up,
then `reps` calls, and print the summed s_memtime cycles of each phase."""
import ctypes
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "lz4-jpeg_amd")]
import torch  # noqa: E402
from lz4jpeg import _lib, lz4, synth  # noqa: E402

PHASES = ["index", "walker queue", "candidates+lcp", "best scan", "nm+jump table", "walk",
          "emission"]
n = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 30
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
d_in = torch.empty(n + 16, dtype=torch.uint8, device="cuda")
synth.random_passages_device(d_in, n, length=30000, seed=1)
L = _lib.lib()
L.lz4r_prof_read.argtypes = [ctypes.c_void_p, ctypes.c_int]
acc = (ctypes.c_ulonglong * 16)()
c = lz4.Compressor()
d_out = torch.empty(n + n // 8 + (1 << 20), dtype=torch.uint8, device="cuda")
c.compress_device(d_in, n, d_out)
torch.cuda.synchronize()
L.lz4r_prof_read(acc, 1)
c.set_timing(True)
for _ in range(reps):
    c.compress_device(d_in, n, d_out)
    print("ms", c.last_timing(), flush=True)
torch.cuda.synchronize()
L.lz4r_prof_read(acc, 0)
tot = sum(acc[i] for i in range(len(PHASES)))
nb = (n + 299) // 300 * reps
for i, name in enumerate(PHASES):
    print(f"{name:16s} {acc[i] / nb:10.1f} cyc/block  {100.0 * acc[i] / tot:5.1f} %")
c.close()
