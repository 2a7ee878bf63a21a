"""Per-phase s_memtime cycles of the fast entropy encoder (tools only):
LZ4JPEG_LIB=tools/ab/libjpegr_entropy_prof.so (built with -DJPEGR_PROF).
Luma phases 0-4, chroma 8-12: load, RLE walk, symbols/heap entries, tree +
codes (after the top-down pass), sequence, heap build, merges, top-down; printed as cycles per wave per call."""
import ctypes
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "lz4-jpeg_amd")]
import torch  # noqa: E402
from lz4jpeg import _lib, jpeg, synth  # noqa: E402

W, H = 3840, 2160
d_img = torch.from_numpy(synth.rand_rgba(W, H, seed=1)).cuda()
d_coef = jpeg.encode_device(d_img, W, H)
ent = jpeg.Entropy(jpeg.tiles(W, H))
lib = _lib.lib() if callable(getattr(_lib, "lib", None)) else _lib.LIB
for _ in range(200):
    ent.encode(d_coef)
torch.cuda.synchronize()
buf = (ctypes.c_ulonglong * 16)()
lib.jpegr_prof_read(buf, 1)
calls = 200
for _ in range(calls):
    ent.encode(d_coef)
torch.cuda.synchronize()
lib.jpegr_prof_read(buf, 0)
names = ["load", "walk", "prep", "codes", "sequence", "heap", "merges", "topdown"]
tiles = jpeg.tiles(W, H)
for base, waves, tag in ((0, (tiles + 63) // 64, "luma"), (8, 2 * ((tiles + 63) // 64), "chroma")):
    vals = [buf[base + k] / (waves * calls) for k in range(8)]
    print(tag, " ".join(f"{n} {v:.0f}" for n, v in zip(names, vals)), f"total {sum(vals):.0f}", flush=True)
