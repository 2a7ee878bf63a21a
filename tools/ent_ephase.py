"""Phase stamps of the entropy encoder's waves (tools only): a diag build of
jpegr_entropy (tools/ab/libjpegr_entropy_<name>.so, from a source with
s_memtime stamps into g_eph[kernel][wave][phase]) encodes one random 4K
image's coefficients; per kernel, the cycles between consecutive stamps.

    python3 tools/ent_ephase.py [name]      (default ediag)

Stamps: 0 start, 1 stream loads issued + table zeroed, 2 RLE + counts done,
3 heap entries / symbols written, 4 tree + codes done, 5 sequence bits done,
6 meta stored (fast-path lanes)."""
import ctypes
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
name = sys.argv[1] if len(sys.argv) > 1 else "ediag"
os.environ["LZ4JPEG_LIB"] = os.path.join(REPO, "tools", "ab", f"libjpegr_entropy_{name}.so")
sys.path[:0] = [os.path.join(REPO, "lz4-jpeg_amd")]
import torch  # noqa: E402
from lz4jpeg import _lib, jpeg, synth  # noqa: E402

W, H = 3840, 2160
d_img = torch.from_numpy(synth.rand_rgba(W, H, seed=1)).cuda()
d_coef = jpeg.encode_device(d_img, W, H)
ent = jpeg.Entropy(jpeg.tiles(W, H))
L = _lib.lib()
for _ in range(4):
    ent.encode(d_coef)
torch.cuda.synchronize()
ph = np.zeros((2, 4096, 8), np.uint32)
assert L.jpegr_eph_read(ph.ctypes.data_as(ctypes.c_void_p)) == 0
back = torch.empty_like(d_coef)
ent.decode(back)
torch.cuda.synchronize()
print("round trip ok", bool(torch.equal(back, d_coef)))
names = ["loads+zero", "RLE+counts", "heap prep", "tree+codes", "sequence", "meta"]
for k, kn in enumerate(("luma", "chroma")):
    p = ph[k].astype(np.int64)
    ok = (p[:, 0] > 0) & (p[:, 6] > 0)
    print(f"{kn}: waves with all stamps {int(ok.sum())}")
    tot = ((p[:, 6] - p[:, 0]) & 0xFFFFFFFF)[ok]
    for j in range(6):
        d = ((p[:, j + 1] - p[:, j]) & 0xFFFFFFFF)[ok]
        print(f"  {names[j]:11s} cycles p10 {np.percentile(d, 10):7.0f} p50 {np.median(d):7.0f}"
              f" max {d.max():7.0f}  share {np.median(d) / np.median(tot):.2f}")
    print(f"  {'whole':11s} cycles p10 {np.percentile(tot, 10):7.0f} p50 {np.median(tot):7.0f} max {tot.max():7.0f}")
