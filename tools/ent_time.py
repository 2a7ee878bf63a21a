"""A/B timing of the entropy stage (LZ4JPEG_LIB selects the build): a 4K
random image's coefficients, 100 ms of settling load, then 300 encodes and
300 decodes, each bracketed by events; prints the medians (tools only)."""
import os
import statistics
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "lz4-jpeg_amd")]
import torch  # noqa: E402
from lz4jpeg import jpeg, synth  # noqa: E402

W, H = 3840, 2160
d_img = torch.from_numpy(synth.rand_rgba(W, H, seed=1)).cuda()
d_coef = jpeg.encode_device(d_img, W, H)
ent = jpeg.Entropy(jpeg.tiles(W, H))
back = torch.empty_like(d_coef)
t0 = time.perf_counter()
while time.perf_counter() - t0 < 0.1:
    ent.encode(d_coef)
    ent.decode(back)
torch.cuda.synchronize()
enc, dec = [], []
for _ in range(300):
    e0, e1, e2 = (torch.cuda.Event(enable_timing=True) for _ in range(3))
    e0.record()
    ent.encode(d_coef)
    e1.record()
    ent.decode(back)
    e2.record()
    torch.cuda.synchronize()
    enc.append(e0.elapsed_time(e1))
    dec.append(e1.elapsed_time(e2))
print(f"encode median {statistics.median(enc):.4f} ms, decode median {statistics.median(dec):.4f} ms, "
      f"ok {bool(torch.equal(back, d_coef))}", flush=True)
