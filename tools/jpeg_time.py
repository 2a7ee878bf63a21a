"""Time the JPEG encoder (and reconstruction) on one 3840x2160 random image:
mean kernel time over 200 launches between HIP events on the current stream."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "lz4-jpeg_amd")]
import torch  # noqa: E402
from lz4jpeg import jpeg, synth  # noqa: E402

w, h = 3840, 2160
img = torch.from_numpy(synth.rand_rgba(w, h, seed=1)).cuda()
out = torch.empty(jpeg.coef_count(w, h), dtype=torch.int16, device="cuda")
for _ in range(20):
    jpeg.encode_device(img, w, h, 1, out)
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(200):
    jpeg.encode_device(img, w, h, 1, out)
e1.record()
torch.cuda.synchronize()
ms = e0.elapsed_time(e1) / 200
print(f"encode {ms * 1e3:.1f} us  {w * h / ms / 1e6:.1f} Gpix/s", flush=True)
