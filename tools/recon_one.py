"""Time the JPEG reconstruction kernel (coefficients -> RGBA) on one 3840x2160
random image: median of HIP-event-timed batches of launches.  LZ4JPEG_LIB
selects an A/B build."""
import os
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "lz4-jpeg_amd")]
import torch  # noqa: E402
from lz4jpeg import jpeg, synth  # noqa: E402

w, h = 3840, 2160
img = torch.from_numpy(synth.rand_rgba(w, h, seed=1)).cuda()
coef = torch.empty(jpeg.coef_count(w, h), dtype=torch.int16, device="cuda")
jpeg.encode_device(img, w, h, 1, coef)
out = jpeg.reconstruct_device(coef, w, h, 1, d_orig=img)
torch.cuda.synchronize()
ts = []
for _ in range(7):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(50):
        jpeg.reconstruct_device(coef, w, h, 1, d_orig=img)
    e1.record()
    torch.cuda.synchronize()
    ts.append(e0.elapsed_time(e1) / 50)
ms = statistics.median(ts)
print(f"reconstruct {ms * 1e3:.1f} us  {w * h / ms / 1e6:.1f} Gpix/s", flush=True)
