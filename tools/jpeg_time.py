"""A/B timing of the JPEG encoder (LZ4JPEG_LIB selects the build): one 4K
image per launch after 100 ms of settling load (the clock ramps over ~40 ms,
DESIGN §4.2), 1000 launches; then 64 images per launch.  Prints us/image."""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "lz4-jpeg_amd")]
import torch  # noqa: E402
from lz4jpeg import jpeg, synth  # noqa: E402

w, h = 3840, 2160
d = torch.empty(4 * w * h * 64, dtype=torch.uint8, device="cuda")
synth.rand_rgba_device(d, 0, w * h * 64, seed=1)
out = torch.empty(64 * jpeg.coef_count(w, h), dtype=torch.int16, device="cuda")
for b, reps in ((1, 1000), (64, 20)):
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 0.1:
        for _ in range(20):
            jpeg.encode_device(d, w, h, b, out)
        torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        jpeg.encode_device(d, w, h, b, out)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    print(f"images {b:3d}: {ms * 1e3 / b:7.2f} us/image  {w * h * b / ms / 1e6:7.1f} Gpix/s",
          flush=True)
