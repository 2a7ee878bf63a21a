"""JPEG encoder time per 3840x2160 image vs images per launch (1 .. 64), from
HIP events over back-to-back launches; images drawn from the rand() stream
in HBM.  LZ4JPEG_LIB selects an A/B build."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "lz4-jpeg_amd")]
import torch  # noqa: E402
from lz4jpeg import jpeg, synth  # noqa: E402

w, h = 3840, 2160
counts = [int(x) for x in sys.argv[1:]] or [1, 2, 4, 16, 64]
maxb = max(counts)
d = torch.empty(4 * w * h * maxb, dtype=torch.uint8, device="cuda")
synth.rand_rgba_device(d, 0, w * h * maxb, seed=1)
out = torch.empty(maxb * jpeg.coef_count(w, h), dtype=torch.int16, device="cuda")
for b in counts:
    reps = max(10, 400 // b)
    for _ in range(5):
        jpeg.encode_device(d, w, h, b, out)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        jpeg.encode_device(d, w, h, b, out)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    print(f"images {b:4d}: {ms * 1e3 / b:7.2f} us/image  {w * h * b / ms / 1e6:7.1f} Gpix/s",
          flush=True)
