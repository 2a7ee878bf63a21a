"""Entropy stage timing on one 3840x2160 image (encode / decode ms, mean of 50
after warm-up) and round-trip check; LZ4JPEG_LIB selects an A/B build."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "lz4-jpeg_amd")]
import torch  # noqa: E402
from lz4jpeg import jpeg, synth  # noqa: E402

W, H = 3840, 2160
d_img = torch.empty(4 * W * H, dtype=torch.uint8, device="cuda")
synth.rand_rgba_device(d_img, 0, W * H, seed=1)
d_coef = jpeg.encode_device(d_img, W, H)
ent = jpeg.Entropy(jpeg.tiles(W, H))
back = torch.empty_like(d_coef)
for _ in range(5):
    ent.encode(d_coef)
    ent.decode(back)
reps = 50
e0, e1, e2 = (torch.cuda.Event(enable_timing=True) for _ in range(3))
e0.record()
for _ in range(reps):
    ent.encode(d_coef)
e1.record()
for _ in range(reps):
    ent.decode(back)
e2.record()
torch.cuda.synchronize()
print(f"encode {e0.elapsed_time(e1) / reps:.4f} ms  decode {e1.elapsed_time(e2) / reps:.4f} ms  "
      f"roundtrip {bool(torch.equal(back, d_coef))} status {ent.status.tolist()}", flush=True)
