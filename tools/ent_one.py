"""Entropy stage on a 4K random image, a few reps (for profilers)."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "lz4-jpeg_amd")]
import torch  # noqa: E402
from lz4jpeg import jpeg, synth  # noqa: E402

W, H = 3840, 2160
reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
d_img = torch.from_numpy(synth.rand_rgba(W, H, seed=1)).cuda()
d_coef = jpeg.encode_device(d_img, W, H)
ent = jpeg.Entropy(jpeg.tiles(W, H))
back = torch.empty_like(d_coef)
for _ in range(reps):
    e0, e1, e2 = (torch.cuda.Event(enable_timing=True) for _ in range(3))
    e0.record()
    ent.encode(d_coef)
    e1.record()
    ent.decode(back)
    e2.record()
    torch.cuda.synchronize()
    print(f"encode ms {e0.elapsed_time(e1):.4f} decode ms {e1.elapsed_time(e2):.4f}", flush=True)
print("ok", bool(torch.equal(back, d_coef)), ent.status.tolist())
