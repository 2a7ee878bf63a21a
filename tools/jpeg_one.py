"""Run the JPEG encoder a few times on 3840x2160 random images (for profilers):
jpeg_one.py [reps] [images per launch]."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "lz4-jpeg_amd")]
import torch  # noqa: E402
from lz4jpeg import jpeg, synth  # noqa: E402

w, h = 3840, 2160
reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
nimg = int(sys.argv[2]) if len(sys.argv) > 2 else 1
if nimg == 1:
    img = torch.from_numpy(synth.rand_rgba(w, h, seed=1)).cuda()
else:
    img = torch.empty(4 * w * h * nimg, dtype=torch.uint8, device="cuda")
    synth.rand_rgba_device(img, 0, w * h * nimg, seed=1)
out = torch.empty(nimg * jpeg.coef_count(w, h), dtype=torch.int16, device="cuda")
for _ in range(reps):
    jpeg.encode_device(img, w, h, nimg, out)
torch.cuda.synchronize()
print("ok", flush=True)
