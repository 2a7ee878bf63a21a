"""Single-image JPEG launch time over a long run of back-to-back launches:
the mean of every 100 launches (HIP events), to see whether the per-launch
time settles (DVFS) and after how many launches."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "lz4-jpeg_amd")]
import torch  # noqa: E402
from lz4jpeg import jpeg, synth  # noqa: E402

w, h = 3840, 2160
nblk = int(sys.argv[1]) if len(sys.argv) > 1 else 30
d = torch.empty(4 * w * h, dtype=torch.uint8, device="cuda")
synth.rand_rgba_device(d, 0, w * h, seed=1)
out = torch.empty(jpeg.coef_count(w, h), dtype=torch.int16, device="cuda")
ev = [torch.cuda.Event(enable_timing=True) for _ in range(nblk + 1)]
ev[0].record()
for b in range(nblk):
    for _ in range(100):
        jpeg.encode_device(d, w, h, 1, out)
    ev[b + 1].record()
torch.cuda.synchronize()
print(" ".join(f"{ev[b].elapsed_time(ev[b + 1]) * 10:.1f}" for b in range(nblk)), flush=True)
