"""Run the LZ4 compressor a few times on the 1 GiB bench corpus (for profilers)."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "lz4-jpeg_amd")]
import torch  # noqa: E402
from lz4jpeg import lz4, synth  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 30
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
host = synth.random_passages(n, length=30000, seed=1)
d_in = torch.from_numpy(host).cuda()
c = lz4.Compressor()
d_out = torch.empty(lz4.compress_bound(n), dtype=torch.uint8, device="cuda")
c.set_timing(True)
for _ in range(reps):
    _, got = c.compress_device(d_in, n, d_out)
    print("len", got, "ms", c.last_timing(), flush=True)
c.close()
