"""Compress the bench corpus once, then run the GPU decoder a few times (for
profilers), on the compressor's device-resident block offsets, and the
bare-stream decode (block boundaries found on the device) as often."""
import time
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "lz4-jpeg_amd")]
import torch  # noqa: E402
from lz4jpeg import lz4, synth  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 30
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
d_in = torch.from_numpy(synth.random_passages(n, length=30000, seed=1)).cuda()
c = lz4.Compressor()
d_stream, length = c.compress_device(d_in)
nb = (n + 299) // 300
d_offs, _ = c.block_offsets_device()          # written by the placement kernel
d_out = torch.empty(n + 300, dtype=torch.uint8, device="cuda")
for _ in range(reps):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    lz4.decompress_device(d_stream, length, d_offs, nb, n + 300, d_out=d_out, check=False)
    e1.record()
    torch.cuda.synchronize()
    print(f"decode ms {e0.elapsed_time(e1):.3f}", flush=True)
_, got = lz4.decompress_device(d_stream, length, d_offs, nb, n + 300, d_out=d_out)
print("ok", got == n and bool(torch.equal(d_out[:n], d_in)))
for _ in range(reps):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    _, got = lz4.decompress_stream_device(d_stream, length, n + 300, d_out=d_out)
    print(f"bare-stream call ms {(time.perf_counter() - t0) * 1e3:.3f}", flush=True)
print("bare ok", got == n and bool(torch.equal(d_out[:n], d_in)))
c.close()
