"""Run the LZ4 compressor on the 1 GiB bench corpus (for profilers and A/B
timing): `reps` calls after 3 warm-up calls; prints each call's (whole call,
lz4_tiles) ms and, last, the medians, with the host wall time of a step (the
call and its length read-back, as bench.py's step)."""
import os
import statistics
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "lz4-jpeg_amd")]
import torch  # noqa: E402
from lz4jpeg import lz4, synth  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 30
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
warm = int(sys.argv[3]) if len(sys.argv) > 3 else 3
d_in = torch.empty(n + 16, dtype=torch.uint8, device="cuda")
synth.random_passages_device(d_in, n, length=30000, seed=1)
c = lz4.Compressor()
d_out = torch.empty(n + n // 8 + (1 << 20), dtype=torch.uint8, device="cuda")
for _ in range(warm):
    c.compress_device(d_in, n, d_out)
c.set_timing(True)
calls, tiles, steps = [], [], []
for _ in range(reps):
    t0 = time.perf_counter()
    _, got = c.compress_device(d_in, n, d_out)
    a, b = c.last_timing()
    steps.append((time.perf_counter() - t0) * 1e3)
    calls.append(a)
    tiles.append(b)
    print("len", got, "ms", (a, b), flush=True)
print(f"median call {statistics.median(calls):.4f} ms, lz4_tiles {statistics.median(tiles):.4f} ms, "
      f"step {statistics.median(steps):.4f} ms")
c.close()
