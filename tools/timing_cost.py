"""What the per-call timing events cost the bench's stream-ordered steps
(tools only): 1 GiB compress, 40 warm-up calls, then alternating blocks of
K back-to-back async calls with the library's timing on / off, wall time per
call between synchronizes.

    python3 tools/timing_cost.py [K] [blocks]"""
import os
import statistics
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "lz4-jpeg_amd")]
import torch  # noqa: E402
from lz4jpeg import lz4, synth  # noqa: E402

K = int(sys.argv[1]) if len(sys.argv) > 1 else 20
B = int(sys.argv[2]) if len(sys.argv) > 2 else 6
n = 1 << 30
d_in = torch.empty(n + 16, dtype=torch.uint8, device="cuda")
synth.random_passages_device(d_in, n, length=30000, seed=1)
c = lz4.Compressor()
d_out = torch.empty(n + n // 8 + (1 << 20), dtype=torch.uint8, device="cuda")
d_len = torch.zeros(1, dtype=torch.int64, device="cuda")
for _ in range(40):
    c.compress_async(d_in, n, d_out, d_len)
torch.cuda.synchronize()
res = {True: [], False: []}
for b in range(B):
    on = b % 2 == 0
    c.set_timing(on)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(K):
        c.compress_async(d_in, n, d_out, d_len)
    torch.cuda.synchronize()
    res[on].append((time.perf_counter() - t0) / K * 1e3)
    if on:
        calls, tiles = c.timed_calls(K)
        print(f"timing on : wall {res[on][-1]:.4f} ms/call, events call {statistics.median(calls):.4f} "
              f"tiles {statistics.median(tiles):.4f}", flush=True)
    else:
        print(f"timing off: wall {res[on][-1]:.4f} ms/call", flush=True)
print(f"median wall: on {statistics.median(res[True]):.4f}  off {statistics.median(res[False]):.4f} ms/call")
