#!/usr/bin/env python3
"""Writes tests/golden/fullsize.json: md5s of the WHOLE outputs of the
full-size workloads, computed by the CPU oracle (oracle/liboracle.so, its
pthread encoders), so that the GPU tests compare every byte of:

  config2      BASELINE config 2: the framed LZ4 stream of 1 GiB of
               random_extract-style text (synth.random_passages, seed 1)
               -- the reference's block loop LZ4.c:707-721 + write_output
  config4_r7   BASELINE config 4 as rank 7 of 8 sees it: the segment (no
               frame byte) of the whole-block shard [lo, hi) of the 64 GiB
               corpus (dist.shard_bytes), which holds the globally last block
  config5_r7   BASELINE config 5 as rank 7 of 8 sees it: the int16 coefficient
               output of images 896..1023 of the continuous rand() stream
               (3840x2160 each) -- JPEG.c:1136-1178 per image

Source "oracle": our restatement, pinned to the reference by golden.json
(make_golden.py).  Inputs are generated in slices (memory stays ~1 GB); the
LZ4 slices are whole 300-byte blocks, so the concatenation of the slices'
block encodings is the stream.  About 5 minutes on 8 cores.

Run from the repo root:  python tests/golden/make_fullsize.py
"""
import ctypes
import hashlib
import json
import os
import sys
import threading
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [os.path.dirname(HERE), os.path.join(REPO, "lz4-jpeg_amd")]
import oracle_api  # noqa: E402
from lz4jpeg import dist, synth  # noqa: E402

THREADS = int(os.environ.get("THREADS", os.cpu_count() or 8))
SLICE = 300 * (1 << 20)          # 314.6 MB of input per slice (whole blocks)
W4K, H4K = 3840, 2160


def lz4_blocks_parallel(o, data):
    """Block encodings of every block of `data` (whole 300-B blocks but the
    last), concatenated: THREADS ctypes calls of lz4o_encode_blocks (ctypes
    releases the GIL)."""
    nb = (data.size + 299) // 300
    per = (nb + THREADS - 1) // THREADS
    parts = [None] * THREADS

    def work(t):
        b0, b1 = min(t * per, nb), min((t + 1) * per, nb)
        parts[t] = o.lz4_blocks(data, b0, b1) if b1 > b0 else b""

    ths = [threading.Thread(target=work, args=(t,)) for t in range(THREADS)]
    for th in ths:
        th.start()
    for th in ths:
        th.join()
    return b"".join(parts)


def lz4_md5(o, lo, hi, framed, total_blocks=None):
    h = hashlib.md5()
    length = 0
    if framed:
        h.update(bytes([total_blocks & 0xFF]))
        length = 1
    for a in range(lo, hi, SLICE):
        b = min(a + SLICE, hi)
        data = synth.random_passages(b - a, length=30000, seed=1, first=a)
        enc = lz4_blocks_parallel(o, data)
        h.update(enc)
        length += len(enc)
        print(f"  lz4 [{a - lo:,} .. {b - lo:,}) of {hi - lo:,}", flush=True)
    return h.hexdigest(), length


def main():
    o = oracle_api.load()
    out = {}
    t0 = time.time()
    n2 = 1 << 30
    md5, ln = lz4_md5(o, 0, n2, True, (n2 + 299) // 300)
    out["config2"] = {"n": n2, "seed": 1, "passage": 30000, "out_len": ln, "md5": md5,
                      "source": "oracle"}
    print("config2", out["config2"], f"{time.time() - t0:.0f}s", flush=True)
    n4, world, rank = 64 << 30, 8, 7
    lo, hi = dist.shard_bytes(n4, world, rank)
    md5, ln = lz4_md5(o, lo, hi, False)
    out["config4_r7"] = {"n_total": n4, "world": world, "rank": rank, "lo": lo, "hi": hi,
                         "seed": 1, "passage": 30000, "seg_len": ln, "md5": md5,
                         "source": "oracle"}
    print("config4_r7", out["config4_r7"], f"{time.time() - t0:.0f}s", flush=True)
    first, count = 896, 128
    px = W4K * H4K
    h = hashlib.md5()
    for k in range(count):
        img = synth.rand_rgba_stream((first + k) * px, px, 1).reshape(H4K, W4K, 4)
        h.update(o.jpeg_encode(img, threads=THREADS).tobytes())
        if k % 16 == 15:
            print(f"  jpeg image {first + k}", flush=True)
    out["config5_r7"] = {"w": W4K, "h": H4K, "first_image": first, "count": count, "seed": 1,
                         "bytes": count * (W4K // 8) * (H4K // 8) * 256, "md5": h.hexdigest(),
                         "source": "oracle"}
    print("config5_r7", out["config5_r7"], f"{time.time() - t0:.0f}s", flush=True)
    with open(os.path.join(HERE, "fullsize.json"), "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
