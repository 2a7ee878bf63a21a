"""Where and when the entropy decode waves ran (tools only): a diag build of
jpegr_entropy (tools/ab/libjpegr_entropy_diag5.so) records per wave its
HW_ID / XCC_ID and s_memrealtime (100 MHz) / s_memtime at start and end.

    python3 tools/ent_diag.py [serial]

serial: the luma and chroma kernels one after the other on one stream
(decoded twice, kernels timed apart)."""
import collections
import ctypes
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["LZ4JPEG_LIB"] = os.path.join(REPO, "tools", "ab", "libjpegr_entropy_diag5.so")
sys.path[:0] = [os.path.join(REPO, "lz4-jpeg_amd")]
import torch  # noqa: E402
from lz4jpeg import _lib, jpeg, synth  # noqa: E402

W, H = 3840, 2160
d_img = torch.from_numpy(synth.rand_rgba(W, H, seed=1)).cuda()
d_coef = jpeg.encode_device(d_img, W, H)
ent = jpeg.Entropy(jpeg.tiles(W, H))
back = torch.empty_like(d_coef)
L = _lib.lib()
ent.encode(d_coef)
for _ in range(3):
    ent.decode(back)
torch.cuda.synchronize()
assert L.jpegr_diag_clear() == 0
ent.decode(back)
torch.cuda.synchronize()
rec = np.zeros((2, 8192, 16), np.uint32)
assert L.jpegr_diag_read(rec.ctypes.data_as(ctypes.c_void_p)) == 0
print("decode ok", bool(torch.equal(back, d_coef)))
t0all = min(int(rec[k, :, 0][rec[k, :, 6] == 1].min()) for k in range(2))
per_simd = collections.Counter()
per_cu = collections.Counter()
for k, name in enumerate(("luma", "chroma")):
    r = rec[k][rec[k, :, 6] == 1]
    t0 = (r[:, 0].astype(np.int64) - t0all) * 10 / 1000.0      # us
    t1 = (r[:, 1].astype(np.int64) - t0all) * 10 / 1000.0
    cyc = (r[:, 3].astype(np.int64) - r[:, 2].astype(np.int64)) & 0xFFFFFFFF
    life = t1 - t0
    hw = r[:, 4]
    simd = (hw >> 4) & 3
    cu = (hw >> 8) & 15
    sh = (hw >> 12) & 1
    se = (hw >> 13) & 7
    xcc = r[:, 5] & 15
    print(f"{name}: waves {len(r)}  start us min {t0.min():.2f} p50 {np.median(t0):.2f} max {t0.max():.2f}"
          f"  end us min {t1.min():.2f} p50 {np.median(t1):.2f} max {t1.max():.2f}"
          f"  life us p10 {np.percentile(life, 10):.2f} p50 {np.median(life):.2f} max {life.max():.2f}"
          f"  cycles/us p50 {np.median(cyc / np.maximum(life, 1e-3)):.0f}")
    keys = list(zip(xcc.tolist(), se.tolist(), sh.tolist(), cu.tolist(), simd.tolist()))
    c = collections.Counter(keys)
    cc = collections.Counter(k4[:4] for k4 in keys)
    for kk, v in c.items():
        per_simd[kk] += v
    for kk, v in cc.items():
        per_cu[kk] += v
    print(f"  {name} SIMDs used {len(c)} waves/SIMD hist {sorted(collections.Counter(c.values()).items())}"
          f"  CUs used {len(cc)} waves/CU hist {sorted(collections.Counter(cc.values()).items())}")
    print(f"  {name} XCCs {sorted(collections.Counter(xcc.tolist()).items())}")
print("both: SIMDs", len(per_simd), "waves/SIMD hist", sorted(collections.Counter(per_simd.values()).items()),
      " CUs", len(per_cu), "waves/CU hist", sorted(collections.Counter(per_cu.values()).items()))

if hasattr(L, "jpegr_ph_read"):
    ph = np.zeros((8192, 8), np.uint32)
    assert L.jpegr_ph_read(ph.ctypes.data_as(ctypes.c_void_p)) == 0
    r = rec[0][rec[0, :, 6] == 1]
    n = len(r)
    ph = ph[:n].astype(np.int64)
    c0 = r[:, 2].astype(np.int64)
    c1 = r[:, 3].astype(np.int64)
    ok = (ph[:, 0] > 0) & (ph[:, 3] > 0)
    d = lambda a, b: ((a - b) & 0xFFFFFFFF)[ok]
    for name, a, b in (("start->stream", ph[:, 0], c0), ("code build", ph[:, 1], ph[:, 0]),
                       ("map build", ph[:, 2], ph[:, 1]), ("walk", ph[:, 3], ph[:, 2]),
                       ("tail+stores", c1, ph[:, 3]), ("whole", c1, c0)):
        x = d(a, b)
        print(f"luma {name:14s} cycles p10 {np.percentile(x, 10):8.0f} p50 {np.median(x):8.0f} max {x.max():8.0f}")
