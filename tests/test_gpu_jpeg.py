"""HIP JPEG path vs the pinned oracle: quantised int16 coefficients bit-exact
(md5 fixtures up to 3840x2160, the 8x8 literal KAT, odd sizes), the
un-quantised fp64 DCT bit-exact, and batches.  All calls go through the C ABI."""
import hashlib
import json
import os

import numpy as np
import pytest

import golden_inputs

pytestmark = pytest.mark.gpu

GOLDEN = json.load(open(os.path.join(golden_inputs.GOLDEN, "golden.json")))


def _enc(img, nimg=1):
    import torch
    from lz4jpeg import jpeg
    h, w = img.shape[-3], img.shape[-2]
    d = torch.from_numpy(np.ascontiguousarray(img)).cuda()
    out = jpeg.encode_device(d, w, h, nimg)
    torch.cuda.synchronize()
    return out.cpu().numpy()


@pytest.mark.parametrize("e", GOLDEN["jpeg"], ids=lambda e: f'{e["w"]}x{e["h"]}')
def test_golden_md5(gpu, e):
    from lz4jpeg import synth
    img = synth.rand_rgba(e["w"], e["h"], e["seed"])
    got = _enc(img).tobytes()
    assert len(got) == e["bytes"]
    assert hashlib.md5(got).hexdigest() == e["md5"]


def test_kat_8x8(gpu):
    from lz4jpeg import synth
    got = _enc(synth.rand_rgba(8, 8, 1))
    kat = GOLDEN["jpeg_kat_8x8"]
    assert list(got[:64]) == kat["Y"]
    assert list(got[64:96]) == kat["Cr"]
    assert list(got[96:]) == kat["Cb"]


@pytest.mark.parametrize("w,h", [(8, 8), (16, 8), (24, 40), (256, 8), (264, 16), (9, 9),
                                 (13, 7), (1, 1), (3, 300), (301, 3), (517, 129), (1000, 1000)])
def test_sizes_vs_oracle(gpu, oracle, w, h):
    rng = np.random.default_rng(w * 1000 + h)
    img = rng.integers(0, 256, (h, w, 4), dtype=np.uint8)
    assert (_enc(img) == oracle.jpeg_encode(img)).all()


@pytest.mark.parametrize("w,h", [(64, 64), (72, 24), (9, 17)])
def test_raw_dct_bit_exact(gpu, oracle, w, h):
    import torch
    from lz4jpeg import jpeg
    rng = np.random.default_rng(3)
    img = rng.integers(0, 256, (h, w, 4), dtype=np.uint8)
    d = torch.from_numpy(img).cuda()
    got = jpeg.dct_raw_device(d, w, h).cpu().numpy()
    assert got.tobytes() == oracle.jpeg_dct_raw(img).tobytes()


def test_extreme_pixels(gpu, oracle):
    """Saturated colours hit the Cr/Cb clamps and exact-integer quotients."""
    vals = np.array([0, 1, 127, 128, 254, 255], np.uint8)
    rng = np.random.default_rng(9)
    img = vals[rng.integers(0, vals.size, (64, 64, 4))]
    assert (_enc(img) == oracle.jpeg_encode(img)).all()
    for c in [(255, 0, 0), (0, 255, 0), (0, 0, 255), (255, 255, 255), (0, 0, 0)]:
        img = np.zeros((16, 16, 4), np.uint8)
        img[..., :3] = c
        assert (_enc(img) == oracle.jpeg_encode(img)).all(), c


def test_batch_equals_singles(gpu, oracle):
    from lz4jpeg import synth
    imgs = np.stack([synth.rand_rgba(264, 40, seed=s) for s in (1, 2, 3, 4)])
    got = _enc(imgs, nimg=4).reshape(4, -1)
    for i in range(4):
        assert (got[i] == oracle.jpeg_encode(imgs[i])).all()


def test_batch_odd_strip_count(gpu, oracle):
    # a batched launch whose images each end in a ragged strip: a 200x24
    # image is 3 tile rows of 25 tiles, i.e. one short strip (25 of 32 tiles)
    # per row, and the strips of image k + 1 follow image k's in one grid
    from lz4jpeg import synth
    imgs = np.stack([synth.rand_rgba(200, 24, seed=s) for s in (7, 8, 9)])
    got = _enc(imgs, nimg=3).reshape(3, -1)
    for i in range(3):
        assert (got[i] == oracle.jpeg_encode(imgs[i])).all()
        assert (got[i] == _enc(imgs[i])).all()


def test_host_api(gpu, oracle):
    from lz4jpeg import jpeg, synth
    img = synth.rand_rgba(120, 80, seed=5)
    assert (jpeg.encode(img).ravel() == oracle.jpeg_encode(img)).all()
