"""GPU reconstruction (jpegr_reconstruct_device) == the oracle's restatement
of the reference's decode side, which is itself pinned to the reference's
whole JPEG.c pipeline (tests/test_oracle.py)."""
import numpy as np
import pytest

import oracle_api

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("w,h,seed", [(8, 8, 1), (64, 48, 2), (38, 21, 3), (37, 21, 4), (1, 1, 5),
                                      (264, 17, 6), (1200, 630, 7), (3840, 2160, 8)])
def test_reconstruct_matches_oracle(gpu, oracle, w, h, seed):
    import torch
    from lz4jpeg import jpeg
    img = oracle.rand_image(w, h, seed=seed)
    d = torch.from_numpy(np.ascontiguousarray(img)).to(gpu)
    coef = jpeg.encode_device(d, w, h)
    rec = jpeg.reconstruct_device(coef, w, h, d_orig=d).cpu().numpy().reshape(h, w, 4)
    assert np.array_equal(rec, oracle_api.reconstruct(oracle, img))


def test_reconstruct_without_orig_decodes_every_tile(gpu, oracle):
    """d_orig = NULL: trailing tiles are decoded from their coefficients, so
    the result equals decoding every tile (differs from the reference only in
    the ceil(W*H/64) quirk tiles)."""
    import torch
    from lz4jpeg import jpeg
    w, h = 40, 16                     # 10 tiles, ceil(640/64) = 10: no quirk tile
    img = oracle.rand_image(w, h, seed=9)
    d = torch.from_numpy(np.ascontiguousarray(img)).to(gpu)
    coef = jpeg.encode_device(d, w, h)
    a = jpeg.reconstruct_device(coef, w, h).cpu().numpy()
    b = jpeg.reconstruct_device(coef, w, h, d_orig=d).cpu().numpy()
    assert np.array_equal(a, b)


def test_reconstruct_batch(gpu, oracle):
    import torch
    from lz4jpeg import jpeg
    w, h, n = 48, 40, 3
    imgs = [oracle.rand_image(w, h, seed=20 + i) for i in range(n)]
    d = torch.from_numpy(np.ascontiguousarray(np.stack(imgs))).to(gpu)
    coef = jpeg.encode_device(d, w, h, nimg=n)
    rec = jpeg.reconstruct_device(coef, w, h, nimg=n, d_orig=d).cpu().numpy().reshape(n, h, w, 4)
    for i in range(n):
        assert np.array_equal(rec[i], oracle_api.reconstruct(oracle, imgs[i]))
