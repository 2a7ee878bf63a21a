"""GPU entropy stage (jpegr_entropy_encode_device / _decode_device, SURVEY.md
§8 f2) against the reference: the committed known answers made by the
reference's own RLE / encode_huffman / generate_encoded_sequence
(tests/golden/entropy.json), the pinned oracle on whole images, and the
decode round trip (the reference's decode_huffman + inverse_RLE is the
identity on every stream).  All calls go through the C ABI."""
import json
import os

import numpy as np
import pytest

import golden_inputs
import oracle_api

pytestmark = pytest.mark.gpu

VECS = json.load(open(os.path.join(golden_inputs.GOLDEN, "entropy.json")))


def _codes_from_lengths(lens):
    out, code, plen = [], 0, 0
    for k, L in enumerate(lens):
        if k:
            code = (code + 1) << (L - plen) if L >= plen else (code + 1) >> (plen - L)
        plen = L
        out.append(code)
    return out


def _pack(vecs):
    """Tiles whose streams are the given vectors (64-int ones in Y slots,
    32-int ones in Cr, then Cb); returns (coef int16 array, placement)."""
    ys = [v for v in vecs if len(v["zz"]) == 64]
    cs = [v for v in vecs if len(v["zz"]) == 32]
    ntiles = max(len(ys), (len(cs) + 1) // 2)
    coef = np.zeros((ntiles, 128), np.int16)
    place = []
    for t, v in enumerate(ys):
        coef[t, :64] = v["zz"]
        place.append((v, t, 0))
    for i, v in enumerate(cs):
        t, c = i // 2, 1 + i % 2
        coef[t, 64 + 32 * (c - 1): 96 + 32 * (c - 1)] = v["zz"]
        place.append((v, t, c))
    return coef, place


def test_golden_vectors(gpu):
    import torch
    from lz4jpeg import jpeg
    coef, place = _pack(VECS)
    d_coef = torch.from_numpy(coef.reshape(-1)).cuda()
    ent = jpeg.Entropy(coef.shape[0])
    ent.encode(d_coef)
    torch.cuda.synchronize()
    assert int(ent.status[0].item()) == 0
    for v, t, c in place:
        got = ent.stream(t, c)
        assert got["rle_len"] == v["rle_len"], v["name"]
        want = [(val, ln) for val, ln, _ in v["table"]]
        assert got["table"] == want, v["name"]
        assert _codes_from_lengths([ln for _, ln in want]) == [int(x) for _, _, x in v["table"]]
        assert got["nbits"] == v["nbits"], v["name"]
        assert got["bits"].hex() == v["bits"], v["name"]
    out = torch.full_like(d_coef, 12345)
    ent.decode(out)
    torch.cuda.synchronize()
    assert int(ent.status[1].item()) == 0
    assert torch.equal(out, d_coef)


def test_deferred_and_slow_paths(gpu, oracle):
    """> 32 distinct symbols (second pass over global scratch) and > 64 codes
    (decode without the LDS table), against the oracle."""
    import torch
    from lz4jpeg import jpeg
    streams = [list(range(100, 164)), list(range(-40, 24)), [(-1) ** i * (i % 37) for i in range(64)],
               list(range(0, 64, 2)) * 2]
    coef = np.zeros((len(streams), 128), np.int16)
    for t, zz in enumerate(streams):
        coef[t, :64] = zz
        coef[t, 64:96] = np.arange(32) - 16
        coef[t, 96:] = np.arange(32) * 3
    d_coef = torch.from_numpy(coef.reshape(-1)).cuda()
    ent = jpeg.Entropy(coef.shape[0])
    ent.encode(d_coef)
    torch.cuda.synchronize()
    assert int(ent.status[0].item()) == 0
    for t in range(coef.shape[0]):
        for c, sl in ((0, slice(0, 64)), (1, slice(64, 96)), (2, slice(96, 128))):
            a = oracle_api.entropy(oracle, coef[t, sl])
            got = ent.stream(t, c)
            assert got["table"] == [(v, ln) for v, ln, _ in a["table"]], (t, c)
            assert (got["nbits"], got["bits"]) == (a["nbits"], a["bits"]), (t, c)
    out = torch.zeros_like(d_coef)
    ent.decode(out)
    torch.cuda.synchronize()
    assert int(ent.status[1].item()) == 0
    assert torch.equal(out, d_coef)


@pytest.mark.parametrize("w,h,kind", [(3840, 2160, "rand"), (512, 384, "smooth"), (40, 24, "rand")])
def test_image_vs_oracle_and_roundtrip(gpu, oracle, w, h, kind):
    import torch
    from lz4jpeg import jpeg
    if kind == "rand":
        img = oracle.rand_image(w, h, seed=1)
    else:
        yy, xx = np.mgrid[0:h, 0:w]
        img = np.ascontiguousarray(np.stack([(xx // 3) % 256, (yy // 2) % 256,
                                             ((xx + yy) // 5) % 256, np.full_like(xx, 255)],
                                            -1).astype(np.uint8))
    d_img = torch.from_numpy(img).cuda()
    d_coef = jpeg.encode_device(d_img, w, h)
    nt = jpeg.tiles(w, h)
    ent = jpeg.Entropy(nt)
    ent.encode(d_coef)
    coef = d_coef.cpu().numpy().reshape(-1, 128)
    torch.cuda.synchronize()
    assert int(ent.status[0].item()) == 0
    rng = np.random.default_rng(3)
    for t in np.unique(np.concatenate([[0, nt - 1], rng.integers(0, nt, 200)])):
        for c, sl in ((0, slice(0, 64)), (1, slice(64, 96)), (2, slice(96, 128))):
            a = oracle_api.entropy(oracle, coef[t, sl])
            got = ent.stream(int(t), c)
            assert got["rle_len"] == len(a["rle"])
            assert got["table"] == [(v, ln) for v, ln, _ in a["table"]], (t, c)
            assert (got["nbits"], got["bits"]) == (a["nbits"], a["bits"]), (t, c)
    out = torch.zeros_like(d_coef)
    ent.decode(out)
    torch.cuda.synchronize()
    assert int(ent.status[1].item()) == 0
    assert torch.equal(out, d_coef)


def _boundary_streams():
    """Luma (64-int) and chroma (32-int) streams at the fast encoder's edges:
    the direct symbol table's key range (luma -64..111, chroma -48..71; one
    past either end is deferred), the distinct-symbol caps (24 / 12; one more
    is deferred), whole-stream runs (count 64 / 32), counts equal to values,
    and symbols met first as a value and later as a count."""
    luma = [
        [-64, 111] * 32, [-65] + [0] * 63, [112] + [1] * 63, [5] * 64, [0] * 64,
        [10 + (i % 23) for i in range(64)],                 # 24 distinct: count 1 + 23 values
        [10 + (i % 24) for i in range(64)],                 # 25: deferred
        [3, 3, 3] + [1] * 61, [2, 2, 7, 7, 7, 2] + [0] * 58,
        [1, 2, 2, 3, 3, 3, 4, 4, 4, 4] * 6 + [-1] * 4,
        [(i * 7) % 5 - 2 for i in range(64)],
    ]
    chroma = [
        [-48, 71] * 16, [-49] + [0] * 31, [72] + [0] * 31, [9] * 32,
        [20 + (i % 11) for i in range(32)],                 # 12 distinct
        [20 + (i % 12) for i in range(32)],                 # 13: deferred
        [2, 2, 1, 1, 1, 3] + [0] * 26, [(i * 3) % 4 - 1 for i in range(32)],
    ]
    return luma, chroma


def test_fast_path_boundaries(gpu, oracle):
    import torch
    from lz4jpeg import jpeg
    luma, chroma = _boundary_streams()
    nt = 70                                  # a second, partial wave of tiles
    rng = np.random.default_rng(11)
    coef = rng.integers(-3, 4, size=(nt, 128)).astype(np.int16)
    for t, zz in enumerate(luma):
        coef[t, :64] = zz
    for i, zz in enumerate(chroma):
        coef[i, 64:96] = zz
        coef[nt - 1 - i, 96:] = zz
    d_coef = torch.from_numpy(coef.reshape(-1)).cuda()
    ent = jpeg.Entropy(nt)
    ent.encode(d_coef)
    torch.cuda.synchronize()
    assert int(ent.status[0].item()) == 0
    for t in range(nt):
        for c, sl in ((0, slice(0, 64)), (1, slice(64, 96)), (2, slice(96, 128))):
            a = oracle_api.entropy(oracle, coef[t, sl])
            got = ent.stream(t, c)
            assert got["rle_len"] == len(a["rle"]), (t, c)
            assert got["table"] == [(v, ln) for v, ln, _ in a["table"]], (t, c)
            assert (got["nbits"], got["bits"]) == (a["nbits"], a["bits"]), (t, c)
    out = torch.zeros_like(d_coef)
    ent.decode(out)
    torch.cuda.synchronize()
    assert int(ent.status[1].item()) == 0
    assert torch.equal(out, d_coef)


def test_decode_counts_malformed_streams(gpu, oracle):
    """status[1] counts exactly the malformed streams of one call -- truncated
    bits (nbits - 1), a wrong RLE length, a meta word past the slot -- in
    workgroup 0 and later ones, is not carried into the next call, and the
    other streams still decode (the decoder zeroes status[1] itself; the
    call's tag in status[2] orders the adds after the zero)."""
    import torch
    from lz4jpeg import jpeg
    w, h = 512, 384
    img = oracle.rand_image(w, h, seed=5)
    d_coef = jpeg.encode_device(torch.from_numpy(img).cuda(), w, h)
    nt = jpeg.tiles(w, h)
    ent = jpeg.Entropy(nt)
    ent.encode(d_coef)
    torch.cuda.synchronize()
    clean = ent.meta.clone()
    meta = clean.cpu().numpy().view(np.uint32).reshape(nt, 3).copy()
    nbits, rle, ncodes = meta & 0xFFFF, (meta >> 16) & 255, meta >> 24
    bad = set()
    for t in (0, 1, 63, 64, 777, nt - 1):                  # truncated luma bits
        assert ncodes[t, 0] > 1 and nbits[t, 0] > 1
        meta[t, 0] -= 1
        bad.add((t, 0))
    for t in (2, 65, 1500, nt - 2):                        # Cr: two RLE ints too many
        assert ncodes[t, 1] > 1
        meta[t, 1] += 2 << 16
        bad.add((t, 1))
    for t in (3, 2000):                                    # Cb: bits past its slot
        meta[t, 2] = (meta[t, 2] & ~np.uint32(0xFFFF)) | np.uint32(600)
        bad.add((t, 2))
    ent.meta.copy_(torch.from_numpy(meta.reshape(-1).view(np.int32)))
    coef = d_coef.view(nt, 128)
    for _ in range(2):                                     # not accumulated over calls
        out = torch.zeros_like(d_coef)
        ent.decode(out)
        torch.cuda.synchronize()
        assert int(ent.status[1].item()) == len(bad)
        ok_rows = torch.ones(nt, dtype=torch.bool, device="cuda")
        ok_rows[sorted({t for t, _ in bad})] = False
        assert torch.equal(out.view(nt, 128)[ok_rows], coef[ok_rows])
    ent.meta.copy_(clean)
    out = torch.zeros_like(d_coef)
    ent.decode(out)
    torch.cuda.synchronize()
    assert int(ent.status[1].item()) == 0
    assert torch.equal(out, d_coef)
