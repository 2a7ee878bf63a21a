"""The entropy-stage oracle (oracle/jpeg_entropy_oracle.c, a restatement of
JPEG.c:767-1097) against the reference's own functions: the committed known
answers (tests/golden/entropy.json, made by make_golden.py from the
reference's RLE / encode_huffman / generate_encoded_sequence) and, where the
reference build exists, live comparisons on further tiles.  CPU only."""
import json
import os

import numpy as np
import pytest

import golden_inputs
import oracle_api

VECS = json.load(open(os.path.join(golden_inputs.GOLDEN, "entropy.json")))


@pytest.mark.parametrize("v", VECS, ids=lambda v: v["name"])
def test_oracle_matches_reference_vectors(oracle, v):
    a = oracle_api.entropy(oracle, v["zz"])
    assert a["rc"] == 0
    assert len(a["rle"]) == v["rle_len"]
    assert [[t[0], t[1], str(t[2])] for t in a["table"]] == v["table"]
    assert a["nbits"] == v["nbits"]
    assert a["bits"].hex() == v["bits"]
    assert oracle_api.entropy_decode(oracle, a, len(v["zz"])) == v["zz"]


def _textbook_lengths(rle):
    """Code lengths from the same construction with a correct insert (the
    merged node sifted up), for comparison."""
    syms, cnt = [], {}
    for s in rle:
        if s not in cnt:
            syms.append(s)
            cnt[s] = 0
        cnt[s] += 1
    nodes = [(cnt[s], s, None, None) for s in syms]
    heap = list(range(len(nodes)))

    def down(size, i):
        while True:
            m, l, r = i, 2 * i + 1, 2 * i + 2
            if l < size and nodes[heap[l]][0] < nodes[heap[m]][0]:
                m = l
            if r < size and nodes[heap[r]][0] < nodes[heap[m]][0]:
                m = r
            if m == i:
                return
            heap[i], heap[m] = heap[m], heap[i]
            i = m
    for i in range(len(heap) // 2 - 1, -1, -1):
        down(len(heap), i)
    while len(heap) > 1:
        lo = heap[0]; heap[0] = heap[-1]; heap.pop(); down(len(heap), 0)
        hi = heap[0]; heap[0] = heap[-1]; heap.pop(); down(len(heap), 0)
        nodes.append((nodes[lo][0] + nodes[hi][0], None, lo, hi))
        heap.append(len(nodes) - 1)
        i = len(heap) - 1
        while i and nodes[heap[(i - 1) // 2]][0] > nodes[heap[i]][0]:
            heap[i], heap[(i - 1) // 2] = heap[(i - 1) // 2], heap[i]
            i = (i - 1) // 2
    out = {}

    def walk(k, d):
        c, s, l, r = nodes[k]
        if s is not None:
            out[s] = d
        else:
            walk(l, d + 1)
            walk(r, d + 1)
    walk(heap[0], 0)
    return out


def test_heap_quirk_is_exercised():
    """The merged node is appended without sifting up (JPEG.c:959-960): the
    committed reference tables include ones a correct insert would not build."""
    differ = 0
    for v in VECS:
        zz = v["zz"]
        rle, cur, cnt = [], zz[0], 1
        for x in zz[1:] + [None]:
            if x == cur:
                cnt += 1
            else:
                rle += [cnt, cur]
                cur, cnt = x, 1
        ref_lens = {t[0]: t[1] for t in v["table"]}
        if _textbook_lengths(rle) != ref_lens:
            differ += 1
    assert differ > 0


def test_oracle_vs_reference_live(oracle):
    """More tiles (random and smooth images) against the live reference build."""
    if oracle_api.ref_jpeg() is None:
        pytest.skip("oracle/_ref not built (no reference tree)")
    rng = np.random.default_rng(3)
    imgs = [oracle.rand_image(64, 32, seed=9)]
    yy, xx = np.mgrid[0:48, 0:64]
    smooth = np.stack([(xx * 4) % 256, (yy * 5) % 256, ((xx + yy) * 2) % 256,
                       np.full_like(xx, 255)], -1).astype(np.uint8)
    imgs.append(np.ascontiguousarray(smooth))
    imgs.append(rng.integers(0, 256, (16, 16, 4), dtype=np.uint8))
    n = 0
    for img in imgs:
        for t in oracle.jpeg_encode(img).reshape(-1, 128):
            for sl in (slice(0, 64), slice(64, 96), slice(96, 128)):
                zz = t[sl]
                a, r = oracle_api.entropy(oracle, zz), oracle_api.ref_entropy(zz)
                assert (a["rle"], a["table"], a["nbits"], a["bits"]) == \
                    (r["rle"], r["table"], r["nbits"], r["bits"])
                assert r["decoded"] == zz.tolist()
                n += 1
    assert n > 200
