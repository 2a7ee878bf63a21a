#!/usr/bin/env python3
"""Writes tests/golden/golden.json -- the known-answer vectors the parity
tests use -- and checks the CPU oracle against every reference-produced one.

Provenance of each entry (field "source"):
  reference-file   a file committed in the reference repository
                   (Output-Input/out/compressed.bin for Output-Input/input/input.txt)
  reference-build  md5s produced by compiling the reference's own
                   Algorithms/sequential/{LZ4,JPEG}/*.c in the survey session
                   (SURVEY.md Appendix A4); the JPEG ones are re-checked here
                   against oracle/_ref/libref_jpeg.so when it exists
  oracle           produced by oracle/liboracle.so (our restatement), for
                   edge cases no reference artefact covers ("parity unpinned"
                   beyond the restatement itself)

Run from the repo root:  python tests/golden/make_golden.py
"""
import hashlib
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
import oracle_api  # noqa: E402
import golden_inputs  # noqa: E402

REF_LZ4 = [  # SURVEY.md Appendix A4 (reference LZ4.c compiled in the survey session)
    {"name": "input.txt", "input": "file:lz4_input.txt", "in_len": 350, "out_len": 377,
     "md5": "a67f911837a68250ccfbccfcd2f82239", "source": "reference-file"},
    {"name": "Metamorphosis raw", "input": "file:Metamorphosis.txt", "in_len": 118489,
     "out_len": 123143, "md5": "92c86420e7b926f9b5b6bff7b5cc6c9c", "source": "reference-build"},
    {"name": "Metamorphosis nl->space", "input": "metamorphosis_spaces", "in_len": 118489,
     "out_len": 122573, "md5": "f79743ece0740c147295f58e3f9461b9", "source": "reference-build"},
    {"name": "Metamorphosis nl->space first 76500", "input": "metamorphosis_spaces:76500",
     "in_len": 76500, "out_len": 79152, "md5": "c753dff5c6eff4fce975d3f1c9c50a4a",
     "source": "reference-build"},
]
REF_JPEG = [  # glibc rand() seed 1, int16 [Y64][Cr32][Cb32] zz per tile
    {"w": 8, "h": 8, "seed": 1, "bytes": 256, "md5": "9c6d56279f0ae49db61099a76b2eddce"},
    {"w": 64, "h": 64, "seed": 1, "bytes": 16384, "md5": "304b2a5b57a1cffeab7d5cd0e6c3d8f0"},
    {"w": 512, "h": 512, "seed": 1, "bytes": 1048576, "md5": "18b16f94bcac063c9db3b86c7d961d91"},
    {"w": 1920, "h": 1080, "seed": 1, "bytes": 8294400, "md5": "6fbe09410185a1cbdad802b61fdad588"},
    {"w": 3840, "h": 2160, "seed": 1, "bytes": 33177600, "md5": "2f534501325d07a4d87edcd18d993363"},
]
JPEG_KAT_8X8 = {  # SURVEY.md Appendix A4, literal coefficients of the 8x8 seed-1 image
    "Y": [-1, -1, 7, -1, -8, 0, -10, 9, 2, 13, 7, -2, -1, -1, 2, -3, 3, 0, -10, -1, 1, 11, -1,
          -1, -1, 8, -3, 0, -2, 0, 3, -2, 0, -2, 0, -1, -1, 1, 0, 0, 1, 3, 4, 2, -1, 0, 0, 3, 2,
          0, 1, -1, 0, 2, 0, -1, 1, 0, 0, -1, 2, -1, 0, -2],
    "Cr": [1, -1, -1, 2, -1, 0, 0, -1, 3, 0, 0, 0, 1] + [0] * 19,
    "Cb": [2, 0, 2, 0, 4, 1, 0, -3, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, -1] + [0] * 13,
}


def entropy_streams(o):
    """Streams (zigzagged ints of one channel of one tile) for the entropy
    stage: the 8x8 KAT tile, edge cases, random and natural-image tiles."""
    import numpy as np
    st = [("kat_Y", JPEG_KAT_8X8["Y"]), ("kat_Cr", JPEG_KAT_8X8["Cr"]),
          ("kat_Cb", JPEG_KAT_8X8["Cb"]),
          ("zeros_Y", [0] * 64), ("zeros_C", [0] * 32),
          ("one_symbol_C", [32] * 32), ("one_symbol_Y", [64] * 64),   # RLE [n, n]: one code, empty
          ("all_distinct_Y", list(range(-32, 32))), ("all_distinct_C", list(range(100, 132))),
          ("alternating_Y", [1, -1] * 32), ("runs_Y", sum([[k] * k for k in range(1, 11)], [])[:64]),
          ("dc_only_Y", [57] + [0] * 63), ("extremes_Y", [-1024, 1016] * 32)]
    rng = np.random.default_rng(11)
    coef = o.jpeg_encode(o.rand_image(32, 16, 7)).reshape(-1, 128)
    for t in range(coef.shape[0]):
        st += [(f"rand_t{t}_Y", coef[t, :64].tolist()), (f"rand_t{t}_Cr", coef[t, 64:96].tolist()),
               (f"rand_t{t}_Cb", coef[t, 96:].tolist())]
    for k in range(12):
        n = 64 if k % 2 == 0 else 32
        alpha = int(rng.integers(2, 40))
        st.append((f"fuzz{k}", (rng.integers(-alpha // 2, alpha // 2 + 1, n)).tolist()))
    return st


def entropy_vectors(o):
    """Known answers from the reference's own entropy functions (oracle/_ref:
    RLE, encode_huffman, generate_encoded_sequence, decode_huffman,
    inverse_RLE); the restatement must agree.  Kept from the previous run
    when the reference build is absent."""
    path = os.path.join(HERE, "entropy.json")
    if oracle_api.ref_jpeg() is None:
        return json.load(open(path))
    vecs = []
    for name, zz in entropy_streams(o):
        r = oracle_api.ref_entropy(zz)
        a = oracle_api.entropy(o, zz)
        assert (a["rle"], a["table"], a["nbits"], a["bits"]) == \
            (r["rle"], r["table"], r["nbits"], r["bits"]), name
        assert r["decoded"] == list(zz), name
        vecs.append({"name": name, "zz": list(zz), "rle_len": len(r["rle"]),
                     "table": [[v, ln, str(c)] for v, ln, c in r["table"]],
                     "nbits": r["nbits"], "bits": r["bits"].hex(), "source": "reference-build"})
    return vecs


def md5(b):
    return hashlib.md5(b).hexdigest()


def main():
    o = oracle_api.load()
    lz4 = []
    for e in REF_LZ4:
        data = golden_inputs.lz4_input(e["input"])
        got = o.lz4_compress(data)
        assert len(data) == e["in_len"], e
        assert (len(got), md5(got)) == (e["out_len"], e["md5"]), (e["name"], len(got), md5(got))
        lz4.append(e)
    for name in golden_inputs.LZ4_EDGE_CASES:
        data = golden_inputs.lz4_input(name)
        got = o.lz4_compress(data)
        lz4.append({"name": name, "input": name, "in_len": len(data), "out_len": len(got),
                    "md5": md5(got), "source": "oracle"})
    ref = oracle_api.ref_jpeg()
    jpeg = []
    for e in REF_JPEG:
        img = o.rand_image(e["w"], e["h"], e["seed"])
        got = o.jpeg_encode(img, threads=8).tobytes()
        assert (len(got), md5(got)) == (e["bytes"], e["md5"]), e
        e = dict(e, source="reference-build")
        if ref is not None and e["w"] * e["h"] <= 512 * 512:
            import numpy as np
            r = np.empty(len(got) // 2, np.int16)
            ref.ref_jpeg_encode_image(img.ctypes.data, e["w"], e["h"], r.ctypes.data)
            assert r.tobytes() == got, "oracle != reference JPEG.c"
            e["rechecked_against_ref_build"] = True
        jpeg.append(e)
    entropy = entropy_vectors(o)
    with open(os.path.join(HERE, "entropy.json"), "w") as f:      # one vector per line
        f.write("[\n" + ",\n".join(json.dumps(v) for v in entropy) + "\n]\n")
    out = {"lz4": lz4, "jpeg": jpeg, "jpeg_kat_8x8": JPEG_KAT_8X8}
    with open(os.path.join(HERE, "golden.json"), "w") as f:
        json.dump(out, f, indent=1)
    print(f"wrote {len(lz4)} lz4 + {len(jpeg)} jpeg + {len(entropy)} entropy vectors")


if __name__ == "__main__":
    main()
