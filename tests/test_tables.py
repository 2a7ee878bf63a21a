"""The JPEG kernel's baked constants equal the reference's libm expressions."""
import math
import os
import re
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(REPO, "lz4-jpeg_amd", "csrc")
PI = 3.14159265358979323846


def test_tables_header_is_generated_output():
    gen = subprocess.run([sys.executable, os.path.join(CSRC, "gen_jpeg_tables.py")],
                         capture_output=True, text=True, check=True).stdout
    assert open(os.path.join(CSRC, "jpeg_tables.h")).read() == gen


def _table(name):
    src = open(os.path.join(CSRC, "jpeg_tables.h")).read()
    body = src.split(f"double {name}[")[1].split("};")[0]
    return [float.fromhex(x) for x in re.findall(r"-?0x[0-9a-f.]+p[+-]\d+", body)]


def test_cos_values_match_libm_expression():
    c8 = _table("C8")
    for x in range(8):
        for u in range(8):
            assert c8[x * 8 + u] == math.cos((PI * (2 * x + 1) * u) / (2.0 * 8))


def test_survey_spot_values():
    c8 = _table("C8")
    # asymmetric last bits
    assert c8[1 * 8 + 3] == float.fromhex("-0x1.8f8b83c69a608p-3")
    assert c8[0 * 8 + 7] == float.fromhex("0x1.8f8b83c69a60dp-3")
    aa = _table("AA88")
    assert aa[0] == float.fromhex("0x1.0000000000001p-3")  # not 0.125


def test_zigzag_chroma_order():
    src = open(os.path.join(CSRC, "jpeg_tables.h")).read()
    pos = [int(v) for v in src.split("ZZ4_POS[32] = {")[1].split("}")[0].split(",")]
    order = [0] * 32
    for i, k in enumerate(pos):
        order[k] = i
    assert order == [0, 1, 4, 8, 5, 2, 3, 6, 9, 12, 16, 13, 10, 7, 11, 14, 17, 20, 24, 21, 18,
                     15, 19, 22, 25, 28, 29, 26, 23, 27, 30, 31]


def test_colour_terms_fp32_equal_fp64():
    """jpeg_recon_kernel's colour terms (assemble_image, JPEG.c:598-600): the
    truncation of the fp32 product fl32(k) * d equals the reference's (int) of
    the fp64 product k * (double)d for every d = Cr - 128 / Cb - 128 in
    -128..127 and each of the four constants, and no product lies within
    0.001 of a nonzero integer (the margin the kernel's comment relies on)."""
    import numpy as np
    d = np.arange(-128, 128)
    for k in (1.402, 0.344136, 0.714136, 1.772):
        ref = np.trunc(k * d.astype(np.float64)).astype(np.int64)
        f32 = np.trunc(np.float32(k) * d.astype(np.float32)).astype(np.int64)
        assert np.array_equal(ref, f32), k
        x = k * d[d != 0]
        assert np.min(np.abs(x - np.round(x))) > 0.001, k


def test_round_clamp_by_truncation():
    """round_clamp_u8 (jpeg_recon_kernel): (int)round(x) clamped to 0..255
    (JPEG.c:440-446) equals trunc + (fraction >= 0.5) clamped, on the values
    where the two could differ: halves, their neighbours, negatives, and
    values past 255."""
    import numpy as np
    xs = []
    for k in range(-3, 259):
        for off in (-0.5, 0.0, 0.5):
            b = k + off
            xs += [b, np.nextafter(b, -1e9), np.nextafter(b, 1e9)]
    xs += list(np.random.default_rng(1).uniform(-300, 600, 20000))
    from decimal import ROUND_HALF_UP, Decimal
    for x in xs:
        x = float(x)
        # C round(): half away from zero, on the exact binary value
        v = int(Decimal(x).quantize(Decimal(1), rounding=ROUND_HALF_UP))
        ref = min(255, max(0, v))
        i = int(x)                                   # toward zero, as v_cvt_i32_f64
        got = min(255, max(0, i + (1 if x - i >= 0.5 else 0)))
        assert got == ref, x
