"""Deterministic LZ4 test inputs, by name (shared by make_golden.py and the
parity tests).  Edge cases target the reference's format quirks
(SURVEY.md Appendix A1): matches clamped at the block end, uint8 length
truncation (len 256 -> literal, 257..259 -> M = 1..3 with the token nibble
overflow and a size field that over-counts), the 0xFF 0x00 literal
extension at L = 270, literal runs of a whole block, short last blocks."""
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _file(name):
    with open(os.path.join(GOLDEN, name), "rb") as f:
        return f.read()


def _rng_bytes(seed, n, alphabet=256):
    r = np.random.default_rng(seed)
    return r.integers(0, alphabet, n, dtype=np.uint8).tobytes()


def _unique_prefix(k, seed=7):
    """k bytes whose 4-grams never repeat (distinct byte values, k <= 256)."""
    r = np.random.default_rng(seed)
    return r.permutation(256)[:k].astype(np.uint8).tobytes()


def _m_truncated(prefix_len, run):
    # `prefix_len` distinct bytes then a run of one byte: the match at
    # prefix_len+1 has length 300-(prefix_len+1) -> uint8 truncation.
    return (_unique_prefix(prefix_len) + b"\xaa" * run)[:300] + _rng_bytes(3, 300)


def _lit270():
    u = _rng_bytes(11, 270)
    return u + u[:30] + _rng_bytes(12, 300)


def _many_sequences(seed=3, nblocks=40):
    """Blocks of a few dozen distinct bytes followed by random 4-byte chunks
    of that prefix: the greedy parse takes many exact-4 matches with no
    literals between them, and some blocks have more than 64 sequences
    (the compressor's multi-round sequence path)."""
    r = np.random.default_rng(seed)
    out = bytearray()
    for _ in range(nblocks):
        pre = bytes(r.permutation(256)[:int(r.integers(10, 60))].astype(np.uint8))
        rest = bytearray()
        while len(pre) + len(rest) < 300:
            s = int(r.integers(0, len(pre) - 4))
            rest += pre[s:s + 4]
        out += (pre + bytes(rest))[:300]
    return bytes(out)


LZ4_EDGE_CASES = [
    "exact_300", "exact_301", "exact_599", "exact_600", "a_x_600", "ab_x_700",
    "zeros_900", "random_bytes_3000", "alphabet2_3000", "alphabet4_3000",
    "m_eq_1", "m_eq_2", "m_eq_3", "len_256", "lit_270", "lit_300",
    "text_last_block_1", "text_last_block_4", "text_10000", "many_sequences",
]


def lz4_input(name):
    if name.startswith("file:"):
        return _file(name[5:])
    meta = _file("Metamorphosis.txt")
    if name.startswith("metamorphosis_spaces"):
        b = meta.replace(b"\n", b" ").replace(b"\r", b" ")
        if ":" in name:
            b = b[: int(name.split(":")[1])]
        return b
    text = meta.replace(b"\n", b" ")
    table = {
        "exact_300": lambda: text[1000:1300],
        "exact_301": lambda: text[2000:2301],
        "exact_599": lambda: text[3000:3599],
        "exact_600": lambda: text[4000:4600],
        "a_x_600": lambda: b"a" * 600,
        "ab_x_700": lambda: b"ab" * 350,
        "zeros_900": lambda: b"\x00" * 900,
        "random_bytes_3000": lambda: _rng_bytes(1, 3000),
        "alphabet2_3000": lambda: bytes(97 + x for x in _rng_bytes(2, 3000, 2)),
        "alphabet4_3000": lambda: bytes(97 + x for x in _rng_bytes(3, 3000, 4)),
        "m_eq_1": lambda: _m_truncated(42, 258),
        "m_eq_2": lambda: _m_truncated(41, 259),
        "m_eq_3": lambda: _m_truncated(40, 260),
        "len_256": lambda: _m_truncated(43, 257),
        "lit_270": _lit270,
        "lit_300": lambda: _unique_prefix(256) + _unique_prefix(44, seed=9) + b"x" * 10,
        "text_last_block_1": lambda: text[5000:5601],
        "text_last_block_4": lambda: text[6000:6604],
        "text_10000": lambda: text[7000:17000],
        "many_sequences": _many_sequences,
    }
    return table[name]()
