"""Tiny PNG reader/writer for tests (8-bit RGB/RGBA, non-interlaced, all five
row filters) -- independent of the product's png_io.c."""
import struct
import zlib

import numpy as np


def read(path):
    b = open(path, "rb").read()
    assert b[:8] == b"\x89PNG\r\n\x1a\n"
    p, idat, w = 8, b"", None
    while p < len(b):
        n = struct.unpack(">I", b[p:p + 4])[0]
        t = b[p + 4:p + 8]
        d = b[p + 8:p + 8 + n]
        if t == b"IHDR":
            w, h, depth, ctype = struct.unpack(">IIBB", d[:10])
            assert depth == 8 and ctype in (2, 6)
            ch = 3 if ctype == 2 else 4
        elif t == b"IDAT":
            idat += d
        p += 12 + n
    raw = np.frombuffer(zlib.decompress(idat), np.uint8).reshape(h, 1 + w * ch)
    out = np.zeros((h, w * ch), np.int32)
    for y in range(h):
        ft, cur = raw[y, 0], raw[y, 1:].astype(np.int32)
        prev = out[y - 1] if y else np.zeros(w * ch, np.int32)
        row = np.zeros(w * ch, np.int32)
        for x in range(w * ch):
            a = row[x - ch] if x >= ch else 0
            bb = prev[x]
            c = prev[x - ch] if x >= ch else 0
            if ft == 0:
                pr = 0
            elif ft == 1:
                pr = a
            elif ft == 2:
                pr = bb
            elif ft == 3:
                pr = (a + bb) >> 1
            else:
                pa, pb, pc = abs(bb - c), abs(a - c), abs(a + bb - 2 * c)
                pr = a if pa <= pb and pa <= pc else (bb if pb <= pc else c)
            row[x] = (cur[x] + pr) & 255
        out[y] = row
    img = out.astype(np.uint8).reshape(h, w, ch)
    if ch == 3:
        img = np.concatenate([img, np.full((h, w, 1), 255, np.uint8)], axis=2)
    return img


def write(path, rgba, filters=(0, 1, 2, 3, 4)):
    """RGBA8 PNG whose rows cycle through the given filter types."""
    h, w, _ = rgba.shape
    img = rgba.astype(np.int32).reshape(h, w * 4)
    rows = []
    for y in range(h):
        ft = filters[y % len(filters)]
        cur = img[y]
        prev = img[y - 1] if y else np.zeros(w * 4, np.int32)
        a = np.concatenate([np.zeros(4, np.int32), cur[:-4]])
        c = np.concatenate([np.zeros(4, np.int32), prev[:-4]])
        if ft == 0:
            pr = 0
        elif ft == 1:
            pr = a
        elif ft == 2:
            pr = prev
        elif ft == 3:
            pr = (a + prev) >> 1
        else:
            pa, pb, pc = np.abs(prev - c), np.abs(a - c), np.abs(a + prev - 2 * c)
            pr = np.where((pa <= pb) & (pa <= pc), a, np.where(pb <= pc, prev, c))
        rows.append(bytes([ft]) + ((cur - pr) & 255).astype(np.uint8).tobytes())

    def chunk(t, d):
        return struct.pack(">I", len(d)) + t + d + struct.pack(">I", zlib.crc32(t + d) & 0xFFFFFFFF)
    data = (b"\x89PNG\r\n\x1a\n" + chunk(b"IHDR", struct.pack(">IIBBBBB", w, h, 8, 6, 0, 0, 0))
            + chunk(b"IDAT", zlib.compress(b"".join(rows), 6)) + chunk(b"IEND", b""))
    open(path, "wb").write(data)
