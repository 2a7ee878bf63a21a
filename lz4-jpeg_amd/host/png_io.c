/*
 * png_io.c -- minimal PNG reader/writer over the system zlib, for the
 * JPEG_seq executable's file contract (the reference reads and writes PNG
 * through its vendored stb_image / stb_image_write: JPEG.c:66-103 read_image,
 * JPEG.c:187-300 create_*_image).  Lossless either way: the pixels handed to
 * the DCT are the same bytes stbi_load returns.
 *
 * Reader: 8-bit, non-interlaced; colour types 0 (grey), 2 (RGB), 3 (palette),
 * 4 (grey+alpha), 6 (RGBA); all five row filters; output RGBA8 with the
 * reference's mapping (r,g,b from the first three channels, a = 255 when the
 * image has no alpha, JPEG.c:90-93).  Writer: RGBA8, filter 0, zlib level 1.
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <zlib.h>

#include "lzj_host.h"

static uint32_t be32(const uint8_t *p) {
  return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3];
}

static void put_be32(uint8_t *p, uint32_t v) {
  p[0] = (uint8_t)(v >> 24); p[1] = (uint8_t)(v >> 16); p[2] = (uint8_t)(v >> 8); p[3] = (uint8_t)v;
}

static uint8_t *slurp(const char *path, size_t *len) {
  FILE *f = fopen(path, "rb");
  if (!f) return NULL;
  if (fseek(f, 0, SEEK_END) != 0) { fclose(f); return NULL; }
  long n = ftell(f);
  if (n < 0) { fclose(f); return NULL; }
  rewind(f);
  uint8_t *b = (uint8_t *)malloc((size_t)n + 1);
  if (b && fread(b, 1, (size_t)n, f) != (size_t)n) { free(b); b = NULL; }
  fclose(f);
  *len = (size_t)n;
  return b;
}

static int paeth(int a, int b, int c) {
  const int p = a + b - c;
  const int pa = abs(p - a), pb = abs(p - b), pc = abs(p - c);
  if (pa <= pb && pa <= pc) return a;
  return pb <= pc ? b : c;
}

int lzj_png_read(const char *path, int *w_out, int *h_out, uint8_t **rgba_out) {
  static const uint8_t sig[8] = {137, 80, 78, 71, 13, 10, 26, 10};
  size_t len = 0;
  uint8_t *f = slurp(path, &len);
  if (!f) return -1;
  int rc = -2;
  uint8_t *idat = NULL, *raw = NULL, *rgba = NULL;
  size_t idat_len = 0;
  uint32_t w = 0, h = 0;
  int ctype = -1, depth = 0, interlace = 0;
  uint8_t pal[256][4];
  memset(pal, 0, sizeof pal);
  for (int i = 0; i < 256; ++i) pal[i][3] = 255;
  if (len < 8 || memcmp(f, sig, 8) != 0) goto done;
  for (size_t p = 8; p + 12 <= len;) {
    const uint32_t clen = be32(f + p);
    const uint8_t *type = f + p + 4, *data = f + p + 8;
    if (p + 12 + (size_t)clen > len) goto done;
    if (!memcmp(type, "IHDR", 4) && clen >= 13) {
      w = be32(data); h = be32(data + 4);
      depth = data[8]; ctype = data[9]; interlace = data[12];
    } else if (!memcmp(type, "PLTE", 4)) {
      for (uint32_t i = 0; i < clen / 3 && i < 256; ++i) {
        pal[i][0] = data[3 * i]; pal[i][1] = data[3 * i + 1]; pal[i][2] = data[3 * i + 2];
      }
    } else if (!memcmp(type, "tRNS", 4) && ctype == 3) {
      for (uint32_t i = 0; i < clen && i < 256; ++i) pal[i][3] = data[i];
    } else if (!memcmp(type, "IDAT", 4)) {
      uint8_t *n = (uint8_t *)realloc(idat, idat_len + clen);
      if (!n) goto done;
      idat = n;
      memcpy(idat + idat_len, data, clen);
      idat_len += clen;
    } else if (!memcmp(type, "IEND", 4)) {
      break;
    }
    p += 12 + (size_t)clen;
  }
  if (w == 0 || h == 0 || w > 65535 || h > 65535 || depth != 8 || interlace != 0) goto done;
  int ch;
  switch (ctype) {
    case 0: ch = 1; break;
    case 2: ch = 3; break;
    case 3: ch = 1; break;
    case 4: ch = 2; break;
    case 6: ch = 4; break;
    default: goto done;
  }
  const size_t stride = (size_t)w * ch;
  uLongf raw_len = (uLongf)((stride + 1) * h);
  raw = (uint8_t *)malloc(raw_len);
  rgba = (uint8_t *)malloc((size_t)w * h * 4);
  if (!raw || !rgba) goto done;
  if (uncompress(raw, &raw_len, idat, (uLong)idat_len) != Z_OK || raw_len != (stride + 1) * h)
    goto done;
  for (uint32_t y = 0; y < h; ++y) {                 /* undo the row filters */
    uint8_t *row = raw + y * (stride + 1);
    const uint8_t ft = row[0];
    uint8_t *cur = row + 1;
    const uint8_t *prev = y ? raw + (y - 1) * (stride + 1) + 1 : NULL;
    for (size_t x = 0; x < stride; ++x) {
      const int a = x >= (size_t)ch ? cur[x - ch] : 0;
      const int b = prev ? prev[x] : 0;
      const int c = (prev && x >= (size_t)ch) ? prev[x - ch] : 0;
      int v = cur[x];
      switch (ft) {
        case 0: break;
        case 1: v += a; break;
        case 2: v += b; break;
        case 3: v += (a + b) >> 1; break;
        case 4: v += paeth(a, b, c); break;
        default: goto done;
      }
      cur[x] = (uint8_t)v;
    }
    for (uint32_t x = 0; x < w; ++x) {
      const uint8_t *s = cur + (size_t)x * ch;
      uint8_t *d = rgba + ((size_t)y * w + x) * 4;
      switch (ctype) {
        case 0: d[0] = d[1] = d[2] = s[0]; d[3] = 255; break;
        case 2: d[0] = s[0]; d[1] = s[1]; d[2] = s[2]; d[3] = 255; break;
        case 3: memcpy(d, pal[s[0]], 4); break;
        case 4: d[0] = d[1] = d[2] = s[0]; d[3] = s[1]; break;
        default: memcpy(d, s, 4); break;
      }
    }
  }
  *w_out = (int)w;
  *h_out = (int)h;
  *rgba_out = rgba;
  rgba = NULL;
  rc = 0;
done:
  free(f);
  free(idat);
  free(raw);
  free(rgba);
  return rc;
}

static int write_chunk(FILE *f, const char *type, const uint8_t *data, uint32_t n) {
  uint8_t hdr[8];
  put_be32(hdr, n);
  memcpy(hdr + 4, type, 4);
  uLong crc = crc32(0L, (const Bytef *)type, 4);
  if (n) crc = crc32(crc, data, n);
  uint8_t tail[4];
  put_be32(tail, (uint32_t)crc);
  return fwrite(hdr, 1, 8, f) == 8 && (n == 0 || fwrite(data, 1, n, f) == n) &&
                 fwrite(tail, 1, 4, f) == 4
             ? 0
             : -1;
}

int lzj_png_write(const char *path, int w, int h, const uint8_t *rgba) {
  static const uint8_t sig[8] = {137, 80, 78, 71, 13, 10, 26, 10};
  if (w <= 0 || h <= 0 || !rgba) return -1;
  const size_t stride = (size_t)w * 4;
  const size_t raw_len = (stride + 1) * (size_t)h;
  uint8_t *raw = (uint8_t *)malloc(raw_len);
  uLongf zlen = compressBound((uLong)raw_len);
  uint8_t *z = (uint8_t *)malloc(zlen);
  int rc = -1;
  FILE *f = NULL;
  if (!raw || !z) goto out;
  for (int y = 0; y < h; ++y) {
    raw[y * (stride + 1)] = 0;
    memcpy(raw + y * (stride + 1) + 1, rgba + (size_t)y * stride, stride);
  }
  if (compress2(z, &zlen, raw, (uLong)raw_len, 1) != Z_OK) goto out;
  f = fopen(path, "wb");
  if (!f) goto out;
  uint8_t ihdr[13];
  put_be32(ihdr, (uint32_t)w);
  put_be32(ihdr + 4, (uint32_t)h);
  ihdr[8] = 8; ihdr[9] = 6; ihdr[10] = 0; ihdr[11] = 0; ihdr[12] = 0;
  if (fwrite(sig, 1, 8, f) != 8 || write_chunk(f, "IHDR", ihdr, 13) ||
      write_chunk(f, "IDAT", z, (uint32_t)zlen) || write_chunk(f, "IEND", NULL, 0))
    goto out;
  rc = 0;
out:
  if (f && fclose(f) != 0) rc = -1;
  free(raw);
  free(z);
  return rc;
}
