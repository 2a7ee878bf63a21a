/*
 * lz4r_decode.c -- host C decoder of the reference's "LZ4" stream
 * (the bytes lz4r_compress / lz4_encode write).
 *
 * Replaces LZ4_decode / interpret_frame / interpret_sequence
 * (Algorithms/sequential/LZ4/LZ4.c:937-1121), which mis-parse streams of
 * >= 256 blocks (the frame byte is nblocks & 0xFF) and literal runs >= 271
 * (the extension byte is (L-15) & 0xFF).  This decoder is exact for every
 * stream the encoder produces:
 *   - blocks are parsed until the input ends; the frame byte is checked
 *     against the block count modulo 256;
 *   - L is recovered from the sequence's u16 size field, which is exact;
 *   - the block header's u16 size field must equal 3 + the sum of its
 *     sequences' size fields (LZ4.c:617), which also prunes wrong readings;
 *   - the format has one genuine ambiguity: a match of length 257..259 is
 *     stored as M = 1..3 (uint8 truncation, LZ4.c:317) and its token
 *     ((L<<4) | (M-4)&0xFF) & 0xFF reads 0xFD..0xFF whatever L was -- the
 *     same token as (L >= 15, M = 17 / 18 / >= 19).  Such tokens are tried
 *     both ways (depth-first, per block) and the reading under which the
 *     block decodes to exactly 300 bytes (or ends the stream) is taken.
 * Host code: decoding is not on the compress hot path.
 */
#include <stddef.h>
#include <stdint.h>
#include <string.h>

#include "../../include/lz4r.h"

typedef struct {
  const uint8_t *in;
  size_t in_len;
  uint8_t *blk;          /* decoded bytes of the current block */
  size_t ip_end;         /* input position after the block (on success) */
  size_t out_len;        /* decoded length of the block (on success) */
  unsigned nseq;
  size_t want;           /* the block header's size field minus 3 = sum of the
                            sequences' size fields (LZ4.c:617) */
} dec_block;

static unsigned litext_len(size_t L) {
  if (L < 15) return 0;
  return ((L - 15) & 255) == 255 ? 2 : 1;
}

/* Literal-extension bytes present at ip for a run of L >= 15 are consistent? */
static int litext_ok(const uint8_t *in, size_t in_len, size_t ip, size_t L) {
  const unsigned r = (unsigned)((L - 15) & 255);
  if (r == 255) return ip + 1 < in_len && in[ip] == 255 && in[ip + 1] == 0;
  return ip < in_len && in[ip] == r;
}

/* Decode sequences s.. of the block from input position ip with `pos` bytes
 * of the block already produced.  Returns 1 on a consistent full parse. */
static int dec_seq(dec_block *d, unsigned s, size_t ip, size_t pos, size_t ssum) {
  const uint8_t *in = d->in;
  if (s == d->nseq) {
    if (ssum != d->want) return 0;
    if ((pos == LZ4R_BLOCK && ip < d->in_len) || (ip == d->in_len && pos >= 1 && pos <= LZ4R_BLOCK)) {
      d->ip_end = ip;
      d->out_len = pos;
      return 1;
    }
    return 0;
  }
  if (ip + 3 > d->in_len) return 0;
  const unsigned tok = in[ip];
  const size_t S = (size_t)in[ip + 1] | ((size_t)in[ip + 2] << 8);
  const size_t ip0 = ip + 3;
  if (ssum + S > d->want) return 0;
  const int last = (s + 1 == d->nseq);

  /* reading A: token nibbles as written for M == 0 or M >= 4 */
  {
    const unsigned tl = tok >> 4, tm = tok & 15;
    const unsigned mx = (tm == 15) ? 1 : 0;
    size_t L, le;
    int ok = 1;
    if (tl == 15) {
      le = (ip0 < d->in_len && in[ip0] == 255) ? 2 : 1;
      if (S < 5 + le + mx) ok = 0;
      L = ok ? S - 5 - le - mx : 0;
      if (ok && (L < 15 || litext_len(L) != le || !litext_ok(in, d->in_len, ip0, L))) ok = 0;
    } else {
      le = 0;
      L = tl;
      if (S != L + 5 + mx) ok = 0;
    }
    size_t ip1 = ip0 + le;
    if (ok && ip1 + L + 2 <= d->in_len && pos + L <= LZ4R_BLOCK) {
      const unsigned dist = in[ip1 + L] | ((unsigned)in[ip1 + L + 1] << 8);
      size_t ip2 = ip1 + L + 2;
      size_t M = 0;
      int good = 1;
      if (dist == 0) {                    /* literal-only tail (LZ4.c:585-613) */
        good = last && tm == 0;
      } else if (tm == 15) {
        if (ip2 >= d->in_len) good = 0;
        else M = 19 + (size_t)in[ip2++];
      } else {
        M = tm + 4;
      }
      if (good && dist != 0 && (dist > pos + L || pos + L + M > LZ4R_BLOCK)) good = 0;
      if (good) {
        memcpy(d->blk + pos, in + ip1, L);
        size_t p = pos + L;
        for (size_t k = 0; k < M; ++k, ++p) d->blk[p] = d->blk[p - dist];
        if (dec_seq(d, s + 1, ip2, p, ssum + S)) return 1;
      }
    }
  }
  /* reading B: a truncated match length M = tok - 0xFC in {1,2,3} */
  if (tok >= 0xFD) {
    const size_t M = tok - 0xFC;
    /* S = L + 5 + litext_len(L) + 1 (the size field counts a match-extension
     * byte that write_sequence does not write, LZ4.c:569-575 vs :393) */
    for (unsigned le = 0; le <= 2; ++le) {
      if (S < 6 + le) continue;
      const size_t L = S - 6 - le;
      if (litext_len(L) != le) continue;
      if (le && !litext_ok(in, d->in_len, ip0, L)) continue;
      const size_t ip1 = ip0 + le;
      if (ip1 + L + 2 > d->in_len || pos + L + M > LZ4R_BLOCK) continue;
      const unsigned dist = in[ip1 + L] | ((unsigned)in[ip1 + L + 1] << 8);
      if (dist == 0 || dist > pos + L) continue;
      memcpy(d->blk + pos, in + ip1, L);
      size_t p = pos + L;
      for (size_t k = 0; k < M; ++k, ++p) d->blk[p] = d->blk[p - dist];
      if (dec_seq(d, s + 1, ip1 + L + 2, p, ssum + S)) return 1;
    }
  }
  return 0;
}

int lz4r_decompress(const uint8_t *in, size_t in_len, uint8_t *out, size_t cap,
                    size_t *out_len) {
  if (!in || !out_len || (!out && cap)) return LZ4R_ERR_ARG;
  if (in_len < 1) return LZ4R_ERR_CORRUPT;
  uint8_t blk[LZ4R_BLOCK];
  size_t ip = 1, op = 0, nb = 0;
  while (ip < in_len) {
    if (ip + 3 > in_len) return LZ4R_ERR_CORRUPT;
    const size_t bsize = (size_t)in[ip + 1] | ((size_t)in[ip + 2] << 8);
    if (bsize < 3) return LZ4R_ERR_CORRUPT;
    dec_block d = {in, in_len, blk, 0, 0, in[ip], bsize - 3};
    if (!dec_seq(&d, 0, ip + 3, 0, 0)) return LZ4R_ERR_CORRUPT;
    if (op + d.out_len > cap) {
      *out_len = op + d.out_len;
      return LZ4R_ERR_CAPACITY;
    }
    memcpy(out + op, blk, d.out_len);
    op += d.out_len;
    ip = d.ip_end;
    ++nb;
  }
  if (nb == 0 || (uint8_t)nb != in[0]) return LZ4R_ERR_CORRUPT;   /* LZ4.c:429 */
  *out_len = op;
  return LZ4R_OK;
}
