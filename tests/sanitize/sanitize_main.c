/*
 * sanitize_main.c -- TEST INFRASTRUCTURE ONLY ("CPU
 * restatement under ASan/UBSan").  Built by `make sanitize` with
 * -fsanitize=address,undefined -fno-sanitize-recover=all together with the
 * host C of the product (lz4r_decode.c, png_io.c, synth.c) and the oracle
 * restatements (oracle/*.c); run by tests/test_sanitize.py.  Exercises:
 *   - the oracle LZ4 encoder on the golden inputs + adversarial blocks, and
 *     the product's exact host decoder (lz4r_decompress) round trip, plus
 *     truncated / corrupted streams (must fail cleanly, never read out of
 *     bounds);
 *   - the synthetic generators (host/synth.c, incl. the jump-ahead);
 *   - PNG write / read round trip (host/png_io.c) and a truncated file;
 *   - the JPEG oracle encode / reconstruct and the entropy oracle round
 *     trip on random tiles;
 *   - the per-block compat API (host/compat_lz4.c: block_encode,
 *     write_output, find_longest_match and its growing block cache) over a
 *     CPU match provider (cpu_matches.c), on 300-B, short and long blocks
 *     (exact-size heap copies), against the oracle's block encoder.
 * Exit 0 and "sanitize ok" when every check passed.
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../include/lz4jpeg_compat.h"
#include "../../include/lz4jpeg_synth.h"
#include "../../include/lz4r.h"
#include "../../lz4-jpeg_amd/host/lzj_host.h"

size_t lz4o_compress(const uint8_t *in, size_t n, uint8_t *out);
size_t lz4o_block_bound(void);
size_t lz4o_encode_block(const uint8_t *blk, size_t n, uint8_t *out);
size_t lz4o_decompress(const uint8_t *in, size_t in_len, uint8_t *out, size_t cap, size_t nb);
void jo_encode_image(const uint8_t *rgba, int w, int h, int16_t *out);
void jo_reconstruct_image(const uint8_t *rgba, int w, int h, uint8_t *out);
int jo_entropy_stream(const int16_t *zz, int n, int *rle, int *rle_len, int *ncodes,
                      int16_t *tab_val, uint8_t *tab_len, uint64_t *tab_code, uint8_t *bits,
                      int cap_bits, int *nbits);
int jo_entropy_decode(const uint8_t *bits, int nbits, int rle_len, int ncodes,
                      const int16_t *tab_val, const uint8_t *tab_len, const uint64_t *tab_code,
                      int n, int16_t *zz);

static int fails = 0;
#define CHECK(c)                                                        \
  do {                                                                  \
    if (!(c)) {                                                         \
      fprintf(stderr, "FAIL %s:%d: %s\n", __FILE__, __LINE__, #c);      \
      ++fails;                                                          \
    }                                                                   \
  } while (0)

static uint8_t *read_file(const char *path, size_t *n) {
  FILE *f = fopen(path, "rb");
  if (!f) return NULL;
  fseek(f, 0, SEEK_END);
  long sz = ftell(f);
  fseek(f, 0, SEEK_SET);
  uint8_t *b = malloc((size_t)sz);
  *n = fread(b, 1, (size_t)sz, f);
  fclose(f);
  return b;
}

/* compress with the oracle, decode with the product's host decoder; also
 * every truncation of the stream's tail and a few corruptions must not
 * read or write out of bounds */
static void lz4_roundtrip(const uint8_t *in, size_t n) {
  uint8_t *comp = malloc(1 + ((n + 299) / 300) * lz4o_block_bound());
  const size_t cl = lz4o_compress(in, n, comp);
  CHECK(cl != (size_t)-1);
  uint8_t *out = malloc(n + 300);
  size_t got = 0;
  CHECK(lz4r_decompress(comp, cl, out, n + 300, &got) == LZ4R_OK);
  CHECK(got == n && memcmp(out, in, n) == 0);
  /* exact-size heap copies, so ASan sees any over-read */
  for (size_t cut = 1; cut < 40 && cut < cl; cut += 3) {
    uint8_t *t = malloc(cl - cut);
    memcpy(t, comp, cl - cut);
    (void)lz4r_decompress(t, cl - cut, out, n + 300, &got);
    free(t);
  }
  for (size_t k = 0; k < 16; k++) {
    uint8_t *t = malloc(cl);
    memcpy(t, comp, cl);
    t[(k * 7919) % cl] ^= (uint8_t)(0x5A + k);
    (void)lz4r_decompress(t, cl, out, n + 300, &got);
    free(t);
  }
  size_t small = 0;
  CHECK(lz4r_decompress(comp, cl, out, n / 2, &small) == LZ4R_ERR_CAPACITY || n / 2 >= n);
  free(out);
  free(comp);
}

/* block_encode + write_output (host/compat_lz4.c) on an exact-size heap copy
 * of n bytes: the stream must be the frame byte 1 + the oracle's block */
static void compat_block(const uint8_t *src, size_t n, const char *tmp) {
  uint8_t *blk = malloc(n);
  memcpy(blk, src, n);
  LZ4Frame frame;
  LZ4Block block;
  memset(&frame, 0, sizeof frame);
  memset(&block, 0, sizeof block);
  block_encode((const char *)blk, n, &block, NULL, NULL, &frame);
  char path[4096];
  snprintf(path, sizeof path, "%s/compat_block.bin", tmp);
  FILE *f = fopen(path, "wb");
  CHECK(f != NULL);
  if (!f) {
    free(blk);
    return;
  }
  write_output(&frame, f);
  fclose(f);
  size_t got = 0;
  uint8_t *bytes = read_file(path, &got);
  uint8_t *want = malloc(1 + 3 + n + 8 * (n / 4 + 8) + 1024);
  want[0] = 1;
  const size_t wl = 1 + lz4o_encode_block(blk, n, want + 1);
  CHECK(bytes && got == wl && memcmp(bytes, want, wl) == 0);
  free(want);
  free(bytes);
  free(blk);
}

int main(int argc, char **argv) {
  const char *golden = argc > 1 ? argv[1] : "tests/golden";
  const char *tmp = argc > 2 ? argv[2] : "/tmp";
  char path[4096];

  /* ---- LZ4 ---- */
  snprintf(path, sizeof path, "%s/Metamorphosis.txt", golden);
  size_t mn = 0;
  uint8_t *meta = read_file(path, &mn);
  CHECK(meta && mn > 100000);
  if (meta) {
    lz4_roundtrip(meta, 300);
    lz4_roundtrip(meta, 301);
    lz4_roundtrip(meta, 10000);
    lz4_roundtrip(meta, mn);
  }
  {
    uint8_t buf[3000];
    memset(buf, 'a', sizeof buf);
    lz4_roundtrip(buf, sizeof buf);                       /* long runs: truncated M */
    for (size_t i = 0; i < sizeof buf; i++) buf[i] = (uint8_t)(i * 2654435761u >> 13);
    lz4_roundtrip(buf, sizeof buf);                       /* no matches */
    for (size_t i = 0; i < sizeof buf; i++) buf[i] = "ab"[(i * 7 / 3) & 1];
    lz4_roundtrip(buf, sizeof buf);
  }

  /* ---- the per-block compat API over the CPU match provider ---- */
  if (meta) {
    compat_block(meta, 300, tmp);
    compat_block(meta + 300, 57, tmp);                    /* short block */
    compat_block(meta + 1000, 1000, tmp);                 /* longer: the cache grows */
    compat_block(meta + 5000, 5000, tmp);
    compat_block(meta + 2000, 300, tmp);                  /* and shrinks back to 300 B */
    /* find_longest_match on its own: the 300 bytes at its pointer */
    uint8_t *b300 = malloc(300);
    memcpy(b300, meta + 7000, 300);
    uint32_t *m = malloc(300 * sizeof(uint32_t));
    lzj_block_matches(b300, 300, m);
    for (size_t p = 0; p < 300; ++p) {
      uint16_t d = 0;
      const uint8_t got = find_longest_match(b300, p, &d);
      const uint32_t len = m[p] & 0xFFFFu;
      CHECK(got == (len >= 4 ? (uint8_t)len : 0));
      CHECK(got == 0 || d == (uint16_t)(m[p] >> 16));
    }
    free(m);
    free(b300);
  }

  /* ---- synthetic generators ---- */
  {
    uint8_t a[4 * 700], b[4 * 100];
    lz4jpeg_rand_rgba(1, 700, 1, a);
    lz4jpeg_rand_rgba_stream(1, 333, 100, b);
    CHECK(memcmp(a + 4 * 333, b, sizeof b) == 0);
    uint32_t st[31 * 3];
    lz4jpeg_rand_states(7, 11, 1000, 3, st);
    uint32_t starts[9];
    CHECK(lz4jpeg_passage_starts(118489, 1, 30000, 5, 9, starts) == 9);
    if (meta) {
      uint8_t *p1 = malloc(100000), *p2 = malloc(40000);
      CHECK(lz4jpeg_random_passages(meta, mn, 3, 30000, 0, 100000, p1) == 100000);
      CHECK(lz4jpeg_random_passages(meta, mn, 3, 30000, 45678, 40000, p2) == 40000);
      CHECK(memcmp(p1 + 45678, p2, 40000) == 0);
      free(p1);
      free(p2);
    }
  }

  /* ---- PNG I/O ---- */
  {
    const int w = 37, h = 21;
    uint8_t *img = malloc((size_t)w * h * 4);
    lz4jpeg_rand_rgba(5, w, h, img);
    snprintf(path, sizeof path, "%s/sanitize_rt.png", tmp);
    CHECK(lzj_png_write(path, w, h, img) == 0);
    int rw = 0, rh = 0;
    uint8_t *back = NULL;
    CHECK(lzj_png_read(path, &rw, &rh, &back) == 0);
    CHECK(rw == w && rh == h && back && memcmp(back, img, (size_t)w * h * 4) == 0);
    free(back);
    size_t pn = 0;
    uint8_t *raw = read_file(path, &pn);
    snprintf(path, sizeof path, "%s/sanitize_cut.png", tmp);
    FILE *f = fopen(path, "wb");
    fwrite(raw, 1, pn / 2, f);
    fclose(f);
    back = NULL;
    CHECK(lzj_png_read(path, &rw, &rh, &back) != 0);     /* truncated: an error, no crash */
    free(back);
    free(raw);

    /* ---- JPEG oracle ---- */
    int16_t *coef = malloc(sizeof(int16_t) * 128 * ((w + 7) / 8) * ((h + 7) / 8));
    uint8_t *rec = malloc((size_t)w * h * 4);
    jo_encode_image(img, w, h, coef);
    jo_reconstruct_image(img, w, h, rec);
    /* entropy round trip on every stream of every tile */
    const int ntiles = ((w + 7) / 8) * ((h + 7) / 8);
    for (int t = 0; t < ntiles; t++) {
      for (int c = 0; c < 3; c++) {
        const int n = c ? 32 : 64;
        const int16_t *zz = coef + 128 * t + (c == 0 ? 0 : c == 1 ? 64 : 96);
        int rle[256], rl = 0, nc = 0, nbits = 0;
        int16_t tv[128];
        uint8_t tl[128], bits[1024];
        uint64_t tc[128];
        int16_t back2[64];
        if (jo_entropy_stream(zz, n, rle, &rl, &nc, tv, tl, tc, bits, 8 * (int)sizeof bits,
                              &nbits) == 0) {
          CHECK(jo_entropy_decode(bits, nbits, rl, nc, tv, tl, tc, n, back2) == 0);
          CHECK(memcmp(back2, zz, sizeof(int16_t) * n) == 0);
        }
      }
    }
    free(coef);
    free(rec);
    free(img);
  }
  free(meta);
  if (fails) {
    fprintf(stderr, "%d check(s) failed\n", fails);
    return 1;
  }
  printf("sanitize ok\n");
  return 0;
}
