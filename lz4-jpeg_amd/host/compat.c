/*
 * compat.c -- the reference's function-level API (include/lz4jpeg_compat.h)
 * on top of the MI355X C ABI.  Host C: file handling, buffer moves and the
 * reference's exit(1) error behaviour; every byte of compression / DCT /
 * quantisation / zigzag is computed by the HIP kernels.
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <hip/hip_runtime_api.h>

#include "../../include/jpegr.h"
#include "../../include/lz4jpeg_compat.h"
#include "../../include/lz4r.h"

/* safe_open, LZ4.c:109-120 */
static FILE *safe_open(const char *name, const char *mode) {
  FILE *f = fopen(name, mode);
  if (f == NULL) {
    perror("Error: Unable to open file");
    exit(1);
  }
  return f;
}

static uint8_t *read_all(FILE *f, size_t *n) {
  if (fseek(f, 0, SEEK_END) != 0) return NULL;
  long sz = ftell(f);
  if (sz < 0 || fseek(f, 0, SEEK_SET) != 0) return NULL;
  uint8_t *b = (uint8_t *)malloc((size_t)sz + 1);
  if (!b) return NULL;
  *n = fread(b, 1, (size_t)sz, f);
  return b;
}

/* dump_to_hex_file, LZ4.c:75-107: every byte as "%02X " */
static void dump_to_hex_file(const char *in_name, const char *out_name) {
  FILE *in = fopen(in_name, "rb");
  if (!in) {
    perror("Error opening input file");
    return;
  }
  FILE *out = fopen(out_name, "w");
  if (!out) {
    perror("Error opening output file");
    fclose(in);
    return;
  }
  int c;
  while ((c = fgetc(in)) != EOF) fprintf(out, "%02X ", (unsigned)c);
  fclose(in);
  fclose(out);
}

static void die_hip(const char *what, int rc) {
  fprintf(stderr, "Error: %s failed (%d)\n", what, rc);
  exit(1);
}

void lz4_encode(void) {
  FILE *log_file = safe_open(LZ4_LOG_FILE, "a");
  FILE *input_file = safe_open(LZ4_INPUT_FILE, "r");
  FILE *output_file = safe_open(LZ4_COMPRESSED_FILE, "ab");
  size_t n = 0;
  uint8_t *data = read_all(input_file, &n);
  fclose(input_file);
  if (!data) {
    perror("Error: Failed to read input file");
    exit(1);
  }
  if (n < LZ4R_BLOCK) {                                   /* LZ4.c:632-637 */
    printf("Error: default block length is too high, please reduce it before proceding.");
    exit(1);
  }
  const size_t cap = lz4r_compress_bound(n);
  uint8_t *comp = (uint8_t *)malloc(cap);
  size_t got = 0;
  if (!comp) {
    perror("Error: Unable to allocate memory");
    exit(1);
  }
  int rc = lz4r_compress(data, n, comp, cap, &got);
  if (rc != LZ4R_OK) die_hip("lz4r_compress", rc);
  if (fwrite(comp, 1, got, output_file) != got) {
    perror("Error: write failed");
    exit(1);
  }
  fclose(log_file);
  fclose(output_file);
  free(comp);
  free(data);
  dump_to_hex_file(LZ4_COMPRESSED_FILE, LZ4_HEX_FILE);
}

/* ---- per-block API: find_longest_match / block_encode / write_output ---- */

/* The block find_longest_match answers for: its bytes, and every position's
 * len | dist << 16 from one launch -- lz4r_block_matches_device for a
 * 300-byte (or shorter) block, lz4r_window_matches_device (the reference's
 * whole 65535-byte window, MAX_MATCH_LENGTH 1024) for a longer block_length.
 * Host and device buffers grow to the block; per thread. */
static __thread struct {
  const uint8_t *ptr;
  size_t n, cap;
  uint8_t *bytes;
  uint32_t *match;
  int valid;
  void *d_in, *d_match;
} fm_cache;
static __thread size_t fm_block_length;   /* set while block_encode runs */

static void fm_reserve(size_t n) {
  if (n <= fm_cache.cap) return;
  free(fm_cache.bytes);
  free(fm_cache.match);
  (void)hipFree(fm_cache.d_in);
  (void)hipFree(fm_cache.d_match);
  fm_cache.bytes = (uint8_t *)malloc(n);
  fm_cache.match = (uint32_t *)malloc(n * sizeof(uint32_t));
  fm_cache.d_in = fm_cache.d_match = NULL;
  fm_cache.valid = 0;
  fm_cache.cap = 0;
  if (!fm_cache.bytes || !fm_cache.match) {
    perror("Error: Unable to allocate memory");
    exit(1);
  }
  /* +16: the block kernel's staging may read a few bytes past a short block */
  if (hipMalloc(&fm_cache.d_in, n + 16) != hipSuccess ||
      hipMalloc(&fm_cache.d_match, n * sizeof(uint32_t)) != hipSuccess)
    die_hip("hipMalloc", LZ4R_ERR_NOMEM);
  fm_cache.cap = n;
}

static void fm_load(const uint8_t *input, size_t n) {
  if (fm_cache.valid && fm_cache.ptr == input && fm_cache.n == n &&
      memcmp(fm_cache.bytes, input, n) == 0)
    return;
  fm_reserve(n < LZ4R_BLOCK ? LZ4R_BLOCK : n);
  int rc = LZ4R_OK;
  if (hipMemcpy(fm_cache.d_in, input, n, hipMemcpyHostToDevice) != hipSuccess) rc = LZ4R_ERR_HIP;
  if (rc == LZ4R_OK)
    rc = n <= LZ4R_BLOCK ? lz4r_block_matches_device(fm_cache.d_in, n, fm_cache.d_match, NULL)
                         : lz4r_window_matches_device(fm_cache.d_in, n, fm_cache.d_match, NULL);
  if (rc == LZ4R_OK &&
      hipMemcpy(fm_cache.match, fm_cache.d_match, n * sizeof(uint32_t), hipMemcpyDeviceToHost) !=
          hipSuccess)
    rc = LZ4R_ERR_HIP;
  if (rc != LZ4R_OK) die_hip("find_longest_match", rc);
  fm_cache.ptr = input;
  fm_cache.n = n;
  memcpy(fm_cache.bytes, input, n);
  fm_cache.valid = 1;
}

uint8_t find_longest_match(uint8_t *input, size_t current_index, uint16_t *match_distance) {
  /* inside block_encode: its block; standalone: the 300 bytes at input */
  const size_t n = fm_block_length ? fm_block_length : LZ4R_BLOCK;
  if (current_index >= n) return 0;
  fm_load(input, n);
  const uint32_t m = fm_cache.match[current_index];
  const size_t len = m & 0xFFFFu;
  if (len < 4) return 0;                               /* MIN_MATCH_LENGTH, LZ4.c:314 */
  *match_distance = (uint16_t)(m >> 16);
  return (uint8_t)len;                                 /* uint8_t return, LZ4.c:317 */
}

static void append_sequence(LZ4Block *block, const LZ4Sequence *q) {   /* LZ4.c:443-459 */
  LZ4Sequence *s = (LZ4Sequence *)realloc(block->sequences,
                                          sizeof(LZ4Sequence) * (block->sequences_count + 1));
  if (!s) {
    perror("Failed to allocate memory for sequences");
    exit(EXIT_FAILURE);
  }
  block->sequences = s;
  s[block->sequences_count++] = *q;
  block->byte_size += q->byte_size;
}

/* bytes of the literal-length extension as the reference counts them: the
 * remainder is a uint8_t, so (L - 15) & 0xFF == 255 takes two (LZ4.c:554-563) */
static size_t litext_len(size_t lits) {
  if (lits < 15) return 0;
  return ((lits - 15) & 0xFFu) == 255u ? 2 : 1;
}

void block_encode(const char *block_entry, size_t block_length, LZ4Block *block,
                  FILE *log_file, FILE *output_file, LZ4Frame *frame) {
  (void)log_file;
  (void)output_file;
  uint8_t *input = (uint8_t *)block_entry;
  const size_t saved = fm_block_length;
  fm_block_length = block_length;
  LZ4Sequence seq = {0};
  size_t pos = 0;
  uint16_t lits = 0;
  while (pos < block_length) {
    uint16_t dist = 0;
    const uint8_t m = find_longest_match(input, pos, &dist);
    if (m == 0) {                                      /* a literal, LZ4.c:522-529 */
      if (lits == 0) seq.literals = &input[pos];
      ++pos;
      ++lits;
      continue;
    }
    /* a match closes the sequence, LZ4.c:533-582.  For m = 1..3 (a 257..259
     * match truncated to uint8_t) (m - 4) wraps and lands in the token's
     * high nibble, and the size counts a match-extension byte */
    const uint8_t tm = m >= 19 ? 15 : (uint8_t)(m - 4);
    seq.match_offset = dist;
    seq.literals_count = lits;
    seq.match_length = m;
    seq.token = (uint8_t)(((lits >= 15 ? 15 : lits) << 4) | tm);
    seq.byte_size = (size_t)lits + 5 + litext_len(lits) + ((uint8_t)(m - 4) >= 15 ? 1 : 0);
    append_sequence(block, &seq);
    lits = 0;
    pos += m;
  }
  if (lits > 0) {                                      /* literal tail, LZ4.c:585-613 */
    seq.match_offset = 0;
    seq.literals_count = lits;
    seq.match_length = 0;
    seq.token = (uint8_t)((lits >= 15 ? 15 : lits) << 4);
    seq.byte_size = (size_t)lits + 5 + litext_len(lits);
    append_sequence(block, &seq);
  }
  block->token = (uint8_t)block->sequences_count;
  block->byte_size += 3;
  fm_block_length = saved;
  /* add_block_to_frame, LZ4.c:461-504 */
  LZ4Block *fb = (LZ4Block *)realloc(frame->frame_blocks, sizeof(LZ4Block) * (frame->blocks + 1));
  if (!fb) {
    perror("Failed to reallocate memory for frame_blocks");
    exit(EXIT_FAILURE);
  }
  frame->frame_blocks = fb;
  fb[frame->blocks++] = *block;
}

static void put_u16(FILE *f, size_t v) {
  const uint8_t b[2] = {(uint8_t)v, (uint8_t)(v >> 8)};   /* low bytes, little endian */
  fwrite(b, 1, 2, f);
}

void write_output(LZ4Frame *frame, FILE *out) {
  const uint8_t nb = (uint8_t)frame->blocks;
  fwrite(&nb, 1, 1, out);
  for (size_t i = 0; i < frame->blocks; i++) {
    const LZ4Block *b = &frame->frame_blocks[i];
    fwrite(&b->token, 1, 1, out);                     /* write_block, LZ4.c:415-425 */
    put_u16(out, b->byte_size);
    for (size_t k = 0; k < b->sequences_count; k++) {
      const LZ4Sequence *q = &b->sequences[k];        /* write_sequence, LZ4.c:365-413 */
      fwrite(&q->token, 1, 1, out);
      put_u16(out, q->byte_size);
      if (q->literals_count >= 15) {
        uint8_t r = (uint8_t)(q->literals_count - 15);
        if (r == 255) {                               /* the uint8_t loop: 255, then 0 */
          const uint8_t ff = 255;
          fwrite(&ff, 1, 1, out);
          r = 0;
        }
        fwrite(&r, 1, 1, out);
      }
      fwrite(q->literals, 1, q->literals_count, out);
      put_u16(out, q->match_offset);
      if (q->match_length >= 4 && (uint8_t)(q->match_length - 4) >= 15) {
        const uint8_t r = (uint8_t)(q->match_length - 4 - 15);
        fwrite(&r, 1, 1, out);
      }
    }
    free(b->sequences);
  }
  free(frame->frame_blocks);
  frame->frame_blocks = NULL;
  frame->blocks = 0;
}

void LZ4_decode(char *input_bin_file, char *log) {
  FILE *input_file = safe_open(input_bin_file, "rb");
  FILE *log_file = safe_open(log, "a");
  size_t n = 0;
  uint8_t *comp = read_all(input_file, &n);
  fclose(input_file);
  fclose(log_file);
  if (!comp) {
    perror("Error: Failed to read input file");
    exit(1);
  }
  /* every block decodes to at most 300 bytes and takes at least 8 */
  size_t cap = (n / 8 + 1) * LZ4R_BLOCK;
  uint8_t *out = (uint8_t *)malloc(cap);
  size_t got = 0;
  if (!out) {
    perror("Error: Unable to allocate memory");
    exit(1);
  }
  /* on the GPU: block boundaries found on the device from the stream alone */
  int rc = lz4r_decompress_stream(comp, n, out, cap, &got);
  if (rc != LZ4R_OK) {
    fprintf(stderr, "Error: %s\n", lz4r_strerror(rc));
    exit(1);
  }
  FILE *f = safe_open(LZ4_UNCOMPRESSED_FILE, "w");
  if (fwrite(out, 1, got, f) != got) {
    perror("Error: write failed");
    exit(1);
  }
  fclose(f);
  free(out);
  free(comp);
}

/* ---- JPEG: one block per call, on the GPU --------------------------------- */

static void *dmalloc(size_t n) {
  void *p = NULL;
  if (hipMalloc(&p, n) != hipSuccess) {
    fprintf(stderr, "Memory allocation failed!\n");
    exit(EXIT_FAILURE);
  }
  return p;
}

void discrete_cosine_transform(uint8_t *data, size_t width, size_t height,
                               double **coefficients) {
  const size_t n = width * height;
  *coefficients = (double *)malloc(n * sizeof(double));
  if (!*coefficients) {
    fprintf(stderr, "Memory allocation failed!\n");
    exit(EXIT_FAILURE);
  }
  uint8_t *din = (uint8_t *)dmalloc(n);
  double *dout = (double *)dmalloc(n * sizeof(double));
  int rc = hipMemcpy(din, data, n, hipMemcpyHostToDevice) == hipSuccess ? JPEGR_OK
                                                                          : JPEGR_ERR_HIP;
  if (rc == JPEGR_OK) rc = jpegr_dct_blocks_device(din, (int)width, (int)height, 1, dout, NULL);
  if (rc == JPEGR_OK &&
      hipMemcpy(*coefficients, dout, n * sizeof(double), hipMemcpyDeviceToHost) != hipSuccess)
    rc = JPEGR_ERR_HIP;
  (void)hipFree(din);
  (void)hipFree(dout);
  if (rc != JPEGR_OK) die_hip("jpegr_dct_blocks_device", rc);
}

void Quantize(double **luminance, size_t *table, size_t size) {
  double *tab = (double *)malloc(size * sizeof(double));
  if (!tab) {
    fprintf(stderr, "Memory allocation failed!\n");
    exit(EXIT_FAILURE);
  }
  for (size_t i = 0; i < size; ++i) tab[i] = (double)table[i];     /* JPEG.c:626 */
  double *dc = (double *)dmalloc(size * sizeof(double));
  double *dt = (double *)dmalloc(size * sizeof(double));
  int rc = JPEGR_OK;
  if (hipMemcpy(dc, *luminance, size * sizeof(double), hipMemcpyHostToDevice) != hipSuccess ||
      hipMemcpy(dt, tab, size * sizeof(double), hipMemcpyHostToDevice) != hipSuccess)
    rc = JPEGR_ERR_HIP;
  if (rc == JPEGR_OK) rc = jpegr_quantize_device(dc, dt, (int)size, size, NULL);
  if (rc == JPEGR_OK &&
      hipMemcpy(*luminance, dc, size * sizeof(double), hipMemcpyDeviceToHost) != hipSuccess)
    rc = JPEGR_ERR_HIP;
  (void)hipFree(dc);
  (void)hipFree(dt);
  free(tab);
  if (rc != JPEGR_OK) die_hip("jpegr_quantize_device", rc);
}

/* Scan order of zigzag_pattern (JPEG.c:693-728): diagonals sum = row + col,
 * even sums bottom-to-top, odd sums top-to-bottom.  perm[k] = source index. */
static size_t zigzag_order(size_t width, size_t height, int *perm) {
  size_t k = 0;
  for (size_t sum = 0; sum + 1 < width + height; ++sum) {
    const size_t r0 = sum < width ? 0 : sum - width + 1;
    const size_t r1 = sum < height ? sum : height - 1;
    if (sum % 2 == 0) {
      for (size_t row = r1 + 1; row-- > r0;)
        if (sum - row < width) perm[k++] = (int)(row * width + (sum - row));
    } else {
      for (size_t row = r0; row <= r1; ++row)
        if (sum - row < width) perm[k++] = (int)(row * width + (sum - row));
    }
  }
  return k;
}

void zigzag_pattern(size_t width, size_t height, double *input, double *output) {
  const size_t n = width * height;
  int *perm = (int *)malloc(n * sizeof(int));
  if (!perm) {
    fprintf(stderr, "Memory allocation failed!\n");
    exit(EXIT_FAILURE);
  }
  const size_t k = zigzag_order(width, height, perm);
  double *din = (double *)dmalloc(n * sizeof(double));
  double *dout = (double *)dmalloc(n * sizeof(double));
  int *dperm = (int *)dmalloc(n * sizeof(int));
  int rc = JPEGR_OK;
  if (hipMemcpy(din, input, n * sizeof(double), hipMemcpyHostToDevice) != hipSuccess ||
      hipMemcpy(dperm, perm, n * sizeof(int), hipMemcpyHostToDevice) != hipSuccess)
    rc = JPEGR_ERR_HIP;
  if (rc == JPEGR_OK && k > 0) rc = jpegr_permute_device(din, dout, dperm, (int)k, k, NULL);
  if (rc == JPEGR_OK &&
      hipMemcpy(output, dout, k * sizeof(double), hipMemcpyDeviceToHost) != hipSuccess)
    rc = JPEGR_ERR_HIP;
  (void)hipFree(din);
  (void)hipFree(dout);
  (void)hipFree(dperm);
  free(perm);
  if (rc != JPEGR_OK) die_hip("jpegr_permute_device", rc);
}
