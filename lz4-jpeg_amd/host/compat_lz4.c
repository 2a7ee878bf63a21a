/*
 * compat_lz4.c -- the reference's per-block LZ4 API (include/lz4jpeg_compat.h:
 * find_longest_match, block_encode, write_output) as host C over the match
 * provider lzj_block_matches (lzj_host.h).  The provider is the GPU in the
 * product (host/compat.c: one launch of the batch match finder per block);
 * this file has no HIP dependency, so the sanitizer build (`make sanitize`)
 * links it with a CPU provider and runs it under ASan/UBSan.
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../include/lz4jpeg_compat.h"
#include "../../include/lz4r.h"
#include "lzj_host.h"

/* ---- per-block API: find_longest_match / block_encode / write_output ---- */

/* The block find_longest_match answers for: its bytes, and every position's
 * len | dist << 16 from the match provider (lzj_block_matches: the GPU in
 * the product, host/compat.c; a CPU restatement in the sanitizer build).
 * The host buffers grow to the block; per thread. */
static __thread struct {
  const uint8_t *ptr;
  size_t n, cap;
  uint8_t *bytes;
  uint32_t *match;
  int valid;
} fm_cache;
static __thread size_t fm_block_length;   /* set while block_encode runs */

static void fm_reserve(size_t n) {
  if (n <= fm_cache.cap) return;
  free(fm_cache.bytes);
  free(fm_cache.match);
  fm_cache.bytes = (uint8_t *)malloc(n);
  fm_cache.match = (uint32_t *)malloc(n * sizeof(uint32_t));
  fm_cache.valid = 0;
  fm_cache.cap = 0;
  if (!fm_cache.bytes || !fm_cache.match) {
    perror("Error: Unable to allocate memory");
    exit(1);
  }
  fm_cache.cap = n;
}

static void fm_load(const uint8_t *input, size_t n) {
  if (fm_cache.valid && fm_cache.ptr == input && fm_cache.n == n &&
      memcmp(fm_cache.bytes, input, n) == 0)
    return;
  fm_reserve(n < LZ4R_BLOCK ? LZ4R_BLOCK : n);
  const int rc = lzj_block_matches(input, n, fm_cache.match);
  if (rc != LZ4R_OK) {
    fprintf(stderr, "Error: find_longest_match failed (%d)\n", rc);
    exit(1);
  }
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

