/*
 * synth.c -- synthetic inputs with the reference generators' semantics
 * (the L2 "input generators" of SURVEY.md §1), seeded so every run is
 * reproducible.
 *
 *   lz4jpeg_rand_rgba      <- generate_noise_image, Experiment/random_image.c:58-74
 *                             (per pixel a = 255, r, g, b = rand() % 256 in that
 *                             order; the reference never seeds, i.e. seed 1)
 *   lz4jpeg_rand_rgba_stream  the same stream from any pixel on, so that a batch
 *                             of images is one continuous rand() sequence
 *                             (BASELINE config 5) and any rank can start at its
 *                             own first image
 *   lz4jpeg_random_passages<- extract_random_passage, Experiment/random_extract.c:8-71
 *                             (start = rand() % (file_size - length), copy
 *                             `length` bytes, '\n' and '\r' -> ' '), repeated
 *                             and concatenated; any byte range of the stream.
 *
 * rand() is glibc's TYPE_3 additive-feedback generator (the one the
 * reference's Linux build calls), restated here so a stream can be entered
 * anywhere: with r[0..30] from the seed's Lehmer sequence (r[i] = 16807 r[i-1]
 * mod 2^31-1), r[i] = r[i-31] for i = 31..33 and r[i] = r[i-31] + r[i-3]
 * (mod 2^32) after, the k-th rand() after srand(seed) is r[344 + k] >> 1.
 * The recurrence is linear, so the 31-word state at any index is the seed
 * state times a power of the 31x31 companion matrix (mod 2^32): a jump of k
 * costs log2(k) matrix squarings.  tests/test_synth.py checks every function
 * against libc's own srand()/rand().
 */
#include <stddef.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../../include/lz4jpeg_synth.h"

#define RDEG 31

/* r[i - 31 .. i - 1] for i = 344 + k: the state just before the k-th output */
typedef struct { uint32_t w[RDEG]; } rstate;

static void seed_state(unsigned seed, uint32_t r[34]) {
    int32_t v = seed ? (int32_t)seed : 1;
    r[0] = (uint32_t)v;
    for (int i = 1; i < 31; i++) {
        /* 16807 * r mod (2^31 - 1) by Schrage's method, as glibc computes it */
        const int32_t hi = v / 127773, lo = v % 127773;
        v = 16807 * lo - 2836 * hi;
        if (v < 0) v += 2147483647;
        r[i] = (uint32_t)v;
    }
    r[31] = r[0];
    r[32] = r[1];
    r[33] = r[2];
}

/* state before output 0: r[313 .. 343] */
static void state_at_zero(unsigned seed, rstate *s) {
    uint32_t r[34 + 310];
    seed_state(seed, r);
    for (int i = 34; i < 344; i++) r[i] = r[i - 31] + r[i - 3];
    memcpy(s->w, r + 344 - RDEG, sizeof(s->w));
}

static uint32_t step(rstate *s, int *pos) {
    /* ring: w[*pos] holds r[i - 31], w[(*pos + 28) % 31] holds r[i - 3] */
    const int p = *pos;
    const uint32_t v = s->w[p] + s->w[(p + 28) % RDEG];
    s->w[p] = v;
    *pos = (p + 1) % RDEG;
    return v;
}

/* 31x31 matrices over Z / 2^32: row-major, M[i][j] */
typedef struct { uint32_t m[RDEG][RDEG]; } rmat;

static void mat_mul(const rmat *a, const rmat *b, rmat *c) {
    rmat t;
    for (int i = 0; i < RDEG; i++)
        for (int j = 0; j < RDEG; j++) {
            uint32_t acc = 0;
            for (int k = 0; k < RDEG; k++) acc += a->m[i][k] * b->m[k][j];
            t.m[i][j] = acc;
        }
    *c = t;
}

/* A^k for the companion matrix of one step: v' = A v, v = (r[i-31] .. r[i-1]) */
static void jump_matrix(uint64_t k, rmat *out) {
    rmat base, acc;
    memset(&base, 0, sizeof(base));
    for (int i = 0; i < RDEG - 1; i++) base.m[i][i + 1] = 1;
    base.m[RDEG - 1][0] = 1;            /* r[i-31] */
    base.m[RDEG - 1][RDEG - 3] = 1;     /* r[i-3]  */
    memset(&acc, 0, sizeof(acc));
    for (int i = 0; i < RDEG; i++) acc.m[i][i] = 1;
    while (k) {
        if (k & 1) mat_mul(&base, &acc, &acc);
        mat_mul(&base, &base, &base);
        k >>= 1;
    }
    *out = acc;
}

static void apply(const rmat *a, const rstate *v, rstate *out) {
    rstate t;
    for (int i = 0; i < RDEG; i++) {
        uint32_t acc = 0;
        for (int k = 0; k < RDEG; k++) acc += a->m[i][k] * v->w[k];
        t.w[i] = acc;
    }
    *out = t;
}

static void state_at(unsigned seed, uint64_t index, rstate *s) {
    state_at_zero(seed, s);
    if (index) {
        rmat a;
        jump_matrix(index, &a);
        apply(&a, s, s);
    }
}

void lz4jpeg_rand_states(unsigned seed, uint64_t first, uint64_t stride, size_t count,
                         uint32_t *states)
{
    rstate s;
    state_at(seed, first, &s);
    rmat a;
    if (count > 1) jump_matrix(stride, &a);
    for (size_t c = 0; c < count; c++) {
        memcpy(states + (size_t)RDEG * c, s.w, sizeof(s.w));
        if (c + 1 < count) apply(&a, &s, &s);
    }
}

void lz4jpeg_rand_rgba_stream(unsigned seed, uint64_t first_pixel, size_t npix, uint8_t *rgba)
{
    rstate s;
    state_at(seed, 3 * first_pixel, &s);
    int pos = 0;
    for (size_t i = 0; i < npix; i++) {
        uint8_t *p = rgba + 4 * i;
        p[0] = (uint8_t)(step(&s, &pos) >> 1);   /* rand() % 256 */
        p[1] = (uint8_t)(step(&s, &pos) >> 1);
        p[2] = (uint8_t)(step(&s, &pos) >> 1);
        p[3] = 255;
    }
}

void lz4jpeg_rand_rgba(unsigned seed, int w, int h, uint8_t *rgba)
{
    lz4jpeg_rand_rgba_stream(seed, 0, (size_t)w * (size_t)h, rgba);
}

size_t lz4jpeg_passage_starts(size_t src_len, unsigned seed, size_t length, uint64_t first_passage,
                              size_t count, uint32_t *starts)
{
    if (!starts || length == 0 || src_len <= length || src_len - length > 0xffffffffu) return 0;
    rstate s;
    state_at(seed, first_passage, &s);
    int pos = 0;
    for (size_t k = 0; k < count; k++)                         /* random_extract.c:36 */
        starts[k] = (uint32_t)((size_t)(step(&s, &pos) >> 1) % (src_len - length));
    return count;
}

/* Bytes [first, first + total) of the infinite stream passage_0 passage_1 ...
 * so that every rank of a sharded job can synthesise exactly its own slice.
 * Returns the number of bytes written (== total) or 0 on bad arguments. */
size_t lz4jpeg_random_passages(const uint8_t *src, size_t src_len, unsigned seed,
                               size_t length, size_t first, size_t total, uint8_t *out)
{
    if (!src || !out || length == 0 || src_len <= length) return 0;
    rstate s;
    const size_t k = first / length;                 /* passages before the slice */
    state_at(seed, k, &s);
    int pos = 0;
    size_t skip = first - k * length;                /* offset inside passage k */
    size_t w = 0;
    while (w < total) {
        const size_t start = (size_t)(step(&s, &pos) >> 1) % (src_len - length);
        const size_t avail = length - skip;
        const size_t take = (total - w < avail) ? total - w : avail;
        for (size_t i = 0; i < take; i++) {
            const uint8_t c = src[start + skip + i];
            out[w + i] = (c == '\n' || c == '\r') ? ' ' : c;   /* :49-53 */
        }
        w += take;
        skip = 0;
    }
    return w;
}
