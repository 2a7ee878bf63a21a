/*
 * lz4jpeg_synth.h -- seeded synthetic inputs with the reference generators'
 * semantics (host C, part of liblz4jpeg.so).
 *
 *   lz4jpeg_rand_rgba       <- generate_noise_image   Experiment/random_image.c:58-74
 *   lz4jpeg_random_passages <- extract_random_passage Experiment/random_extract.c:8-71
 * plus entry at any point of either stream and device-side generators.
 */
#ifndef LZ4JPEG_SYNTH_H
#define LZ4JPEG_SYNTH_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* w*h RGBA8 pixels from glibc rand() after srand(seed): a = 255,
 * r, g, b = rand() % 256 (seed 1 == the reference's unseeded stream). */
void lz4jpeg_rand_rgba(unsigned seed, int w, int h, uint8_t *rgba);

/* Pixels [first_pixel, first_pixel + npix) of that stream (pixel i takes the
 * rand() outputs 3i, 3i+1, 3i+2): image k of a batch of w x h images drawn
 * from one continuous stream starts at pixel k*w*h. */
void lz4jpeg_rand_rgba_stream(unsigned seed, uint64_t first_pixel, size_t npix,
                              uint8_t *rgba);

/* The generator's 31-word state (r[i-31 .. i-1], see host/synth.c) just
 * before rand() output first + c*stride, for c < count, into
 * states[31*c .. 31*c + 30] (jump-ahead by companion-matrix powers). */
void lz4jpeg_rand_states(unsigned seed, uint64_t first, uint64_t stride, size_t count,
                         uint32_t *states);

/* Start offsets of passages [first_passage, first_passage + count) of the
 * random_extract stream (rand() % (src_len - length), random_extract.c:36).
 * Returns count, or 0 on bad arguments. */
size_t lz4jpeg_passage_starts(size_t src_len, unsigned seed, size_t length,
                              uint64_t first_passage, size_t count, uint32_t *starts);

/* Device-side synthesis (csrc/synth.hip), byte-identical to the host
 * functions above, for inputs too large to build on the host (config 4's
 * 64 GiB corpus, config 5's 1024 4K images).  Synchronous: they return once
 * d_out is written on `stream` (a hipStream_t as void *).  0 or a negative
 * error (-1 bad argument, -4 HIP error). */
int lz4jpeg_rand_rgba_device(unsigned seed, uint64_t first_pixel, size_t npix, void *d_rgba,
                             void *stream);
int lz4jpeg_random_passages_device(const uint8_t *src_host, size_t src_len, unsigned seed,
                                   size_t length, uint64_t first, size_t total, void *d_out,
                                   void *stream);

/* Bytes [first, first+total) of the stream of random `length`-byte passages
 * of src (newlines -> spaces), passage k starting at the k-th
 * rand() % (src_len - length) after srand(seed).  Returns bytes written
 * (== total), or 0 on bad arguments. */
size_t lz4jpeg_random_passages(const uint8_t *src, size_t src_len, unsigned seed,
                               size_t length, size_t first, size_t total,
                               uint8_t *out);

#ifdef __cplusplus
}
#endif
#endif /* LZ4JPEG_SYNTH_H */
