/*
 * lz4jpeg_synth.h -- seeded synthetic inputs with the reference generators'
 * semantics (host C, part of liblz4jpeg.so).
 *
 *   lz4jpeg_rand_rgba       <- generate_noise_image   Experiment/random_image.c:58-74
 *   lz4jpeg_random_passages <- extract_random_passage Experiment/random_extract.c:8-71
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
