/*
 * synth.c -- synthetic inputs with the reference's generator semantics
 * (the L2 "input generators" of SURVEY.md §1), seeded so every run is
 * reproducible.
 *
 *   lz4jpeg_rand_rgba      <- generate_noise_image, Experiment/random_image.c:58-74
 *                             (per pixel a = 255, r, g, b = rand() % 256 in that
 *                             order; the reference never seeds, i.e. seed 1)
 *   lz4jpeg_random_passages<- extract_random_passage, Experiment/random_extract.c:8-71
 *                             (start = rand() % (file_size - length), copy
 *                             `length` bytes, '\n' and '\r' -> ' '), repeated
 *                             and concatenated; any byte range of the stream.
 *
 * rand() is glibc's (TYPE_3 additive feedback), the same generator the
 * reference's Linux build uses.
 */
#include <stddef.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

void lz4jpeg_rand_rgba(unsigned seed, int w, int h, uint8_t *rgba)
{
    srand(seed);
    const size_t np = (size_t)w * (size_t)h;
    for (size_t i = 0; i < np; i++) {
        uint8_t *p = rgba + 4 * i;
        p[3] = 255;
        p[0] = (uint8_t)(rand() % 256);
        p[1] = (uint8_t)(rand() % 256);
        p[2] = (uint8_t)(rand() % 256);
    }
}

/* Bytes [first, first + total) of the infinite stream passage_0 passage_1 ...
 * so that every rank of a sharded job can synthesise exactly its own slice.
 * Returns the number of bytes written (== total) or 0 on bad arguments. */
size_t lz4jpeg_random_passages(const uint8_t *src, size_t src_len, unsigned seed,
                               size_t length, size_t first, size_t total, uint8_t *out)
{
    if (!src || !out || length == 0 || src_len <= length) return 0;
    srand(seed);
    size_t k = first / length;                 /* passages before the slice */
    for (size_t i = 0; i < k; i++) (void)rand();
    size_t skip = first - k * length;          /* offset inside passage k */
    size_t w = 0;
    while (w < total) {
        size_t start = (size_t)rand() % (src_len - length);    /* random_extract.c:36 */
        size_t avail = length - skip;
        size_t take = (total - w < avail) ? total - w : avail;
        for (size_t i = 0; i < take; i++) {
            uint8_t c = src[start + skip + i];
            out[w + i] = (c == '\n' || c == '\r') ? ' ' : c;   /* :49-53 */
        }
        w += take;
        skip = 0;
    }
    return w;
}
