/* lzj_host.h -- host-side helpers of the drop-in executables and the
 * compatibility layer (not part of the C ABI in include/): PNG I/O over zlib,
 * and the match provider of the per-block LZ4 API. */
#ifndef LZJ_HOST_H
#define LZJ_HOST_H
#include <stddef.h>
#include <stdint.h>

/* RGBA8 pixels of an 8-bit non-interlaced PNG (malloc'd; caller frees).
 * 0 on success, <0 on I/O or format error. */
int lzj_png_read(const char *path, int *w, int *h, uint8_t **rgba);
/* Write w x h RGBA8 pixels as a PNG.  0 on success. */
int lzj_png_write(const char *path, int w, int h, const uint8_t *rgba);

/* Every position's longest match of the n-byte block at `in` (the
 * reference's find_longest_match, LZ4.c:290-323, matches clamped at the block
 * end): match[p] = len | dist << 16, or 0 when len < 4.  0 or an LZ4R_ERR_*
 * code.  The product's provider runs on the GPU (host/compat.c). */
__attribute__((visibility("hidden"))) int lzj_block_matches(const uint8_t *in, size_t n,
                                                          uint32_t *match);

#endif
