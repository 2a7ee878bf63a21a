/* lzj_host.h -- host-side helpers of the drop-in executables (not part of
 * the C ABI in include/): PNG I/O over zlib. */
#ifndef LZJ_HOST_H
#define LZJ_HOST_H
#include <stdint.h>

/* RGBA8 pixels of an 8-bit non-interlaced PNG (malloc'd; caller frees).
 * 0 on success, <0 on I/O or format error. */
int lzj_png_read(const char *path, int *w, int *h, uint8_t **rgba);
/* Write w x h RGBA8 pixels as a PNG.  0 on success. */
int lzj_png_write(const char *path, int w, int h, const uint8_t *rgba);

#endif
