/*
 * jpegr.h -- C ABI of the MI355X JPEG hot path (colour conversion, 4:2:2
 * odd-column subsampling, 8x8/8x4 tiling, fp64 DCT-II, truncating
 * quantisation, zigzag), bit-exact to the reference's sequential C.
 *
 * Replaces, for a whole image (or a batch of images) at once, the reference's
 * per-tile host loop in Algorithms/sequential/JPEG/JPEG.c:
 *   build_luminance_matrix / build_rChrominance_matrix /
 *   build_bChrominance_matrix   JPEG.c:114-185
 *   chroma_subsample            JPEG.c:302-375
 *   divide_image                JPEG.c:496-550
 *   discrete_cosine_transform   JPEG.c:451-494
 *   Quantize                    JPEG.c:621-629
 *   zigzag_pattern              JPEG.c:693-728
 *   (driven by main, JPEG.c:1110-1178)
 *
 * Input: RGBA8 pixels, row-major, 4 bytes/pixel (the reference's Pixel,
 * JPEG.c:29-32; alpha ignored).  Output: per 8x8 tile, 128 int16
 * little-endian = [Y 64 zigzag][Cr 32 zigzag][Cb 32 zigzag]; tiles in raster
 * order (this layout is defined by this library: the reference keeps the
 * quantised coefficients as doubles in memory).  Pixels outside the image
 * read as 0, as divide_image's zero-initialised tiles do (JPEG.c:512-523).
 *
 * No torch types; device pointers are plain `void *` from hipMalloc (or a
 * torch tensor's data_ptr()), `stream` is a hipStream_t (NULL = default).
 * All functions return JPEGR_OK (0) or a negative JPEGR_ERR_* code.
 */
#ifndef JPEGR_H
#define JPEGR_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define JPEGR_OK 0
#define JPEGR_ERR_ARG (-1)     /* bad dimensions / NULL pointer */
#define JPEGR_ERR_HIP (-2)     /* HIP runtime error (no GPU, launch failure) */
#define JPEGR_ERR_NOMEM (-3)   /* device allocation failed */

/* Number of int16 coefficients one w x h image produces: tiles * 128. */
size_t jpegr_coef_count(int w, int h);

/* Device API, asynchronous on `stream`.  `nimg` images of identical size,
 * contiguous (image i at d_rgba + i*w*h*4, output at d_out + i*coef_count). */
int jpegr_encode_device(const void *d_rgba, int w, int h, int nimg,
                        void *d_out_i16, void *stream);

/* Same tiles, but the un-quantised fp64 DCT coefficients in row-major
 * (u*W+v) order per plane: [Y 64][Cr 32][Cb 32] doubles per tile.  This is
 * the value discrete_cosine_transform (JPEG.c:451) leaves in *coefficients;
 * exposed for bit-exact parity checks. */
int jpegr_dct_raw_device(const void *d_rgba, int w, int h, int nimg,
                         void *d_out_f64, void *stream);

/* Host convenience: copies in, runs on the current device, copies out,
 * synchronises.  `out` holds jpegr_coef_count(w, h) int16. */
int jpegr_encode(const uint8_t *rgba, int w, int h, int16_t *out);

/* Event-timed device run for measurement: runs jpegr_encode_device `iters`
 * times on `stream` bracketed by HIP events recorded on that same stream and
 * returns the mean milliseconds per launch in *ms_per_launch. */
int jpegr_time_device(const void *d_rgba, int w, int h, int nimg,
                      void *d_out_i16, int iters, void *stream,
                      float *ms_per_launch);

/* Reconstruction (the decode side of the reference's main, JPEG.c:1131-1425;
 * the RLE/Huffman round trip there is the identity on the coefficients):
 * per tile, reverse zigzag + Inverse_quantize (:631-638), fp64 IDCT in the
 * reference's order with (int)round(x + 128) clamped (:399-448), and
 * assemble_image's YCbCr 4:2:2 -> RGB (:553-619), RGBA8 out (a = 255).
 * d_coef is jpegr_encode_device's layout.  Tiles at raster index >=
 * ceil(w*h/64) are never transformed by the reference (:1131) and keep their
 * original samples: pass the source image as d_rgba_orig to reproduce that
 * (NULL decodes them like the others).  Asynchronous on `stream`. */
int jpegr_reconstruct_device(const void *d_coef, const void *d_rgba_orig, int w, int h,
                             int nimg, void *d_rgba_out, void *stream);

/* Block-level kernels (jpegr_blocks.hip) behind the reference-named API in
 * lz4jpeg_compat.h, asynchronous on `stream`:
 *   jpegr_planes_device: full-resolution uint8 Y, Cr, Cb planes of an RGBA8
 *     image (build_luminance_matrix / build_r,bChrominance_matrix,
 *     JPEG.c:114-185), w*h bytes each.
 *   jpegr_dct_blocks_device: discrete_cosine_transform (JPEG.c:451-494) of
 *     nblocks planar uint8 blocks of `height` rows x `width` columns
 *     (width 8 or 4, height 8), fp64 out, u*width+v order.
 *   jpegr_quantize_device: Quantize (JPEG.c:621-629) in place on n doubles,
 *     element i divided by table[i % size] (fp64 table) and truncated.
 *   jpegr_permute_device: out[i] = in[(i/size)*size + perm[i%size]] for n
 *     doubles (zigzag_pattern, JPEG.c:693-728, with perm = its scan order). */
int jpegr_planes_device(const void *d_rgba, int w, int h, void *d_y, void *d_cr,
                        void *d_cb, void *stream);
int jpegr_dct_blocks_device(const void *d_blocks, int width, int height, int nblocks,
                            void *d_out_f64, void *stream);
int jpegr_quantize_device(void *d_coef_f64, const void *d_table_f64, int size,
                          size_t n, void *stream);
int jpegr_permute_device(const void *d_in_f64, void *d_out_f64, const void *d_perm_i32,
                         int size, size_t n, void *stream);

const char *jpegr_strerror(int code);

/* Entropy stage (JPEG.c:767-1097, run by main at :1211-1349): per tile and
 * channel -- Y 64, Cr 32, Cb 32 zigzagged ints in jpegr_encode_device's
 * layout -- the RLE (count, value) ints (RLE, :767), the per-stream Huffman
 * code exactly as encode_huffman builds it (first-occurrence frequencies
 * :864, heap :895-936, tree :938 with its append-without-sift-up, DFS codes
 * :964), and the encoded sequence (:993).  Output per tile (ntiles = all
 * tiles of all images):
 *   d_bits   256 B: [Y 128][Cr 64][Cb 64] bytes, bits packed MSB-first
 *            (the reference's '0'/'1' chars); the final byte's unused low
 *            bits are 0, bytes past it unspecified
 *   d_meta   3 u32 (Y, Cr, Cb): nbits | rle_len << 16 | ncodes << 24
 *   d_table  256 u32: [Y 128][Cr 64][Cb 64]; entry k = value (int16) |
 *            code length << 16, in the reference's codes[] (DFS) order;
 *            the codes follow from the lengths: code[0] = 0, code[k] =
 *            (code[k-1] + 1) shifted left (or right) to length len[k]
 * d_coef 16-B aligned; d_bits 4-B aligned to encode, d_bits and d_table
 * 16-B aligned to decode (JPEGR_ERR_ARG otherwise).
 * d_scratch: jpegr_entropy_scratch_bytes(ntiles) device bytes.  d_status:
 * 3 u32 on the device, shared by both calls; [0] = streams whose code or
 * sequence would overflow the reference's char code[32] / sequence[1024|512]
 * buffers (undefined behaviour there; truncated here).  Asynchronous on
 * `stream`. */
size_t jpegr_entropy_scratch_bytes(size_t ntiles);
int jpegr_entropy_encode_device(const void *d_coef, size_t ntiles, void *d_bits,
                                void *d_meta, void *d_table, void *d_scratch,
                                void *d_status, void *stream);

/* Inverse: bits + table -> RLE ints (decode_huffman, :1009; a one-code
 * stream has an empty sequence and stands for rle_len copies of its symbol,
 * which the reference keeps in its RLE array) -> ints (inverse_RLE, :810:
 * counts clamped to the stream length, zero fill), written in
 * jpegr_encode_device's layout.  d_status[1] = malformed streams, set by
 * the call itself (no memset needed); d_status[2] is the call's tag, which
 * orders the kernel's own zeroing of [1] before any count is added (keep it
 * to the library; one decode at a time per status array). */
int jpegr_entropy_decode_device(const void *d_bits, const void *d_meta,
                                const void *d_table, size_t ntiles, void *d_coef,
                                void *d_status, void *stream);

#ifdef __cplusplus
}
#endif
#endif /* JPEGR_H */
