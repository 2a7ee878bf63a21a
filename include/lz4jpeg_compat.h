/*
 * lz4jpeg_compat.h -- the reference's own in-process entry points, with the
 * reference's names and signatures, implemented on the MI355X path
 * (liblz4jpeg.so).  Code written against Algorithms/sequential/{LZ4,JPEG}
 * links against these unchanged; the batch C ABI in lz4r.h / jpegr.h is the
 * fast interface.
 *
 *   lz4_encode                 <- Algorithms/sequential/LZ4/LZ4.c:670-742
 *       reads LZ4_INPUT_FILE, appends the stream to LZ4_COMPRESSED_FILE,
 *       writes the "%02X " dump to LZ4_HEX_FILE; compression runs on the GPU
 *       (lz4r_compress).  Input < 300 B: message + exit(1) (LZ4.c:632-637).
 *   LZ4_decode                 <- LZ4.c:1038-1121
 *       decodes input_bin_file into LZ4_UNCOMPRESSED_FILE with the exact
 *       decoder (lz4r_decompress); `log` is opened for append like the
 *       reference and left untouched.
 *   discrete_cosine_transform  <- Algorithms/sequential/JPEG/JPEG.c:451-494
 *       width 8 or 4, height 8 (the shapes the reference calls); mallocs
 *       *coefficients (caller frees, JPEG.c:1447).  GPU: jpegr_dct_blocks_device.
 *   Quantize                   <- JPEG.c:621-629   GPU: jpegr_quantize_device
 *   zigzag_pattern             <- JPEG.c:693-728   GPU: jpegr_permute_device
 *
 * Paths are relative to the working directory, as the reference's #defines
 * (LZ4.c:24-28) are: the drivers run the executables from Experiment/.
 */
#ifndef LZ4JPEG_COMPAT_H
#define LZ4JPEG_COMPAT_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define LZ4_LOG_FILE "../Output-Input/log/encoding_log.txt"
#define LZ4_COMPRESSED_FILE "../Output-Input/out/compressed.bin"
#define LZ4_UNCOMPRESSED_FILE "../Output-Input/out/uncompressed.txt"
#define LZ4_INPUT_FILE "../Output-Input/input/input.txt"
#define LZ4_HEX_FILE "../Output-Input/out/compressed.txt"

void lz4_encode(void);
void LZ4_decode(char *input_bin_file, char *log);

void discrete_cosine_transform(uint8_t *data, size_t width, size_t height,
                               double **coefficients);
void Quantize(double **luminance, size_t *table, size_t size);
void zigzag_pattern(size_t width, size_t height, double *input, double *output);

#ifdef __cplusplus
}
#endif
#endif /* LZ4JPEG_COMPAT_H */
