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
 *   find_longest_match         <- LZ4.c:290-323 (GPU, per block)
 *   block_encode               <- LZ4.c:506-620, with LZ4Sequence / LZ4Block /
 *                                 LZ4Frame (LZ4.c:30-52)
 *   write_output               <- LZ4.c:365-441
 *   LZ4_decode                 <- LZ4.c:1038-1121
 *       decodes input_bin_file into LZ4_UNCOMPRESSED_FILE on the GPU from
 *       the stream alone (lz4r_decompress_stream: block boundaries found on
 *       the device); `log` is opened for append like the reference and left
 *       untouched.
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
#include <stdio.h>

#ifdef __cplusplus
extern "C" {
#endif

#define LZ4_LOG_FILE "../Output-Input/log/encoding_log.txt"
#define LZ4_COMPRESSED_FILE "../Output-Input/out/compressed.bin"
#define LZ4_UNCOMPRESSED_FILE "../Output-Input/out/uncompressed.txt"
#define LZ4_INPUT_FILE "../Output-Input/input/input.txt"
#define LZ4_HEX_FILE "../Output-Input/out/compressed.txt"

/* LZ4.c:30-58, field for field (size_t fields serialise as their low bytes) */
typedef struct {
  uint8_t token;
  size_t byte_size;
  uint8_t *literals;          /* points into the caller's block buffer (LZ4.c:525) */
  size_t literals_count;
  uint16_t match_offset;
  size_t match_length;
} LZ4Sequence;

typedef struct {
  uint8_t token;              /* = sequences_count & 0xFF (LZ4.c:615) */
  size_t byte_size;
  size_t sequences_count;
  LZ4Sequence *sequences;
} LZ4Block;

typedef struct {
  size_t blocks;
  LZ4Block *frame_blocks;
} LZ4Frame;

typedef struct {
  uint8_t *input_data;
  size_t input_size;
} LZ4Context;

void lz4_encode(void);
void LZ4_decode(char *input_bin_file, char *log);

/* find_longest_match <- LZ4.c:290-323.  The longest match at current_index
 * of the block starting at `input` (earliest source among equals), as
 * (uint8_t)len with *match_distance set, or 0 when len < 4.  The block is
 * the one block_encode is encoding (its block_length, any length), otherwise
 * the 300 bytes at input (DEFAULT_BLOCK_LENGTH, LZ4.c:23: a standalone call
 * needs 300 readable bytes there, as the reference reads up to
 * MAX_MATCH_LENGTH past current_index); matches are clamped at the block end
 * (the reference reads past it).  GPU: the first call for a
 * block computes every position of it in one launch
 * (lz4r_block_matches_device; lz4r_window_matches_device with the 65535-byte
 * window for a block longer than 300); later calls on the same bytes are
 * lookups. */
uint8_t find_longest_match(uint8_t *input, size_t current_index, uint16_t *match_distance);

/* block_encode <- LZ4.c:506-620: the greedy parse of one block into `block`
 * (sequences appended with their token / byte_size quirks), then
 * block->token = sequence count, byte_size += 3, and a copy of *block is
 * appended to frame->frame_blocks.  log_file / output_file are unused, as in
 * the reference.  Matches come from find_longest_match (the GPU). */
void block_encode(const char *block_entry, size_t block_length, LZ4Block *block,
                  FILE *log_file, FILE *output_file, LZ4Frame *frame);

/* write_output <- LZ4.c:427-441: u8 frame->blocks, then every block
 * (write_block / write_sequence, LZ4.c:365-425) -- compressed.bin's bytes.
 * Releases frame->frame_blocks and the sequence arrays the blocks own (the
 * reference leaks the latter) and resets the frame. */
void write_output(LZ4Frame *frame, FILE *output_file);

void discrete_cosine_transform(uint8_t *data, size_t width, size_t height,
                               double **coefficients);
void Quantize(double **luminance, size_t *table, size_t size);
void zigzag_pattern(size_t width, size_t height, double *input, double *output);

#ifdef __cplusplus
}
#endif
#endif /* LZ4JPEG_COMPAT_H */
