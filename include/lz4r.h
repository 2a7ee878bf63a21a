/*
 * lz4r.h -- C ABI of the MI355X "LZ4" compressor: the reference's exhaustive
 * per-300-byte-block longest-match finder, greedy parser and custom
 * token/sequence byte emitter, bit-exact to Algorithms/sequential/LZ4/LZ4.c
 * (canonical semantics: matches are clamped at the block end).
 *
 * Entry points and the reference interface each replaces
 * (Algorithms/sequential/LZ4/LZ4.c):
 *   lz4r_compress_device / lz4r_compress   <- lz4_encode()            :670-742
 *        (divide_input :123-177, the block loop :707-721, write_output
 *         :427-441 minus the fixed file paths; the bytes written equal
 *         compressed.bin)
 *   per block inside the kernels            <- block_encode()          :506-620
 *                                              find_longest_match()    :290-323
 *                                              add_sequence_to_block() :443-459
 *                                              write_sequence/_block() :365-425
 *   lz4r_compress_segment_device            <- the same, for a run of whole
 *        blocks without the frame header byte (multi-GPU shards)
 *
 * Stream format (frame := u8 nblocks&0xFF, block*; block := u8 nseq&0xFF,
 * u16le (sum of sequence sizes + 3), sequence*).
 *
 * Errors: negative LZ4R_ERR_* codes instead of the reference's
 * perror()+exit(1).  An input shorter than one block (300 B) is
 * LZ4R_ERR_TOO_SMALL, the reference's exit(1) at LZ4.c:632-637.
 *
 * No torch types: device pointers are plain `void *`, `stream` is a
 * hipStream_t passed as `void *` (NULL = legacy default stream).  A context
 * owns the scratch buffers; one context per thread (or serialise).
 */
#ifndef LZ4R_H
#define LZ4R_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define LZ4R_BLOCK 300            /* DEFAULT_BLOCK_LENGTH, LZ4.c:23 */
#define LZ4R_BLOCK_BOUND 1152     /* max encoded bytes of one block */

#define LZ4R_OK 0
#define LZ4R_ERR_ARG (-1)         /* NULL pointer / bad argument */
#define LZ4R_ERR_TOO_SMALL (-2)   /* input < LZ4R_BLOCK (LZ4.c:632) */
#define LZ4R_ERR_CAPACITY (-3)    /* output buffer too small; *out_len = need */
#define LZ4R_ERR_HIP (-4)         /* HIP runtime error */
#define LZ4R_ERR_NOMEM (-5)       /* device allocation failed */
#define LZ4R_ERR_CORRUPT (-6)     /* decoder: malformed stream; compressor: corrupt LDS index */
/* bit 63 of an async call's length word: the call met a corrupt LDS index */
#define LZ4R_LEN_CORRUPT (1ull << 63)

/* Inputs up to 2^40 bytes per call; the kernels run in chunks of 2^24 blocks
 * (5.03 GB), so device scratch is ~10.7 GB of block slots at most plus
 * 16 B per block of the whole input. */

typedef struct lz4r_ctx lz4r_ctx;

/* Create a context bound to the current HIP device. */
int lz4r_ctx_create(lz4r_ctx **ctx);
void lz4r_ctx_destroy(lz4r_ctx *ctx);

/* Worst-case compressed size of n input bytes (frame header included). */
size_t lz4r_compress_bound(size_t n);
size_t lz4r_nblocks(size_t n);

/* Compress n bytes at d_in (device) into d_out (device, cap bytes) on
 * `stream`, then synchronise it and return the compressed length in
 * *out_len.  Frame header included.  Bytes equal lz4_encode()'s
 * compressed.bin for the same input. */
int lz4r_compress_device(lz4r_ctx *ctx, const void *d_in, size_t n,
                         void *d_out, size_t cap, size_t *out_len,
                         void *stream);

/* Asynchronous form: enqueue only.  The compressed length (or the required
 * capacity, if larger than cap: nothing past cap is written) is stored as a
 * uint64 at d_out_len (device) when the stream reaches it.  Bit 63 of that
 * word (LZ4R_LEN_CORRUPT) is set, instead of an error return, when the call
 * met a corrupt bucket head in lz4_tiles' LDS index (see lz4r_check): the
 * caller gets the verdict in the same read-back as the length and must not
 * use the stream then.  The length is the word without that bit. */
int lz4r_compress_async(lz4r_ctx *ctx, const void *d_in, size_t n,
                        void *d_out, size_t cap, void *d_out_len,
                        void *stream);

/* A run of whole 300-byte blocks without the frame header byte, for shards
 * of a multi-GPU job; asynchronous, length at d_out_len like
 * lz4r_compress_async.  Only the globally last shard (final_shard != 0) may
 * end in a short block: a non-final shard whose n is not a multiple of 300
 * is rejected with LZ4R_ERR_ARG (its stream would differ from the single-GPU
 * one).  n == 0 (more ranks than blocks) enqueues a zero length.
 * Concatenating the segments of consecutive shards after one header byte
 * (u8 total_blocks & 0xFF) yields the single-GPU stream. */
int lz4r_compress_segment_async(lz4r_ctx *ctx, const void *d_in, size_t n,
                                void *d_out, size_t cap, void *d_out_len,
                                int final_shard, void *stream);

/* find_longest_match (LZ4.c:290-323) at every position of every 300-byte
 * block of the n bytes at d_in, in one launch, asynchronous on `stream`:
 * d_matches[300 b + p] (uint32, n entries, device) = len | dist << 16 for
 * the longest match at p of block b (the earliest source among equals,
 * LZ4.c:307; matches clamped at the block end), or 0 when len < 4
 * (MIN_MATCH_LENGTH).  len is not truncated: the reference's uint8_t return
 * value is len & 0xFF. */
int lz4r_block_matches_device(const void *d_in, size_t n, void *d_matches, void *stream);

/* find_longest_match (LZ4.c:290-323) at every position of ONE block of any
 * length n (what block_encode does for a block_length other than 300): the
 * reference's whole window (sources i >= p - WINDOW_SIZE, LZ4.c:295), match
 * length capped at MAX_MATCH_LENGTH (1024, LZ4.c:20) and at the block end.
 * d_matches[p] = len | dist << 16, or 0 when len < 4.  O(n * min(n, 65535))
 * work: a compatibility path.  Asynchronous on `stream`; n < 2^32. */
int lz4r_window_matches_device(const void *d_in, size_t n, void *d_matches, void *stream);

/* After a compress call: copy the encoded byte count (uint16) of each of the
 * first `count` blocks of the last call to `dst` (host or device memory),
 * then synchronise `stream`.  Block b's bytes start at sum(sizes[0..b)) after
 * the frame header byte.  Written by the kernel on every call (2 B/block). */
int lz4r_copy_block_sizes(const lz4r_ctx *ctx, void *dst, size_t count,
                          void *stream);

/* After a compress call: copy the first `count` per-block output offsets
 * (uint64, exclusive scan, relative to the first block byte -- add 1 for a
 * framed stream) of the last call to `dst` (host or device memory), then
 * synchronise `stream`.  The placement kernel writes them on the device as
 * it computes them (8 B/block); no host prefix sum. */
int lz4r_copy_block_offsets(const lz4r_ctx *ctx, void *dst, size_t count,
                            void *stream);

/* The same offsets in place: *d_offsets = the context's device array of the
 * last call's *count block offsets (valid until the next call on ctx; ready
 * when the call's stream reaches its end).  This is what the block-parallel
 * decoder takes, without a host round trip. */
int lz4r_block_offsets_device(const lz4r_ctx *ctx, const void **d_offsets,
                              size_t *count);

/* Decode a framed stream (bytes as lz4r_compress writes them) back to the
 * input.  Host C; replaces LZ4_decode / interpret_frame (LZ4.c:937-1121),
 * which mis-parse streams of >= 256 blocks or literal runs >= 271: blocks are
 * read until the input ends (the frame byte is checked modulo 256), literal
 * lengths come from the exact u16 size field, and the format's one
 * ambiguous token (a match of 257..259 stored as M = 1..3, LZ4.c:317) is
 * resolved per block by backtracking.  LZ4R_ERR_CAPACITY sets *out_len to
 * the length needed so far; LZ4R_ERR_CORRUPT on a malformed stream. */
int lz4r_decompress(const uint8_t *in, size_t in_len, uint8_t *out, size_t cap,
                    size_t *out_len);

/* Block-parallel GPU decoder (csrc/lz4r_gpudec.hip), asynchronous on
 * `stream`.  d_in: the framed stream (in_len bytes, device); d_block_offsets:
 * nb uint64 offsets of each block's first byte relative to the first block
 * byte, as lz4r_copy_block_offsets returns them for the compressing call
 * (the format cannot be split without them).  Block b decodes to
 * d_out[300 b ...]; nothing at or past out_cap is written.  d_result: two
 * uint64 on the device: [0] = decoded length (if it exceeds out_cap, only
 * out_cap bytes were written), [1] = ~0 if every block was consistent, else
 * 1 + the index of the first malformed block. */
int lz4r_decompress_device(const void *d_in, size_t in_len, const void *d_block_offsets,
                           size_t nb, void *d_out, size_t out_cap, void *d_result,
                           void *stream);

/* Decode a bare framed stream on the GPU -- only the stream, as LZ4_decode
 * (LZ4.c:1038) takes the file: the block boundaries are found on the device
 * (csrc/lz4r_gpudec.hip: a candidate header per 8 KiB chunk, a lane per
 * chunk walking the size fields, one wave re-walking any chunk whose
 * predecessor does not end on its candidate), then lz4_decode_blocks checks
 * every block against them.  Streams with truncated matches (whose size
 * fields over-count, LZ4.c:569-575) take a second pass that parses every
 * block.  d_in / d_out are device pointers; synchronises `stream`;
 * *out_len = decoded length.  LZ4R_ERR_CORRUPT when the blocks do not chain
 * from the frame byte to the end of the stream or a block does not decode;
 * LZ4R_ERR_CAPACITY (with *out_len = need, or a lower bound on it when the
 * stream has more blocks than out_cap can hold) when out_cap is too small.
 * One host read-back per pass when out_cap / 300 + 1 <= (in_len - 1) / 8 + 1
 * (the output bounds the block count); a larger out_cap reads the block
 * count back first.  Device scratch: ~20 B per 8 KiB of stream + 8 B per
 * block out_cap can hold (stream-ordered allocation from a per-device pool
 * the library keeps: returned to the pool on return, not to the device, so
 * the next call does not map it again). */
int lz4r_decompress_stream_device(const void *d_in, size_t in_len, void *d_out,
                                  size_t out_cap, size_t *out_len, void *stream);

/* Host-buffer form of lz4r_decompress_stream_device (copies in and out). */
int lz4r_decompress_stream(const uint8_t *in, size_t in_len, uint8_t *out, size_t cap,
                           size_t *out_len);

/* Host convenience wrapper around lz4r_compress_device (copies in and out). */
int lz4r_compress(const uint8_t *in, size_t n, uint8_t *out, size_t cap,
                  size_t *out_len);

/* Synchronise `stream` and report whether the last compress call on ctx met
 * a corrupt bucket head in lz4_tiles' LDS index (a head that is neither empty
 * nor an earlier position of the block: never on a sound LDS; the walk ends
 * anyway, chains strictly decrease): LZ4R_ERR_CORRUPT or LZ4R_OK.  It reads a
 * verdict word the context owns, written by the call's last scan kernel
 * beside LZ4R_LEN_CORRUPT of the call's length word (so the caller's length
 * buffer may already be freed).  Every call folds the kernel's status into
 * its own length word and clears it, so an async caller that reads the
 * length needs no separate check.  lz4r_compress_device checks by itself.
 * Ordering: the verdict word is one per context and every call overwrites it,
 * whatever stream that call runs on.  Pass the stream the compress call ran
 * on, and call lz4r_check before the next compress call on this context;
 * otherwise the word read is unordered with, or belongs to, another call
 * (the length word's bit 63 has no such restriction). */
int lz4r_check(lz4r_ctx *ctx, void *stream);

/* Measurement: when enabled, every compress call records HIP events on its
 * own launch stream around the whole call and around each launch of the
 * compressor kernel lz4_tiles (one per 2^24-block chunk of the input).
 * lz4r_last_timing waits for the last call's end event and returns the
 * call's duration and the summed lz4_tiles durations in milliseconds.
 * Enabling starts a new record; each timed call has its own events (a ring
 * of the newest 4096 calls), so back-to-back async calls are timed without a
 * host wait between them: lz4r_timed_calls then waits for the newest call and
 * fills ms_call/ms_match with the newest min(calls, 4096, max) calls' times,
 * oldest first, and their number in *count. */
int lz4r_set_timing(lz4r_ctx *ctx, int enable);
int lz4r_last_timing(lz4r_ctx *ctx, float *ms_call, float *ms_match);
int lz4r_timed_calls(lz4r_ctx *ctx, size_t max, float *ms_call, float *ms_match, size_t *count);

const char *lz4r_strerror(int code);

#ifdef __cplusplus
}
#endif
#endif /* LZ4R_H */
