/*
 * oracle/lz4_oracle.c -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the reference's "LZ4" compressor (a brute-force LZ77 over
 * 300-byte blocks with a custom byte format).  It is the *checker* for the HIP
 * path: only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg
 * may load it.  The product library (lz4-jpeg_amd/) never links or calls it.
 *
 * Parity pin: reproduces Output-Input/out/compressed.bin committed in the
 * reference (tests/golden/lz4_input.compressed.bin) byte-for-byte, plus the
 * oracle-produced md5s of SURVEY.md Appendix A4 (tests/test_oracle.py).
 * The reference's own LZ4.c is NOT buildable here (it #includes the
 * Windows-only <direct.h>, LZ4.c:17) -- see DESIGN.md "Oracle".
 *
 * Canonical semantics: a match never extends past the end of
 * its block.  The reference reads past the block (LZ4.c:302, heap over-read);
 * for text inputs under MALLOC_PERTURB_ the two agree.
 *
 * Citations are to /root/reference/Algorithms/sequential/LZ4/LZ4.c.
 */
#include <stddef.h>
#include <stdint.h>
#include <string.h>
#include <pthread.h>

#define LZ4O_BLOCK 300        /* DEFAULT_BLOCK_LENGTH, LZ4.c:23 */
#define LZ4O_MAX_MATCH 1024   /* MAX_MATCH_LENGTH, LZ4.c:20 */
#define LZ4O_MIN_MATCH 4      /* MIN_MATCH_LENGTH, LZ4.c:21 */
#define LZ4O_WINDOW 65535     /* WINDOW_SIZE, LZ4.c:22 */

/* find_longest_match, LZ4.c:290-323: scan every earlier position of the
 * block, strict '>' so the smallest i wins ties; the length is returned
 * through a uint8_t (truncation), distance through a uint16_t. */
static unsigned lz4o_find_longest_match(const uint8_t *blk, size_t n, size_t p,
                                        unsigned *dist)
{
    size_t best = 0, best_dist = 0;
    size_t start = (p >= LZ4O_WINDOW) ? p - LZ4O_WINDOW : 0;     /* LZ4.c:295 */
    for (size_t i = start; i < p; ++i) {                          /* LZ4.c:297 */
        size_t l = 0;
        /* LZ4.c:301-305, clamped at the block end (p + l < n) */
        while (l < LZ4O_MAX_MATCH && p + l < n && blk[i + l] == blk[p + l])
            l++;
        if (l > best) {                                           /* LZ4.c:307 */
            best = l;
            best_dist = p - i;
        }
    }
    if (best >= LZ4O_MIN_MATCH) {                                 /* LZ4.c:314 */
        *dist = (uint16_t)best_dist;
        return (uint8_t)best;                                     /* LZ4.c:317 */
    }
    return 0;
}

/* byte count of the literal-length extension, LZ4.c:548-560 / 372-386 */
static unsigned litext_len(size_t L)
{
    if (L < 15) return 0;
    uint8_t r = (uint8_t)(L - 15);
    return (r == 255) ? 2u : 1u;
}

static uint8_t *put_litext(uint8_t *o, size_t L)
{
    if (L >= 15) {                                                /* LZ4.c:372 */
        uint8_t r = (uint8_t)(L - 15);
        while (r >= 255) { *o++ = 255; r -= 255; }
        *o++ = r;
    }
    return o;
}

/* block_encode (LZ4.c:506-620) + write_block/write_sequence (LZ4.c:365-425).
 * Writes the block record to `out` and returns the number of bytes written. */
size_t lz4o_encode_block(const uint8_t *blk, size_t n, uint8_t *out)
{
    uint8_t *o = out + 3;
    size_t nseq = 0, size_sum = 0;
    size_t p = 0, L = 0, lit = 0;
    while (p < n) {                                               /* LZ4.c:516 */
        unsigned dist = 0;
        unsigned M = lz4o_find_longest_match(blk, n, p, &dist);   /* uint8_t */
        if (M == 0) {                                             /* LZ4.c:521 */
            if (L == 0) lit = p;
            p++;
            L++;
            continue;
        }
        uint8_t tl = (L >= 15) ? 15 : (uint8_t)L;                 /* LZ4.c:540 */
        uint8_t tm = (M >= 19) ? 15 : (uint8_t)(M - LZ4O_MIN_MATCH); /* :542 */
        uint8_t tok = (uint8_t)((tl << 4) | tm);                  /* LZ4.c:544 */
        uint8_t adj = (uint8_t)(M - 4);                           /* LZ4.c:562 */
        size_t S = L + 5 + litext_len(L) + (adj >= 15 ? 1 : 0);   /* :546-575 */
        *o++ = tok;                                               /* LZ4.c:367 */
        *o++ = (uint8_t)(S & 0xFF);                               /* LZ4.c:369 */
        *o++ = (uint8_t)((S >> 8) & 0xFF);
        o = put_litext(o, L);
        memcpy(o, blk + lit, L);                                  /* LZ4.c:388 */
        o += L;
        *o++ = (uint8_t)(dist & 0xFF);                            /* LZ4.c:390 */
        *o++ = (uint8_t)((dist >> 8) & 0xFF);
        if (M >= 4 && adj >= 15)                                  /* LZ4.c:393-411 */
            *o++ = (uint8_t)(adj - 15);
        size_sum += S;
        nseq++;
        L = 0;
        p += M;                                                   /* LZ4.c:581 */
    }
    if (L > 0) {                                                  /* LZ4.c:585-613 */
        uint8_t tl = (L >= 15) ? 15 : (uint8_t)L;
        size_t S = L + 5 + litext_len(L);
        *o++ = (uint8_t)(tl << 4);
        *o++ = (uint8_t)(S & 0xFF);
        *o++ = (uint8_t)((S >> 8) & 0xFF);
        o = put_litext(o, L);
        memcpy(o, blk + lit, L);
        o += L;
        *o++ = 0;                                                 /* offset 0 */
        *o++ = 0;
        size_sum += S;
        nseq++;
    }
    size_t bsize = size_sum + 3;                                  /* LZ4.c:617 */
    out[0] = (uint8_t)nseq;                                       /* LZ4.c:615 */
    out[1] = (uint8_t)(bsize & 0xFF);                             /* LZ4.c:419 */
    out[2] = (uint8_t)((bsize >> 8) & 0xFF);
    return (size_t)(o - out);
}

/* Upper bound of one encoded block (<=120 sequences of <= L+8 bytes). */
size_t lz4o_block_bound(void) { return 3 + LZ4O_BLOCK + 8 * 121; }

size_t lz4o_nblocks(size_t n) { return (n + LZ4O_BLOCK - 1) / LZ4O_BLOCK; }

/* Encode a run of whole blocks [b0, b1) of the input `in` (total length n),
 * concatenated, no frame header.  Returns bytes written. */
size_t lz4o_encode_blocks(const uint8_t *in, size_t n, size_t b0, size_t b1,
                          uint8_t *out)
{
    size_t w = 0;
    for (size_t b = b0; b < b1; b++) {                            /* LZ4.c:707 */
        size_t off = b * LZ4O_BLOCK;
        size_t len = (n - off < LZ4O_BLOCK) ? n - off : LZ4O_BLOCK; /* :712 */
        w += lz4o_encode_block(in + off, len, out + w);
    }
    return w;
}

/* lz4_encode (LZ4.c:670-742) minus the file I/O: frame header byte
 * (write_output, LZ4.c:429) followed by every block.  Returns bytes written,
 * or (size_t)-1 if the input is shorter than one block (LZ4.c:632-637). */
size_t lz4o_compress(const uint8_t *in, size_t n, uint8_t *out)
{
    if (n < LZ4O_BLOCK) return (size_t)-1;
    size_t nb = lz4o_nblocks(n);
    out[0] = (uint8_t)nb;
    return 1 + lz4o_encode_blocks(in, n, 0, nb, out + 1);
}

/* ---- multi-threaded CPU baseline (bench.py cpu_baseline leg) ---------- */
typedef struct {
    const uint8_t *in;
    size_t n, b0, b1;
    uint8_t *out;
    size_t written;
} lz4o_job;

static void *lz4o_worker(void *arg)
{
    lz4o_job *j = (lz4o_job *)arg;
    j->written = lz4o_encode_blocks(j->in, j->n, j->b0, j->b1, j->out);
    return NULL;
}

/* Encode blocks [0, nb) on `threads` pthreads over contiguous block ranges.
 * Each thread writes into its own region out + t*stride_per_block*blocks;
 * returns the total number of encoded bytes (segments are not compacted). */
size_t lz4o_encode_parallel(const uint8_t *in, size_t n, int threads,
                            uint8_t *scratch)
{
    if (threads < 1) threads = 1;
    if (threads > 256) threads = 256;
    size_t nb = lz4o_nblocks(n);
    pthread_t tid[256];
    lz4o_job jobs[256];
    size_t per = (nb + threads - 1) / threads;
    for (int t = 0; t < threads; t++) {
        size_t b0 = (size_t)t * per, b1 = b0 + per;
        if (b0 > nb) b0 = nb;
        if (b1 > nb) b1 = nb;
        jobs[t].in = in; jobs[t].n = n; jobs[t].b0 = b0; jobs[t].b1 = b1;
        jobs[t].out = scratch + b0 * lz4o_block_bound();
        jobs[t].written = 0;
        pthread_create(&tid[t], NULL, lz4o_worker, &jobs[t]);
    }
    size_t total = 0;
    for (int t = 0; t < threads; t++) {
        pthread_join(tid[t], NULL);
        total += jobs[t].written;
    }
    return total;
}

/* ---- decoder of the same format, for round-trip properties ----------- *
 * Parses sequences as sequence_decode/interpret_sequence do (LZ4.c:744-843,
 * 937-982) except that the literal count of a sequence whose token nibble is
 * 15 is recovered from its u16 size field (S = L + 5 + litext + matchext,
 * LZ4.c:546-575): the reference's one-byte literal extension wraps for
 * L >= 270 (LZ4.c:374), so its own decoder cannot round-trip such blocks.
 * Streams with uint8-truncated matches (M = 1..3, len 257..259) are not
 * decodable by construction (the token nibble overflows, LZ4.c:542-544).
 * Returns decoded length or (size_t)-1 on a malformed stream. */
size_t lz4o_decompress(const uint8_t *in, size_t in_len, uint8_t *out,
                       size_t cap, size_t nblocks)
{
    size_t ip = 1, op = 0;
    for (size_t b = 0; b < nblocks; b++) {
        if (ip + 3 > in_len) return (size_t)-1;
        unsigned nseq = in[ip];
        ip += 3;
        for (unsigned s = 0; s < nseq; s++) {
            if (ip + 3 > in_len) return (size_t)-1;
            uint8_t tok = in[ip];
            size_t S = in[ip + 1] | ((size_t)in[ip + 2] << 8);
            ip += 3;
            size_t L = tok >> 4;
            size_t tm = tok & 15;
            if (L == 15) {
                if (ip >= in_len) return (size_t)-1;
                size_t le = 1;
                if (in[ip] == 255) {
                    if (ip + 1 >= in_len || in[ip + 1] != 0) return (size_t)-1;
                    le = 2;
                }
                size_t mx = (tm == 15) ? 1 : 0;
                if (S < 5 + le + mx) return (size_t)-1;
                L = S - 5 - le - mx;
                ip += le;
            }
            if (ip + L + 2 > in_len || op + L > cap) return (size_t)-1;
            memcpy(out + op, in + ip, L);
            ip += L;
            op += L;
            unsigned dist = in[ip] | (in[ip + 1] << 8);
            ip += 2;
            if (dist == 0) continue;            /* literal-only tail sequence */
            size_t M = tm;
            if (M == 15) {
                if (ip >= in_len) return (size_t)-1;
                M += in[ip++];
            }
            M += 4;
            if (dist > op || op + M > cap) return (size_t)-1;
            for (size_t k = 0; k < M; k++, op++) out[op] = out[op - dist];
        }
    }
    return op;
}
