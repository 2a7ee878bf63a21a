// lz4r.hip -- MI355X (gfx950) "LZ4" compressor, bit-exact to the reference's
// Algorithms/sequential/LZ4/LZ4.c (canonical block-clamped matches).
//
// The reference cuts the input into 300-byte blocks (LZ4.c:23, 123-177) and,
// in every block, greedily parses with an exhaustive longest-match search over
// the whole block prefix (find_longest_match, LZ4.c:290-323; strict '>' so the
// smallest i -- farthest offset -- wins ties; length truncated to uint8_t).
// Blocks are independent; the compressor is one compute kernel, a scan and
// an emission pass:
//
// lz4_tiles: workgroup = one wave = one 300-B block (4,976 B of LDS, <= 64
// VGPRs -> 8 waves per SIMD; occupancy is what this LDS- and issue-bound
// kernel lives on).  Per block:
//   stage    the block's 75 dwords -> LDS (the only read of the input).
//   position-major (lane l owns p = 64 r + l, r = 0..4):
//     index  per-bucket chains of the 4-gram starts by a 10-bit hash: each
//            position empties its bucket's u32 head, then exchanges itself
//            into it (ds_wrxchg_rtn_b32) in ascending position order and keeps
//            the old head as its link (byte offsets 4 p), so every chain
//            strictly decreases; entry = link | (p == 0) << 15 | preceding
//            byte << 16 | own byte (the tag) << 24, stored by add-TID.
//     local  every unordered pair of a bucket is met once, by the later
//            position walking its chain (deepest walkers first); a lane
//            keeps its walker until the chain ends -- or a link fails to
//            decrease: the walk ends on any input -- and then takes the next
//            queued one.  A pair (j < p) is a candidate when the tags agree
//            and it is LEFT-MAXIMAL (j == 0 or blk[j-1] != blk[p-1]): one
//            v_xad + one compare of the two entries; a balanced lcp pass over
//            the 4-gram keys takes the longest candidate per p, ties to the
//            smallest j (LDS atomicMax of end << 19 | end << 9 | dist: the end
//            twice, so that subtracting p << 9 later leaves the record word).
//   blocked (lane l owns p = 5 l .. 5 l + 4):
//     best   a candidate that is not left-maximal is the pair (j-1, p-1)
//            shifted by one, whose match is one byte longer.  Hence
//              best(p) = lexmax over q <= p of (q + local_len(q), q - local_j(q))
//            i.e. the longest match ends furthest right and, among equals,
//            has the largest distance (= smallest source, LZ4.c:307).  A
//            running max over the lane's five and one wave max-scan give
//            best() for all p.  M = len & 0xFF (the uint8_t return, LZ4.c:317).
//     parse  word[x] = the record word (dist | M << 9 | 4 (c + M) << 17) of
//            c = the first matchable position >= x (a suffix pass over the
//            positions); the greedy parse (LZ4.c:516-583) is the walk
//            w_0 = word[0], w_{k+1} = word[c_k + M_k], one LDS read per
//            sequence.
//   records  sequence k on lane k: one packed wave scan of the bytes the block
//            takes and of its size fields; record k = the sequence's match
//            word dist | M << 9 | (match start + M) << 19 (its literal run
//            starts where sequence k - 1's match ends; the literal tail is
//            n << 19) -> the block's record scratch (a dense 96-B head: header
//            and records 0..22; an overflow slot for the rest), after a header
//            dword (sum of the size
//            fields | sequence count << 16); the block's byte count -> usz
//            (u32, for the scan) and bsizes (u16).
// lz4_scan_reduce / lz4_scan_partials: exclusive scan of the block sizes.
// lz4_emit: 32 blocks per workgroup of 8 waves, 4 blocks per wave.  The
// blocks' input is staged in LDS, their records flattened over the lanes (one
// round = 64 sequences of one or more blocks), and the bytes of write_block /
// write_sequence (LZ4.c:365-425) land by aligned ds_or in a zeroed LDS image
// of the output range -- header bytes from the sequence lanes, literal runs
// flattened over the lanes as aligned 16-byte words -- which leaves as aligned
// 16-B stores.  Splitting the emission off lz4_tiles (which is bound by
// instruction issue, one block per wave) lets a round of lz4_emit serve
// several blocks: lz4_tiles 3.44 -> 2.97 ms per GiB, and the slot round trip
// shrinks from ~310 B of bytes to ~100 B of records per block.
// No workgroup ever waits on another (a fused decoupled look-back ran the
// waves in lock-step at the pace of the slowest block of each round).
// lz4_emit issues every global load of a workgroup (scan inputs, record
// heads, staged input) before waiting on any: one memory round trip per
// workgroup instead of three (0.91 -> 0.75 ms per GiB).
// HBM traffic per input byte: 1 B read + ~0.35 B of records written by
// lz4_tiles; ~1 B of input + ~0.33 B of record heads read and ~1.03 B
// written by lz4_emit (+14 B/block of sizes and offsets).
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>
#include <limits.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <algorithm>
#include <type_traits>
#include <new>
#include <vector>

#include "../../include/lz4r.h"

// LZ4R_VARIANT: per-phase timing ablations for the instruction budget in
// DESIGN.md, compiled only by tools/build_variants.sh into tools/variants/
// (the Makefile's product build never defines it): 1 = no match search,
// 2 = no index/match phase, 3 = index only (no candidates), 4 = candidates
// without the lcp verification, 5 = the lcp without its result (no
// matches downstream), 11 = no sequence emission; lz4_emit: 31 = no literal
// words, 32 = no header bytes.
#ifndef LZ4R_VARIANT
#define LZ4R_VARIANT 0
#endif
// LZ4R_PROF (tools builds only, like LZ4R_VARIANT): per-phase s_memtime
// cycles of every wave summed into lz4r_prof[] (read by lz4r_prof_read).
#ifdef LZ4R_PROF
__device__ unsigned long long lz4r_prof_acc[16];
#define PROF_DECL uint64_t prof_t = __builtin_amdgcn_s_memtime()
#define PROF_MARK(k)                                                     \
  do {                                                                   \
    const uint64_t prof_n = __builtin_amdgcn_s_memtime();                \
    if (threadIdx.x == 0) atomicAdd(&lz4r_prof_acc[k], prof_n - prof_t); \
    prof_t = prof_n;                                                     \
  } while (0)
#elif defined(LZ4R_MARK)
// static phase markers in the assembly (tools: per-phase instruction counts)
#define PROF_DECL
#define PROF_MARK(k) asm volatile(";PHASE_END " #k ::: "memory")
#else
#define PROF_DECL
#define PROF_MARK(k) \
  do {               \
  } while (0)
#endif


namespace {

constexpr int kBlk = LZ4R_BLOCK;          // 300
constexpr int kBlkOutMax = 560;           // >= 548: worst-case bytes of one block, 16-B multiple
constexpr int kHB = 10;                   // hash bits: 1024 buckets
constexpr int kH = 1 << kHB;
constexpr int kArr = 320;                // per-position arrays: every lane's five positions
                                         // (p = 5 l + r <= 319) in range, no index clamps
constexpr int kQ = kBlk + 64;            // walker queue: reads run up to 63 past the last
constexpr int kCand = 128;               // candidate list (drained when a pass could fill it)
constexpr uint32_t kEmptyHead = 0xFFFFFFFCu;   // an emptied bucket head; as an entry's
                                              // 11-bit link field it reads kNoLink
constexpr uint32_t kNoLink = 2044;       // chain end: an empty head (0x07FC), a dword-aligned
                                         // offset, so the reads past a chain's end stay aligned
static_assert(kArr >= 64 * 5, "blocked positions of all 64 lanes");
static_assert((kEmptyHead & 0x7FFu) == kNoLink && kNoLink >= 4 * kArr, "the chain-end link");

// LDS of one wave (4,976 B: 32 waves per CU).  Byte offsets in TileLds::buf:
//   [kInOff, +348)     the block (byte kInOff - 1 is read as blk[-1]) + an
//                      over-read pad (lcp reads)
//   [kQOff, +1456)     chain walkers (q), or the slow walk's sequence starts (seq)
//   [kCandOff, +512)   candidate pairs
// then ent[320] and rec[320].  While the block is indexed, the 1024 u32
// bucket heads overlay [kHeadOff, +4096) = q, cand, ent and rec[0..192), all
// dead until the index is built (ent and rec are written after the heads'
// last exchange).
constexpr int kInOff = 16;
constexpr int kQOff = 368;
constexpr int kCandOff = kQOff + 4 * kQ;
constexpr int kHeadOff = kQOff;
constexpr int kBufBytes = kHeadOff + 2 * kH > kCandOff + 4 * kCand ? kHeadOff + 2 * kH
                                                                   : kCandOff + 4 * kCand;
static_assert(kInOff + kBlk + 48 <= kQOff && kQOff % 16 == 0 && kInOff % 16 == 0 &&
                  kBlk == 75 * 4,
              "dword staging (75 dwords), aligned regions");

// Record scratch per block: the header dword and <= 121 sequence records.
// The first kHeadW dwords (header + 23 records: all of a text block's but for
// ~7 % of blocks) go to a dense head array, kHead bytes per block, so lz4_emit
// reads its 32 blocks' heads as one contiguous 3 KB run of 16-B loads (no
// 128-B line per block of which ~60 B were used); records 23.. go to a
// per-block overflow slot of kOvf bytes.
constexpr int kHeadW = 24;
constexpr int kHead = 4 * kHeadW;        // 96 B
constexpr int kOvf = 400;                // records 23..120: <= 98 dwords
constexpr int kSlot = kHead + kOvf;      // scratch bytes per block
static_assert(kHead % 16 == 0 && kOvf % 16 == 0 && 4 * (121 + 1 - kHeadW) <= kOvf,
              "aligned head and overflow slots");

struct TileLds {
  alignas(16) uint8_t buf[kBufBytes];
  union {
    uint32_t ent[kArr];   // per position: link | (p == 0) << 15 | blk[p - 1] << 16 | blk[p] << 24
    uint32_t word[kArr];  // then: the first match at or after x, as its record word
  };
  uint32_t rec[kArr];     // local(p) accumulator: end << 19 | end << 9 | dist (end = p + len)
  // chain walkers: the walker's byte offset 4 p (candidate phase)
  __device__ __forceinline__ uint32_t *q() { return reinterpret_cast<uint32_t *>(buf + kQOff); }
  // per sequence, its match start (slow walk only)
  __device__ __forceinline__ uint32_t *seq() { return reinterpret_cast<uint32_t *>(buf + kQOff); }
  // candidate pairs p | j << 16 awaiting the lcp pass
  __device__ __forceinline__ uint32_t *cand() { return reinterpret_cast<uint32_t *>(buf + kCandOff); }
};

constexpr int kWordOff = kBufBytes;             // byte offset of ent / word in TileLds
constexpr int kRecOff = kBufBytes + 4 * kArr;   // byte offset of rec in TileLds
// word[] past the last match: its field (the next read's byte offset) is
// 4 * 319 > 4 n, the walk's exit, and stays inside the array
constexpr uint32_t kWordEnd = (uint32_t)(4 * (kArr - 1)) << 17;
static_assert(kHeadOff + 4 * kH <= kRecOff + 4 * 192, "u32 heads end before rec[192]");
static_assert(kRecOff + 4 * kArr <= 4976, "LDS of one wave");

// Five ds_wrxchg_rtn_b32 back to back, one wait: old = *(head base + a); *(...) = v.
// The addresses are relative to the head array (kHeadOff, the instruction's
// offset field); the LDS serves one wave's operations in order, so a later
// exchange of the same head sees the earlier.
// Each head this block uses is first emptied by the positions that hash to
// it (five ds_write_b32 of kEmptyHead, before any exchange; the LDS serves one
// wave's operations in order): a head no position of the block maps to is
// never read, so the other ~800 of the 1024 need no reset (5 scattered
// stores instead of 16 ds_write_addtid_b32 over the whole 4 KB).
__device__ __forceinline__ void xchg_rtn5(uint32_t (&old)[5], const uint32_t (&a)[5],
                                          const uint32_t (&v)[5]) {
  asm volatile(
      "ds_write_b32 %5, %15 offset:368\n\t"
      "ds_write_b32 %6, %15 offset:368\n\t"
      "ds_write_b32 %7, %15 offset:368\n\t"
      "ds_write_b32 %8, %15 offset:368\n\t"
      "ds_write_b32 %9, %15 offset:368\n\t"
      "ds_wrxchg_rtn_b32 %0, %5, %10 offset:368\n\t"
      "ds_wrxchg_rtn_b32 %1, %6, %11 offset:368\n\t"
      "ds_wrxchg_rtn_b32 %2, %7, %12 offset:368\n\t"
      "ds_wrxchg_rtn_b32 %3, %8, %13 offset:368\n\t"
      "ds_wrxchg_rtn_b32 %4, %9, %14 offset:368\n\t"
      "s_waitcnt lgkmcnt(0)"
      : "=&v"(old[0]), "=&v"(old[1]), "=&v"(old[2]), "=&v"(old[3]), "=&v"(old[4])
      : "v"(a[0]), "v"(a[1]), "v"(a[2]), "v"(a[3]), "v"(a[4]),
        "v"(v[0]), "v"(v[1]), "v"(v[2]), "v"(v[3]), "v"(v[4]), "v"(kEmptyHead)
      : "memory");
}

static_assert(kHeadOff == 368 && kH == 1024, "xchg_rtn5 offsets");

// ent[64 r + lane] = e[r] (the position-major entries, r = 0..4) and zero
// rec[0 .. 320) (1,280 B at kRecOff, the local(p) accumulators) with
// ds_write_addtid_b32: 10 stores of 2 LDS cycles each, one m0 set.  Called
// after the heads' last exchange (ent and rec[0 .. 192) lie under the heads).
__device__ __forceinline__ void ent_store_rec_zero_addtid(const uint32_t (&e)[5]) {
  asm volatile(
      "s_mov_b32 m0, 0\n\t"
      "s_nop 0\n\t"
      "ds_write_addtid_b32 %0 offset:%c6\n\t"
      "ds_write_addtid_b32 %1 offset:%c7\n\t"
      "ds_write_addtid_b32 %2 offset:%c8\n\t"
      "ds_write_addtid_b32 %3 offset:%c9\n\t"
      "ds_write_addtid_b32 %4 offset:%c10\n\t"
      "ds_write_addtid_b32 %5 offset:%c11\n\t"
      "ds_write_addtid_b32 %5 offset:%c12\n\t"
      "ds_write_addtid_b32 %5 offset:%c13\n\t"
      "ds_write_addtid_b32 %5 offset:%c14\n\t"
      "ds_write_addtid_b32 %5 offset:%c15"
      :
      : "v"(e[0]), "v"(e[1]), "v"(e[2]), "v"(e[3]), "v"(e[4]), "v"(0u),
        "i"(kBufBytes), "i"(kBufBytes + 256), "i"(kBufBytes + 512), "i"(kBufBytes + 768),
        "i"(kBufBytes + 1024), "i"(kRecOff), "i"(kRecOff + 256), "i"(kRecOff + 512),
        "i"(kRecOff + 768), "i"(kRecOff + 1024)
      : "memory");
}

// key[64 r + lane] = k[r] over the walker queue (kQOff), one m0 set.
__device__ __forceinline__ void keys_store_addtid(const uint32_t (&k)[5]) {
  asm volatile(
      "s_mov_b32 m0, 0\n\t"
      "s_nop 0\n\t"
      "ds_write_addtid_b32 %0 offset:%c5\n\t"
      "ds_write_addtid_b32 %1 offset:%c6\n\t"
      "ds_write_addtid_b32 %2 offset:%c7\n\t"
      "ds_write_addtid_b32 %3 offset:%c8\n\t"
      "ds_write_addtid_b32 %4 offset:%c9"
      :
      : "v"(k[0]), "v"(k[1]), "v"(k[2]), "v"(k[3]), "v"(k[4]), "i"(kQOff), "i"(kQOff + 256),
        "i"(kQOff + 512), "i"(kQOff + 768), "i"(kQOff + 1024)
      : "memory");
}

__device__ __forceinline__ uint32_t ffbl(uint32_t x) {   // v_ffbl_b32: -1 when x == 0
  uint32_t r;
  asm("v_ffbl_b32 %0, %1" : "=v"(r) : "v"(x));
  return r;
}

// Longest common prefix of the byte runs at a and b (a < b), capped at
// `limit` = n - b: the canonical clamp (a match never crosses the block end).
// Each operand's 16 bytes come from aligned dwords and v_alignbyte: a
// misaligned ds_read_b128 is replayed at ~64 LDS cycles, and the kernel's
// LDS array is ~80 % busy (SQ_LDS_IDX_ACTIVE), so the 4 extra VALU per
// operand pay (-1 % lz4_tiles; an earlier 8-byte funnel-shift form cost ~30
// VALU per block and lost).  Reads past the region land in its pad (>= 48 B
// past any block end; the aligned form reads at most 19 past it).
__device__ __forceinline__ int lcp(const uint8_t *d, int a, int b, int limit) {
  // a step continues only after 16 equal bytes, so both operands keep their
  // byte alignment: the shifts are loop-invariant and the dword pointers
  // advance by 16 bytes
  const uint32_t sa = (uint32_t)a & 3u, sb = (uint32_t)b & 3u;
  const uint32_t *wa = reinterpret_cast<const uint32_t *>(d + (a & ~3));
  const uint32_t *wb = reinterpret_cast<const uint32_t *>(d + (b & ~3));
  int l = 0;
  for (;;) {                              // 16 bytes per step
    // 16 bytes from five aligned dwords (two ds_read2_b32 and a ds_read_b32:
    // no misaligned replay), byte-aligned by v_alignbyte
    auto at16 = [](const uint32_t *w, uint32_t sh) {
      const uint32_t w0 = w[0], w1 = w[1], w2 = w[2], w3 = w[3], w4 = w[4];
      return make_uint4(__builtin_amdgcn_alignbyte(w1, w0, sh),
                        __builtin_amdgcn_alignbyte(w2, w1, sh),
                        __builtin_amdgcn_alignbyte(w3, w2, sh),
                        __builtin_amdgcn_alignbyte(w4, w3, sh));
    };
    const uint4 A = at16(wa, sa), B = at16(wb, sb);
    // first differing bit of the 16 bytes: v_ffbl per dword (-1 when equal),
    // offset by 32 k with an OR (each is < 32 or all ones), min over the four
    const uint32_t m = min(min(ffbl(A.x ^ B.x), ffbl(A.y ^ B.y) | 32u),
                           min(ffbl(A.z ^ B.z) | 64u, ffbl(A.w ^ B.w) | 96u));
    l += (int)min(m >> 3, 16u);
    if (m != 0xFFFFFFFFu || l >= limit) break;
    wa += 4;
    wb += 4;
  }
  return l < limit ? l : limit;
}

// The same over the 4-gram keys (kj = &key[j], kp = &key[p], j < p): the
// 16 bytes at a position are key[x], key[x + 4], key[x + 8], key[x + 12].
// key[] covers positions 0 .. 319 and a step reads at most 12 past p + l
// < n <= 300.
__device__ __forceinline__ int lcp_keys(const uint32_t *kj, const uint32_t *kp, int limit) {
  int l = 0;
  for (;;) {
    const uint32_t a0 = kj[0], a1 = kj[4], a2 = kj[8], a3 = kj[12];
    const uint32_t b0 = kp[0], b1 = kp[4], b2 = kp[8], b3 = kp[12];
    const uint32_t m = min(min(ffbl(a0 ^ b0), ffbl(a1 ^ b1) | 32u),
                           min(ffbl(a2 ^ b2) | 64u, ffbl(a3 ^ b3) | 96u));
    l += (int)min(m >> 3, 16u);
    if (m != 0xFFFFFFFFu || l >= limit) break;
    kj += 16;
    kp += 16;
  }
  return l < limit ? l : limit;
}

// The same from global memory (kFull blocks, whose bytes are not staged in
// LDS: only a drain in the middle of the walk, when a pass could overflow the
// candidate list, uses it): 16 bytes per operand and step as one unaligned
// global_load_dwordx4 (L1/L2-resident: the block was just read).  Reads reach
// at most 15 bytes past the block end, into the next block.
__device__ __forceinline__ int lcp_global(const uint8_t *a, const uint8_t *b, int limit) {
  int l = 0;
  for (;;) {
    uint4 A, B;
    __builtin_memcpy(&A, a + l, 16);
    __builtin_memcpy(&B, b + l, 16);
    const uint32_t m = min(min(ffbl(A.x ^ B.x), ffbl(A.y ^ B.y) | 32u),
                           min(ffbl(A.z ^ B.z) | 64u, ffbl(A.w ^ B.w) | 96u));
    l += (int)min(m >> 3, 16u);
    if (m != 0xFFFFFFFFu || l >= limit) break;
  }
  return l < limit ? l : limit;
}

// DPP helpers (gfx9 row_shr / row_bcast; identity 0 for lanes without a source)
template <int CTRL, int ROW, int BANK>
__device__ __forceinline__ uint32_t dpp(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, ROW, BANK, false);
}

__device__ __forceinline__ uint32_t wave_incl_add(uint32_t v) {
  v += dpp<0x111, 0xf, 0xf>(v);
  v += dpp<0x112, 0xf, 0xf>(v);
  v += dpp<0x114, 0xf, 0xf>(v);
  v += dpp<0x118, 0xf, 0xf>(v);
  v += dpp<0x142, 0xa, 0xf>(v);
  v += dpp<0x143, 0xc, 0xf>(v);
  return v;
}

__device__ __forceinline__ uint32_t wave_incl_max(uint32_t v) {
  v = max(v, dpp<0x111, 0xf, 0xf>(v));
  v = max(v, dpp<0x112, 0xf, 0xf>(v));
  v = max(v, dpp<0x114, 0xf, 0xf>(v));
  v = max(v, dpp<0x118, 0xf, 0xf>(v));
  v = max(v, dpp<0x142, 0xa, 0xf>(v));
  v = max(v, dpp<0x143, 0xc, 0xf>(v));
  return v;
}

__device__ __forceinline__ uint32_t lane63(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_readlane((int)v, 63);
}

__device__ __forceinline__ int ctz64(uint64_t m) { return __builtin_ctzll(m); }

// lane mask of a predicate, straight from the compare (hip's __ballot goes
// through a 0/1 VGPR and a second compare)
__device__ __forceinline__ uint64_t ballot(bool b) { return __builtin_amdgcn_ballot_w64(b); }

// set bits of m in the lanes below this one (v_mbcnt_lo / v_mbcnt_hi)
__device__ __forceinline__ int rank_below(uint64_t m) {
  return (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                        __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}




// acc + the set bits of m in the lanes below this one (the adds fold into
// v_mbcnt's accumulator)
__device__ __forceinline__ uint32_t rank_below_plus(uint64_t m, uint32_t acc) {
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                   __builtin_amdgcn_mbcnt_lo((uint32_t)m, acc));
}

// per lane: t where the lane's bit of m is set, else f (v_cndmask with the
// mask straight from an SGPR pair)
__device__ __forceinline__ uint32_t sel_mask(uint64_t m, uint32_t t, uint32_t f) {
  uint32_t r;
  asm("v_cndmask_b32_e64 %0, %1, %2, %3" : "=v"(r) : "v"(f), "v"(t), "s"(m));
  return r;
}

// base[1 + off / 4] = v in the lanes of m: EXEC = EXEC & m around one
// global_store_dword, straight from the SGPR pair (a condition built from the
// mask costs a 0/1 select and a compare per store).  The untracked store only
// makes the compiler's later vmcnt waits conservative.
__device__ __forceinline__ void store_lanes1(uint64_t m, uint32_t *base, uint32_t off, uint32_t v) {
  uint64_t save;
  asm volatile(
      "s_and_saveexec_b64 %0, %1\n\t"
      "global_store_dword %2, %3, %4 offset:4\n\t"
      "s_or_b64 exec, exec, %0"
      : "=&s"(save)
      : "s"(m), "v"(off), "v"(v), "s"(base)
      : "memory", "scc");
}

// S.buf[kOff + addr] = v (a dword) in the lanes of m, the same way: no
// select of a dummy address for the other lanes (the wave's LDS operations
// are served in order, so later reads see the store; lz4_tiles' TileLds sits
// at LDS address 0, as xchg_rtn5's offsets assume)
template <int kOff>
__device__ __forceinline__ void lds_store_lanes(uint64_t m, uint32_t addr, uint32_t v) {
  uint64_t save;
  asm volatile(
      "s_and_saveexec_b64 %0, %1\n\t"
      "ds_write_b32 %2, %3 offset:%c4\n\t"
      "s_or_b64 exec, exec, %0"
      : "=&s"(save)
      : "s"(m), "v"(addr), "v"(v), "i"(kOff)
      : "memory", "scc");
}

// The compressor's workgroup is one wave.  A wave's LDS operations are
// served in order, so its phase boundaries need neither s_barrier nor the
// s_waitcnt vmcnt(0) lgkmcnt(0) that __syncthreads() implies: a compiler
// barrier that keeps the LDS accesses of both phases in program order is
// enough, and loads still in flight (LDS or global) stay in flight.
__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_wave_barrier();
  asm volatile("" ::: "memory");
}

// Encode the staged block (n bytes at S.buf[kInOff]) as sequence records:
// dwords 0 .. kHeadW - 1 (header, records 0..22) at head, record k >= 23 at
// ovf[k + 1 - kHeadW]; returns the bytes its stream takes.
// kMatchesOnly: stop after the best-match scan and store every position's
// find_longest_match result to mout instead (lz4r_block_matches_device).
template <bool kMatchesOnly, bool kFull>
__device__ __forceinline__ int encode_block(TileLds &S, int n_arg, const uint8_t *__restrict__ gsrc,
                                            uint32_t *__restrict__ mout,
                                            uint32_t *__restrict__ head,
                                            uint32_t *__restrict__ ovf,
                                            uint32_t *__restrict__ status) {
  // kFull: a whole 300-byte block of a 4-byte aligned input that is not the
  // launch's last (every block but one): n is a constant, only round 4's
  // lanes 41..63 hold positions past the last 4-gram start, and the block is
  // NOT staged in LDS -- each lane loads the two dwords its 4-grams need
  // straight from gsrc (L1/L2: the 24 bytes past the block end that row 4
  // reads belong to the next block); otherwise the block is staged at
  // S.buf[kInOff] by the caller.
  const int n = kFull ? kBlk : n_arg;
  const int lane = threadIdx.x;
  constexpr int base = kInOff;

  // ---- index: per-bucket chains of the 4-gram starts -----------------------
  // Position-major: lane l owns p_r = 64 r + l (r = 0..4; positions 297..319
  // of a full block start no 4-gram).  Round r exchanges the 64 positions
  // 64 r .. 64 r + 63 into their buckets' u32 heads (ds_wrxchg_rtn_b32, the
  // five rounds back to back, one wait) and keeps each old head as the
  // position's link.  Insertion is in ascending position order (rounds
  // ascend; within one exchange the LDS serves the lanes in ascending order),
  // so every link is a smaller byte offset than its position or empty: a
  // chain strictly decreases, and a walk that stops at the first link not
  // below the current one ends on any input -- even on a corrupted head.
  // Entry (byte offsets 4 p):  link (bits 0..10) | p == 0 (bit 15) |
  // preceding byte (16..23) | tag (24..31: the position's own byte, which
  // equal 4-grams share).  Entries are written by ds_write_addtid_b32
  // (2 LDS cycles per round instead of 4-6 for a strided store).
  PROF_DECL;
  const bool search = LZ4R_VARIANT != 1 && LZ4R_VARIANT != 2;
  const int nk = n >= 4 ? n - 3 : 0;     // positions that start a 4-gram

  bool walk[5];                          // p_r has a link (a walker)
  uint32_t qn = 0;                       // walkers queued
  uint32_t key[5];                       // p_r's 4-gram (kept for the lcp drain)
  {
    // bytes p .. p + 3 from two aligned dwords: sh = p & 3 = lane & 3
    const uint32_t sh = (uint32_t)lane & 3u;
    const uint32_t *bw = kFull ? reinterpret_cast<const uint32_t *>(gsrc) + (lane >> 2)
                               : reinterpret_cast<const uint32_t *>(S.buf) + (kInOff >> 2) +
                                     (lane >> 2);
    uint32_t pt[5], adr[5], set[5];
    // inactive positions (p >= nk) exchange with a dword of rec[192 + lane]
    // (past the heads, zeroed after the exchanges; distinct per lane)
    const uint32_t dummy = (uint32_t)(kRecOff + 4 * (192 + lane) - kHeadOff);
#pragma unroll
    for (int r = 0; r < 5; ++r) {
      // one global_load_dwordx2 (kFull) or ds_read2_b32
      const uint32_t w1 = bw[16 * r], w2 = bw[16 * r + 1];
      key[r] = __builtin_amdgcn_alignbyte(w2, w1, sh);
      const uint32_t hv = key[r] * 2654435761u;                    // bucket = top 10 bits
      // [0, 0, blk[p - 1], blk[p]]: the entry without its link.  The tag
      // (byte 3) is the position's own first byte: any function of the 4-gram
      // serves (equal 4-grams always agree; a pair that agrees by chance is
      // a candidate whose lcp is < 4), and this one costs no hash bits
      if (r == 0) {
        // blk[p - 1] = byte 0 of the lane below's key (DPP wave_shr:1; lane 0
        // is p = 0, whose byte is the sentinel bit below)
        const uint32_t pb = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)key[0], 0x138, 0xf,
                                                                 0xf, false);
        pt[0] = __builtin_amdgcn_perm(pb, key[0], 0x00040C0Cu);
      } else {
        // rows 1..4: bytes 3 + sh and 4 + sh of the dword pair before (one
        // more dword in the same load, no cross-lane step)
        const uint32_t w0 = bw[16 * r - 1];
        pt[r] = __builtin_amdgcn_perm(w1, w0, 0x04030C0Cu + sh * 0x01010000u);
      }
      const int p = 64 * r + lane;
      // (full block: rounds 0..3 are all 4-gram starts)
      const bool act = search && ((kFull && r < 4) || p < nk);
      adr[r] = act ? (hv >> (32 - kHB)) << 2 : dummy;
      set[r] = (uint32_t)(4 * p);
    }
    if (lane == 0) pt[0] |= 1u << 15;     // p = 0: left-maximal with every later position
    uint32_t old[5];
    xchg_rtn5(old, adr, set);
#if LZ4R_VARIANT == 20
    // tools build: one stale head (a forward link, as a missed reset would
    // leave) -- the walk must still end and the call report LZ4R_ERR_CORRUPT
    if (lane == 7) old[2] = 4u * 250u;
#endif
    uint32_t e[5];
    int d[5];
#pragma unroll
    for (int r = 0; r < 5; ++r) {
      // the link field is 11 bits: kEmptyHead reads kNoLink (2044)
      e[r] = (old[r] & 0x7FFu) | pt[r];  // inactive: never read (no chain reaches it)
      // a link (not an empty head, -4 as an int); on a sound LDS an earlier
      // position -- checked below, and a walk ends at any non-decreasing link
      walk[r] = (int)old[r] >= 0;
      // a link is an earlier position (old - 4 p < 0) or an empty head
      // (kEmptyHead = -4 as an int: old - 4 p < 0 too); anything else is a
      // corrupt head.  One subtraction per position and two v_max3.
      d[r] = (int)(old[r] - set[r]);
    }
    const int y = max(max(max(d[0], d[1]), d[2]), max(d[3], d[4]));
    // (never on a sound LDS; the batch match finder has no status word)
    if (!kMatchesOnly && ballot(y >= 0)) atomicOr(status, 1u);
    // queue the walkers row by row from r = 4 down (later positions first:
    // the deepest chains start early, which keeps the walk passes near the
    // longest chain), lanes ascending within a row; the queue overlays the
    // heads, dead after the exchanges (the LDS serves the wave in order)
#pragma unroll
    for (int r = 4; r >= 0; --r) {
      const uint64_t m = ballot(walk[r]);
      // only the walkers' lanes store (EXEC = m around the store)
      lds_store_lanes<kQOff>(m, rank_below_plus(m, qn) << 2, set[r]);
      qn += (uint32_t)__popcll(m);
    }
    ent_store_rec_zero_addtid(e);        // ent[64 r + lane] = e[r]; rec[] = 0
  }
  PROF_MARK(0);                       // index + walker queue
  wave_sync();
  const int qwr = (int)qn;               // walkers queued (S.q()[0 .. qwr))
  wave_sync();

  PROF_MARK(1);                       // walker queue
  // ---- candidates: walk the chains ------------------------------------------
  // A pair (j < p) of one bucket is a candidate when the tags agree and the
  // match is left-maximal (j == 0 or blk[j-1] != blk[p-1]): with x = the two
  // entries xor'ed, exactly when 2^15 <= x < 2^24 (bits 24..31 zero: the
  // tags agree; some bit 15..23 set: the preceding bytes differ or j == 0).
  // Candidates go to a list in S.cand, drained by a balanced lcp pass with
  // LDS atomicMax into S.rec (end << 19 | end << 9 | (p - j), end = p + len:
  // the longest, ties to
  // the smallest j).
  uint32_t longm = 0;                    // this lane verified a candidate of >= 256 bytes
  if (search && LZ4R_VARIANT != 3) {
    constexpr int kTrash = kCand - 1;
    int ncand = 0;
    const uint8_t *const entb = reinterpret_cast<const uint8_t *>(S.ent);
    auto ent_at = [&](int off) { return *reinterpret_cast<const uint32_t *>(entb + off); };
    // kKeys: the walk is over and the queue region holds every position's
    // 4-gram key (key[p] = bytes p .. p + 3 as a dword), so a 16-byte lcp
    // step is four aligned dword reads per operand (two ds_read2_b32), with
    // no byte alignment; a drain in the middle of the walk (more than 63
    // candidates) reads the staged block with v_alignbyte
    auto drain = [&](auto keys) {
      constexpr bool kKeys = decltype(keys)::value;
      wave_sync();
      for (int i = lane; i < ncand && LZ4R_VARIANT != 4; i += 64) {
        const uint32_t pr = S.cand()[i];
        const int p = (int)(pr & 0xFFFFu) >> 2, j = (int)(pr >> 18);   // j < p: chains decrease
        const int l = kKeys ? lcp_keys(S.q() + j, S.q() + p, n - p)
                      : kFull ? lcp_global(gsrc + j, gsrc + p, n - p)
                              : lcp(S.buf, base + j, base + p, n - p);
        // (end, dist) as the best scan wants it: for one p the larger end is
        // the longer match and the larger dist the smaller source
        if (LZ4R_VARIANT == 5) {          // ablation: the lcp without its result
          if (l == 12345) S.rec[0] = 1u;
        } else if (l >= 4) {
          // end << 19 | end << 9 | dist (the end twice: see the word pass)
          atomicMax(&S.rec[p], (uint32_t)(p + l) * 0x80200u | (uint32_t)(p - j));
        }
        longm |= l >= 256 ? 1u : 0u;     // (a match the uint8_t return truncates)
      }
      wave_sync();
    };
    // Persistent walkers: a lane keeps its walker (a walks, b = the next chain
    // entry) in registers until the chain ends, and an idle lane takes the
    // next queued walker.  The queue is read once, front to back: no ring,
    // no re-queue stores.  The walkers' liveness is a scalar lane mask (the
    // selects read it straight from SGPRs, written by SALU ops only).
    int qrd4 = 0;
    const int qwr4 = 4 * qwr;
    const uint8_t *const qb = reinterpret_cast<const uint8_t *>(S.q());
    int a = 0, b = 0;
    uint32_t me = 0;                       // the walker's own entry (re-read only on a take)
    uint64_t vm = 0;                       // lanes holding a walker
    // one pass: every live walker meets its next chain entry
    auto pass = [&]() {
      const uint32_t o = ent_at(b);
      const uint64_t cm = vm & ballot(((me ^ o) - (1u << 15)) < (1u << 24) - (1u << 15));
      // the pair (walker, chain entry): the entry is the earlier position
      lds_store_lanes<kCandOff>(cm, rank_below_plus(cm, (uint32_t)ncand) << 2,
                                (uint32_t)a | ((uint32_t)b << 16));
      ncand += __popcll(cm);
      const int bn = (int)(o & 2047u);
      vm &= ballot(bn < b);                // the chain ends (kNoLink, or any non-decreasing link)
      b = bn;
      if (ncand > kTrash - 64) {           // (rare: a full list drains mid-walk)
        drain(std::false_type{});
        ncand = 0;
      }
    };
    // while walkers are queued, idle lanes take them (uniform); then the
    // passes go on without the take
    while (qrd4 < qwr4) {
      const uint64_t em = ~vm;
      const int idx4 = qrd4 + (rank_below(em) << 2);
      const uint64_t nm_ = em & ballot(idx4 < qwr4);
      const uint32_t it = *reinterpret_cast<const uint32_t *>(qb + idx4);   // idx <= qwr + 63 < kQ
      a = (int)sel_mask(nm_, it, (uint32_t)a);
      vm |= nm_;
      qrd4 += 4 * __popcll(em);
      me = ent_at(a);                      // (lanes that kept their walker read the same word)
      b = (int)sel_mask(nm_, me & 2047u, (uint32_t)b);   // a new walker starts at its link
      pass();
    }
    while (vm) {                         // (unrolled by two: -0.6 % lz4_tiles)
      pass();
      if (!vm) break;
      pass();
    }
    if (ncand) {
      keys_store_addtid(key);            // the queue is dead: keys over it
      drain(std::true_type{});
    }
  }
  wave_sync();
  PROF_MARK(2);                       // candidates + lcp
  // ---- best(p) = prefix lexmax of (end, dist) -------------------------------
  // (from here on the per-position phases are BLOCKED: lane l owns
  // p = 5 l .. 5 l + 4, so a prefix over positions is a running max over the
  // lane's five plus one wave scan; the arrays in LDS are indexed by p in
  // either layout)
  const int p0 = 5 * lane;
  // blocked: a running max over the lane's five positions, one wave scan of
  // the lane totals, the exclusive prefix folded back in
  uint32_t v[5];
#pragma unroll
  for (int r = 0; r < 5; ++r) {
    // local(p) as end << 19 | end << 9 | dist; 0 without a candidate and at
    // and past n
    v[r] = S.rec[p0 + r];
    if (r) v[r] = max(v[r], v[r - 1]);
  }
  {
    const uint32_t incl = wave_incl_max(v[4]);
    const uint32_t excl = dpp<0x138, 0xf, 0xf>(incl);     // wave_shr:1, lane 0 gets 0
#pragma unroll
    for (int r = 0; r < 5; ++r) v[r] = max(v[r], excl);
  }
  if constexpr (kMatchesOnly) {
    // find_longest_match (LZ4.c:290-323) at every p: len | dist << 16, both 0
    // below MIN_MATCH_LENGTH (the uint8_t truncation is the caller's)
#pragma unroll
    for (int r = 0; r < 5; ++r) {
      const int p = p0 + r;
      const int len = (int)(v[r] >> 19) - p;
      if (p < n) mout[p] = len >= 4 ? (uint32_t)len | ((v[r] & 511u) << 16) : 0u;
    }
    return 0;
  }
  // The scan values are end << 19 | end << 9 | dist (the lexicographic order
  // of (end, dist): the middle copy follows the end), so x = v - p << 9 =
  // end << 19 | len << 9 | dist; a match covers p when end >= p + 4 (one
  // compare of the scan value), and M = len & 0xFF (the uint8_t return,
  // LZ4.c:317).  A match starts at p when len >= 4 and M != 0 (len 256 is a
  // literal, LZ4.c:521).
  // The greedy parse (LZ4.c:516-583) at x -- 0, then the end of the previous
  // match -- takes the first matchable position c = nm(x) >= x with its M and
  // dist.  word[x] holds exactly that, as the match's own record word
  //   dist | M << 9 | (c + M) << 19
  // -- x itself when the match is not truncated (len < 256) -- whose top
  // field, as the shifted word >> 17 = 4 (c + M), is the byte offset of the
  // next word the walk reads, or kWordEnd when no match starts at or after x.
  // So the walk reads one word per sequence and needs no successor table (no
  // gathers, no second array).
  // (the word pass is instantiated for both cases below, so the match flags
  // stay lane masks in SGPRs: merged across a branch they were packed into
  // a VGPR and unpacked again, ~15 VALU)
  const uint32_t nP9 = 0u - ((uint32_t)p0 << 9);
  const uint32_t K0 = (uint32_t)(p0 + 4) << 19;
  auto word_pass = [&](auto fast) -> uint32_t {
    uint32_t rw[5];               // p's own word (where a match starts at p)
    bool mt[5];                   // a match starts at p (len >= 4, M != 0)
#pragma unroll
    for (int r = 0; r < 5; ++r) {
      const uint32_t x = v[r] + nP9 + (0u - ((uint32_t)r << 9));   // one v_add3
      const bool m4 = v[r] >= K0 + ((uint32_t)r << 19);             // len >= 4
      if constexpr (decltype(fast)::value) {
        mt[r] = m4;
        rw[r] = x;
      } else {
        const uint32_t M = __builtin_amdgcn_ubfe(x, 9, 8);
        mt[r] = m4 && M != 0u;
        rw[r] = ((M + (uint32_t)(p0 + r)) << 19) | (x & 0x1FFFFu);
      }
    }
    PROF_MARK(3);                     // best scan
    // ---- word[x] for x in [0, n]: a suffix "next match" over the positions
    uint32_t loc = kWordEnd;      // the lane's own first match word
#pragma unroll
    for (int r = 4; r >= 0; --r) loc = mt[r] ? rw[r] : loc;
    const uint64_t has = ballot(loc != kWordEnd);
    const uint64_t up = has & ~((2ull << lane) - 1ull);  // lanes above this one
    const int src = up ? ctz64(up) : lane;
    const uint32_t nx = (uint32_t)__builtin_amdgcn_ds_bpermute(src << 2, (int)loc);
    uint32_t w = up ? nx : kWordEnd;
    uint32_t wr[5];
#pragma unroll
    for (int r = 4; r >= 0; --r) wr[r] = w = mt[r] ? rw[r] : w;
#pragma unroll
    for (int r = 0; r < 5; ++r)
      S.word[p0 + r] = wr[r];            // past n: kWordEnd (no match starts there)
    return (uint32_t)__builtin_amdgcn_readlane((int)wr[0], 0);   // word[0]
  };
  // No verified candidate reached 256 bytes, so no best(p) does (a scan term
  // is a candidate shifted right, never longer): len < 256, M = len, every
  // len >= 4 is a match, and the word is x (its bits 17..18, len's bits
  // 8..9, are zero).  Otherwise the general form (M = len & 0xFF, len 256 no
  // match).  The records rounds are instantiated the same way: without a
  // truncated match no M is 1..3, so a sequence's size field is its byte
  // count and one plain wave sum gives both.
  const bool fastw = !ballot(longm != 0u);   // no truncated match: M = len, never 1..3
  const uint32_t w0 = fastw ? word_pass(std::true_type{}) : word_pass(std::false_type{});
  wave_sync();

  PROF_MARK(4);                       // word
  // ---- greedy parse = walk over the match words (LZ4.c:516-583) -------------
  // The walk is the serial part of the block: w_0 = word[0], w_{k+1} =
  // word[c_k + M_k], one LDS read per sequence; sequence k's word is kept in
  // lane k of a register (v_writelane).  The loop is one asm block: m0 is both
  // the lane select and the sequence counter, the next address is the loaded
  // word shifted in a VGPR, and the loop goes on while the word is a match,
  // i.e. its field 4 (c + M) <= 4 n (kWordEnd's is 4 * 319 > 4 n): three VALU
  // and two SALU per sequence.
  const uint32_t lim = (uint32_t)(4 * n + 1) << 17;
  int it = 0;
  uint32_t seqv = 0;
  // The walk is the block's one serial chain: the wave issues it at raised
  // priority, so on a SIMD shared with waves in their parallel phases each
  // step goes first (-0.3 % lz4_tiles, tools/ab_inproc.py; raising the index,
  // candidate, scan or records phases instead measured 0.2-5 % slower)
  __builtin_amdgcn_s_setprio(3);
  if (w0 < lim) {
    static_assert(kWordOff < 65536, "ds_read offset field");
    uint32_t w = w0, va = w0 >> 17, vt;
    asm volatile(
        "s_mov_b32 m0, 0\n"
        "1:\n\t"
        "v_writelane_b32 %0, %1, m0\n\t"
        "ds_read_b32 %3, %2 offset:%c6\n\t"
        "s_add_u32 m0, m0, 1\n\t"
        "s_waitcnt lgkmcnt(0)\n\t"
        "v_readfirstlane_b32 %1, %3\n\t"
        "v_lshrrev_b32 %2, 17, %3\n\t"
        "s_cmp_lt_u32 %1, %5\n\t"
        "s_cbranch_scc1 1b\n\t"
        "s_mov_b32 %4, m0"
        : "+v"(seqv), "+s"(w), "+v"(va), "=&v"(vt), "=s"(it)
        : "s"(lim), "i"(kWordOff)
        : "scc", "memory");
  }
  __builtin_amdgcn_s_setprio(0);
  // Past 64 sequences (only with truncated matches) the walk is redone into S.seq.
  const bool slow = it > 64;
  int Sv_slow = 0;
  if (slow) {
    const uint8_t *const wb = reinterpret_cast<const uint8_t *>(S.word);
    for (uint32_t w = w0; w < lim;
         w = (uint32_t)__builtin_amdgcn_readfirstlane(
             (int)*reinterpret_cast<const uint32_t *>(wb + (w >> 17)))) {
      if (lane == 0) S.seq()[Sv_slow] = w;
      ++Sv_slow;
    }
    wave_sync();
  }
  PROF_MARK(5);                       // walk
#if LZ4R_VARIANT >= 40 && LZ4R_VARIANT <= 42
  // tools build: probes of the binding resource -- 40: +16 conflict-free LDS
  // reads, 41: +16 VOP3 VALU (v_perm), 42: +32 plain VALU (v_xor) per block
  {
    uint32_t acc = (uint32_t)lane;
#if LZ4R_VARIANT == 40
#pragma unroll
    for (int i = 0; i < 16; ++i)
      acc ^= *reinterpret_cast<volatile uint32_t *>(&S.rec[(lane + 64 * (i & 3)) % kArr]);
#elif LZ4R_VARIANT == 41
#pragma unroll
    for (int i = 0; i < 16; ++i) asm volatile("v_perm_b32 %0, %0, %0, %1" : "+v"(acc) : "s"(0x05040100u));
#else
#pragma unroll
    for (int i = 0; i < 32; ++i) asm volatile("v_xor_b32 %0, 0x9e3779b1, %0" : "+v"(acc));
#endif
    if (acc == 0x7FFFFFFFu) S.seq()[0] = acc;   // never on a real block; keeps the probe
  }
#endif
  // ---- sequence records: lane kk = sequence kk -----------------------------
  // A round is 64 consecutive sequences; the match sequences are a prefix
  // (cpos < n), followed by the literal-only tail when the last match ends
  // before n (LZ4.c:585-612).  Rounds go on while a round is all matches.
  // The block leaves as records -- sequence k: its match word dist | M << 9 |
  // (match start + M) << 19 as the walk read it (its literal run starts where
  // sequence k - 1's match ends; the tail is n << 19) -- after a header dword,
  // the sum of the sequences' size fields | the sequence count << 16.  lz4_emit writes the bytes
  // (write_sequence / write_block, LZ4.c:365-425) straight into the stream.
  int nseq = 0;
  int ocar = 3;                      // block header: u8 nseq, u16 size
  int szsum = 0;
  int end_prev = 0;                  // end of the previous round's last match
  // one round: sequence kk = s0 + lane has the match word wv (n << 19 -- no
  // match, M = dist = 0, ending at n -- past the matches); returns false once
  // the round holds the last sequence
  auto round = [&](auto fast, int s0, uint32_t wv) {
    const int kk = s0 + lane;
    const int M = (int)((wv >> 9) & 255u);
    const int end = (int)(wv >> 19);
    const uint32_t cq = (uint32_t)(end - M);                       // the match start
    const uint64_t ismm = ballot((int)cq < n);                     // ends with a match
    const int nm_r = __popcll(ismm);                               // a prefix of the round
    const uint32_t upv = dpp<0x138, 0xf, 0xf>((uint32_t)end);   // wave_shr:1
    const int pend = lane == 0 ? end_prev : (int)upv;             // literal run start
    end_prev = (int)lane63((uint32_t)end);
    const int L = (int)cq - pend;
    // + the tail (lane nm_r, when literals are left); the mask from ballots
    // of the compares (a ballot of a combined bool costs two VALU)
    const uint64_t am = ismm | (ballot(lane == nm_r) & ballot(pend < n));
    // bytes written (LZ4.c:365-413) | the size field (LZ4.c:546-575) << 16:
    // 5 + L + the literal-extension bytes (one from 15, two at L = 270, where
    // the uint8_t remainder is 255: LZ4.c:376-385) + a match-extension byte
    // (M >= 19); the size field also counts one for M = 1..3, which
    // write_sequence never writes (LZ4.c:393 vs :562-575)
    if constexpr (decltype(fast)::value) {
      // no M = 1..3 (no truncated match): the size fields are the bytes
      const uint32_t ws = (uint32_t)(L + 5) + (L >= 15 ? 1u : 0u) + (L == 270 ? 1u : 0u) +
                          (M >= 19 ? 1u : 0u);
      const uint32_t tot = lane63(wave_incl_add(sel_mask(am, ws, 0u)));
      ocar += (int)tot;
      szsum += (int)tot;
    } else {
      uint32_t ws = (uint32_t)(L + 5 + (L >= 15 ? 1 : 0) + (L == 270 ? 1 : 0)) * 0x10001u;
      ws += M >= 19 ? 0x10001u : 0u;
      ws += (uint32_t)(M - 1) < 3u ? 0x10000u : 0u;
      const uint32_t tot = lane63(wave_incl_add(sel_mask(am, ws, 0u)));
      ocar += (int)(tot & 0xFFFFu);
      szsum += (int)(tot >> 16);
    }
    // record dword 1 + kk (the sequence's word; the tail: n << 19): the head
    // for kk < kHeadW - 1, the overflow slot after (the same lane offset off
    // a base kHeadW dwords back)
    if (s0 == 0) {
      store_lanes1(am & ((1ull << (kHeadW - 1)) - 1), head, 4u * (uint32_t)kk, wv);
      if (am >> (kHeadW - 1)) store_lanes1(am >> (kHeadW - 1) << (kHeadW - 1), ovf - kHeadW,
                                           4u * (uint32_t)kk, wv);
    } else {
      store_lanes1(am, ovf - kHeadW, 4u * (uint32_t)kk, wv);
    }
    nseq += (int)__popcll(am);
    return nm_r == 64;
  };
  if (LZ4R_VARIANT != 11) {
    // round 0 from the walk's register; more than 64 sequences (the walk's
    // register wrapped) come from the redone walk in S.seq
    const uint32_t wtail = (uint32_t)n << 19;
    const uint32_t c0 = slow ? S.seq()[lane] : (lane < it ? seqv : wtail);
    auto rounds = [&](auto fast) {
      if (round(fast, 0, c0)) {        // 64 match sequences: the tail or more follow
        for (int s0 = 64;; s0 += 64) {
          const int kk = s0 + lane;
          if (!round(fast, s0, slow && kk < Sv_slow ? S.seq()[kk] : wtail)) break;
        }
      }
    };
    if (fastw)
      rounds(std::true_type{});
    else
      rounds(std::false_type{});
  }
  PROF_MARK(6);                       // records
  if (lane == 0) head[0] = (uint32_t)szsum | ((uint32_t)nseq << 16);
  return ocar;
}

template <bool kAligned>   // the input is 4-byte aligned (the host checks)
__global__ __launch_bounds__(64) void lz4_tiles(
    const uint8_t *__restrict__ in, uint32_t nb, uint32_t per, uint32_t last_n,
    uint8_t *__restrict__ heads, uint8_t *__restrict__ ovfs, uint32_t *__restrict__ usz,
    uint16_t *__restrict__ bsizes, uint32_t *__restrict__ status) {
  __shared__ TileLds S;
  const int lane = threadIdx.x;
  // XCD-aware order: workgroups w and w + 8 share an XCD (observed round-robin
  // dealing), so XCD w % 8 takes the contiguous slice [(w % 8) per, ...) of
  // the blocks and a 128-B line shared by two neighbouring blocks is fetched
  // into one L2, not two (a speed matter only: any mapping is correct).
  const uint32_t t = (blockIdx.x & 7u) * per + (blockIdx.x >> 3);
  if (t >= nb) return;
  const int n = t == nb - 1 ? (int)last_n : kBlk;
  const uint8_t *src = in + (size_t)t * kBlk;

  uint32_t *const head = reinterpret_cast<uint32_t *>(heads + (size_t)t * kHead);
  uint32_t *const ovf = reinterpret_cast<uint32_t *>(ovfs + (size_t)t * kOvf);
  int W;
  if (kAligned && (t + 2 < nb || (t + 2 == nb && last_n >= 24))) {
    // no staging, the keys come straight from global memory
    // (encode_block<kFull>): row 4's lanes read 24 bytes past the block end
    // (and a mid-walk lcp drain up to 15), so only where those bytes are the
    // launch's own -- every block but the last, and the one before it when
    // the last holds at least 24 bytes
    W = encode_block<false, true>(S, kBlk, src, nullptr, head, ovf, status);
  } else {
    // the last block (n <= 300: nothing may be read past the input), the one
    // before a last block of < 24 bytes, or an unaligned input: staged
    // bytewise, 16-B zero pad
    for (int i = lane; i < n; i += 64) S.buf[kInOff + i] = src[i];
    if (lane < 16) S.buf[kInOff + n + lane] = 0;
    wave_sync();
    W = encode_block<false, false>(S, n, nullptr, nullptr, head, ovf, status);
  }
  if (lane == 0) {
    usz[t] = (uint32_t)W;
    bsizes[t] = (uint16_t)W;
  }
}


// Per-position longest matches of every block (the batch form of
// find_longest_match): the same staging and match finder as lz4_tiles.
__global__ __launch_bounds__(64) void lz4_matches(const uint8_t *__restrict__ in, uint32_t nb,
                                                   uint32_t last_n, uint32_t *__restrict__ mout) {
  __shared__ TileLds S;
  const int lane = threadIdx.x;
  const uint32_t t = blockIdx.x;
  if (t >= nb) return;
  const int n = t == nb - 1 ? (int)last_n : kBlk;
  const uint8_t *src = in + (size_t)t * kBlk;
  for (int i = lane; i < n; i += 64) S.buf[kInOff + i] = src[i];
  if (lane < 16) S.buf[kInOff + n + lane] = 0;
  wave_sync();
  encode_block<true, false>(S, n, nullptr, mout + (size_t)t * kBlk, nullptr, nullptr, nullptr);
}

// find_longest_match over a block of any length n (block_encode with a
// block_length other than 300): the reference's whole window, LZ4.c:295-312
// -- sources i in [max(0, p - WINDOW_SIZE), p), match length capped at
// MAX_MATCH_LENGTH (1024) and, canonically, at the block end n - p; the
// longest wins, ties to the smallest i (strict '>', LZ4.c:307).  One wave
// per position, its lanes striding over the window, a max-reduction of
// len << 17 | dist (the larger dist is the smaller source).  A compatibility
// path, O(n * window): the 300-byte blocks of the compressor use lz4_tiles.
constexpr int kWindow = 65535;          // WINDOW_SIZE, LZ4.c:22
constexpr int kMaxMatch = 1024;         // MAX_MATCH_LENGTH, LZ4.c:20

__global__ __launch_bounds__(256) void lz4_window_matches(const uint8_t *__restrict__ in,
                                                          uint32_t n, uint32_t p_first,
                                                          uint32_t *__restrict__ mout) {
  const int lane = threadIdx.x & 63;
  const uint32_t p = p_first + blockIdx.x * 4u + (threadIdx.x >> 6);
  if (p >= n) return;
  const uint32_t cap = min((uint32_t)kMaxMatch, n - p);
  const uint32_t i0 = p >= (uint32_t)kWindow ? p - (uint32_t)kWindow : 0u;
  const uint8_t c0 = in[p];
  uint32_t best = 0;
  for (uint32_t i = i0 + (uint32_t)lane; i < p; i += 64) {
    if (in[i] != c0) continue;
    uint32_t l = 1;
    while (l < cap && in[i + l] == in[p + l]) ++l;
    best = max(best, (l << 17) | (p - i));
  }
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) best = max(best, (uint32_t)__shfl_xor((int)best, d, 64));
  if (lane == 0) {
    const uint32_t len = best >> 17;
    mout[p] = len >= 4 ? len | ((best & 0x1FFFFu) << 16) : 0u;   // MIN_MATCH_LENGTH, LZ4.c:314
  }
}

// ---- placement: exclusive scan of tile sizes, then gather -----------------
constexpr int kGT = 64;              // tiles per gather group (one workgroup)
constexpr int kPart = 64 * kGT;      // tiles per scan partial (64 groups)

// per group of 64 tiles: gsum; per 64 groups: part.  Coalesced: load k of
// the workgroup reads tiles [1024 k, 1024 k + 1024) of the partial as uint4,
// 16 lanes (one DPP row) per group of 64 tiles.
__global__ __launch_bounds__(256) void lz4_scan_reduce(const uint32_t *__restrict__ tsz,
                                                       size_t ntiles, size_t p_first,
                                                       uint32_t *__restrict__ gsum,
                                                       uint64_t *__restrict__ part) {
  __shared__ uint32_t ws[4];
  const int tid = threadIdx.x;
  const size_t pi = p_first + blockIdx.x;                            // partial index
  const size_t q0 = pi * (kPart / 4);                                // its first uint4
  uint32_t v[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const size_t q = q0 + (size_t)(256 * k + tid);                   // tiles 4q .. 4q + 3
    if (4 * q + 4 <= ntiles) {
      const uint4 x = reinterpret_cast<const uint4 *>(tsz)[q];
      v[k] = x.x + x.y + x.z + x.w;
    } else {
      v[k] = 0;
      for (int j = 0; j < 4; ++j)
        if (4 * q + j < ntiles) v[k] += tsz[4 * q + j];
    }
  }
  uint32_t tot = 0;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    uint32_t x = v[k];                       // row prefix: lane 15 of the row holds the group
    x += dpp<0x111, 0xf, 0xf>(x);
    x += dpp<0x112, 0xf, 0xf>(x);
    x += dpp<0x114, 0xf, 0xf>(x);
    x += dpp<0x118, 0xf, 0xf>(x);
    const size_t g = pi * 64 + (size_t)(16 * k + (tid >> 4));
    if ((tid & 15) == 15) {
      if (g * kGT < ntiles) gsum[g] = x;
      tot += x;
    }
  }
  tot = wave_incl_add(tot);                  // < 2^32: 4096 tiles of <= 548 B
  if ((tid & 63) == 63) ws[tid >> 6] = tot;
  __syncthreads();
  if (tid == 0) part[pi] = (uint64_t)ws[0] + ws[1] + ws[2] + ws[3];
}

// one workgroup: exclusive scan of the partials in place, as absolute stream
// offsets.  The scan starts at `hdr` (first != 0) or at *len (a continuation)
// and leaves its end in *len.  The call's last scan (last != 0) also folds
// lz4_tiles' corrupt-index status word into bit 63 of *len (kLenCorrupt) and
// clears the word: every async caller gets the verdict in the length it
// reads anyway, and the next call starts clean.  The same verdict goes to
// *verdict, a word the context owns (lz4r_check reads it: the caller's
// length buffer may be gone by then).
constexpr uint64_t kLenCorrupt = 1ull << 63;
__global__ __launch_bounds__(1024) void lz4_scan_partials(uint64_t *__restrict__ part,
                                                          size_t nparts, uint64_t hdr,
                                                          int first, int last,
                                                          uint32_t *__restrict__ status,
                                                          uint64_t *__restrict__ len,
                                                          uint64_t *__restrict__ verdict) {
  __shared__ uint64_t ws[16];
  __shared__ uint64_t carry;
  if (threadIdx.x == 0) carry = first ? hdr : *len;
  __syncthreads();
  for (size_t c0 = 0; c0 < nparts; c0 += 1024) {
    const size_t i = c0 + threadIdx.x;
    const uint64_t v = i < nparts ? part[i] : 0;
    uint64_t x = v;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const uint64_t o = __shfl_up(x, d, 64);
      if ((threadIdx.x & 63) >= d) x += o;
    }
    if ((threadIdx.x & 63) == 63) ws[threadIdx.x >> 6] = x;
    __syncthreads();
    uint64_t pre = carry;
    for (int w = 0; w < (int)(threadIdx.x >> 6); ++w) pre += ws[w];
    if (i < nparts) part[i] = pre + x - v;
    __syncthreads();
    if (threadIdx.x == 1023) carry = pre + x;
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    uint64_t v = carry;
    if (last) {
      const bool bad = atomicExch(status, 0u) != 0u;
      if (bad) v |= kLenCorrupt;
      *verdict = bad ? 1u : 0u;
    }
    *len = v;
  }
}



// lz4_emit: workgroup = 32 consecutive blocks (half a scan group of 64).
//   offsets  the blocks' stream offsets from the partials, the group sums and
//            a wave scan; also stored to boff (the decoder's side input)
//   stage    the 32 blocks' input -> LDS (the literals' source; 16-B loads)
//   bytes    each wave takes 8 blocks and flattens their sequence records over
//            the lanes (one round = 64 sequences of one or more blocks); per
//            sequence the token / size / literal-extension / offset /
//            match-extension bytes (write_sequence, LZ4.c:365-413) and per
//            block the u8 count + u16 size header (write_block, :415-425)
//            land by aligned ds_or in a zeroed LDS image of the output range,
//            and the literal runs are flattened over the lanes as aligned
//            16-byte image words funnel-shifted out of the staged input
//   store    the image -> the stream as aligned 16-B stores (the edge chunks
//            bytewise); nothing at or past `cap` is written.
// This is the emission lz4_tiles used to do one block per wave; here a round
// serves several blocks and the kernel is bound by its HBM traffic, not by
// instruction issue as lz4_tiles is.
// lz4_emit reads its input, the record heads and writes the stream exactly
// once: 16-B accesses with the non-temporal hint (the nontemporal builtins take
// a native vector type), -1.3 % emit time (tools/ab_inproc.py)
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
constexpr int kGH = 32;                              // blocks per emit workgroup
constexpr int kEW = 8;                               // waves per emit workgroup (4 blocks each)
constexpr int kRecPre = kHeadW;                      // record dwords per block staged in LDS
constexpr int kGSplit = kGT / kGH;                   // workgroups per group
constexpr int kEmitImg = kGH * kBlkOutMax + 32;      // worst case: every block 548 B
constexpr int kStagePad = 16;                        // literal words reach 15 B before a run
constexpr int kStage = kStagePad + kGH * kBlk + 32;  // ... and 16 B past its end
static_assert(kStage < (1 << 16), "stage offsets fit 16 bits");

// OR the (<= 4) bytes of v into the zeroed byte area at offset x: two
// aligned dwords (ds_or_b32), never a misaligned access
__device__ __forceinline__ void or_bytes(uint32_t *buf32, int x, uint32_t v) {
  const uint64_t w = (uint64_t)v << (8 * (x & 3));
  atomicOr(&buf32[x >> 2], (uint32_t)w);
  atomicOr(&buf32[(x >> 2) + 1], (uint32_t)(w >> 32));
}

// Records -> bytes of one emit task (lz4_emit): wave wv takes
// blocks [h0 + 4 wv, ...) of the task's [h0, h1); the image img[lead] is
// stream byte G0; block h's input is stage[kStagePad + 300 (h - h0) + p].
__device__ __forceinline__ void emit_records(const int wv, const int lane, const int h0,
                                             const int h1, const uint64_t G0, const int lead,
                                             const uint64_t *toff, uint8_t *img,
                                             const uint8_t *stage,
                                             const uint32_t (*recst)[kRecPre],
                                             uint32_t (*marks)[64], const uint4 *pmask,
                                             const uint8_t *__restrict__ wovf) {
  {
    constexpr int kBW = kGH / kEW;                   // blocks per wave
    const int bl0 = h0 + wv * kBW, bl1 = min(h1, bl0 + kBW);
    // (33, 37: tools ablations without the records -> bytes phase)
    if (bl0 < bl1 && LZ4R_VARIANT != 33 && LZ4R_VARIANT != 37) {
      uint32_t *const out32 = reinterpret_cast<uint32_t *>(img);
      const int nbk = bl1 - bl0;
      // lanes 0..nbk-1: the blocks' sequence counts -> first flattened index
      const uint32_t hd = lane < nbk ? recst[bl0 - h0 + lane][0] : 0u;
      const uint32_t ns = hd >> 16;
      const uint32_t sinc = wave_incl_add(ns);
      const int Stot = (int)lane63(sinc);
      const int sst = (int)(sinc - ns);
      int st[kBW];                                 // wave-uniform block starts
#pragma unroll
      for (int i = 0; i < kBW; ++i)
        st[i] = i < nbk ? __builtin_amdgcn_readlane(sst, i) : 0x7fffffff;
      // the wave's blocks are contiguous in the image, each its 3 header bytes
      // and then its sequences' bytes (tsz counts the bytes written): sequence f
      // lands at the wave's first image byte + 3 (its block's rank + 1) + the
      // bytes of the wave's sequences before it
      int end_prev = 0, wcur = lead + (int)(toff[bl0] - G0) + 3;
      for (int f0 = 0; f0 < Stot; f0 += 64) {
        const int f = f0 + lane;
        const bool valid = f < Stot;
        int bi = 0, sb = 0;                        // the lane's block: the last start <= f
#pragma unroll
        for (int i = 1; i < kBW; ++i) {
          const bool ge = f >= st[i];
          bi += ge ? 1 : 0;
          sb = ge ? st[i] : sb;
        }
        const int k = f - sb;                      // sequence index in the block
        const int hb = bl0 + bi;
        const uint32_t *rp = reinterpret_cast<const uint32_t *>(wovf + (hb - h0) * kOvf);
        const uint32_t r =
            !valid ? 0u : (1 + k < kRecPre ? recst[hb - h0][1 + k] : rp[1 + k - kRecPre]);
        // record = the sequence's match word: dist | M << 9 | (match start +
        // M) << 19 (the literal tail: n << 19)
        const int M = (int)((r >> 9) & 255u), D = (int)(r & 511u);
        const int end = (int)(r >> 19);
        const int cpos = end - M;
        const uint32_t upv = dpp<0x138, 0xf, 0xf>((uint32_t)end);   // wave_shr:1
        const int pend = k == 0 ? 0 : (lane == 0 ? end_prev : (int)upv);   // literal run start
        end_prev = (int)lane63((uint32_t)end);
        const int L = cpos - pend;
        const int rem = (L - 15) & 255;
        const int le = L >= 15 ? (rem == 255 ? 2 : 1) : 0;         // literal-extension bytes
        const int mx = (M - 4) & 255;
        const bool mextW = M >= 4 && mx >= 15, mextS = M != 0 && mx >= 15;
        const int bytes = valid ? 5 + le + L + (mextW ? 1 : 0) : 0;
        const uint32_t inc = wave_incl_add((uint32_t)bytes);
        const int o = wcur + 3 * bi + (int)inc - bytes;               // the sequence's token
        const int ib = o - 3;                                         // (k == 0) its block's header
        const int ol = o + 3 + le;                                   // first literal byte
        if (valid && LZ4R_VARIANT != 32) {                            // (32: tools ablation)
          const int tl = L >= 15 ? 15 : L;                            // LZ4.c:540
          const int tm = M == 0 ? 0 : (M >= 19 ? 15 : mx);            // LZ4.c:542
          const uint32_t ext = le == 0 ? 0u : (rem == 255 ? 255u : (uint32_t)rem);
          const uint32_t SZ = (uint32_t)(5 + le + L + (mextS ? 1 : 0));   // LZ4.c:546-575
          or_bytes(out32, o, (uint32_t)((tl << 4) | tm) | (SZ << 8) | (ext << 24));
          or_bytes(out32, ol + L, (uint32_t)D | (mextW ? ((uint32_t)(mx - 15) & 255u) << 16 : 0u));
          if (k == 0) {                                               // LZ4.c:417-419
            const uint32_t bh = recst[hb - h0][0];
            or_bytes(out32, ib, ((bh >> 16) & 255u) | ((((bh & 0xFFFFu) + 3u) & 0xFFFFu) << 8));
          }
        }
        // literals (LZ4.c:388), flattened over the lanes: one aligned 16-byte
        // image word per lane and pass, funnel-shifted out of five aligned
        // staged input dwords and masked to the run (16-B words: half the
        // passes of 8-B ones; two ds_or_b64 per word)
        {
          const int cw = valid && L > 0 ? ((ol + L - 1) >> 4) - (ol >> 4) + 1 : 0;
          const uint32_t cinc = wave_incl_add((uint32_t)cw);
          const int C = LZ4R_VARIANT == 31 ? 0 : (int)lane63(cinc);   // (31: tools ablation)
          const int stw = (int)dpp<0x138, 0xf, 0xf>(cinc);
          // the run, as its owning lanes use it: image word w = (ol >> 3) - stw + gw,
          // stage byte of that word's first image byte xs = 8 w + (src - ol), and
          // its bytes [ol, ol + L) of the image (two 16-bit fields per dword)
          const int src = kStagePad + kBlk * (hb - h0) + pend;
          const uint32_t rw = ((uint32_t)((ol >> 4) - stw) & 0xFFFFu) | ((uint32_t)(src - ol) << 16);
          const uint32_t rb = (uint32_t)ol | ((uint32_t)(ol + L) << 16);
          uint32_t carry = 0;                    // 1 + the last run owning a word so far
          for (int w0 = 0; w0 < C; w0 += 64) {
            wave_sync();
            marks[wv][lane] = 0u;
            if (cw > 0 && stw >= w0 && stw < w0 + 64) marks[wv][stw - w0] = (uint32_t)lane + 1u;
            wave_sync();
            const uint32_t k1 = max(wave_incl_max(marks[wv][lane]), carry);
            carry = lane63(k1);
            const int gw = w0 + lane;
            const int kr = ((int)k1 - 1) & 63;   // the run owning word gw
            const uint32_t kw = (uint32_t)__shfl((int)rw, kr, 64);
            const uint32_t kb = (uint32_t)__shfl((int)rb, kr, 64);
            if (gw < C) {
              const int t = 16 * ((int)(int16_t)(kw & 0xFFFFu) + gw);  // image word's first byte
              const int xs = t + ((int)kw >> 16);                      // its input bytes
              const uint32_t *iw = reinterpret_cast<const uint32_t *>(stage + (xs & ~3));
              const uint32_t d0 = iw[0], d1 = iw[1], d2 = iw[2], d3 = iw[3], d4 = iw[4];
              const uint32_t sh = (uint32_t)xs & 3u;
              const int lb = max((int)(kb & 0xFFFFu) - t, 0), hb = min((int)(kb >> 16) - t, 16);
              const uint4 ml = pmask[lb], mh = pmask[hb];
              const uint32_t v0 = __builtin_amdgcn_alignbyte(d1, d0, sh) & (ml.x ^ mh.x);
              const uint32_t v1 = __builtin_amdgcn_alignbyte(d2, d1, sh) & (ml.y ^ mh.y);
              const uint32_t v2 = __builtin_amdgcn_alignbyte(d3, d2, sh) & (ml.z ^ mh.z);
              const uint32_t v3 = __builtin_amdgcn_alignbyte(d4, d3, sh) & (ml.w ^ mh.w);
              atomicOr(reinterpret_cast<unsigned long long *>(img + t),
                       (unsigned long long)v1 << 32 | v0);
              atomicOr(reinterpret_cast<unsigned long long *>(img + t + 8),
                       (unsigned long long)v3 << 32 | v2);
            }
          }
        }
        wcur += (int)lane63(inc);
      }
    }
  }
}

// The task's image -> the stream (aligned 16-B stores; the two edge chunks a
// byte per lane of the last wave); nothing at or past G1 (<= cap) is written.
__device__ __forceinline__ void emit_store(const int tid, const int wv, const int lane,
                                           const uint64_t G0, const uint64_t G1, const int lead,
                                           const uint8_t *img, uint8_t *__restrict__ out) {
  if (G1 <= G0) return;
  // chunk ci covers stream bytes [F + 16 ci, F + 16 ci + 16), F = G0 - lead
  // (16-B aligned), as 32-bit offsets (the range is at most kEmitImg bytes) from
  // out + F, so the stores stay global_store (a pointer rebuilt from an integer
  // is a flat address: every flat store also counts in lgkmcnt and serialised
  // this loop behind its LDS reads)
  const uint64_t F = G0 - (uint64_t)lead;
  uint8_t *const outF = out + F;
  const uint32_t nrel = (uint32_t)(G1 - F);
  const uint32_t c0 = lead ? 1u : 0u, c1 = nrel >> 4;   // the whole chunks: [c0, c1)
  for (uint32_t ci = c0 + (uint32_t)tid; ci < c1; ci += 64 * kEW)
    __builtin_nontemporal_store(reinterpret_cast<const u32x4 *>(img)[ci],
                                reinterpret_cast<u32x4 *>(outF + 16u * ci));
  // the partial chunks at either end, a byte per lane: lanes 0-15 the first
  // chunk's bytes [lead, 16), lanes 16-31 the last one's [16 c1, nrel) (when it
  // is not the first)
  if (wv == kEW - 1 && lane < 32) {
    const uint32_t x = lane < 16 ? (uint32_t)lane : 16u * c1 + (uint32_t)(lane - 16);
    const bool own = lane < 16 ? (c0 && x >= (uint32_t)lead && x < nrel) : (c1 >= c0 && x < nrel);
    if (own) outF[x] = img[x];
  }}

__global__ __launch_bounds__(64 * kEW) void lz4_emit(
    const uint8_t *__restrict__ in, const uint8_t *__restrict__ heads,
    const uint8_t *__restrict__ ovfs, size_t slot_base,
    const uint32_t *__restrict__ tsz, size_t ntiles, size_t g_first,
    const uint32_t *__restrict__ gsum, const uint64_t *__restrict__ part,
    uint8_t *__restrict__ out, uint64_t cap, int hdr, uint64_t nb_total, uint32_t last_n,
    uint64_t *__restrict__ boff) {
  __shared__ uint64_t toff[kGT + 1];
  __shared__ alignas(16) uint8_t img[kEmitImg];
  __shared__ alignas(16) uint8_t stage[kStage];
  __shared__ uint32_t marks[kEW][64];                // per wave: literal-run starts
  __shared__ uint4 pmask[17];                        // pmask[k]: the low k bytes of 16 set
  __shared__ uint32_t recst[kGH][kRecPre];           // each block's header + first records
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  // XCD-aware order (workgroups b and b + 8 share an XCD): XCD b % 8 takes a
  // contiguous eighth of the workgroups, so neighbouring outputs' boundary
  // lines meet in one L2
  const uint32_t nwg = (uint32_t)((ntiles - g_first * kGT + kGT - 1) / kGT) * kGSplit;
  const uint32_t per = (nwg + 7) / 8;
  const uint32_t wg = (blockIdx.x & 7u) * per + (blockIdx.x >> 3);
  if (wg >= nwg) return;
  const size_t g = g_first + wg / kGSplit;
  const int h0 = (int)(wg % kGSplit) * kGH;          // this workgroup: blocks [h0, h0 + kGH)
  const size_t g0 = g * kGT;
  const int nt = (int)min((size_t)kGT, ntiles - g0);
  if (h0 >= nt) return;
  const int h1 = min(nt, h0 + kGH);
  // Every global load of the workgroup is issued before any of them is
  // waited on (the scan inputs, the record heads, the staged input): one
  // memory round trip per workgroup, not three.
  const size_t b0 = g0 + h0;
  const int len = (h1 - h0 - 1) * kBlk + (g0 + h1 == nb_total ? (int)last_n : kBlk);
  const uint8_t *src = in + b0 * kBlk;
  const bool al16 = ((uintptr_t)src & 15) == 0;    // b0 is a multiple of 32: 9600 B steps
  const int n16 = al16 ? len >> 4 : 0;
  uint64_t pt = 0;
  uint32_t gs = 0, tv = 0;
  if (tid < 64) {
    // wave 0 carries the workgroup's critical path to the first barrier (its
    // scan loads, then two wave sums): raised priority until the barrier
    // (emit 0.622 -> 0.603 ms, tools/ab_inproc.py)
    __builtin_amdgcn_s_setprio(3);
    const size_t p = g0 / kPart;
    const size_t gfirst = p * 64;                  // first group of the partial
    gs = (gfirst + tid < g) ? gsum[gfirst + tid] : 0u;
    pt = part[p];                                  // part[] holds absolute offsets
    tv = tid < nt ? tsz[g0 + tid] : 0u;
  }
  constexpr int kPerSlot = kRecPre / 4;            // record heads: 32 x 96 B, contiguous
  static_assert(kGH * kPerSlot <= 64 * kEW, "one record load per thread");
  uint4 rv = make_uint4(0, 0, 0, 0);
  const int rhb = tid / kPerSlot, rj = tid % kPerSlot;
  // the workgroup's heads (one contiguous run) and overflow slots
  const uint8_t *const wheads = heads + (b0 - slot_base) * (size_t)kHead;
  const uint8_t *const wovf = ovfs + (b0 - slot_base) * (size_t)kOvf;
  if (tid < (h1 - h0) * kPerSlot) {
    const u32x4 t = __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(wheads) + tid);
    rv = make_uint4(t.x, t.y, t.z, t.w);
  }
  constexpr int kSt16 = (kGH * kBlk) / 16;         // 600 16-B chunks of staged input
  constexpr int kStPer = (kSt16 + 64 * kEW - 1) / (64 * kEW);
  uint4 sv[kStPer];
#pragma unroll
  for (int k = 0; k < kStPer; ++k) {
    const int i = tid + k * 64 * kEW;
    u32x4 t = {0u, 0u, 0u, 0u};
    if (i < n16) t = __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(src) + i);
    sv[k] = make_uint4(t.x, t.y, t.z, t.w);
  }
  // the image is zeroed in full while the loads are in flight
  for (int i = tid; i < kEmitImg / 16 && LZ4R_VARIANT != 35; i += 64 * kEW)   // (35: ablation)
    reinterpret_cast<uint4 *>(img)[i] = make_uint4(0, 0, 0, 0);
  if (tid < 64) {
    // the groups before g in its partial: <= 63 sums of <= 64 blocks of
    // <= 548 B, so the total fits 32 bits -- a DPP sum, not a 64-bit
    // shuffle reduction (12 dependent ds_bpermute round trips on wave 0,
    // which every wave of the workgroup waits for at the barrier)
    const uint64_t base = pt + lane63(wave_incl_add(gs));
    const uint32_t inc = wave_incl_add(tv);
    toff[tid] = base + inc - tv;
    if (tid == 63) toff[kGT] = base + inc;
    // device-resident block offsets (relative to the first block byte) for
    // the block-parallel decoder: no host prefix sum, no host round trip
    if (h0 == 0 && tid < nt) boff[g0 + tid] = base + inc - tv - (uint64_t)hdr;
  }
  if (hdr && g == 0 && h0 == 0 && tid == 0 && cap > 0) out[0] = (uint8_t)nb_total;
  if (tid < (h1 - h0) * kPerSlot) reinterpret_cast<uint4 *>(&recst[rhb][0])[rj] = rv;
  if (tid < 17) {
    uint32_t m[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int n = min(max(tid - 4 * j, 0), 4);
      m[j] = n == 4 ? ~0u : (1u << (8 * n)) - 1u;
    }
    pmask[tid] = make_uint4(m[0], m[1], m[2], m[3]);
  }
  // ---- stage: byte p of block h is stage[kStagePad + 300 (h - h0) + p] ----------
  {
    uint8_t *dst = stage + kStagePad;
#pragma unroll
    for (int k = 0; k < kStPer; ++k) {
      const int i = tid + k * 64 * kEW;
      if (i < n16) reinterpret_cast<uint4 *>(dst)[i] = sv[k];
    }
    for (int i = (n16 << 4) + tid; i < len; i += 64 * kEW) dst[i] = src[i];   // tail / unaligned
  }
  __syncthreads();
  __builtin_amdgcn_s_setprio(0);
#if LZ4R_VARIANT == 31 || LZ4R_VARIANT == 33 || LZ4R_VARIANT == 37
  // tools ablations: the staged input and record heads kept alive (a read the
  // compiler cannot drop), so their loads stay in the ablated build
  if (reinterpret_cast<const uint32_t *>(stage)[tid] == 0x9E3779B1u &&
      recst[tid & 31][tid >> 5 & 15] == 0x7F4A7C15u && cap == 12345u)
    out[tid] = 1;
#endif
  const uint64_t G0 = toff[h0];
  const int lead = (int)(((uintptr_t)out + G0) & 15);   // img[lead] = stream byte G0
  emit_records(wv, lane, h0, h1, G0, lead, toff, img, stage, recst, marks, pmask, wovf);
  __syncthreads();
#if LZ4R_VARIANT == 34 || LZ4R_VARIANT == 37
  // tools ablations without the image -> stream stores (the image kept alive)
  if (reinterpret_cast<const uint32_t *>(img)[tid] == 0x9E3779B1u && cap == 12345u) out[tid] = 1;
  return;
#endif
  // ---- LDS image -> stream (aligned 16-B stores) --------------------------------
  emit_store(tid, wv, lane, G0, min(toff[h1], cap), lead, img, out);
}

}  // namespace

// Launch chunking: lz4_tiles is a 64-lane workgroup per block, and a HIP
// grid may not exceed 2^32 work-items, so a call is cut into chunks of at
// most kChunk blocks (5.03 GB of input; a multiple of the scan partial, so
// every chunk starts on a gather group and a partial).  The block slots are
// sized for one chunk (10.7 GB at most) and reused; the per-block arrays and
// the scan state span the whole call.  Each chunk is a full compress ->
// scan -> gather pass that continues the stream offset the previous chunk
// left in *d_len; the per-chunk launch cost (four launches) is noise against
// the ~19 ms of encoder work in a full chunk.
#ifndef LZ4R_CHUNK_LOG2
#define LZ4R_CHUNK_LOG2 24
#endif
constexpr size_t kChunk = size_t(1) << LZ4R_CHUNK_LOG2;
static_assert(kChunk % kPart == 0, "chunks start on a scan partial");
static_assert((kChunk / 8) * 8 * 64 < (size_t(1) << 32), "chunk grid fits HIP's limit");
// largest input one call accepts (block indices are u32 in the per-call arrays)
constexpr size_t kMaxInput = size_t(1) << 40;

struct lz4r_ctx {
  int device = 0;
  size_t cap_blocks = 0;       // capacity of the per-call per-block arrays
  size_t cap_slots = 0;        // capacity of the slot scratch, in blocks (<= kChunk)
  uint16_t *bsizes = nullptr;  // encoded bytes of every block of the last call
  uint64_t *boff = nullptr;    // every block's offset from the first block byte
  uint8_t *slots = nullptr;    // per-block record scratch, one chunk: cap_slots heads of
                               // kHead bytes, then cap_slots overflow slots of kOvf
  uint32_t *tsz = nullptr;     // encoded bytes per block (u32, for the scan)
  uint32_t *gsum = nullptr;    // encoded bytes per group of kGT blocks
  uint64_t *part = nullptr;    // scan partials, one per kPart blocks
  uint64_t *len = nullptr;     // default device length slot, the status word, the verdict
  uint32_t *status = nullptr;  // (len + 1) nonzero once a block saw a corrupt bucket head
  uint64_t *verdict = nullptr; // (len + 2) the last call's corrupt-index verdict (0 / 1)
  size_t last_nb = 0;
  bool checkable = false;      // a call has launched (lz4r_check has a verdict to read)
  // timing: per timed call since lz4r_set_timing(1), the call's start/end
  // events and lz4_tiles' start/end in every chunk (a ring of kTimedCalls
  // sets, so back-to-back async calls need no host wait between them)
  struct timed_set {
    hipEvent_t a = nullptr, c = nullptr;
    std::vector<hipEvent_t> tiles;   // 2 per chunk (chunk 0 starts at a: tiles[0] unused)
    size_t chunks = 0;
  };
  std::vector<timed_set> tsets;
  size_t timed_calls = 0;      // calls recorded since timing was enabled
  bool timing = false;
};
constexpr size_t kTimedCalls = 4096;

namespace {

void free_scratch(lz4r_ctx *c) {
  (void)hipFree(c->bsizes);
  (void)hipFree(c->boff);
  (void)hipFree(c->tsz);
  (void)hipFree(c->gsum);
  (void)hipFree(c->part);
  (void)hipFree(c->slots);
  c->bsizes = nullptr;
  c->boff = nullptr;
  c->slots = nullptr;
  c->tsz = nullptr;
  c->gsum = nullptr;
  c->part = nullptr;
  c->cap_blocks = 0;
  c->cap_slots = 0;
}

int ensure_scratch(lz4r_ctx *c, size_t nb) {
  const size_t need_slots = std::min(nb, kChunk);
  if (nb <= c->cap_blocks && need_slots <= c->cap_slots) return LZ4R_OK;
  free_scratch(c);
  const size_t cap = nb + nb / 8 + 1024;
  const size_t cap_slots = std::min(cap, kChunk);
  const size_t parts = (cap + kPart - 1) / kPart;
  const size_t groups = (cap + kGT - 1) / kGT;
  // hipMalloc: 256-B aligned; heads and overflow slots are 16-B multiples
  if (hipMalloc(&c->slots, cap_slots * (size_t)kSlot) != hipSuccess ||
      hipMalloc(&c->bsizes, cap * sizeof(uint16_t)) != hipSuccess ||
      hipMalloc(&c->boff, cap * sizeof(uint64_t)) != hipSuccess ||
      hipMalloc(&c->tsz, cap * sizeof(uint32_t)) != hipSuccess ||
      hipMalloc(&c->gsum, groups * sizeof(uint32_t)) != hipSuccess ||
      hipMalloc(&c->part, parts * sizeof(uint64_t)) != hipSuccess) {
    (void)hipGetLastError();
    free_scratch(c);
    return LZ4R_ERR_NOMEM;
  }
  c->cap_blocks = cap;
  c->cap_slots = cap_slots;
  return LZ4R_OK;
}

// A timing event: no system-scope fence when it is recorded (the events only
// time the work; the call's results reach the host by their own copies).  With
// the default fence every record writes back and invalidates the caches: four
// records cost a back-to-back call 13 us (tools/timing_cost.py).
int make_event(hipEvent_t *e) {
  return hipEventCreateWithFlags(e, hipEventDisableSystemFence) == hipSuccess ? LZ4R_OK
                                                                               : LZ4R_ERR_HIP;
}

// the event set of the next timed call (created on first use)
int next_timed_set(lz4r_ctx *c, size_t nchunks, lz4r_ctx::timed_set **out) {
  const size_t i = c->timed_calls % kTimedCalls;
  if (c->tsets.size() <= i) c->tsets.resize(i + 1);
  lz4r_ctx::timed_set &t = c->tsets[i];
  if ((!t.a && make_event(&t.a) != LZ4R_OK) || (!t.c && make_event(&t.c) != LZ4R_OK))
    return LZ4R_ERR_HIP;
  while (t.tiles.size() < 2 * nchunks) {
    hipEvent_t e = nullptr;
    if (make_event(&e) != LZ4R_OK) return LZ4R_ERR_HIP;
    t.tiles.push_back(e);
  }
  t.chunks = nchunks;
  *out = &t;
  return LZ4R_OK;
}

void destroy_events(lz4r_ctx *c) {
  for (auto &t : c->tsets) {
    if (t.a) (void)hipEventDestroy(t.a);
    if (t.c) (void)hipEventDestroy(t.c);
    for (hipEvent_t e : t.tiles) (void)hipEventDestroy(e);
  }
  c->tsets.clear();
}

// milliseconds of timed call set t: the whole call and its lz4_tiles launches
int timed_ms(const lz4r_ctx::timed_set &t, float *ms_call, float *ms_match) {
  if (hipEventSynchronize(t.c) != hipSuccess) return LZ4R_ERR_HIP;
  float a = 0.f, b = 0.f;
  if (hipEventElapsedTime(&a, t.a, t.c) != hipSuccess) return LZ4R_ERR_HIP;
  for (size_t k = 0; k < t.chunks; ++k) {
    float x = 0.f;
    if (hipEventElapsedTime(&x, k == 0 ? t.a : t.tiles[2 * k], t.tiles[2 * k + 1]) != hipSuccess)
      return LZ4R_ERR_HIP;
    b += x;
  }
  *ms_call = a;
  *ms_match = b;
  return LZ4R_OK;
}

// hdr = 1: a framed stream (frame byte first).  hdr = 0: a segment of whole
// blocks for one shard of a multi-GPU job (no frame byte).
int run(lz4r_ctx *c, const void *d_in, size_t n, void *d_out, size_t cap,
        void *d_len, int hdr, void *stream) {
  if (!c || !d_in || !d_out || !d_len) return LZ4R_ERR_ARG;
  if (hdr && n < (size_t)kBlk) return LZ4R_ERR_TOO_SMALL;
  if (n == 0 || n > kMaxInput) return LZ4R_ERR_ARG;
  const size_t nb = (n + kBlk - 1) / kBlk;
  const size_t nchunks = (nb + kChunk - 1) / kChunk;
  int rc = ensure_scratch(c, nb);
  if (rc != LZ4R_OK) return rc;
  static_assert(kPart % kGT == 0, "partials hold whole groups");
  hipStream_t s = static_cast<hipStream_t>(stream);
  const bool timed = c->timing;
  lz4r_ctx::timed_set *ts = nullptr;
  if (timed && (rc = next_timed_set(c, nchunks, &ts)) != LZ4R_OK) return rc;
  // A timed call's events ride on its kernels' own dispatch packets
  // (hipExtLaunchKernelGGL: start / stop timestamps of the dispatch), so
  // timing adds no marker packet between the kernels: call = the first
  // lz4_tiles start .. the last lz4_emit stop.
  auto ev = [&](hipEvent_t e) { return timed ? e : nullptr; };
  const uint8_t *in = static_cast<const uint8_t *>(d_in);
  // the block scratch: cap_slots heads of kHead bytes, then the overflow slots
  uint8_t *const ovfs = c->slots + c->cap_slots * (size_t)kHead;
  for (size_t k = 0; k < nchunks; ++k) {
    const size_t b0 = k * kChunk;                      // first block of the chunk
    const size_t nbc = std::min(kChunk, nb - b0);
    const size_t b1 = b0 + nbc;
    const uint32_t last_n = (uint32_t)(b1 == nb ? n - (nb - 1) * kBlk : kBlk);
    // one block per workgroup: the hardware dispatcher balances the uneven
    // per-block cost (a static grid-stride split leaves a tail; measured
    // slower also with the next block prefetched into registers)
    const uint32_t per = (uint32_t)((nbc + 7) / 8);    // blocks per XCD slice
    hipEvent_t t0 = timed ? (k == 0 ? ts->a : ts->tiles[2 * k]) : nullptr;   // chunk 0 starts the call
    hipEvent_t t1 = timed ? ts->tiles[2 * k + 1] : nullptr;
    // (every chunk starts 300 b0 bytes in: a multiple of 4)
    if (((uintptr_t)in & 3) == 0) {
      hipExtLaunchKernelGGL(lz4_tiles<true>, dim3(8 * per), dim3(64), 0, s, t0, t1, 0u,
                            in + b0 * kBlk, (uint32_t)nbc, per, last_n, c->slots, ovfs,
                            c->tsz + b0, c->bsizes + b0, c->status);
    } else
      hipExtLaunchKernelGGL(lz4_tiles<false>, dim3(8 * per), dim3(64), 0, s, t0, t1, 0u,
                            in + b0 * kBlk, (uint32_t)nbc, per, last_n, c->slots, ovfs,
                            c->tsz + b0, c->bsizes + b0, c->status);
    const size_t p0 = b0 / kPart, np = (nbc + kPart - 1) / kPart;
    hipLaunchKernelGGL(lz4_scan_reduce, dim3((unsigned)np), dim3(256), 0, s, c->tsz, b1, p0,
                       c->gsum, c->part);
    hipLaunchKernelGGL(lz4_scan_partials, dim3(1), dim3(1024), 0, s, c->part + p0, np,
                       (uint64_t)hdr, k == 0 ? 1 : 0, k + 1 == nchunks ? 1 : 0, c->status,
                       static_cast<uint64_t *>(d_len), c->verdict);
    const size_t g0 = b0 / kGT, ng = (nbc + kGT - 1) / kGT;
    hipExtLaunchKernelGGL(lz4_emit, dim3((unsigned)(8 * ((ng * kGSplit + 7) / 8))), dim3(64 * kEW), 0, s, nullptr,
                          k + 1 == nchunks ? ev(ts ? ts->c : nullptr) : nullptr, 0u, in,
                          (const uint8_t *)c->slots, (const uint8_t *)ovfs, b0,
                          (const uint32_t *)c->tsz, b1, g0, (const uint32_t *)c->gsum,
                          (const uint64_t *)c->part, static_cast<uint8_t *>(d_out), (uint64_t)cap,
                          hdr, (uint64_t)nb, (uint32_t)(n - (nb - 1) * kBlk), c->boff);
  }
  if (timed) ++c->timed_calls;
  c->last_nb = nb;
  c->checkable = true;
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess && getenv("LZ4R_DEBUG"))
    fprintf(stderr, "lz4r: %s\n", hipGetErrorString(e));
  return e == hipSuccess ? LZ4R_OK : LZ4R_ERR_HIP;
}

}  // namespace

extern "C" {

#ifdef LZ4R_PROF
int lz4r_prof_read(unsigned long long *host16, int reset) {
  if (hipMemcpyFromSymbol(host16, HIP_SYMBOL(lz4r_prof_acc), 16 * sizeof(unsigned long long)) !=
      hipSuccess)
    return LZ4R_ERR_HIP;
  if (reset) {
    static const unsigned long long zero[16] = {};
    if (hipMemcpyToSymbol(HIP_SYMBOL(lz4r_prof_acc), zero, sizeof(zero)) != hipSuccess)
      return LZ4R_ERR_HIP;
  }
  return LZ4R_OK;
}
#endif

int lz4r_ctx_create(lz4r_ctx **out) {
  if (!out) return LZ4R_ERR_ARG;
  lz4r_ctx *c = new (std::nothrow) lz4r_ctx();
  if (!c) return LZ4R_ERR_NOMEM;
  if (hipGetDevice(&c->device) != hipSuccess ||
      hipMalloc(&c->len, 3 * sizeof(uint64_t)) != hipSuccess ||
      hipMemset(c->len, 0, 3 * sizeof(uint64_t)) != hipSuccess) {
    lz4r_ctx_destroy(c);
    return LZ4R_ERR_HIP;
  }
  c->status = reinterpret_cast<uint32_t *>(c->len + 1);
  c->verdict = c->len + 2;
  *out = c;
  return LZ4R_OK;
}

void lz4r_ctx_destroy(lz4r_ctx *c) {
  if (!c) return;
  free_scratch(c);
  (void)hipFree(c->len);
  destroy_events(c);
  delete c;
}

size_t lz4r_nblocks(size_t n) { return (n + kBlk - 1) / kBlk; }

size_t lz4r_compress_bound(size_t n) { return 1 + lz4r_nblocks(n) * (size_t)LZ4R_BLOCK_BOUND; }

int lz4r_compress_async(lz4r_ctx *c, const void *d_in, size_t n, void *d_out, size_t cap,
                        void *d_len, void *stream) {
  return run(c, d_in, n, d_out, cap, d_len, 1, stream);
}

int lz4r_compress_segment_async(lz4r_ctx *c, const void *d_in, size_t n, void *d_out,
                                size_t cap, void *d_len, int final_shard, void *stream) {
  if (!c || !d_len) return LZ4R_ERR_ARG;
  // a non-final shard must end on the 300-B grid, or the blocks after it
  // (and so the concatenated stream) would differ from the single-GPU one
  if (!final_shard && n % kBlk != 0) return LZ4R_ERR_ARG;
  if (n == 0) {                      // an empty shard (more ranks than blocks)
    c->last_nb = 0;
    c->checkable = false;     // nothing launched: lz4r_check reports OK
    hipStream_t s = static_cast<hipStream_t>(stream);
    if (c->timing) {          // a timed call of no launches
      lz4r_ctx::timed_set *ts = nullptr;
      const int rc = next_timed_set(c, 0, &ts);
      if (rc != LZ4R_OK) return rc;
      (void)hipEventRecord(ts->a, s);
      (void)hipEventRecord(ts->c, s);
      ++c->timed_calls;
    }
    return hipMemsetAsync(d_len, 0, sizeof(uint64_t), s) == hipSuccess ? LZ4R_OK : LZ4R_ERR_HIP;
  }
  return run(c, d_in, n, d_out, cap, d_len, 0, stream);
}

int lz4r_compress_device(lz4r_ctx *c, const void *d_in, size_t n, void *d_out, size_t cap,
                         size_t *out_len, void *stream) {
  if (!c || !out_len) return LZ4R_ERR_ARG;
  int rc = run(c, d_in, n, d_out, cap, c->len, 1, stream);
  if (rc != LZ4R_OK) return rc;
  uint64_t got = 0;                    // the length, with the corrupt flag: one read-back
  hipStream_t s = static_cast<hipStream_t>(stream);
  hipError_t e = hipMemcpyAsync(&got, c->len, sizeof(got), hipMemcpyDeviceToHost, s);
  if (e == hipSuccess) e = hipStreamSynchronize(s);
  if (e != hipSuccess) {
    if (getenv("LZ4R_DEBUG")) fprintf(stderr, "lz4r: %s\n", hipGetErrorString(e));
    return LZ4R_ERR_HIP;
  }
  *out_len = (size_t)(got & ~kLenCorrupt);
  if (got & kLenCorrupt) return LZ4R_ERR_CORRUPT;   // a corrupt bucket head
  return *out_len > cap ? LZ4R_ERR_CAPACITY : LZ4R_OK;
}

int lz4r_block_matches_device(const void *d_in, size_t n, void *d_matches, void *stream) {
  if (!d_in || !d_matches || n == 0 || n > kMaxInput) return LZ4R_ERR_ARG;
  const size_t nb = (n + kBlk - 1) / kBlk;
  const uint8_t *in = static_cast<const uint8_t *>(d_in);
  uint32_t *mo = static_cast<uint32_t *>(d_matches);
  // a grid of 64-lane workgroups stays under HIP's 2^32 work-items: launch
  // chunks of kChunk blocks, as run() does
  for (size_t b0 = 0; b0 < nb; b0 += kChunk) {
    const size_t nbc = std::min(kChunk, nb - b0);
    const uint32_t last_n = (uint32_t)(b0 + nbc == nb ? n - (nb - 1) * kBlk : kBlk);
    hipLaunchKernelGGL(lz4_matches, dim3((unsigned)nbc), dim3(64), 0,
                       static_cast<hipStream_t>(stream), in + b0 * kBlk, (uint32_t)nbc, last_n,
                       mo + b0 * kBlk);
  }
  return hipGetLastError() == hipSuccess ? LZ4R_OK : LZ4R_ERR_HIP;
}

int lz4r_window_matches_device(const void *d_in, size_t n, void *d_matches, void *stream) {
  if (!d_in || !d_matches || n == 0 || n > 0xFFFFFFFFull) return LZ4R_ERR_ARG;
  constexpr size_t kPosChunk = size_t(1) << 26;       // 2^24 workgroups of 256 per launch
  for (size_t p0 = 0; p0 < n; p0 += kPosChunk) {
    const size_t np = std::min(kPosChunk, n - p0);
    hipLaunchKernelGGL(lz4_window_matches, dim3((unsigned)((np + 3) / 4)), dim3(256), 0,
                       static_cast<hipStream_t>(stream), static_cast<const uint8_t *>(d_in),
                       (uint32_t)n, (uint32_t)p0, static_cast<uint32_t *>(d_matches));
  }
  return hipGetLastError() == hipSuccess ? LZ4R_OK : LZ4R_ERR_HIP;
}

int lz4r_copy_block_sizes(const lz4r_ctx *c, void *dst, size_t count, void *stream) {
  if (!c || !dst || count > c->last_nb) return LZ4R_ERR_ARG;
  if (count == 0) return LZ4R_OK;
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (hipMemcpyAsync(dst, c->bsizes, count * sizeof(uint16_t), hipMemcpyDefault, s) !=
          hipSuccess ||
      hipStreamSynchronize(s) != hipSuccess)
    return LZ4R_ERR_HIP;
  return LZ4R_OK;
}

int lz4r_copy_block_offsets(const lz4r_ctx *c, void *dst, size_t count, void *stream) {
  if (!c || !dst || count > c->last_nb) return LZ4R_ERR_ARG;
  if (count == 0) return LZ4R_OK;
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (hipMemcpyAsync(dst, c->boff, count * sizeof(uint64_t), hipMemcpyDefault, s) !=
          hipSuccess ||
      hipStreamSynchronize(s) != hipSuccess)
    return LZ4R_ERR_HIP;
  return LZ4R_OK;
}

int lz4r_block_offsets_device(const lz4r_ctx *c, const void **d_offsets, size_t *count) {
  if (!c || !d_offsets || !count) return LZ4R_ERR_ARG;
  *d_offsets = c->boff;
  *count = c->last_nb;
  return LZ4R_OK;
}

int lz4r_compress(const uint8_t *in, size_t n, uint8_t *out, size_t cap, size_t *out_len) {
  if (!in || !out || !out_len) return LZ4R_ERR_ARG;
  if (n < (size_t)kBlk) return LZ4R_ERR_TOO_SMALL;
  lz4r_ctx *c = nullptr;
  int rc = lz4r_ctx_create(&c);
  if (rc != LZ4R_OK) return rc;
  void *din = nullptr, *dout = nullptr;
  const size_t dcap = lz4r_compress_bound(n);
  if (hipMalloc(&din, n + 16) != hipSuccess || hipMalloc(&dout, dcap) != hipSuccess) {
    (void)hipFree(din);
    lz4r_ctx_destroy(c);
    return LZ4R_ERR_NOMEM;
  }
  if (hipMemcpy(din, in, n, hipMemcpyHostToDevice) != hipSuccess) rc = LZ4R_ERR_HIP;
  size_t got = 0;
  if (rc == LZ4R_OK) rc = lz4r_compress_device(c, din, n, dout, dcap, &got, nullptr);
  if (rc == LZ4R_OK) {
    *out_len = got;
    if (got > cap) rc = LZ4R_ERR_CAPACITY;
    else if (hipMemcpy(out, dout, got, hipMemcpyDeviceToHost) != hipSuccess) rc = LZ4R_ERR_HIP;
  }
  (void)hipFree(din);
  (void)hipFree(dout);
  lz4r_ctx_destroy(c);
  return rc;
}

int lz4r_check(lz4r_ctx *c, void *stream) {
  if (!c) return LZ4R_ERR_ARG;
  if (!c->checkable) return LZ4R_OK;     // no launch yet (or an empty segment)
  uint64_t v = 0;                        // the context's own verdict word
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (hipMemcpyAsync(&v, c->verdict, sizeof(v), hipMemcpyDeviceToHost, s) != hipSuccess ||
      hipStreamSynchronize(s) != hipSuccess)
    return LZ4R_ERR_HIP;
  return v ? LZ4R_ERR_CORRUPT : LZ4R_OK;
}

int lz4r_set_timing(lz4r_ctx *c, int enable) {
  if (!c) return LZ4R_ERR_ARG;
  c->timing = enable != 0;
  if (c->timing) c->timed_calls = 0;
  return LZ4R_OK;
}

int lz4r_last_timing(lz4r_ctx *c, float *ms_call, float *ms_match) {
  if (!c || c->timed_calls == 0) return LZ4R_ERR_ARG;
  float a = 0.f, b = 0.f;
  const int rc = timed_ms(c->tsets[(c->timed_calls - 1) % kTimedCalls], &a, &b);
  if (rc != LZ4R_OK) return rc;
  if (ms_call) *ms_call = a;
  if (ms_match) *ms_match = b;
  return LZ4R_OK;
}

int lz4r_timed_calls(lz4r_ctx *c, size_t max, float *ms_call, float *ms_match, size_t *count) {
  if (!c || !count || (max && (!ms_call || !ms_match))) return LZ4R_ERR_ARG;
  // the newest min(calls, ring, max) calls, oldest first
  const size_t n = std::min(std::min(c->timed_calls, kTimedCalls), max);
  for (size_t j = 0; j < n; ++j) {
    const size_t i = (c->timed_calls - n + j) % kTimedCalls;
    const int rc = timed_ms(c->tsets[i], &ms_call[j], &ms_match[j]);
    if (rc != LZ4R_OK) return rc;
  }
  *count = n;
  return LZ4R_OK;
}

const char *lz4r_strerror(int code) {
  switch (code) {
    case LZ4R_OK: return "ok";
    case LZ4R_ERR_ARG: return "invalid argument";
    case LZ4R_ERR_TOO_SMALL: return "input shorter than one 300-byte block";
    case LZ4R_ERR_CAPACITY: return "output buffer too small";
    case LZ4R_ERR_HIP: return "HIP runtime error";
    case LZ4R_ERR_NOMEM: return "device allocation failed";
    case LZ4R_ERR_CORRUPT: return "corrupt stream";
    default: return "unknown error";
  }
}

}  // extern "C"
