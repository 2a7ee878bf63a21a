// lz4r_gpudec.hip -- block-parallel MI355X decoder of the reference's "LZ4"
// stream (the bytes lz4r_compress / lz4_encode write).
//
// The reference decoder (LZ4_decode / interpret_frame, LZ4.c:937-1121) walks
// the stream serially and mis-parses >= 256 blocks and literal runs >= 271.
// Here every 300-byte block is decoded independently into its fixed output
// slot [300 b, 300 b + 300).  Block boundaries come from the compressor's
// per-block offsets (lz4r_copy_block_offsets): the format itself cannot be
// split in parallel (the u16 size field over-counts the truncated-length
// sequences, LZ4.c:569-575).
//
// Mapping: one LANE per block, 32 consecutive blocks per wave (a wave per
// block would issue every serial parsing step as a full wave instruction).
// The walk is issue-bound (the divergent per-lane loop), so the kernel keeps
// LDS small for occupancy (10.1 KB per wave: 32 output slots of 300 B + 16 B
// of slack; 15 waves/CU) and the loop free of exec-mask bookkeeping:
//   - every block first goes through decode_block_plain: every token read
//     plainly, the header decoded as selects and lane masks, the window's
//     bytes by v_alignbyte of selected dwords, whole 16-B stores only (the
//     slot's slack takes what passes its end); anything unusual (a reading
//     that does not fit, an inconsistent end) returns -1 and the general
//     decode_block below redoes the block;
//   - the lane reads its encoded bytes with single unaligned 8/16-byte
//     global loads (L1/L2 absorb the re-reads of the wave's ~20 KB range),
//     after touching the block's next four 128-B lines up front so that the
//     serial walk does not wait on HBM once per line; a sequence's distance
//     word, up to four literal chunks past the window and the next window
//     are issued together, so the walk waits on memory once per sequence of
//     up to ~77 literals (a load per chunk, each waited for, cost 1.28 ->
//     1.18 ms per GiB: tools/r06_r.sh; two chunks instead of four, 1.068 ->
//     1.015), longer runs take four chunks per round trip, and each load runs
//     only on the lanes that need it: the vector memory address unit is the
//     bound (TA busy ~80 % of the kernel, ~45 cycles per scattered wave load,
//     tools/r06_w.sh), and a lane with exec off costs it nothing (1.17 ->
//     1.06 ms per GiB);
//   - literals move in 16-byte chunks; a match of distance D is copied in
//     chunks of min(16, d) bytes at a distance d that grows from D (the
//     match is D-periodic, so any multiple of D up to the bytes already
//     written + D is a valid distance), with D < 8 seeded by replicating
//     its period over 8 bytes;
//   - the general path's stores within 16 bytes of the 300-B end are
//     exact-size (b64/b32/b16/b8 pieces);
//   - the wave's 32 x 300 = 9600 contiguous output bytes leave as 16-B
//     stores gathered across the slot ends (one v_perm per dword).
// Measured alternatives that lost (1 GiB text, MI355X): one wave per block
// (15.5 ms), nested copy loops with byte stores (3.4 ms), staging the wave's
// input in LDS (halves occupancy: 2x slower), output slots in global memory
// (read-after-write through L2: 2.4x slower), a one-chunk-per-step state
// machine (the header path then runs every step: 2x slower).
// L comes from the exact u16 size field; the one ambiguous token family
// (0xFD..0xFF: L >= 15 with M = 17 / 18 / >= 19, or a truncated match
// M = 1..3 whatever L, LZ4.c:317 + :540-544) is resolved by a per-lane
// stack of choice points (registers): the plain reading is taken first and undone if the
// block does not then end exactly at its last byte with 300 decoded bytes
// (or 1..300 for the last block) and size fields summing to the block
// header's (LZ4.c:617).  A plain reading of such a token decodes >= 32
// bytes, so at most 9 choice points are ever pending; a backtrack rewrites
// the tail.  A sequence's size field equals the bytes it occupies, plus one
// for a truncated reading, so the running sum is (ip - 3) + #truncated.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <map>
#include <mutex>

#include "../../include/lz4r.h"

namespace {

constexpr int kBlk = LZ4R_BLOCK;
constexpr int kInMax = LZ4R_BLOCK_BOUND;   // bytes of one encoded block (bound)
constexpr int kLanes = 64;                 // threads per workgroup (one wave)
// blocks per wave (lanes 0 .. kBPW-1 decode; all 64 lanes store the wave's
// output): 32 x 300 B of LDS lets 16 waves share a CU where 64 blocks per wave
// allowed 8 -- the walk is latency-bound, so more, narrower waves win (1 GiB:
// 64 -> 1.68 ms, 48 -> 1.68, 40 -> 1.68, 32 -> 1.59, 24 -> 1.61, 16 -> 1.95)
constexpr int kBPW = 32;
constexpr int kDepth = 10;                 // choice points per lane (<= 9 needed)
constexpr int kMaxSteps = 1 << 16;         // header budget: a hostile stream cannot spin a lane
constexpr int kPfN = 4;                    // L2 lines touched ahead of the walk
constexpr int kPfS = 128;                  // (2 / 4 / 8 lines, 64 or 128 B apart: same time)

typedef uint64_t u64u __attribute__((aligned(1)));
typedef uint32_t u32u __attribute__((aligned(1)));
typedef uint16_t u16u __attribute__((aligned(1)));

// Slots kSlotS apart: 300 bytes of output and 16 of slack, so a 16-B store
// that starts inside the block never reaches the next lane's slot (no
// exact-size stores at the slot end).
constexpr int kSlotS = kBlk + 16;

struct DecLds {
  alignas(16) uint8_t out[kBPW * kSlotS + 48];  // lane l's block at out[kSlotS l] (+ slack)
  uint4 sel[17];                                 // sel[k]: v_perm selectors, bytes < k from A
  uint32_t qlen[kLanes];                         // decoded bytes per block (0 = failed)
};

struct V16 {
  uint64_t lo, hi;
};

// The lane's encoded block in global memory; `avail` = readable bytes from p.
// kSafe: bounds-checked (only the wave holding the stream's last bytes needs
// it; everywhere else a 16-byte read past a block stays inside the stream).
template <bool kSafe>
struct Bytes {
  const uint8_t *p;
  size_t avail;

  __device__ __forceinline__ uint64_t ld8(int a) const {
    if (!kSafe || (size_t)a + 8 <= avail) return *reinterpret_cast<const u64u *>(p + a);
    uint64_t r = 0;
    for (int t = 0; t < 8; ++t)
      if ((size_t)(a + t) < avail) r |= (uint64_t)p[a + t] << (8 * t);
    return r;
  }
  __device__ __forceinline__ V16 ld16(int a) const {
    if (!kSafe || (size_t)a + 16 <= avail) {
      const u64u *q = reinterpret_cast<const u64u *>(p + a);
      return {q[0], q[1]};
    }
    return {ld8(a), ld8(a + 8)};
  }
};

// The same, unchecked, as a wave-uniform base and the lane's 32-bit offset
// from it: every load is global_load with an SGPR base and a VGPR offset,
// with no 64-bit address arithmetic on the walk's dependency chain (64-bit
// VALU issues at ~5.6 cycles per wave-instruction on gfx950, a 32-bit add at
// ~2.3: tools/valu_rate).
struct BytesW {
  const uint8_t *base;
  uint32_t off;

  __device__ __forceinline__ uint64_t ld8(int a) const {
    return *reinterpret_cast<const u64u *>(base + (off + (uint32_t)a));
  }
  __device__ __forceinline__ V16 ld16(int a) const {
    const uint32_t x = off + (uint32_t)a;
    return {*reinterpret_cast<const u64u *>(base + x), *reinterpret_cast<const u64u *>(base + x + 8u)};
  }
};

// The lane's 300-byte output slot in LDS.  Reads may run past the slot
// (into a neighbour or the slack) and are masked by the caller; writes are
// exact.
struct Slot {
  uint8_t *o;

  __device__ __forceinline__ uint64_t ld8(int a) const {
    return *reinterpret_cast<const u64u *>(o + a);
  }
  __device__ __forceinline__ V16 ld16(int a) const {
    const u64u *q = reinterpret_cast<const u64u *>(o + a);
    return {q[0], q[1]};
  }
  // v at o[a .. a+16) when that stays inside the slot, else exactly n bytes.
  // Bytes past the n meant ones land beyond the lane's write frontier and
  // are overwritten before anything reads them (output is produced in
  // order; a backtrack rewrites from the choice point on).
  __device__ __forceinline__ void st_fast(int a, V16 v, int n) const {
    if (a + 16 <= kBlk) {
      *reinterpret_cast<u64u *>(o + a) = v.lo;
      *reinterpret_cast<u64u *>(o + a + 8) = v.hi;
    } else {
      st(a, v, n);
    }
  }
  // the first n (1..16) bytes of v at o[a]
  __device__ __forceinline__ void st(int a, V16 v, int n) const {
    if (n == 16) {
      *reinterpret_cast<u64u *>(o + a) = v.lo;
      *reinterpret_cast<u64u *>(o + a + 8) = v.hi;
      return;
    }
    uint64_t w = v.lo;
    if (n & 8) {
      *reinterpret_cast<u64u *>(o + a) = w;
      a += 8;
      w = v.hi;
    }
    if (n & 4) {
      *reinterpret_cast<u32u *>(o + a) = (uint32_t)w;
      a += 4;
      w >>= 32;
    }
    if (n & 2) {
      *reinterpret_cast<u16u *>(o + a) = (uint16_t)w;
      a += 2;
      w >>= 16;
    }
    if (n & 1) o[a] = (uint8_t)w;
  }
};

// The output slot of the fast path: every store is a whole 16-B store (the
// slot's 16-B slack takes what passes its 300 bytes).
struct SlotW {
  uint8_t *o;
  __device__ __forceinline__ uint64_t ld8(int a) const {
    return *reinterpret_cast<const u64u *>(o + a);
  }
  __device__ __forceinline__ V16 ld16(int a) const {
    const u64u *q = reinterpret_cast<const u64u *>(o + a);
    return {q[0], q[1]};
  }
  __device__ __forceinline__ void st_fast(int a, V16 v, int) const {
    *reinterpret_cast<u64u *>(o + a) = v.lo;
    *reinterpret_cast<u64u *>(o + a + 8) = v.hi;
  }
};

// the low D (1..7) bytes of w repeated over 8 bytes
__device__ __forceinline__ uint64_t replicate(uint64_t w, int D) {
  uint64_t x = w & ((1ull << (8 * D)) - 1);
  x |= x << (8 * D);
  if (2 * D < 8) x |= x << (16 * D);
  if (4 * D < 8) x |= x << (32 * D);
  return x;
}

// v >> (8 * nbytes), nbytes in 0..15
__device__ __forceinline__ V16 shr_bytes(V16 v, int nbytes) {
  const int s = 8 * nbytes;
  if (s == 0) return v;
  if (s < 64) return {(v.lo >> s) | (v.hi << (64 - s)), v.hi >> s};
  return {v.hi >> (s - 64), 0};
}

__device__ __forceinline__ int litext_len(int L) {
  if (L < 15) return 0;
  return ((L - 15) & 255) == 255 ? 2 : 1;
}

// Truncated reading of the sequence at ip: match length M = alt in 1..3
// (tokens 0xFD..0xFF only); size field S = L + 5 + litext_len(L) + 1
// (LZ4.c:569-575).  e0, e1 = the two bytes after the size field.
template <typename BytesT>
__device__ bool read_truncated(const BytesT &p, int len, int ip, int Sz, int e0, int e1, int pos,
                               int alt, int &L, int &M, int &D, int &lit, int &nip) {
  const int ip0 = ip + 3;
  M = alt;
  for (int le = 0; le <= 2; ++le) {
    L = Sz - 6 - le;
    if (L < 0 || litext_len(L) != le) continue;
    if (le) {
      const int r = (L - 15) & 255;
      const bool ok = r == 255 ? (ip0 + 1 < len && e0 == 255 && e1 == 0) : (ip0 < len && e0 == r);
      if (!ok) continue;
    }
    lit = ip0 + le;
    if (lit + L + 2 > len || pos + L + M > kBlk) continue;
    D = (int)(p.ld8(lit + L) & 0xFFFF);
    if (D == 0 || D > pos + L) continue;
    nip = lit + L + 2;
    return true;
  }
  return false;
}

// choice point: k 8 | ip 11 | pos 9 | #truncated 2 | next reading 2
__device__ __forceinline__ uint32_t pack_choice(int k, int ip, int pos, int ntr, int alt) {
  return (uint32_t)k | ((uint32_t)ip << 8) | ((uint32_t)pos << 19) | ((uint32_t)ntr << 28) |
         ((uint32_t)alt << 30);
}

// literals p[lit, lit+L) -> o[pos, pos+L), 32 bytes per step
template <typename SlotT, typename BytesT>
__device__ __forceinline__ void copy_literals(const SlotT &o, int pos, const BytesT &p, int lit,
                                              int L) {
  for (int i = 0; i < L; i += 32) {
    const V16 a = p.ld16(lit + i), b = p.ld16(lit + i + 16);
    o.st_fast(pos + i, a, L - i < 16 ? L - i : 16);
    if (i + 16 < L) o.st_fast(pos + i + 16, b, L - i - 16 < 16 ? L - i - 16 : 16);
  }
}

// o[q + i] = o[q - D + i] for i < M, in order (D-periodic when D < M)
template <typename SlotT>
__device__ __forceinline__ void copy_match(const SlotT &o, int q, int D, int M) {
  int i = 0, d = D;
  if (D < 8) {                                   // seed: whole periods within 8 bytes
    const uint64_t x = replicate(o.ld8(q - D), D);
    const int per = (int)((0x76586880u >> (4 * D)) & 15u);   // 8 - 8 % D, nibble D
    i = M < per ? M : per;
    o.st_fast(q, {x, x}, i);
    d = i + D;                                   // i is a multiple of D (or M: done)
  }
  // while d < 16 every step copies d bytes, so i stays a multiple of D and the
  // next distance is i + D (no modulo); from d >= 16 on, d no longer changes
  while (i < M) {
    int n = M - i < 16 ? M - i : 16;
    if (n > d) n = d;
    o.st_fast(q + i, o.ld16(q + i - d), n);
    i += n;
    if (d < 16) d = i + D;                       // grow while short
  }
}

// Decode one block into its slot.  Returns the decoded length, or 0 if the
// block is malformed.  Each sequence is decoded from a 16-byte window h of
// the stream at ip; its distance bytes and literals come from the window
// when they lie inside it, and the next sequence's window is requested as
// soon as the next ip is known (it does not depend on the distance: the
// literal-only tail has tm = 0, so no match-extension byte either way), so
// its load overlaps this sequence's copies.
// kFindLen: the block's end is unknown (a bare stream, lz4_bare_walk's exact
// mode): `len` is the bytes readable from the block start (<= kInMax), the
// block ends at the first complete reading (300 bytes, or 1..300 ending at
// `len` when `last`), and the return value is its byte length, not the
// decoded length (0 = no reading).
template <typename BytesT, typename SlotT, bool kFindLen = false>
__device__ __forceinline__ int decode_block(const BytesT &p, int len, bool last, const SlotT &o) {
  uint32_t stk[kDepth];                              // choice points (registers; rare)
  const uint64_t h0 = p.ld8(0);
  const int nseq = (int)(h0 & 255);                  // nseq & 0xFF; <= 76 in practice
  const int want = (int)((h0 >> 8) & 0xFFFF) - 3;    // LZ4.c:617
  if (len < 3 || nseq == 0 || want < 0) return 0;
  int k = 0, ip = 3, pos = 0, ntr = 0, nch = 0, alt = 0, steps = 0;
  V16 h = p.ld16(3);
  for (;;) {
    bool ok = false;
    int L = 0, M = 0, D = 0, lit = 0, nip = 0;
    V16 hn = {0, 0};
    if (++steps > kMaxSteps) return 0;
    if (k == nseq) {
      if constexpr (kFindLen) {
        if (ip - 3 + ntr == want && (pos == kBlk || (last && ip == len && pos >= 1))) return ip;
      } else {
        if (ip == len && ip - 3 + ntr == want && (pos == kBlk || (last && pos >= 1))) return pos;
      }
    } else if (ip + 3 <= len) {
      const int tok = (int)(h.lo & 255), Sz = (int)((h.lo >> 8) & 0xFFFF);
      const int e0 = (int)((h.lo >> 24) & 255), e1 = (int)((h.lo >> 32) & 255);
      const bool fits = ip - 3 + ntr + Sz <= want;
      if (alt == 0) {
        // plain reading, branch-free: token nibbles as written (M == 0 or M >= 4)
        const int tl = tok >> 4, tm = tok & 15;
        const int mx = tm == 15 ? 1 : 0;
        const bool big = tl == 15;
        const int le = big ? (e0 == 255 ? 2 : 1) : 0;
        L = big ? Sz - 5 - le - mx : tl;
        const int r = (L - 15) & 255;
        bool okp = big ? (L >= 15 && (e0 == 255 ? (r == 255 && e1 == 0) : r == e0))
                       : Sz == L + 5 + mx;
        lit = ip + 3 + le;
        okp = okp && fits && lit + L + 2 <= len && pos + L <= kBlk;
        nip = lit + L + 2 + mx;
        hn = p.ld16(okp ? nip : ip);                 // next window, in flight during the copies
        const int off = lit + L - ip;                // distance bytes within the window?
        const uint32_t t = off + 3 <= 16 ? (uint32_t)shr_bytes(h, off).lo
                                         : (uint32_t)p.ld8(okp ? lit + L : 0);
        D = (int)(t & 0xFFFF);
        const bool hasm = D != 0;
        M = hasm ? (mx ? 19 + (int)((t >> 16) & 255) : tm + 4) : 0;
        okp = okp && (hasm ? (nip <= len && D <= pos + L && pos + L + M <= kBlk)
                           : (k + 1 == nseq && tm == 0));   // literal-only tail, LZ4.c:585-613
        ok = okp;
        if (tok >= 0xFD) {
          if (okp) {                                 // the truncated reading remains
            if (nch == kDepth) return 0;
            stk[nch++] = pack_choice(k, ip, pos, ntr, tok - 0xFC);
          } else {
            alt = tok - 0xFC;
          }
        }
      }
      if (alt != 0) {                                // truncated reading (rare)
        ok = fits && ntr < 3 &&
             read_truncated(p, len, ip, Sz, e0, e1, pos, alt, L, M, D, lit, nip);
        ntr += ok ? 1 : 0;
        if (ok) hn = p.ld16(nip);
      }
    }
    if (ok) {
      if (lit + L <= ip + 16) {                      // literals inside the window
        if (L) o.st_fast(pos, shr_bytes(h, lit - ip), L);
      } else {
        copy_literals(o, pos, p, lit, L);
      }
      if (M) copy_match(o, pos + L, D, M);
      ++k;
      ip = nip;
      h = hn;
      pos += L + M;
      alt = 0;
      continue;
    }
    // dead end: resume the most recent choice point with its other reading
    if (nch == 0) return 0;
    const uint32_t c = stk[--nch];
    k = (int)(c & 255); ip = (int)((c >> 8) & 2047); pos = (int)((c >> 19) & 511);
    ntr = (int)((c >> 28) & 3); alt = (int)(c >> 30);
    h = p.ld16(ip);
  }
}

// The common case of decode_block, for the hot path: every token read
// plainly (no choice points, no truncated readings), one loop iteration per
// sequence with no data-dependent branch but the copies' own loops, so the
// wave issues little exec-mask bookkeeping.  Returns the decoded length, or -1
// when anything is unusual -- a reading that does not fit, or a block that
// does not end consistently -- and decode_block then redoes the block: it
// takes the same plain readings first and backtracks only where they fail,
// so when this path succeeds the general one would return the same bytes.
template <typename BytesT, typename SlotT>
__device__ __forceinline__ int decode_block_plain(const BytesT &p, int len, bool last,
                                                  const SlotT &o) {
  const uint64_t h0 = p.ld8(0);
  const int nseq = (int)(h0 & 255);
  const int want = (int)((h0 >> 8) & 0xFFFF) - 3;    // LZ4.c:617
  if (len < 3 || nseq == 0 || want < 0) return -1;
  int k = 0, ip = 3, pos = 0;
  V16 h = p.ld16(3);
  bool bad = false;
  while (k < nseq) {
    // the window as dwords; bytes [o, o + 4) of it by one v_alignbyte of two
    // selected dwords (no 64-bit shifts, no branches)
    const uint32_t w0 = (uint32_t)h.lo, w1 = (uint32_t)(h.lo >> 32);
    const uint32_t w2 = (uint32_t)h.hi, w3 = (uint32_t)(h.hi >> 32);
    const int tok = (int)(w0 & 255), Sz = (int)((w0 >> 8) & 0xFFFF);
    const int e0 = (int)(w0 >> 24), e1 = (int)(w1 & 255);
    const int tl = tok >> 4, tm = tok & 15;
    const int mx = tm == 15 ? 1 : 0;
    const bool big = tl == 15;
    // the plain reading as selects and lane masks, not branches
    const bool ff = e0 == 255;
    const int le = (big ? 1 : 0) + ((big & ff) ? 1 : 0);
    const int Lb = Sz - 5 - le - mx;
    const int L = big ? Lb : tl;
    const int r = (L - 15) & 255;
    const bool okb = (L >= 15) & ((ff & (r == 255) & (e1 == 0)) | (!ff & (r == e0)));
    const bool oks = Sz == L + 5 + mx;
    bool okp = (big & okb) | (!big & oks);
    const int lit = ip + 3 + le;
    // (bitwise & and |: every test is evaluated, no short-circuit branches;
    // the size-field sum is checked once, after the walk: ip - 3 == want;
    // lit + L + 2 <= len keeps this sequence's reads inside the stream)
    okp = okp & (ip + 3 <= len) & (lit + L + 2 <= len) & (pos + L <= kBlk);
    const int nip = lit + L + 2 + mx;
    // the distance word and up to four literal chunks past the window, loaded
    // together: one wait where a long literal run waited for the distance
    // word, then for each chunk (all inside the stream: the plain path runs
    // only with kInMax + 64 bytes after the block); the next window last, so
    // that waiting for these (vmcnt counts in issue order) does not wait for it
    const int wl = min(L, ip + 16 - lit);
    const int off = lit + L - ip;                    // distance bytes within the window?
    // each load only on the lanes that need it: the vector memory address
    // unit is the decoder's bound (TA busy ~80 % of the kernel, ~45 cycles
    // per scattered wave load), and a lane with exec off costs it nothing
    uint32_t tw = 0;
    V16 c1 = {0, 0}, c2 = {0, 0}, c3 = {0, 0}, c4 = {0, 0};
    if (okp & (off + 3 > 16)) tw = (uint32_t)p.ld8(lit + L);
    if (okp & (L > wl)) c1 = p.ld16(lit + wl);
    if (okp & (L > wl + 16)) c2 = p.ld16(lit + wl + 16);
    if (okp & (L > wl + 32)) c3 = p.ld16(lit + wl + 32);
    if (okp & (L > wl + 48)) c4 = p.ld16(lit + wl + 48);
    const V16 hn = p.ld16(okp ? nip : ip);           // next window, in flight during the copies
    uint32_t t;
    {
      const int wi = off >> 2;
      const uint32_t a = wi == 0 ? w0 : wi == 1 ? w1 : wi == 2 ? w2 : w3;
      const uint32_t c = wi == 0 ? w1 : wi == 1 ? w2 : w3;
      t = __builtin_amdgcn_alignbyte(c, a, (uint32_t)off & 3u);
    }
    if (off + 3 > 16) t = tw;
    const int D = (int)(t & 0xFFFF);
    const bool hasm = D != 0;
    const int Mx = 19 + (int)((t >> 16) & 255), Ms = tm + 4;
    const int M = hasm ? (mx ? Mx : Ms) : 0;
    const bool mok = (nip <= len) & (D <= pos + L) & (pos + L + M <= kBlk);
    const bool tailok = (k + 1 == nseq) & (tm == 0);   // literal-only tail, LZ4.c:585-613
    okp = okp & ((hasm & mok) | (!hasm & tailok));
    if (!okp) {
      // a use of the chunks and the next window on this path too, so that
      // their loads are not sunk below this test (issued apart, they would be
      // waited for apart)
      asm volatile("" ::"v"(c1.lo), "v"(c1.hi), "v"(c2.lo), "v"(c2.hi), "v"(c3.lo), "v"(c3.hi),
                   "v"(c4.lo), "v"(c4.hi), "v"(hn.lo), "v"(hn.hi));
      bad = true;
      break;
    }
    // literals: the window's bytes, the two chunks, then 16 at a time.  The
    // first two stores are unconditional: they stay inside the slot and its
    // slack (pos + wl <= pos + L <= 300), and what they write past the run is
    // overwritten by the match or the next sequence before anything reads it
    {
      // the window from byte d = lit - ip (3, 4 or 5): dwords from w[d >> 2]
      const bool d4 = le > 0;                         // d = 3 + le
      const uint32_t sh = (uint32_t)(3 + le) & 3u;
      const uint32_t s0 = d4 ? w1 : w0, s1 = d4 ? w2 : w1, s2 = d4 ? w3 : w2, s3 = d4 ? 0u : w3;
      const uint32_t o0 = __builtin_amdgcn_alignbyte(s1, s0, sh);
      const uint32_t o1 = __builtin_amdgcn_alignbyte(s2, s1, sh);
      const uint32_t o2 = __builtin_amdgcn_alignbyte(s3, s2, sh);
      const uint32_t o3 = __builtin_amdgcn_alignbyte(0u, s3, sh);
      o.st_fast(pos, {(uint64_t)o1 << 32 | o0, (uint64_t)o3 << 32 | o2}, wl);
    }
    o.st_fast(pos + wl, c1, min(16, L - wl));
    if (L > wl + 16) o.st_fast(pos + wl + 16, c2, min(16, L - wl - 16));
    if (L > wl + 32) o.st_fast(pos + wl + 32, c3, min(16, L - wl - 32));
    if (L > wl + 48) o.st_fast(pos + wl + 48, c4, min(16, L - wl - 48));
    // longer runs: four chunks per memory round trip (loaded on the lanes
    // that need each, then stored), not one
    for (int i = wl + 64; i < L; i += 64) {
      V16 v[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        v[j] = {0, 0};
        if (i + 16 * j < L) v[j] = p.ld16(lit + i + 16 * j);
      }
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if (i + 16 * j < L) o.st_fast(pos + i + 16 * j, v[j], min(16, L - i - 16 * j));
    }
    // match: one 16-B piece, unconditionally (with no match it writes inside
    // the slot's slack what the next sequence overwrites), then the general
    // copy when the match overlaps itself or exceeds 16 bytes
    const int q = pos + L;
    o.st_fast(q, o.ld16(q - D), M);
    if ((M > 16) | ((M > 0) & (D < 16))) copy_match(o, q, D, M);
    ++k;
    ip = nip;
    h = hn;
    pos += L + M;
  }
  if (bad || ip != len || ip - 3 != want || !(pos == kBlk || (last && pos >= 1))) return -1;
  return pos;
}

// nb_dev (bare streams): the block count is read on the device, the grid is
// sized for an upper bound, and nothing is decoded unless *gate is 0
__global__ __launch_bounds__(kLanes) void lz4_decode_blocks(
    const uint8_t *__restrict__ in, size_t in_len, const uint64_t *__restrict__ boff,
    size_t nb, uint8_t *__restrict__ out, size_t out_cap,
    unsigned long long *__restrict__ result, const unsigned long long *__restrict__ nb_dev,
    const unsigned long long *__restrict__ gate) {
  __shared__ DecLds S;
  const int lane = threadIdx.x;
  const size_t b0 = (size_t)blockIdx.x * kBPW;
  if (nb_dev) {
    if (*gate != 0) return;
    nb = (size_t)*nb_dev;
  }
  if (b0 >= nb) return;
  const int nl = (int)(nb - b0 < (size_t)kBPW ? nb - b0 : kBPW);       // blocks here
  const size_t b = b0 + lane;

  int q = 0;                                         // decoded bytes (0 = failed / absent)
  uint32_t pfv[kPfN] = {};
  // the wave's base: its first block's first byte (a uniform load)
  const size_t wbeg = 1 + boff[b0];
  const uint8_t *const wbase = in + wbeg;
  if (lane < nl) {
    const bool last = b == nb - 1;
    const size_t beg = 1 + boff[b];
    const size_t end = last ? in_len : 1 + boff[b + 1];
    if (end >= beg + 3 && end <= in_len && end - beg <= (size_t)kInMax) {
      const Slot o{S.out + lane * kSlotS};
      // touch the block's next four 128-B lines now: the walk's header loads
      // then hit L2 instead of waiting on HBM one line at a time (the values
      // are folded into pfx after the walk; 1.82 -> 1.66 ms per GiB)
      {
        const uint8_t *q0 = in + ((beg + kPfS) & ~(size_t)(kPfS - 1));
        const uint8_t *qe = in + end;
#pragma unroll
        for (int t = 0; t < kPfN; ++t) {
          const uint8_t *q = q0 + kPfS * t;
          pfv[t] = *(q < qe ? q : q0 - kPfS);          // one byte: never past the stream
        }
      }
      // a lane's reads reach at most 32 bytes past its block (<= kInMax bytes):
      // unchecked loads only when that stays inside the stream, decided per
      // lane from its own offsets (caller-supplied offsets need not be
      // monotone; only the stream's last few blocks take the checked path)
      // (compressor offsets are monotone: the wave's blocks lie within
      // 32 x kInMax bytes of its base; other offsets take the checked path)
      if (beg + (size_t)kInMax + 64 <= in_len && beg >= wbeg && beg - wbeg < (1u << 30)) {
        const BytesW bw{wbase, (uint32_t)(beg - wbeg)};
        q = decode_block_plain(bw, (int)(end - beg), last, SlotW{S.out + lane * kSlotS});
        if (q < 0) q = decode_block(bw, (int)(end - beg), last, o);
      } else {
        q = decode_block(Bytes<true>{in + beg, in_len - beg}, (int)(end - beg), last, o);
      }
    }
    if (q == 0) atomicMin(&result[1], (unsigned long long)b + 1);
    else if (last) result[0] = (unsigned long long)(b * kBlk + q);
  }
  // keeps the prefetch loads alive; never true for a decoded block (q <= 300)
  uint32_t pfx = 0;
#pragma unroll
  for (int t = 0; t < kPfN; ++t) pfx ^= pfv[t];
  if (pfx == 0x5A5A5A5Au && q == 1000) q = 0;
  S.qlen[lane] = (uint32_t)q;
  if (lane < 17) {                                   // sel[k]: dword j, byte m from A iff 4 j + m < k
    uint32_t w[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      uint32_t x = 0;
#pragma unroll
      for (int m = 0; m < 4; ++m) x |= (uint32_t)(4 * j + m < lane ? m : 4 + m) << (8 * m);
      w[j] = x;
    }
    S.sel[lane] = make_uint4(w[0], w[1], w[2], w[3]);
  }
  __syncthreads();

  // ---- store the wave's contiguous output -----------------------------------
  // every block but the last decodes to exactly 300 bytes, so the valid range
  // is [300 b0, 300 b0 + sum q); a failed block leaves garbage (error raised).
  // Output byte x is slot l = x / 300, byte x - 300 l; a 16-B chunk that
  // crosses a slot end takes its first k bytes from slot l (A) and the rest
  // from slot l + 1, 16 B further on (B): one v_perm per dword.
  size_t total = 0;
  for (int l = 0; l < nl; ++l) total += l + 1 < nl ? kBlk : S.qlen[l];
  const size_t o0 = b0 * (size_t)kBlk;
  if (o0 >= out_cap) return;
  if (o0 + total > out_cap) total = out_cap - o0;
  auto src_of = [](uint32_t x) {                     // LDS offset of output byte x (< 2^15)
    const uint32_t l = (x * 27963u) >> 23;           // x / 300
    return x + 16u * l;
  };
  if (((reinterpret_cast<uintptr_t>(out) + o0) & 15) == 0) {
    const int nv = (int)(total >> 4);
    uint4 *dst = reinterpret_cast<uint4 *>(out + o0);
    typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
    for (int v = lane; v < nv; v += kLanes) {
      const uint32_t x = 16u * (uint32_t)v;
      const uint32_t l = (x * 27963u) >> 23;
      const uint32_t off = x - 300u * l;
      const uint32_t k = min(300u - off, 16u);
      const uint8_t *a = S.out + x + 16u * l;
      const uint4 A = *reinterpret_cast<const uint4 *>(a);
      const uint4 B = *reinterpret_cast<const uint4 *>(a + 16);
      const uint4 sl = S.sel[k];
      const u32x4 m = {__builtin_amdgcn_perm(B.x, A.x, sl.x), __builtin_amdgcn_perm(B.y, A.y, sl.y),
                       __builtin_amdgcn_perm(B.z, A.z, sl.z), __builtin_amdgcn_perm(B.w, A.w, sl.w)};
      // written once: non-temporal 16-B stores (-1.3 %, tools/ab_dec_inproc.py)
      __builtin_nontemporal_store(m, reinterpret_cast<u32x4 *>(dst) + v);
    }
    for (size_t i = (size_t)nv * 16 + lane; i < total; i += kLanes)
      out[o0 + i] = S.out[src_of((uint32_t)i)];
  } else {
    for (size_t i = lane; i < total; i += kLanes) out[o0 + i] = S.out[src_of((uint32_t)i)];
  }
}

// ---- bare streams: block boundaries found on the device ---------------------
// LZ4_decode (LZ4.c:1038) takes only the file.  The stream is cut into
// chunks of kChunkB bytes; in each chunk the first position that parses as
// a block header is a candidate start (lz4_bare_cand), a lane per chunk
// walks the blocks from its candidate to the next chunk (lz4_bare_walk),
// and one wave checks that every chunk's walk ends on the next chunk's
// candidate, re-walking a chunk from its predecessor's exit where it does
// not (lz4_bare_fix).  By induction from position 1 the candidates are then
// on the stream's own block chain.  A block's length is its u16 size field
// (fast mode) unless it holds truncated matches (M = 1..3, LZ4.c:317), whose
// size fields count a byte that is never written (LZ4.c:569-575): the exact
// mode parses every block (decode_block<kFindLen>).  The host tries the
// fast mode first; the decoder checks every block against its boundaries,
// so a wrong fast-mode boundary is an error, never wrong bytes.
constexpr int kChunkB = 8192;                        // stream bytes per chunk
constexpr int kWin = 2 * kInMax + 32;                // candidate window (LDS)
constexpr uint64_t kNone = ~0ull;                    // no candidate in the chunk
constexpr uint64_t kBad = ~0ull - 1;                 // the walk met an impossible block

// a slot that stores nothing and reads zeros: decode_block as a parser
struct NullSlot {
  __device__ __forceinline__ uint64_t ld8(int) const { return 0; }
  __device__ __forceinline__ V16 ld16(int) const { return {0, 0}; }
  __device__ __forceinline__ void st_fast(int, V16, int) const {}
  __device__ __forceinline__ void st(int, V16, int) const {}
};

__device__ __forceinline__ int rd_u16(const uint8_t *w, int a) {
  return (int)w[a] | ((int)w[a + 1] << 8);
}

// Candidate start of every chunk: a wave per chunk, its window
// [s, s + kWin) of the stream in LDS.  x passes when its header is
// plausible (1 <= nseq, 3 + 5 nseq <= size <= kInMax, inside the stream) and
// the nseq sequence size fields, hopped as written, end exactly at x + size
// (a true block without truncated matches always does), and the next header
// is plausible too (or x + size is the stream end).
__global__ __launch_bounds__(256) void lz4_bare_cand(const uint8_t *__restrict__ in,
                                                      size_t in_len, size_t nchunks,
                                                      uint64_t *__restrict__ cand) {
  constexpr int kWin16 = (kWin + 16 + 15) / 16;       // 16-B pieces of the window
  __shared__ alignas(16) uint8_t win[4][kWin16 * 16];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const size_t c = (size_t)blockIdx.x * 4 + wv;
  if (c >= nchunks) return;
  if (c == 0) {                                      // the first block starts after the frame byte
    if (lane == 0) cand[0] = 1;
    return;
  }
  const size_t s = 1 + c * (size_t)kChunkB;
  // the window [s, s + kWin) as aligned 16-B loads from s & ~15 (pieces
  // past the stream end bytewise, zero-filled)
  const size_t a0 = s & ~(size_t)15;
  uint8_t *const w = win[wv] + (s - a0);            // w[i] = in[s + i]
  for (int k = lane; k < kWin16; k += 64) {
    const size_t at = a0 + 16 * (size_t)k;
    uint4 v = make_uint4(0, 0, 0, 0);
    if (at + 16 <= in_len) {
      v = *reinterpret_cast<const uint4 *>(in + at);
    } else {
      uint32_t t[4] = {0, 0, 0, 0};
      for (int b = 0; b < 16; ++b)
        if (at + b < in_len) t[b >> 2] |= (uint32_t)in[at + b] << (8 * (b & 3));
      v = make_uint4(t[0], t[1], t[2], t[3]);
    }
    reinterpret_cast<uint4 *>(win[wv])[k] = v;
  }
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  const int avail = (int)min((size_t)kWin, in_len - s);   // window bytes inside the stream
  uint64_t found = kNone;
  for (int x0 = 0; x0 < kInMax && x0 < avail; x0 += 64) {
    const int x = x0 + lane;
    bool ok = x + 3 <= avail;
    int nseq = 0, size = 0;
    if (ok) {
      nseq = w[x];
      size = rd_u16(w, x + 1);
      ok = nseq >= 1 && size >= 3 + 5 * nseq && size <= kInMax && x + size <= avail;
    }
    if (ok) {
      int y = x + 3;
      for (int k = 0; k < nseq && ok; ++k) {
        const int S = y + 3 <= x + size ? rd_u16(w, y + 1) : 0;
        ok = S >= 5;
        y += S;
        ok = ok && y <= x + size;
      }
      ok = ok && y == x + size;
      if (ok && s + (size_t)(x + size) < in_len) {   // the next header
        const int z = x + size;
        ok = z + 3 <= avail && w[z] >= 1 && rd_u16(w, z + 1) >= 8 && rd_u16(w, z + 1) <= kInMax;
      }
    }
    const uint64_t m = __builtin_amdgcn_ballot_w64(ok);
    if (m) {
      found = s + (size_t)(x0 + __builtin_ctzll(m));
      break;
    }
  }
  if (lane == 0) cand[c] = found;
}

// the byte length of the block at x (0: no block can start there)
template <bool kExact>
__device__ __forceinline__ int bare_block_len(const uint8_t *in, size_t in_len, size_t x) {
  if (x + 3 > in_len) return 0;
  if (!kExact) {
    // the header as one unaligned dword load (three byte loads were three
    // scattered wave loads for the vector memory address unit)
    const uint32_t h = x + 4 <= in_len ? *reinterpret_cast<const u32u *>(in + x)
                                       : (uint32_t)in[x] | (uint32_t)in[x + 1] << 8 | (uint32_t)in[x + 2] << 16;
    const int size = (int)((h >> 8) & 0xFFFF);
    return (h & 255) >= 1 && size >= 8 && size <= kInMax && x + size <= in_len ? size : 0;
  }
  const size_t rem = in_len - x;
  const int len = rem < (size_t)kInMax ? (int)rem : kInMax;
  return decode_block<Bytes<true>, NullSlot, true>(Bytes<true>{in + x, rem}, len,
                                                   rem <= (size_t)kInMax, NullSlot{});
}

// the blocks of chunk c from x: count and exit (the first position at or
// past the next chunk), or kBad; kWrite: their offsets to boff[base ...]
// lst (walk only): the first kList block starts, relative to the chunk start
constexpr int kList = 32;
template <bool kExact, bool kWrite>
__device__ __forceinline__ uint64_t bare_walk_chunk(const uint8_t *in, size_t in_len, size_t c,
                                                    uint64_t x, uint32_t &cnt,
                                                    uint64_t *boff, uint64_t base,
                                                    uint64_t boff_cap = 0,
                                                    uint16_t *lst = nullptr) {
  cnt = 0;
  if (x == kNone || x == kBad) return kBad;
  const uint64_t c0 = 1 + c * (uint64_t)kChunkB;
  const uint64_t lim = c0 + kChunkB;
  while (x < lim && x < in_len) {
    const int L = bare_block_len<kExact>(in, in_len, x);
    if (L == 0) return kBad;
    if (kWrite && base + cnt < boff_cap) boff[base + cnt] = x - 1;
    if (!kWrite && lst && cnt < (uint32_t)kList) lst[cnt] = (uint16_t)(x - c0);
    ++cnt;
    x += (uint64_t)L;
  }
  return x;
}

// a lane per chunk: count and exit from the candidate, and per wave of 64
// chunks the block count (gsum)
template <bool kExact>
__global__ __launch_bounds__(64) void lz4_bare_walk(const uint8_t *__restrict__ in, size_t in_len,
                                                    size_t nchunks,
                                                    const uint64_t *__restrict__ cand,
                                                    uint32_t *__restrict__ cnt,
                                                    uint64_t *__restrict__ exitp,
                                                    unsigned long long *__restrict__ gsum,
                                                    uint16_t *__restrict__ lists,
                                                    uint32_t *__restrict__ lok) {
  // the lanes' lists are staged in LDS (a global store per block would make
  // every next header load wait for it: in-order vmcnt) and leave as one
  // coalesced 4 KB copy per wave
  __shared__ alignas(16) uint16_t ls[64 * kList];
  const size_t c = (size_t)blockIdx.x * 64 + threadIdx.x;
  uint32_t n = 0;
  if (c < nchunks) {
    exitp[c] = bare_walk_chunk<kExact, false>(in, in_len, c, cand[c], n, nullptr, 0, 0,
                                              ls + threadIdx.x * kList);
    cnt[c] = n;
    lok[c] = n <= (uint32_t)kList ? 1u : 0u;   // the list holds every block start
  }
  __syncthreads();
  {
    const size_t c0 = (size_t)blockIdx.x * 64;
    const int nl = (int)min((size_t)64, nchunks - c0);
    uint4 *dst = reinterpret_cast<uint4 *>(lists + c0 * kList);
    const uint4 *src = reinterpret_cast<const uint4 *>(ls);
    for (int i = threadIdx.x; i < nl * kList / 8; i += 64) dst[i] = src[i];
  }
  unsigned long long t = n;
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) t += __shfl_xor(t, d, 64);
  if (threadIdx.x == 0) gsum[blockIdx.x] = t;
}

// A lane per chunk: chunk c is consistent when its exit is the next chunk's
// candidate (the last chunk's: the stream end).  The inconsistent ones go to
// an unordered list (count in *nmis; the list holds at most kMisCap).
constexpr int kMisCap = 1024;
__global__ __launch_bounds__(256) void lz4_bare_check(size_t in_len, size_t nchunks,
                                                      const uint64_t *__restrict__ cand,
                                                      const uint64_t *__restrict__ exitp,
                                                      unsigned int *__restrict__ nmis,
                                                      unsigned int *__restrict__ mis) {
  const size_t c = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (c >= nchunks) return;
  const uint64_t e = exitp[c];
  const bool bad = e == kBad || (c + 1 < nchunks ? e != cand[c + 1] : e != (uint64_t)in_len);
  if (bad) {
    const unsigned int k = atomicAdd(nmis, 1u);
    if (k < (unsigned)kMisCap) mis[k] = (unsigned int)c;
  }
}

// One wave, in stream order over the listed chunks: a chunk whose exit is
// not the next chunk's candidate has the next chunk re-walked from that exit
// (the stream's own chain, by induction from position 1), which is then
// checked in turn; the others keep what lz4_bare_walk found.  More than
// kMisCap inconsistent chunks: every chunk is checked in order.
// status[0] = 0 when the chain is consistent, else 1 + the chunk where it broke.
template <bool kExact>
__global__ __launch_bounds__(64) void lz4_bare_fix(const uint8_t *__restrict__ in, size_t in_len,
                                                   size_t nchunks, uint64_t *__restrict__ cand,
                                                   uint32_t *__restrict__ cnt,
                                                   uint64_t *__restrict__ exitp,
                                                   unsigned long long *__restrict__ gsum,
                                                   const unsigned int *__restrict__ nmis_p,
                                                   const unsigned int *__restrict__ mis,
                                                   unsigned long long *__restrict__ status,
                                                   uint32_t *__restrict__ lok) {
  __shared__ unsigned int list[kMisCap];
  const int lane = threadIdx.x;
  const unsigned int nmis = *nmis_p;
  const bool all = nmis > (unsigned)kMisCap;         // too many: check every chunk
  const int nl = all ? 0 : (int)nmis;
  for (int i = lane; i < nl; i += 64) list[i] = mis[i];
  __syncthreads();
  size_t ov_c = ~(size_t)0;                          // chunk re-walked last, and its exit
  uint64_t ov_exit = 0;                              // (a later load may not see the store)
  size_t pos = 0;                                    // chunks below pos are consistent
  size_t force = ~(size_t)0;                         // a re-walked chunk, checked next
  unsigned long long st = 0;
  for (;;) {
    size_t f;
    if (force != ~(size_t)0) {
      f = force;
    } else if (all) {
      f = pos;                                       // (slow path: every chunk in order)
    } else {
      size_t m = ~(size_t)0;                         // smallest listed chunk >= pos
      for (int i = lane; i < nl; i += 64)
        if (list[i] >= pos && list[i] < m) m = list[i];
#pragma unroll
      for (int d = 32; d >= 1; d >>= 1) {
        const size_t o = __shfl_xor(m, d, 64);
        m = o < m ? o : m;
      }
      f = m;
    }
    if (f >= nchunks) break;
    force = ~(size_t)0;
    const uint64_t e = f == ov_c ? ov_exit : exitp[f];
    const bool bad =
        e == kBad || (f + 1 < nchunks ? e != cand[f + 1] : e != (uint64_t)in_len);
    if (!bad) {
      pos = f + 1;
      continue;
    }
    if (f + 1 >= nchunks || e == kBad) {             // no way on: a corrupt stream
      st = 1 + f;
      break;
    }
    // chunk f + 1 starts where chunk f's walk left off
    uint32_t n = 0;
    uint64_t ex = 0;
    if (lane == 0) ex = bare_walk_chunk<kExact, false>(in, in_len, f + 1, e, n, nullptr, 0);
    ex = __shfl(ex, 0, 64);
    n = (uint32_t)__shfl((int)n, 0, 64);
    if (lane == 0) {
      const uint32_t old = cnt[f + 1];
      cand[f + 1] = e;
      cnt[f + 1] = n;
      exitp[f + 1] = ex;
      lok[f + 1] = 0u;                               // its list is stale: re-walked for offsets
      atomicAdd(&gsum[(f + 1) / 64], (unsigned long long)n - (unsigned long long)old);
    }
    ov_c = f + 1;
    ov_exit = ex;
    pos = f + 1;
    force = f + 1;
  }
  if (lane == 0) status[0] = st;
}

// exclusive scan of the per-wave block counts (one workgroup) -> gbase; the
// total block count -> *nb
__global__ __launch_bounds__(1024) void lz4_bare_scan(const unsigned long long *__restrict__ gsum,
                                                      size_t ng,
                                                      unsigned long long *__restrict__ gbase,
                                                      unsigned long long *__restrict__ nb) {
  __shared__ unsigned long long ws[16];
  __shared__ unsigned long long carry;
  if (threadIdx.x == 0) carry = 0;
  __syncthreads();
  for (size_t c0 = 0; c0 < ng; c0 += 1024) {
    const size_t i = c0 + threadIdx.x;
    const unsigned long long v = i < ng ? gsum[i] : 0;
    unsigned long long x = v;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const unsigned long long o = __shfl_up(x, d, 64);
      if ((threadIdx.x & 63) >= d) x += o;
    }
    if ((threadIdx.x & 63) == 63) ws[threadIdx.x >> 6] = x;
    __syncthreads();
    unsigned long long pre = carry;
    for (int w = 0; w < (int)(threadIdx.x >> 6); ++w) pre += ws[w];
    if (i < ng) gbase[i] = pre + x - v;
    __syncthreads();
    if (threadIdx.x == 1023) carry = pre + x;
    __syncthreads();
  }
  if (threadIdx.x == 0) *nb = carry;
}

// a lane per chunk: its blocks' offsets (relative to the first block byte)
template <bool kExact>
__global__ __launch_bounds__(64) void lz4_bare_offsets(const uint8_t *__restrict__ in,
                                                       size_t in_len, size_t nchunks,
                                                       const uint64_t *__restrict__ cand,
                                                       const uint32_t *__restrict__ cnt,
                                                       const unsigned long long *__restrict__ gbase,
                                                       uint64_t *__restrict__ boff,
                                                       uint64_t boff_cap,
                                                       const uint16_t *__restrict__ lists,
                                                       const uint32_t *__restrict__ lok) {
  const size_t c = (size_t)blockIdx.x * 64 + threadIdx.x;
  const uint32_t v = c < nchunks ? cnt[c] : 0u;
  uint32_t x = v;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t o = (uint32_t)__shfl_up((int)x, d, 64);
    if ((int)threadIdx.x >= d) x += o;
  }
  // the wave's offsets are one contiguous range [wbase, wbase + total):
  // staged in LDS and stored coalesced when they fit, else stored per lane
  constexpr int kStageN = 1024;
  __shared__ uint64_t st[kStageN];
  const uint32_t total = (uint32_t)__shfl((int)x, 63, 64);
  const uint64_t wbase = gbase[blockIdx.x];
  const bool staged = total <= (uint32_t)kStageN;
  if (c < nchunks) {
    const uint32_t rel = x - v;
    if (lok[c]) {
      // the walk's list: no second walk of the chain (its loads wait on
      // memory once per block)
      const uint64_t c0 = 1 + c * (uint64_t)kChunkB;
      const uint16_t *l = lists + c * kList;
      for (uint32_t i = 0; i < v; ++i) {
        const uint64_t o = c0 + l[i] - 1;
        if (staged) st[rel + i] = o;
        else if (wbase + rel + i < boff_cap) boff[wbase + rel + i] = o;
      }
    } else {
      uint32_t n = 0;
      if (staged)
        bare_walk_chunk<kExact, true>(in, in_len, c, cand[c], n, st, rel, (uint64_t)kStageN);
      else
        bare_walk_chunk<kExact, true>(in, in_len, c, cand[c], n, boff, wbase + rel, boff_cap);
    }
  }
  if (staged) {
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < total; i += 64)
      if (wbase + i < boff_cap) boff[wbase + i] = st[i];
  }
}

// One thread: the chain's verdict before any block is decoded -- 0 = go,
// 1 = corrupt (a broken chain, no block, or a frame byte that is not the
// block count mod 256), 2 = more blocks than the output can hold (and so
// than the offsets array) -- and the decoder's result slots reset.
__global__ void lz4_bare_gate(const uint8_t *__restrict__ in, unsigned long long *small,
                              uint64_t nb_cap) {
  const unsigned long long nb = small[0], st = small[1];
  unsigned long long g = 0;
  if (st != 0 || nb == 0 || (uint8_t)(nb & 0xFF) != in[0]) g = 1;
  else if (nb > nb_cap) g = 2;
  small[2] = 0ull;
  small[3] = ~0ull;
  small[4] = g;
}

__global__ void lz4_decode_init(unsigned long long *result) {
  result[0] = 0ull;
  result[1] = ~0ull;
}

}  // namespace

extern "C" int lz4r_decompress_device(const void *d_in, size_t in_len, const void *d_block_offsets,
                                      size_t nb, void *d_out, size_t out_cap, void *d_result,
                                      void *stream) {
  if (!d_in || !d_block_offsets || !d_out || !d_result || nb == 0 || in_len < 4 ||
      nb > 0x7fffffffULL * kBPW)
    return LZ4R_ERR_ARG;
  hipStream_t s = static_cast<hipStream_t>(stream);
  hipLaunchKernelGGL(lz4_decode_init, dim3(1), dim3(1), 0, s,
                     static_cast<unsigned long long *>(d_result));
  const unsigned grid = (unsigned)((nb + kBPW - 1) / kBPW);
  hipLaunchKernelGGL(lz4_decode_blocks, dim3(grid), dim3(kLanes), 0, s,
                     static_cast<const uint8_t *>(d_in), in_len,
                     static_cast<const uint64_t *>(d_block_offsets), nb,
                     static_cast<uint8_t *>(d_out), out_cap,
                     static_cast<unsigned long long *>(d_result), nullptr, nullptr);
  return hipGetLastError() == hipSuccess ? LZ4R_OK : LZ4R_ERR_HIP;
}

namespace {

// one pass of the bare-stream decode in mode kExact; returns LZ4R_OK, or
// LZ4R_ERR_CORRUPT when the chain or a block does not hold together.  With
// The bare path's per-call scratch comes from a pool of the library's own
// per device that keeps its memory (release threshold: all): from the
// default pool, whose threshold is 0, every call re-mapped its ~34 MB per GiB
// of stream after the previous call's synchronise returned it.
hipMemPool_t scratch_pool() {
  static std::mutex mu;
  static std::map<int, hipMemPool_t> pools;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return nullptr;
  std::lock_guard<std::mutex> g(mu);
  auto it = pools.find(dev);
  if (it != pools.end()) return it->second;
  hipMemPoolProps props = {};
  props.allocType = hipMemAllocationTypePinned;
  props.location.type = hipMemLocationTypeDevice;
  props.location.id = dev;
  hipMemPool_t p = nullptr;
  if (hipMemPoolCreate(&p, &props) != hipSuccess) return nullptr;
  uint64_t keep = ~0ull;
  (void)hipMemPoolSetAttribute(p, hipMemPoolAttrReleaseThreshold, &keep);
  pools[dev] = p;
  return p;
}

hipError_t scratch_alloc(void **ptr, size_t bytes, hipStream_t s) {
  hipMemPool_t p = scratch_pool();
  return p ? hipMallocFromPoolAsync(ptr, bytes, p, s) : hipMallocAsync(ptr, bytes, s);
}

// boff given (nb_cap of them: the most blocks out_cap can hold), one host
// read-back: the block count stays on the device, the decoder's grid is sized
// for nb_cap and lz4_bare_gate decides on the device whether anything is
// decoded.  Without (an out_cap far above the stream's possible output), the
// block count is read back first and sizes both.
template <bool kExact>
int bare_pass(const uint8_t *in, size_t in_len, uint8_t *out, size_t out_cap, size_t nchunks,
              uint64_t *cand, uint32_t *cnt, uint64_t *exitp, unsigned long long *gsum,
              unsigned long long *gbase, unsigned long long *small, unsigned int *nmis,
              unsigned int *mis, uint16_t *lists, uint32_t *lok, uint64_t *boff, size_t nb_cap,
              size_t *out_len, hipStream_t s) {
  const unsigned ng = (unsigned)((nchunks + 63) / 64);
  unsigned long long *d_nb = small, *d_status = small + 1, *d_res = small + 2, *d_gate = small + 4;
  hipLaunchKernelGGL(lz4_bare_walk<kExact>, dim3(ng), dim3(64), 0, s, in, in_len, nchunks, cand,
                     cnt, exitp, gsum, lists, lok);
  if (hipMemsetAsync(nmis, 0, sizeof(unsigned int), s) != hipSuccess) return LZ4R_ERR_HIP;
  hipLaunchKernelGGL(lz4_bare_check, dim3((unsigned)((nchunks + 255) / 256)), dim3(256), 0, s,
                     in_len, nchunks, cand, exitp, nmis, mis);
  hipLaunchKernelGGL(lz4_bare_fix<kExact>, dim3(1), dim3(64), 0, s, in, in_len, nchunks, cand, cnt,
                     exitp, gsum, nmis, mis, d_status, lok);
  hipLaunchKernelGGL(lz4_bare_scan, dim3(1), dim3(1024), 0, s, gsum, (size_t)ng, gbase, d_nb);
  uint64_t *own = nullptr;
  if (!boff) {
    // no useful bound from out_cap: read the block count first
    unsigned long long h2[2] = {0, 0};
    if (hipMemcpyAsync(h2, small, sizeof(h2), hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipStreamSynchronize(s) != hipSuccess)
      return LZ4R_ERR_HIP;
    if (h2[1] != 0 || h2[0] == 0) return LZ4R_ERR_CORRUPT;
    nb_cap = (size_t)h2[0];
    if (scratch_alloc(reinterpret_cast<void **>(&own), nb_cap * sizeof(uint64_t), s) !=
        hipSuccess)
      return LZ4R_ERR_NOMEM;
    boff = own;
  }
  hipLaunchKernelGGL(lz4_bare_offsets<kExact>, dim3(ng), dim3(64), 0, s, in, in_len, nchunks, cand,
                     cnt, gbase, boff, (uint64_t)nb_cap, lists, lok);
  hipLaunchKernelGGL(lz4_bare_gate, dim3(1), dim3(1), 0, s, in, small, (uint64_t)nb_cap);
  hipLaunchKernelGGL(lz4_decode_blocks, dim3((unsigned)((nb_cap + kBPW - 1) / kBPW)),
                     dim3(kLanes), 0, s, in, in_len, static_cast<const uint64_t *>(boff), nb_cap,
                     out, out_cap, d_res, d_nb, d_gate);
  if (own) (void)hipFreeAsync(own, s);
  unsigned long long h[5] = {0, 0, 0, 0, 0};          // nb, status, result[2], gate
  if (hipMemcpyAsync(h, small, sizeof(h), hipMemcpyDeviceToHost, s) != hipSuccess ||
      hipStreamSynchronize(s) != hipSuccess)
    return LZ4R_ERR_HIP;
  if (h[4] == 1) return LZ4R_ERR_CORRUPT;
  if (h[4] == 2) {                                    // at least this much output
    *out_len = (size_t)(h[0] - 1) * kBlk + 1;
    return LZ4R_ERR_CAPACITY;
  }
  if (h[3] != ~0ull) return LZ4R_ERR_CORRUPT;
  *out_len = (size_t)h[2];
  return h[2] > out_cap ? LZ4R_ERR_CAPACITY : LZ4R_OK;
}

}  // namespace

extern "C" int lz4r_decompress_stream_device(const void *d_in, size_t in_len, void *d_out,
                                             size_t out_cap, size_t *out_len, void *stream) {
  if (!d_in || !d_out || !out_len) return LZ4R_ERR_ARG;
  *out_len = 0;
  if (in_len < 9) return LZ4R_ERR_CORRUPT;          // a frame byte and one 8-byte block at least
  hipStream_t s = static_cast<hipStream_t>(stream);
  const uint8_t *in = static_cast<const uint8_t *>(d_in);
  uint8_t *out = static_cast<uint8_t *>(d_out);
  const size_t nchunks = (in_len - 1 + kChunkB - 1) / kChunkB;
  const size_t ng = (nchunks + 63) / 64;
  // blocks the output can hold (every block but the last decodes to 300
  // bytes): the size of the offsets array and of the decoder's grid -- when
  // that is tighter than what the stream can hold (a block is >= 8 bytes);
  // else (an oversized out_cap) the count is read back first (nb_cap 0)
  const size_t nb_out = out_cap / kBlk + 1, nb_in = (in_len - 1) / 8 + 1;
  const size_t nb_cap = nb_out <= nb_in ? nb_out : 0;
  // scratch: cand, exit (u64) per chunk; gsum, gbase per 64 chunks; 8 u64 of
  // nb, status, result[2], gate, the inconsistent-chunk count; the list
  // (kMisCap u32); cnt, list-valid (u32) and the first kList block starts
  // (u16) per chunk; the block offsets (nb_cap u64)
  const size_t o_gsum = 16 * nchunks, o_small = o_gsum + 16 * ng, o_mis = o_small + 64;
  const size_t o_cnt = o_mis + 4 * (size_t)kMisCap;
  // every region 16-B aligned: lz4_bare_walk stores the lists as uint4
  auto al16 = [](size_t x) { return (x + 15) & ~(size_t)15; };
  const size_t o_lok = al16(o_cnt + 4 * nchunks);            // u32 per chunk
  const size_t o_lst = al16(o_lok + 4 * nchunks);            // kList u16 per chunk
  const size_t o_boff = al16(o_lst + 2 * (size_t)kList * nchunks);
  const size_t bytes = o_boff + 8 * nb_cap;
  uint8_t *scr = nullptr;
  if (scratch_alloc(reinterpret_cast<void **>(&scr), bytes, s) != hipSuccess) return LZ4R_ERR_NOMEM;
  uint64_t *cand = reinterpret_cast<uint64_t *>(scr);
  uint64_t *exitp = cand + nchunks;
  unsigned long long *gsum = reinterpret_cast<unsigned long long *>(scr + o_gsum);
  unsigned long long *gbase = gsum + ng;
  unsigned long long *small = reinterpret_cast<unsigned long long *>(scr + o_small);
  unsigned int *nmis = reinterpret_cast<unsigned int *>(small + 5);
  unsigned int *mis = reinterpret_cast<unsigned int *>(scr + o_mis);
  uint32_t *cnt = reinterpret_cast<uint32_t *>(scr + o_cnt);
  uint32_t *lok = reinterpret_cast<uint32_t *>(scr + o_lok);
  uint16_t *lists = reinterpret_cast<uint16_t *>(scr + o_lst);
  uint64_t *boff = reinterpret_cast<uint64_t *>(scr + o_boff);
  hipLaunchKernelGGL(lz4_bare_cand, dim3((unsigned)((nchunks + 3) / 4)), dim3(256), 0, s, in,
                     in_len, nchunks, cand);
  // fast mode (block length = its size field); the exact mode parses every
  // block and is needed only for streams with truncated matches
  int rc = bare_pass<false>(in, in_len, out, out_cap, nchunks, cand, cnt, exitp, gsum, gbase,
                            small, nmis, mis, lists, lok, nb_cap ? boff : nullptr, nb_cap,
                            out_len, s);
  if (rc == LZ4R_ERR_CORRUPT) {
    hipLaunchKernelGGL(lz4_bare_cand, dim3((unsigned)((nchunks + 3) / 4)), dim3(256), 0, s, in,
                       in_len, nchunks, cand);
    rc = bare_pass<true>(in, in_len, out, out_cap, nchunks, cand, cnt, exitp, gsum, gbase, small,
                         nmis, mis, lists, lok, nb_cap ? boff : nullptr, nb_cap, out_len, s);
  }
  (void)hipFreeAsync(scr, s);
  if (hipStreamSynchronize(s) != hipSuccess) return LZ4R_ERR_HIP;
  return rc;
}

extern "C" int lz4r_decompress_stream(const uint8_t *in, size_t in_len, uint8_t *out, size_t cap,
                                      size_t *out_len) {
  if (!in || !out || !out_len) return LZ4R_ERR_ARG;
  void *din = nullptr, *dout = nullptr;
  if (hipMalloc(&din, in_len ? in_len : 1) != hipSuccess ||
      hipMalloc(&dout, cap ? cap : 1) != hipSuccess) {
    (void)hipFree(din);
    return LZ4R_ERR_NOMEM;
  }
  int rc = hipMemcpy(din, in, in_len, hipMemcpyHostToDevice) == hipSuccess ? LZ4R_OK
                                                                          : LZ4R_ERR_HIP;
  if (rc == LZ4R_OK) rc = lz4r_decompress_stream_device(din, in_len, dout, cap, out_len, nullptr);
  if (rc == LZ4R_OK && hipMemcpy(out, dout, *out_len, hipMemcpyDeviceToHost) != hipSuccess)
    rc = LZ4R_ERR_HIP;
  (void)hipFree(din);
  (void)hipFree(dout);
  return rc;
}
