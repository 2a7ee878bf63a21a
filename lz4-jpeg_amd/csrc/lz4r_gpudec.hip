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
// Mapping: one LANE per block, 64 consecutive blocks per wave (a wave per
// block would issue every serial parsing step as a full wave instruction).
// The walk is latency- and issue-bound, so the kernel keeps LDS small for
// occupancy (19.5 KB of LDS per wave: the 64 output slots; 8 waves/CU) and
// keeps instruction counts low:
//   - the lane reads its encoded bytes with single unaligned 8/16-byte
//     global loads (L1/L2 absorb the re-reads of the wave's ~20 KB range),
//     after touching the block's next four 128-B lines up front so that the
//     serial walk does not wait on HBM once per line;
//   - a sequence header is decoded branch-free for the plain reading; the
//     rare truncated readings (below) take a separate path;
//   - literals move in 16-byte chunks; a match of distance D is copied in
//     chunks of min(16, d) bytes at a distance d that grows from D (the
//     match is D-periodic, so any multiple of D up to the bytes already
//     written + D is a valid distance), with D < 8 seeded by replicating
//     its period over 8 bytes;
//   - stores into the LDS slot are unaligned 16-byte stores (the hardware
//     runs in unaligned mode) whose bytes past the wanted ones fall beyond
//     the lane's write frontier; within 16 bytes of the slot end they are
//     exact-size (b64/b32/b16/b8 pieces), so no lane touches a neighbour;
//   - the wave's 64 x 300 = 19200 contiguous bytes leave as 16-B stores.
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

#include "../../include/lz4r.h"

namespace {

constexpr int kBlk = LZ4R_BLOCK;
constexpr int kInMax = LZ4R_BLOCK_BOUND;   // bytes of one encoded block (bound)
constexpr int kLanes = 64;                 // blocks per workgroup (one wave)
constexpr int kDepth = 10;                 // choice points per lane (<= 9 needed)
constexpr int kMaxSteps = 1 << 16;         // header budget: a hostile stream cannot spin a lane
constexpr int kPfN = 4;                    // L2 lines touched ahead of the walk
constexpr int kPfS = 128;                  // (2 / 4 / 8 lines, 64 or 128 B apart: same time)

typedef uint64_t u64u __attribute__((aligned(1)));
typedef uint32_t u32u __attribute__((aligned(1)));
typedef uint16_t u16u __attribute__((aligned(1)));

struct DecLds {
  alignas(16) uint8_t out[kLanes * kBlk + 32];   // lane l's block at out[300 l] (+ slack)
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
    const int per = 8 - 8 % D;
    i = M < per ? M : per;
    o.st_fast(q, {x, x}, i);
    d = i + D - i % D;                           // multiple of D, <= i + D
  }
  while (i < M) {
    int n = M - i < 16 ? M - i : 16;
    if (n > d) n = d;
    o.st_fast(q + i, o.ld16(q + i - d), n);
    i += n;
    if (d < 16) d = i + D - i % D;               // grow while short
  }
}

// Decode one block into its slot.  Returns the decoded length, or 0 if the
// block is malformed.  Each sequence is decoded from a 16-byte window h of
// the stream at ip; its distance bytes and literals come from the window
// when they lie inside it, and the next sequence's window is requested as
// soon as the next ip is known (it does not depend on the distance: the
// literal-only tail has tm = 0, so no match-extension byte either way), so
// its load overlaps this sequence's copies.
template <typename BytesT, typename SlotT>
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
      if (ip == len && ip - 3 + ntr == want && (pos == kBlk || (last && pos >= 1))) return pos;
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

__global__ __launch_bounds__(kLanes) void lz4_decode_blocks(
    const uint8_t *__restrict__ in, size_t in_len, const uint64_t *__restrict__ boff,
    size_t nb, uint8_t *__restrict__ out, size_t out_cap,
    unsigned long long *__restrict__ result) {
  __shared__ DecLds S;
  const int lane = threadIdx.x;
  const size_t b0 = (size_t)blockIdx.x * kLanes;
  const int nl = (int)(nb - b0 < (size_t)kLanes ? nb - b0 : kLanes);   // blocks here
  const size_t b = b0 + lane;

  int q = 0;                                         // decoded bytes (0 = failed / absent)
  uint32_t pfv[kPfN] = {};
  if (lane < nl) {
    const bool last = b == nb - 1;
    const size_t beg = 1 + boff[b];
    const size_t end = last ? in_len : 1 + boff[b + 1];
    if (end >= beg + 3 && end <= in_len && end - beg <= (size_t)kInMax) {
      const Slot o{S.out + lane * kBlk};
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
      if (beg + (size_t)kInMax + 64 <= in_len)
        q = decode_block(Bytes<false>{in + beg, in_len - beg}, (int)(end - beg), last, o);
      else
        q = decode_block(Bytes<true>{in + beg, in_len - beg}, (int)(end - beg), last, o);
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
  __syncthreads();

  // ---- store the wave's contiguous output -----------------------------------
  // every block but the last decodes to exactly 300 bytes, so the valid range
  // is [300 b0, 300 b0 + sum q); a failed block leaves garbage (error raised)
  size_t total = 0;
  for (int l = 0; l < nl; ++l) total += l + 1 < nl ? kBlk : S.qlen[l];
  const size_t o0 = b0 * (size_t)kBlk;
  if (o0 >= out_cap) return;
  if (o0 + total > out_cap) total = out_cap - o0;
  if (((reinterpret_cast<uintptr_t>(out) + o0) & 15) == 0) {
    const int nv = (int)(total >> 4);
    const uint4 *src = reinterpret_cast<const uint4 *>(S.out);
    uint4 *dst = reinterpret_cast<uint4 *>(out + o0);
    for (int v = lane; v < nv; v += kLanes) dst[v] = src[v];
    for (size_t i = (size_t)nv * 16 + lane; i < total; i += kLanes) out[o0 + i] = S.out[i];
  } else {
    for (size_t i = lane; i < total; i += kLanes) out[o0 + i] = S.out[i];
  }
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
      nb > 0x7fffffffULL * kLanes)
    return LZ4R_ERR_ARG;
  hipStream_t s = static_cast<hipStream_t>(stream);
  hipLaunchKernelGGL(lz4_decode_init, dim3(1), dim3(1), 0, s,
                     static_cast<unsigned long long *>(d_result));
  const unsigned grid = (unsigned)((nb + kLanes - 1) / kLanes);
  hipLaunchKernelGGL(lz4_decode_blocks, dim3(grid), dim3(kLanes), 0, s,
                     static_cast<const uint8_t *>(d_in), in_len,
                     static_cast<const uint64_t *>(d_block_offsets), nb,
                     static_cast<uint8_t *>(d_out), out_cap,
                     static_cast<unsigned long long *>(d_result));
  return hipGetLastError() == hipSuccess ? LZ4R_OK : LZ4R_ERR_HIP;
}
