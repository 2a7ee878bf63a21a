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
// Mapping: one LANE per block, 64 consecutive blocks per wave.  Parsing a
// block is a serial walk over its sequence headers; running 64 of them side
// by side makes each wave instruction do 64 blocks' work (a wave-per-block
// walk issues the same instructions for one block).  Each lane
//   parse  reads its block straight from global memory (aligned dword loads,
//          L1/L2 absorb the re-reads; the wave's 64 blocks are one
//          contiguous ~20 KB range).  L comes from the exact u16 size field;
//          the one ambiguous token family (0xFD..0xFF: L >= 15 with
//          M = 17 / 18 / >= 19, or a truncated match M = 1..3 whatever L,
//          LZ4.c:317 + :540-544) is resolved by a per-lane LDS stack of
//          choice points: the plain reading is taken first and undone if the
//          block does not then end exactly at its last byte with 300 decoded
//          bytes (or 1..300 for the last block) and size fields summing to
//          the block header's (LZ4.c:617).  A plain reading of such a token
//          decodes >= 32 bytes, so at most 9 choice points are ever pending.
//   emit   writes literals and (periodic) match copies into its 300-byte
//          LDS slot as it parses; a backtrack simply rewrites the tail.
// The wave then stores its 64 x 300 = 19200 contiguous bytes as 16-B stores.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/lz4r.h"

namespace {

constexpr int kBlk = LZ4R_BLOCK;
constexpr int kInMax = LZ4R_BLOCK_BOUND;   // bytes of one encoded block (bound)
constexpr int kLanes = 64;                 // blocks per workgroup (one wave)
constexpr int kDepth = 10;                 // choice points per lane (<= 9 needed)
constexpr int kMaxSteps = 1 << 16;         // parse budget: a hostile stream cannot spin a lane

struct DecLds {
  alignas(16) uint8_t out[kLanes * kBlk];  // lane l's block at out[300 l]
  uint64_t stk[kDepth][kLanes];            // choice points, column per lane
  uint32_t qlen[kLanes];                   // decoded bytes per block (0 = failed)
};

__device__ __forceinline__ uint32_t funnel(uint32_t hi, uint32_t lo, uint32_t s) {
  return __builtin_amdgcn_alignbyte(hi, lo, s);
}

// Bytes a .. a+7 after p, little-endian; `avail` = readable bytes after p.
__device__ __forceinline__ uint64_t ld8(const uint8_t *p, int a, int avail) {
  const uint8_t *q = p + a;
  if (a + 12 <= avail) {
    const uint32_t *w = reinterpret_cast<const uint32_t *>((uintptr_t)q & ~(uintptr_t)3);
    const uint32_t s = (uint32_t)((uintptr_t)q & 3);
    const uint32_t w0 = w[0], w1 = w[1], w2 = w[2];
    return funnel(w1, w0, s) | ((uint64_t)funnel(w2, w1, s) << 32);
  }
  uint64_t r = 0;
  for (int t = 0; t < 8; ++t)
    if (a + t < avail) r |= (uint64_t)q[t] << (8 * t);
  return r;
}

__device__ __forceinline__ uint32_t ld4(const uint8_t *p, int a, int avail) {
  const uint8_t *q = p + a;
  if (a + 8 <= avail) {
    const uint32_t *w = reinterpret_cast<const uint32_t *>((uintptr_t)q & ~(uintptr_t)3);
    return funnel(w[1], w[0], (uint32_t)((uintptr_t)q & 3));
  }
  uint32_t r = 0;
  for (int t = 0; t < 4; ++t)
    if (a + t < avail) r |= (uint32_t)q[t] << (8 * t);
  return r;
}

__device__ __forceinline__ int litext_len(int L) {
  if (L < 15) return 0;
  return ((L - 15) & 255) == 255 ? 2 : 1;
}

__device__ __forceinline__ bool litext_ok(int ip0, int len, int e0, int e1, int L) {
  const int r = (L - 15) & 255;
  return r == 255 ? (ip0 + 1 < len && e0 == 255 && e1 == 0) : (ip0 < len && e0 == r);
}

// One reading of the sequence at ip (output position pos) whose first eight
// bytes are h.  alt 0: the token's nibbles as written for M == 0 or M >= 4;
// alt 1..3: a truncated match M = alt, tokens 0xFD..0xFF only, size field
// S = L + 5 + litext_len(L) + 1 (LZ4.c:569-575).
__device__ __forceinline__ bool read_seq(const uint8_t *p, int avail, int len, int ip,
                                         uint64_t h, int pos, bool last, int alt, int &L,
                                         int &M, int &D, int &lit, int &nip) {
  const int tok = (int)(h & 255), Sz = (int)((h >> 8) & 0xFFFF);
  const int e0 = (int)((h >> 24) & 255), e1 = (int)((h >> 32) & 255);
  const int ip0 = ip + 3;
  if (alt == 0) {
    const int tl = tok >> 4, tm = tok & 15, mx = tm == 15 ? 1 : 0;
    int le = 0;
    if (tl == 15) {
      le = (ip0 < len && e0 == 255) ? 2 : 1;
      L = Sz - 5 - le - mx;
      if (L < 15 || litext_len(L) != le || !litext_ok(ip0, len, e0, e1, L)) return false;
    } else {
      L = tl;
      if (Sz != L + 5 + mx) return false;
    }
    lit = ip0 + le;
    if (lit + L + 2 > len || pos + L > kBlk) return false;
    const uint32_t t = ld4(p, lit + L, avail);
    D = (int)(t & 0xFFFF);
    nip = lit + L + 2;
    if (D == 0) {                            // literal-only tail (LZ4.c:585-613)
      M = 0;
      return last && tm == 0;
    }
    if (tm == 15) {
      if (nip >= len) return false;
      M = 19 + (int)((t >> 16) & 255);
      ++nip;
    } else {
      M = tm + 4;
    }
    return D <= pos + L && pos + L + M <= kBlk;
  }
  M = alt;
  for (int le = 0; le <= 2; ++le) {
    L = Sz - 6 - le;
    if (L < 0 || litext_len(L) != le) continue;
    if (le && !litext_ok(ip0, len, e0, e1, L)) continue;
    lit = ip0 + le;
    if (lit + L + 2 > len || pos + L + M > kBlk) continue;
    D = (int)(ld4(p, lit + L, avail) & 0xFFFF);
    if (D == 0 || D > pos + L) continue;
    nip = lit + L + 2;
    return true;
  }
  return false;
}

// literals p[lit, lit+L) -> o[pos, pos+L)
__device__ __forceinline__ void emit_literals(uint8_t *o, int pos, const uint8_t *p, int lit,
                                              int L, int avail) {
  int i = 0;
  for (; i + 8 <= L; i += 8) {
    const uint64_t w = ld8(p, lit + i, avail);
#pragma unroll
    for (int t = 0; t < 8; ++t) o[pos + i + t] = (uint8_t)(w >> (8 * t));
  }
  if (i < L) {
    const uint64_t w = ld8(p, lit + i, avail);
    for (int t = 0; i + t < L; ++t) o[pos + i + t] = (uint8_t)(w >> (8 * t));
  }
}

// match of length M at distance D: o[q + i] = o[q - D + i] in order, i.e.
// periodic with period D when D < M
__device__ __forceinline__ void emit_match(uint8_t *o, int q, int D, int M) {
  if (D >= 8) {
    int i = 0;
    for (; i + 8 <= M; i += 8) {
      uint8_t c[8];
#pragma unroll
      for (int t = 0; t < 8; ++t) c[t] = o[q - D + i + t];
#pragma unroll
      for (int t = 0; t < 8; ++t) o[q + i + t] = c[t];
    }
    for (; i < M; ++i) o[q + i] = o[q - D + i];
  } else {
    // period D < 8: X = the period repeated over 16 bytes (lo, hi); the
    // 8 bytes at q + i are X[s .. s+8) with s = i mod D
    uint64_t pat = 0;
    for (int t = 0; t < D; ++t) pat |= (uint64_t)o[q - D + t] << (8 * t);
    uint64_t lo = 0, hi = 0;
    int r = 0;
#pragma unroll
    for (int t = 0; t < 16; ++t) {
      const uint64_t c = (pat >> (8 * r)) & 255;
      if (t < 8) lo |= c << (8 * t);
      else hi |= c << (8 * (t - 8));
      r = r + 1 == D ? 0 : r + 1;
    }
    int s = 0;
    for (int i = 0; i < M; i += 8) {
      const uint64_t w = s ? (lo >> (8 * s)) | (hi << (64 - 8 * s)) : lo;
      const int n = M - i < 8 ? M - i : 8;
      for (int t = 0; t < n; ++t) o[q + i + t] = (uint8_t)(w >> (8 * t));
      s += 8 % D;
      if (s >= D) s -= D;
    }
  }
}

__device__ __forceinline__ uint64_t pack_choice(int k, int ip, int pos, int ssum, int alt) {
  return (uint64_t)k | ((uint64_t)ip << 8) | ((uint64_t)pos << 24) | ((uint64_t)ssum << 40) |
         ((uint64_t)alt << 56);
}

__global__ __launch_bounds__(kLanes) void lz4_decode_blocks(
    const uint8_t *__restrict__ in, size_t in_len, const uint64_t *__restrict__ boff,
    size_t nb, uint8_t *__restrict__ out, size_t out_cap,
    unsigned long long *__restrict__ result) {
  __shared__ DecLds S;
  const int lane = threadIdx.x;
  const size_t b0 = (size_t)blockIdx.x * kLanes;
  const size_t b = b0 + lane;
  uint8_t *o = S.out + lane * kBlk;
  int q = 0;                                       // decoded bytes (0 = failed / absent)

  if (b < nb) {
    const bool last = b == nb - 1;
    const size_t beg = 1 + boff[b];
    const size_t end = last ? in_len : 1 + boff[b + 1];
    bool ok = end >= beg + 3 && end <= in_len && end - beg <= (size_t)kInMax;
    const uint8_t *p = in + (ok ? beg : 0);
    const int len = ok ? (int)(end - beg) : 0;
    const int avail = ok ? (int)(in_len - beg < (size_t)(1 << 30) ? in_len - beg : 1 << 30) : 0;
    int k = 0, ip = 3, pos = 0, nch = 0, alt = 0, steps = 0, ssum = 0, nseq = 0, want = 0;
    if (ok) {
      const uint64_t h0 = ld8(p, 0, avail);
      nseq = (int)(h0 & 255);                        // nseq & 0xFF; <= 76 in practice
      want = (int)((h0 >> 8) & 0xFFFF) - 3;          // LZ4.c:617
      ok = nseq > 0 && want >= 0;
    }
    while (ok) {
      if (++steps > kMaxSteps) { ok = false; break; }
      if (k == nseq) {
        if (ip == len && ssum == want && (pos == kBlk || (last && pos >= 1))) break;
      } else if (ip + 3 <= len) {
        const uint64_t h = ld8(p, ip, avail);
        const int tok = (int)(h & 255), Sz = (int)((h >> 8) & 0xFFFF);
        int L = 0, M = 0, D = 0, lit = 0, nip = 0;
        bool got = false;
        if (ssum + Sz <= want && alt <= 3) {
          got = read_seq(p, avail, len, ip, h, pos, k + 1 == nseq, alt, L, M, D, lit, nip);
          if (alt == 0 && tok >= 0xFD) {
            if (got) {                               // the truncated reading remains
              if (nch == kDepth) { ok = false; break; }
              S.stk[nch++][lane] = pack_choice(k, ip, pos, ssum, tok - 0xFC);
            } else {
              got = read_seq(p, avail, len, ip, h, pos, k + 1 == nseq, tok - 0xFC, L, M, D,
                             lit, nip);
            }
          }
        }
        if (got) {
          emit_literals(o, pos, p, lit, L, avail);
          emit_match(o, pos + L, D, M);
          ++k;
          ssum += Sz;
          ip = nip;
          pos += L + M;
          alt = 0;
          continue;
        }
      }
      // dead end: resume the most recent choice point with its other reading
      if (nch == 0) { ok = false; break; }
      const uint64_t c = S.stk[--nch][lane];
      k = (int)(c & 255); ip = (int)((c >> 8) & 0xFFFF); pos = (int)((c >> 24) & 0xFFFF);
      ssum = (int)((c >> 40) & 0xFFFF); alt = (int)(c >> 56);
    }
    if (ok) {
      q = pos;
      if (last) result[0] = (unsigned long long)(b * kBlk + q);
    } else {
      atomicMin(&result[1], (unsigned long long)b + 1);
    }
  }
  S.qlen[lane] = (uint32_t)q;
  __syncthreads();

  // ---- store the wave's contiguous output -----------------------------------
  // every block but the last decodes to exactly 300 bytes, so the valid range
  // is [300 b0, 300 b0 + sum q); a failed block leaves garbage (error raised)
  __shared__ uint32_t s_total;
  if (lane == 0) {
    uint32_t t = 0;
    const int nl = (int)(nb - b0 < (size_t)kLanes ? nb - b0 : kLanes);
    for (int l = 0; l < nl; ++l) t += l + 1 < nl ? kBlk : S.qlen[l];
    s_total = t;
  }
  __syncthreads();
  const size_t o0 = b0 * (size_t)kBlk;
  size_t total = s_total;
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
