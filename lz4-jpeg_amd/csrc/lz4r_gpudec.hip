// lz4r_gpudec.hip -- block-parallel MI355X decoder of the reference's "LZ4"
// stream (the bytes lz4r_compress / lz4_encode write).
//
// The reference decoder (LZ4_decode / interpret_frame, LZ4.c:937-1121) walks
// the stream serially and mis-parses >= 256 blocks and literal runs >= 271.
// Here every block is decoded independently, one wave per block, into its
// fixed output slot [300 b, 300 b + 300): block boundaries come from the
// compressor's per-block offsets (lz4r_copy_block_offsets), because the
// format itself cannot be split in parallel (the u16 size field over-counts
// the truncated-length sequences, LZ4.c:569-575).
//
// Per block:
//   parse  wave-uniform walk over the sequence headers held in LDS.  L comes
//          from the exact u16 size field; the one ambiguous token family
//          (0xFD..0xFF: L >= 15 with M = 17 / 18 / >= 19, or a truncated
//          match M = 1..3 whatever L, LZ4.c:317 + :540-544) is resolved by a
//          small LDS stack of choice points: the first consistent reading is
//          taken and undone if the block does not then end exactly at its
//          last byte with 300 decoded bytes (or 1..300 for the last block)
//          and size fields summing to the block header's (LZ4.c:617).
//   copy   lane-parallel: literals from the block's bytes; a match of
//          distance d at position q is periodic, out[q + i] =
//          out[q - d + (i mod d)], so every match copy is one parallel pass.
//   store  the 300 decoded bytes leave LDS as 16-B-aligned stores.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/lz4r.h"

namespace {

constexpr int kBlk = LZ4R_BLOCK;
constexpr int kInMax = LZ4R_BLOCK_BOUND;   // bytes of one encoded block (bound)
constexpr int kMaxSeq = 304;               // a sequence decodes to >= 1 byte
constexpr int kMaxChoice = 32;             // ambiguous tokens kept for backtracking
constexpr int kMaxSteps = 1 << 14;         // parse budget: a hostile stream cannot spin a wave

struct DecLds {
  alignas(16) uint8_t in[kInMax + 32];
  alignas(16) uint8_t out[kBlk + 16];
  // per sequence: literal source (ip), literal count, match length, distance
  uint16_t s_ip[kMaxSeq], s_L[kMaxSeq], s_M[kMaxSeq], s_D[kMaxSeq];
  // choice points: sequence index, ip, pos at the token; next reading to try
  uint16_t c_k[kMaxChoice], c_ip[kMaxChoice], c_pos[kMaxChoice], c_alt[kMaxChoice];
  uint16_t c_sum[kMaxChoice];     // sum of the size fields before the token
};

__device__ __forceinline__ int litext_len(int L) {
  if (L < 15) return 0;
  return ((L - 15) & 255) == 255 ? 2 : 1;
}

__device__ __forceinline__ bool litext_ok(const uint8_t *in, int len, int ip, int L) {
  const int r = (L - 15) & 255;
  if (r == 255) return ip + 1 < len && in[ip] == 255 && in[ip + 1] == 0;
  return ip < len && in[ip] == r;
}

// One reading of the sequence at `ip` (output position `pos`).  alt 0: the
// token's nibbles as written for M == 0 or M >= 4; alt 1..3: a truncated
// match M = alt (only for tokens 0xFD..0xFF).  Returns false if the bytes
// are inconsistent with that reading; else fills L, M, D, the literal start
// and the next ip.
__device__ bool read_seq(const uint8_t *in, int len, int ip, int pos, bool last, int alt,
                         int &L, int &M, int &D, int &lit, int &nip) {
  if (ip + 3 > len) return false;
  const int tok = in[ip];
  const int S = in[ip + 1] | (in[ip + 2] << 8);
  const int ip0 = ip + 3;
  if (alt == 0) {
    const int tl = tok >> 4, tm = tok & 15, mx = tm == 15 ? 1 : 0;
    int le = 0;
    if (tl == 15) {
      le = (ip0 < len && in[ip0] == 255) ? 2 : 1;
      L = S - 5 - le - mx;
      if (L < 15 || litext_len(L) != le || !litext_ok(in, len, ip0, L)) return false;
    } else {
      L = tl;
      if (S != L + 5 + mx) return false;
    }
    lit = ip0 + le;
    if (lit + L + 2 > len || pos + L > kBlk) return false;
    D = in[lit + L] | (in[lit + L + 1] << 8);
    nip = lit + L + 2;
    if (D == 0) {                          // literal-only tail (LZ4.c:585-613)
      if (!last || tm != 0) return false;
      M = 0;
      return true;
    }
    if (tm == 15) {
      if (nip >= len) return false;
      M = 19 + in[nip++];
    } else {
      M = tm + 4;
    }
    return D <= pos + L && pos + L + M <= kBlk;
  }
  // truncated match length: S = L + 5 + litext_len(L) + 1 (LZ4.c:569-575)
  if (tok - 0xFC != alt) return false;
  M = alt;
  for (int le = 0; le <= 2; ++le) {
    L = S - 6 - le;
    if (L < 0 || litext_len(L) != le) continue;
    if (le && !litext_ok(in, len, ip0, L)) continue;
    lit = ip0 + le;
    if (lit + L + 2 > len || pos + L + M > kBlk) continue;
    D = in[lit + L] | (in[lit + L + 1] << 8);
    if (D == 0 || D > pos + L) continue;
    nip = lit + L + 2;
    return true;
  }
  return false;
}

__global__ __launch_bounds__(64) void lz4_decode_blocks(
    const uint8_t *__restrict__ in, size_t in_len, const uint64_t *__restrict__ boff,
    size_t nb, uint8_t *__restrict__ out, size_t out_cap,
    unsigned long long *__restrict__ result) {
  __shared__ DecLds S;
  const int lane = threadIdx.x;
  const size_t b = blockIdx.x;
  const bool last = b == nb - 1;
  const size_t beg = 1 + boff[b];
  const size_t end = last ? in_len : 1 + boff[b + 1];
  if (end < beg + 3 || end - beg > (size_t)kInMax) {
    if (lane == 0) atomicMin(&result[1], (unsigned long long)b + 1);
    return;
  }
  const int len = (int)(end - beg);
  for (int i = lane; i < len; i += 64) S.in[i] = in[beg + i];
  if (lane < 32) S.in[len + lane] = 0;
  __syncthreads();

  // ---- parse (wave-uniform) ------------------------------------------------
  const int nseq = S.in[0];                          // nseq & 0xFF; <= 255 in practice
  // header size field = 3 + sum of the sequences' size fields (LZ4.c:617)
  const int want = (S.in[1] | (S.in[2] << 8)) - 3;
  int k = 0, ip = 3, pos = 0, nch = 0, alt = 0, steps = 0, ssum = 0;
  bool ok = nseq > 0 && want >= 0;
  while (ok) {
    if (++steps > kMaxSteps) { ok = false; break; }
    if (k == nseq) {
      if (ip == len && ssum == want && (pos == kBlk || (last && pos >= 1))) break;
    } else {
      int L, M, D, lit, nip;
      bool got = false;
      const int tok = S.in[ip < len ? ip : 0];
      const int maxalt = (ip < len && tok >= 0xFD) ? 3 : 0;
      const int sz = ip + 3 <= len ? (S.in[ip + 1] | (S.in[ip + 2] << 8)) : 0;
      if (ssum + sz > want) alt = maxalt + 1;            // no reading fits the header
      for (; alt <= maxalt && !got; ++alt)
        got = read_seq(S.in, len, ip, pos, k + 1 == nseq, alt, L, M, D, lit, nip);
      if (got) {
        if (maxalt && alt <= maxalt) {                 // other readings remain: choice point
          if (nch == kMaxChoice) { ok = false; break; }
          if (lane == 0) {
            S.c_k[nch] = (uint16_t)k; S.c_ip[nch] = (uint16_t)ip;
            S.c_pos[nch] = (uint16_t)pos; S.c_alt[nch] = (uint16_t)alt;
            S.c_sum[nch] = (uint16_t)ssum;
          }
          ++nch;
        }
        if (lane == 0) {
          S.s_ip[k] = (uint16_t)lit; S.s_L[k] = (uint16_t)L;
          S.s_M[k] = (uint16_t)M; S.s_D[k] = (uint16_t)D;
        }
        ++k;
        ssum += sz;
        ip = nip;
        pos += L + M;
        alt = 0;
        continue;
      }
    }
    // dead end: resume the most recent choice point with its next reading
    if (nch == 0) { ok = false; break; }
    --nch;
    __syncthreads();
    k = S.c_k[nch]; ip = S.c_ip[nch]; pos = S.c_pos[nch]; alt = S.c_alt[nch];
    ssum = S.c_sum[nch];
    __syncthreads();
  }
  if (!ok) {
    if (lane == 0) atomicMin(&result[1], (unsigned long long)b + 1);
    return;
  }
  __syncthreads();

  // ---- copy: literals and periodic matches, lane-parallel ------------------
  int q = 0;
  for (int s = 0; s < nseq; ++s) {
    const int L = S.s_L[s], M = S.s_M[s], D = S.s_D[s], lit = S.s_ip[s];
    for (int i = lane; i < L; i += 64) S.out[q + i] = S.in[lit + i];
    q += L;
    __syncthreads();
    for (int i = lane; i < M; i += 64) S.out[q + i] = S.out[q - D + (i % D)];
    q += M;
    __syncthreads();
  }

  // ---- store -----------------------------------------------------------------
  const size_t o0 = b * (size_t)kBlk;
  for (int i = lane; i < q; i += 64)
    if (o0 + i < out_cap) out[o0 + i] = S.out[i];
  if (last && lane == 0) result[0] = (unsigned long long)(o0 + q);
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
      nb > 0x7fffffffULL)
    return LZ4R_ERR_ARG;
  hipStream_t s = static_cast<hipStream_t>(stream);
  hipLaunchKernelGGL(lz4_decode_init, dim3(1), dim3(1), 0, s,
                     static_cast<unsigned long long *>(d_result));
  hipLaunchKernelGGL(lz4_decode_blocks, dim3((unsigned)nb), dim3(64), 0, s,
                     static_cast<const uint8_t *>(d_in), in_len,
                     static_cast<const uint64_t *>(d_block_offsets), nb,
                     static_cast<uint8_t *>(d_out), out_cap,
                     static_cast<unsigned long long *>(d_result));
  return hipGetLastError() == hipSuccess ? LZ4R_OK : LZ4R_ERR_HIP;
}
