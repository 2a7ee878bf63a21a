// lz4r.hip -- MI355X (gfx950) "LZ4" compressor, bit-exact to the reference's
// Algorithms/sequential/LZ4/LZ4.c (canonical block-clamped matches).
//
// The reference cuts the input into 300-byte blocks (LZ4.c:23, 123-177) and,
// in every block, greedily parses with an exhaustive longest-match search over
// the whole block prefix (find_longest_match, LZ4.c:290-323; strict '>' so the
// smallest i -- farthest offset -- wins ties; length truncated to uint8_t).
// Every block is independent, so the GPU decomposition is:
//
//   lz4_analyze  one wave per group of kG blocks staged in LDS.
//     index (wave-parallel, per block): every position p <= n-4 gets its
//       4-byte key; positions are chained into per-bucket circular lists
//       (LDS hash table, atomic exchange); a lane per position walks its
//       cycle to set has_match[p] (exists i < p with an equal key, i.e. a
//       match of length >= 4).  Exact: any match >= 4 starts with an equal
//       4-gram, every equal 4-gram is in the same bucket, and the result
//       does not depend on the order the atomics ran in.
//     parse (lane per block): greedy walk that jumps over literal runs with
//       the has_match bitmask (find-first-set) and, at each candidate
//       position, walks the cycle: lcp with every earlier equal-key position
//       (4 bytes per compare), best = max length, ties -> smallest i.
//       Emits one packed record per sequence (L | M<<9 | dist<<17) and the
//       block's encoded byte count.
//   lz4_scan_*   exclusive scan of per-block byte counts -> output offsets.
//   lz4_emit     one wave per block: records -> token/size/ext/literals/
//       offset bytes at the block's output offset (write_sequence,
//       LZ4.c:365-413; write_block :415-425; frame byte :429).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>
#include <new>

#include "../../include/lz4r.h"

namespace {

constexpr int kBlk = LZ4R_BLOCK;   // 300
constexpr int kG = 16;             // blocks per analyze wave
constexpr int kH = 512;            // hash buckets of the per-block index
constexpr int kHashShift = 32 - 9;
constexpr int kMaxRec = 128;       // >= 75 (M>=4) + 44 (M in 1..3, q<=43) + 1
constexpr uint32_t kEmpty = 0xFFFFFFFFu;
constexpr int kChunkBytes = kG * kBlk;          // 4800, multiple of 16
constexpr int kDataWords = (kChunkBytes + 16) / 4;

struct AnalyzeLds {
  uint32_t data[kDataWords];       // the kG blocks, contiguous, + 16 B pad
  uint64_t mask[kG][5];            // has_match bit per position
  uint32_t head[kH];               // bucket -> last inserted position
  uint32_t keys[kBlk + 4];         // 4-byte key per position (current block)
  uint16_t nxt[kG][kBlk];          // circular bucket lists
};

__device__ __forceinline__ uint32_t load4u(const uint32_t *d, int off) {
  const uint32_t w0 = d[off >> 2], w1 = d[(off >> 2) + 1];
  return __builtin_amdgcn_alignbyte(w1, w0, (uint32_t)(off & 3));
}

__device__ __forceinline__ uint32_t hash_key(uint32_t k) {
  return (k * 2654435761u) >> kHashShift;
}

// Longest common prefix of the byte runs at a and b (a < b), capped at
// `limit` = n - q: the canonical clamp (match never crosses the block end).
__device__ __forceinline__ int lcp(const uint32_t *d, int a, int b, int limit) {
  int l = 0;
  while (l < limit) {
    const uint32_t x = load4u(d, a + l) ^ load4u(d, b + l);
    if (x) {
      l += __builtin_ctz(x) >> 3;
      return l < limit ? l : limit;
    }
    l += 4;
  }
  return limit;
}

// litext bytes (LZ4.c:548-560 accounting == 372-386 writing)
__device__ __forceinline__ int litext_len(int L) {
  if (L < 15) return 0;
  return ((L - 15) & 255) == 255 ? 2 : 1;
}

// bytes write_sequence emits for (L, M); M == 0 marks the literal-only tail
__device__ __forceinline__ int seq_written(int L, int M) {
  const int mext = (M >= 4 && ((M - 4) & 255) >= 15) ? 1 : 0;   // LZ4.c:393-411
  return 3 + litext_len(L) + L + 2 + mext;
}

// byte_size the reference stores in the sequence (LZ4.c:546-575, :597-610)
__device__ __forceinline__ int seq_size_field(int L, int M) {
  const int mext = (M != 0 && ((M - 4) & 255) >= 15) ? 1 : 0;
  return L + 5 + litext_len(L) + mext;
}

__global__ __launch_bounds__(64) void lz4_analyze(
    const uint8_t *__restrict__ in, size_t n_total, size_t nb_total,
    uint32_t *__restrict__ recs, uint32_t *__restrict__ info) {
  __shared__ AnalyzeLds S;
  const int lane = threadIdx.x;
  const size_t b0 = (size_t)blockIdx.x * kG;
  const int nb = (int)min((size_t)kG, nb_total - b0);
  const size_t byte0 = b0 * kBlk;
  const int len = (int)min((size_t)kChunkBytes, n_total - byte0);
  const uint8_t *src = in + byte0;

  // ---- stage the chunk in LDS (coalesced 16-B loads) ----------------------
  uint8_t *lds_bytes = reinterpret_cast<uint8_t *>(S.data);
  const int nvec = (((uintptr_t)src & 15) == 0) ? (len >> 4) : 0;
  for (int i = lane; i < nvec; i += 64)
    reinterpret_cast<uint4 *>(S.data)[i] = reinterpret_cast<const uint4 *>(src)[i];
  for (int i = nvec * 16 + lane; i < len; i += 64) lds_bytes[i] = src[i];
  if (lane < 16) lds_bytes[len + lane] = 0;
  for (int i = lane; i < kH; i += 64) S.head[i] = kEmpty;
  __syncthreads();

  // ---- index phase: wave-parallel per block --------------------------------
  for (int blk = 0; blk < nb; ++blk) {
    const size_t gb = b0 + blk;
    const int n = (gb == nb_total - 1) ? (int)(n_total - gb * kBlk) : kBlk;
    const int nk = n >= 4 ? n - 3 : 0;      // positions that can start a >=4 match
    const int base = blk * kBlk;
    uint32_t key[5], hh[5];
#pragma unroll
    for (int r = 0; r < 5; ++r) {
      const int p = r * 64 + lane;
      key[r] = 0;
      hh[r] = 0;
      if (p < nk) {
        key[r] = load4u(S.data, base + p);
        hh[r] = hash_key(key[r]);
        S.keys[p] = key[r];
      }
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < 5; ++r) {
      const int p = r * 64 + lane;
      if (p < nk) S.nxt[blk][p] = (uint16_t)atomicExch(&S.head[hh[r]], (uint32_t)p);
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < 5; ++r) {            // close each list into a cycle
      const int p = r * 64 + lane;
      if (p < nk && S.nxt[blk][p] == 0xFFFF) S.nxt[blk][p] = (uint16_t)S.head[hh[r]];
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < 5; ++r) {
      const int p = r * 64 + lane;
      bool found = false;
      if (p < nk) {
        int j = S.nxt[blk][p];
        while (j != p) {
          if (j < p && S.keys[j] == key[r]) { found = true; break; }
          j = S.nxt[blk][j];
        }
      }
      const uint64_t m = __ballot(found);
      if (lane == 0) S.mask[blk][r] = m;
    }
#pragma unroll
    for (int r = 0; r < 5; ++r) {
      const int p = r * 64 + lane;
      if (p < nk) S.head[hh[r]] = kEmpty;
    }
    __syncthreads();
  }

  // ---- parse phase: one lane per block -------------------------------------
  if (lane < nb) {
    const int blk = lane;
    const size_t gb = b0 + blk;
    const int n = (gb == nb_total - 1) ? (int)(n_total - gb * kBlk) : kBlk;
    const int base = blk * kBlk;
    uint32_t *out = recs + gb * kMaxRec;
    int p = 0, L = 0, nrec = 0, W = 3;
    while (true) {
      int q = n;
      for (int wi = p >> 6; wi < 5; ++wi) {           // next has_match >= p
        uint64_t m = S.mask[blk][wi];
        if (wi == (p >> 6)) m &= ~0ull << (p & 63);
        if (m) { q = wi * 64 + __builtin_ctzll(m); break; }
      }
      if (q >= n) { L += n - p; break; }
      L += q - p;
      const int limit = n - q;
      int best = 0, bj = 0;
      int j = S.nxt[blk][q];
      while (j != q) {                                // every equal-key i < q
        if (j < q) {
          const int l = lcp(S.data, base + j, base + q, limit);
          if (l > best || (l == best && j < bj)) { best = l; bj = j; }
        }
        j = S.nxt[blk][j];
      }
      const int M = best >= 4 ? (best & 255) : 0;     // uint8_t return, LZ4.c:317
      if (M == 0) {                                   // literal (len 256 -> 0)
        L += 1;
        p = q + 1;
        if (p >= n) break;
        continue;
      }
      out[nrec++] = (uint32_t)L | ((uint32_t)M << 9) | ((uint32_t)(q - bj) << 17);
      W += seq_written(L, M);
      L = 0;
      p = q + M;                                      // LZ4.c:581
      if (p >= n) break;
    }
    if (L > 0) {                                      // LZ4.c:585-613
      out[nrec++] = (uint32_t)L;
      W += seq_written(L, 0);
    }
    info[gb] = (uint32_t)W | ((uint32_t)nrec << 16);
  }
}

// ---- exclusive scan of per-block byte counts (info & 0xFFFF) --------------
constexpr int kScanThreads = 256;
constexpr int kScanPer = 16;
constexpr int kScanTile = kScanThreads * kScanPer;   // 4096 blocks per tile

__device__ __forceinline__ uint64_t wave_incl_scan(uint64_t v) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint64_t o = __shfl_up(v, d, 64);
    if (lane >= d) v += o;
  }
  return v;
}

__global__ __launch_bounds__(kScanThreads) void lz4_scan_reduce(
    const uint32_t *__restrict__ info, size_t nb, uint64_t *__restrict__ part) {
  __shared__ uint64_t ws[kScanThreads / 64];
  const size_t t0 = (size_t)blockIdx.x * kScanTile;
  uint64_t s = 0;
  for (int k = 0; k < kScanPer; ++k) {
    const size_t i = t0 + (size_t)k * kScanThreads + threadIdx.x;
    if (i < nb) s += info[i] & 0xFFFFu;
  }
  s = wave_incl_scan(s);
  if ((threadIdx.x & 63) == 63) ws[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) part[blockIdx.x] = ws[0] + ws[1] + ws[2] + ws[3];
}

// single workgroup: exclusive scan of the tile partials; total -> *len
__global__ __launch_bounds__(1024) void lz4_scan_partials(
    uint64_t *__restrict__ part, size_t nparts, uint64_t hdr,
    uint64_t *__restrict__ len) {
  __shared__ uint64_t ws[16];
  __shared__ uint64_t carry;
  if (threadIdx.x == 0) carry = 0;
  __syncthreads();
  for (size_t c0 = 0; c0 < nparts; c0 += 1024) {
    const size_t i = c0 + threadIdx.x;
    const uint64_t v = i < nparts ? part[i] : 0;
    uint64_t s = wave_incl_scan(v);
    if ((threadIdx.x & 63) == 63) ws[threadIdx.x >> 6] = s;
    __syncthreads();
    uint64_t pre = carry;
    for (int w = 0; w < (int)(threadIdx.x >> 6); ++w) pre += ws[w];
    if (i < nparts) part[i] = pre + s - v;
    __syncthreads();
    if (threadIdx.x == 1023) carry = pre + s;
    __syncthreads();
  }
  if (threadIdx.x == 0) *len = hdr + carry;
}

__global__ __launch_bounds__(kScanThreads) void lz4_scan_apply(
    const uint32_t *__restrict__ info, size_t nb, const uint64_t *__restrict__ part,
    uint64_t *__restrict__ off) {
  __shared__ uint64_t ws[kScanThreads / 64];
  const size_t t0 = (size_t)blockIdx.x * kScanTile + (size_t)threadIdx.x * kScanPer;
  uint32_t v[kScanPer];
  uint64_t s = 0;
  for (int k = 0; k < kScanPer; ++k) {
    const size_t i = t0 + k;
    v[k] = i < nb ? (info[i] & 0xFFFFu) : 0u;
    s += v[k];
  }
  const uint64_t incl = wave_incl_scan(s);
  if ((threadIdx.x & 63) == 63) ws[threadIdx.x >> 6] = incl;
  __syncthreads();
  uint64_t pre = part[blockIdx.x] + incl - s;
  for (int w = 0; w < (int)(threadIdx.x >> 6); ++w) pre += ws[w];
  for (int k = 0; k < kScanPer; ++k) {
    const size_t i = t0 + k;
    if (i < nb) off[i] = pre;
    pre += v[k];
  }
}

// ---- emit: one wave per block ----------------------------------------------
__device__ __forceinline__ void put(uint8_t *out, uint64_t cap, uint64_t pos, uint8_t b) {
  if (pos < cap) out[pos] = b;
}

__global__ __launch_bounds__(256) void lz4_emit(
    const uint8_t *__restrict__ in, size_t n_total, size_t nb_total,
    const uint32_t *__restrict__ recs, const uint32_t *__restrict__ info,
    const uint64_t *__restrict__ off, uint8_t *__restrict__ out, uint64_t cap,
    int hdr) {
  const int lane = threadIdx.x & 63;
  const size_t b = (size_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (b >= nb_total) return;
  if (hdr && b == 0 && lane == 0) put(out, cap, 0, (uint8_t)nb_total);  // LZ4.c:429
  const int nrec = (int)(info[b] >> 16);
  const uint64_t obase = (uint64_t)hdr + off[b];
  const uint8_t *blk = in + b * kBlk;
  const uint32_t *r = recs + b * kMaxRec;

  // packed (in_len:10 | written:11 | size_field:11) per record, two halves
  int Lk[2], Mk[2], Dk[2];
  uint32_t pk[2];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int k = h * 64 + lane;
    const uint32_t rv = k < nrec ? r[k] : 0u;
    Lk[h] = (int)(rv & 511u);
    Mk[h] = (int)((rv >> 9) & 255u);
    Dk[h] = (int)(rv >> 17);
    pk[h] = 0;
    if (k < nrec)
      pk[h] = (uint32_t)(Lk[h] + Mk[h]) | ((uint32_t)seq_written(Lk[h], Mk[h]) << 10) |
              ((uint32_t)seq_size_field(Lk[h], Mk[h]) << 21);
  }
  uint32_t inc0 = (uint32_t)wave_incl_scan(pk[0]);
  const uint32_t tot0 = __shfl(inc0, 63, 64);
  uint32_t inc1 = (uint32_t)wave_incl_scan(pk[1]) + tot0;
  const uint32_t tot = __shfl(inc1, 63, 64);
  if (lane == 0) {                                                  // LZ4.c:417-419
    const uint32_t bsize = (tot >> 21) + 3;
    put(out, cap, obase + 0, (uint8_t)nrec);
    put(out, cap, obase + 1, (uint8_t)(bsize & 255));
    put(out, cap, obase + 2, (uint8_t)((bsize >> 8) & 255));
  }
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int k = h * 64 + lane;
    if (k >= nrec) continue;
    const uint32_t excl = (h ? inc1 : inc0) - pk[h];
    const int L = Lk[h], M = Mk[h], D = Dk[h];
    const int lit = (int)(excl & 1023u);
    uint64_t o = obase + 3 + ((excl >> 10) & 2047u);
    const int S = seq_size_field(L, M);
    const int tl = L >= 15 ? 15 : L;                                // LZ4.c:540
    const int tm = M == 0 ? 0 : (M >= 19 ? 15 : ((M - 4) & 255));   // LZ4.c:542
    put(out, cap, o++, (uint8_t)((tl << 4) | tm));                  // LZ4.c:367
    put(out, cap, o++, (uint8_t)(S & 255));                         // LZ4.c:369
    put(out, cap, o++, (uint8_t)((S >> 8) & 255));
    if (L >= 15) {                                                  // LZ4.c:372-386
      const int rem = (L - 15) & 255;
      if (rem == 255) { put(out, cap, o++, 255); put(out, cap, o++, 0); }
      else put(out, cap, o++, (uint8_t)rem);
    }
    for (int i = 0; i < L; ++i) put(out, cap, o++, blk[lit + i]);  // LZ4.c:388
    put(out, cap, o++, (uint8_t)(D & 255));                         // LZ4.c:390
    put(out, cap, o++, (uint8_t)((D >> 8) & 255));
    if (M >= 4 && ((M - 4) & 255) >= 15)                            // LZ4.c:393-411
      put(out, cap, o++, (uint8_t)(((M - 4) & 255) - 15));
  }
}

}  // namespace

struct lz4r_ctx {
  int device = 0;
  size_t cap_blocks = 0;       // capacity of the per-block arrays
  uint32_t *recs = nullptr;
  uint32_t *info = nullptr;
  uint64_t *off = nullptr;
  uint64_t *part = nullptr;
  uint64_t *len = nullptr;     // default device length slot
  hipEvent_t ev_a = nullptr, ev_b = nullptr, ev_c = nullptr;
  bool timing = false;
  bool timed_call = false;     // the last call recorded the events
};

namespace {

void free_scratch(lz4r_ctx *c) {
  (void)hipFree(c->recs);
  (void)hipFree(c->info);
  (void)hipFree(c->off);
  (void)hipFree(c->part);
  c->recs = nullptr; c->info = nullptr; c->off = nullptr; c->part = nullptr;
  c->cap_blocks = 0;
}

int ensure_scratch(lz4r_ctx *c, size_t nb) {
  if (nb <= c->cap_blocks) return LZ4R_OK;
  free_scratch(c);
  const size_t cap = nb + nb / 8 + 1024;
  const size_t nparts = (cap + kScanTile - 1) / kScanTile;
  if (hipMalloc(&c->recs, cap * kMaxRec * sizeof(uint32_t)) != hipSuccess ||
      hipMalloc(&c->info, cap * sizeof(uint32_t)) != hipSuccess ||
      hipMalloc(&c->off, cap * sizeof(uint64_t)) != hipSuccess ||
      hipMalloc(&c->part, (nparts + 1) * sizeof(uint64_t)) != hipSuccess) {
    free_scratch(c);
    return LZ4R_ERR_NOMEM;
  }
  c->cap_blocks = cap;
  return LZ4R_OK;
}

int run(lz4r_ctx *c, const void *d_in, size_t n, void *d_out, size_t cap,
        void *d_len, int hdr, void *stream) {
  if (!c || !d_in || !d_out || !d_len) return LZ4R_ERR_ARG;
  if (hdr && n < (size_t)kBlk) return LZ4R_ERR_TOO_SMALL;
  if (n == 0) return LZ4R_ERR_ARG;
  const size_t nb = (n + kBlk - 1) / kBlk;
  int rc = ensure_scratch(c, nb);
  if (rc != LZ4R_OK) return rc;
  hipStream_t s = static_cast<hipStream_t>(stream);
  const size_t ntiles = (nb + kScanTile - 1) / kScanTile;
  const size_t ga = (nb + kG - 1) / kG;
  if (ga > 0x7fffffffULL) return LZ4R_ERR_ARG;
  const bool timed = c->timing;
  c->timed_call = timed;
  if (timed) (void)hipEventRecord(c->ev_a, s);
  hipLaunchKernelGGL(lz4_analyze, dim3((unsigned)ga), dim3(64), 0, s,
                     static_cast<const uint8_t *>(d_in), n, nb, c->recs, c->info);
  if (timed) (void)hipEventRecord(c->ev_b, s);
  hipLaunchKernelGGL(lz4_scan_reduce, dim3((unsigned)ntiles), dim3(kScanThreads), 0, s,
                     c->info, nb, c->part);
  hipLaunchKernelGGL(lz4_scan_partials, dim3(1), dim3(1024), 0, s, c->part, ntiles,
                     (uint64_t)hdr, static_cast<uint64_t *>(d_len));
  hipLaunchKernelGGL(lz4_scan_apply, dim3((unsigned)ntiles), dim3(kScanThreads), 0, s,
                     c->info, nb, c->part, c->off);
  hipLaunchKernelGGL(lz4_emit, dim3((unsigned)((nb + 3) / 4)), dim3(256), 0, s,
                     static_cast<const uint8_t *>(d_in), n, nb, c->recs, c->info, c->off,
                     static_cast<uint8_t *>(d_out), (uint64_t)cap, hdr);
  if (timed) (void)hipEventRecord(c->ev_c, s);
  return hipGetLastError() == hipSuccess ? LZ4R_OK : LZ4R_ERR_HIP;
}

}  // namespace

extern "C" {

int lz4r_ctx_create(lz4r_ctx **out) {
  if (!out) return LZ4R_ERR_ARG;
  lz4r_ctx *c = new (std::nothrow) lz4r_ctx();
  if (!c) return LZ4R_ERR_NOMEM;
  if (hipGetDevice(&c->device) != hipSuccess ||
      hipMalloc(&c->len, sizeof(uint64_t)) != hipSuccess ||
      hipEventCreate(&c->ev_a) != hipSuccess || hipEventCreate(&c->ev_b) != hipSuccess ||
      hipEventCreate(&c->ev_c) != hipSuccess) {
    lz4r_ctx_destroy(c);
    return LZ4R_ERR_HIP;
  }
  *out = c;
  return LZ4R_OK;
}

void lz4r_ctx_destroy(lz4r_ctx *c) {
  if (!c) return;
  free_scratch(c);
  (void)hipFree(c->len);
  if (c->ev_a) (void)hipEventDestroy(c->ev_a);
  if (c->ev_b) (void)hipEventDestroy(c->ev_b);
  if (c->ev_c) (void)hipEventDestroy(c->ev_c);
  delete c;
}

size_t lz4r_nblocks(size_t n) { return (n + kBlk - 1) / kBlk; }

size_t lz4r_compress_bound(size_t n) { return 1 + lz4r_nblocks(n) * (size_t)LZ4R_BLOCK_BOUND; }

int lz4r_compress_async(lz4r_ctx *c, const void *d_in, size_t n, void *d_out, size_t cap,
                        void *d_len, void *stream) {
  return run(c, d_in, n, d_out, cap, d_len, 1, stream);
}

int lz4r_compress_segment_async(lz4r_ctx *c, const void *d_in, size_t n, void *d_out,
                                size_t cap, void *d_len, void *stream) {
  return run(c, d_in, n, d_out, cap, d_len, 0, stream);
}

int lz4r_compress_device(lz4r_ctx *c, const void *d_in, size_t n, void *d_out, size_t cap,
                         size_t *out_len, void *stream) {
  if (!c || !out_len) return LZ4R_ERR_ARG;
  int rc = run(c, d_in, n, d_out, cap, c->len, 1, stream);
  if (rc != LZ4R_OK) return rc;
  uint64_t need = 0;
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (hipMemcpyAsync(&need, c->len, sizeof(need), hipMemcpyDeviceToHost, s) != hipSuccess ||
      hipStreamSynchronize(s) != hipSuccess)
    return LZ4R_ERR_HIP;
  *out_len = (size_t)need;
  return need > cap ? LZ4R_ERR_CAPACITY : LZ4R_OK;
}

int lz4r_copy_block_offsets(const lz4r_ctx *c, void *dst, size_t count, void *stream) {
  if (!c || !dst || count > c->cap_blocks) return LZ4R_ERR_ARG;
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (hipMemcpyAsync(dst, c->off, count * sizeof(uint64_t), hipMemcpyDefault, s) != hipSuccess ||
      hipStreamSynchronize(s) != hipSuccess)
    return LZ4R_ERR_HIP;
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

int lz4r_set_timing(lz4r_ctx *c, int enable) {
  if (!c) return LZ4R_ERR_ARG;
  c->timing = enable != 0;
  return LZ4R_OK;
}

int lz4r_last_timing(lz4r_ctx *c, float *ms_call, float *ms_match) {
  if (!c || !c->timed_call) return LZ4R_ERR_ARG;
  if (hipEventSynchronize(c->ev_c) != hipSuccess) return LZ4R_ERR_HIP;
  float a = 0.f, b = 0.f;
  if (hipEventElapsedTime(&a, c->ev_a, c->ev_c) != hipSuccess ||
      hipEventElapsedTime(&b, c->ev_a, c->ev_b) != hipSuccess)
    return LZ4R_ERR_HIP;
  if (ms_call) *ms_call = a;
  if (ms_match) *ms_match = b;
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
