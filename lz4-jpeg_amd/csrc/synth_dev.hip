// synth_dev.hip -- device-side synthetic inputs, byte-identical to host/synth.c
// (the reference generators Experiment/random_image.c:58-74 and
// random_extract.c:8-71), for inputs too large to build on the host: config
// 4's 64 GiB text corpus and config 5's 1024 4K images drawn from one
// continuous rand() stream.  Not on the timed path: a rank synthesises its
// shard in HBM before the benchmark's warm-up.
//
// rand_rgba_chunks: thread = a run of kRunPix consecutive pixels.  The host
// jumps the generator to every run's start (lz4jpeg_rand_states); the thread
// keeps the 31-word lagged-Fibonacci state in registers (a ring whose slot
// indices are compile-time constants: 31 pixels = 93 outputs = three turns of
// the ring per unrolled step) and emits one RGBA dword per pixel.
// passages_kernel: thread = 16 output bytes, each byte looked up in the
// (L2-resident) corpus at its passage's start.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/lz4jpeg_synth.h"

namespace {

constexpr int kDeg = 31;
constexpr int kRunPix = 31 * 256;       // pixels per thread (7,936)

__global__ __launch_bounds__(256) void rand_rgba_chunks(const uint32_t *__restrict__ states,
                                                        uint64_t npix,
                                                        uint32_t *__restrict__ out) {
  const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint64_t p0 = t * kRunPix;
  if (p0 >= npix) return;
  uint32_t w[kDeg];
#pragma unroll
  for (int j = 0; j < kDeg; ++j) w[j] = states[t * kDeg + j];
  const uint64_t np = npix - p0 < (uint64_t)kRunPix ? npix - p0 : (uint64_t)kRunPix;
  uint32_t *o = out + p0;
  for (uint64_t g = 0; g < np; g += 31) {
    // outputs m = 0..92 of this step: slot m % 31 holds r[i-31], slot
    // (m + 28) % 31 holds r[i-3]
    uint32_t px[31];
#pragma unroll
    for (int m = 0; m < 93; ++m) {
      const int s = m % kDeg;
      w[s] += w[(m + 28) % kDeg];
      const uint32_t b = (w[s] >> 1) & 0xffu;       // rand() % 256
      const int q = m / 3, c = m % 3;
      if (c == 0) px[q] = b;
      else if (c == 1) px[q] |= b << 8;
      else px[q] |= (b << 16) | 0xff000000u;        // a = 255
    }
#pragma unroll
    for (int q = 0; q < 31; ++q)
      if (g + q < np) o[g + q] = px[q];
  }
}

__global__ __launch_bounds__(256) void passages_kernel(const uint8_t *__restrict__ src,
                                                       const uint32_t *__restrict__ starts,
                                                       uint64_t length, uint64_t first,
                                                       uint64_t total, uint8_t *__restrict__ out) {
  const uint64_t i0 = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) * 16;
  if (i0 >= total) return;
  const uint64_t k0 = first / length;
  uint32_t v[4] = {0, 0, 0, 0};
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    const uint64_t g = first + i0 + j;
    uint32_t c = 0;
    if (i0 + j < total) {
      const uint64_t k = g / length;
      c = src[starts[k - k0] + (g - k * length)];
      if (c == '\n' || c == '\r') c = ' ';
    }
    v[j >> 2] |= c << (8 * (j & 3));
  }
  if (i0 + 16 <= total) {
    *reinterpret_cast<uint4 *>(out + i0) = make_uint4(v[0], v[1], v[2], v[3]);
  } else {
    for (int j = 0; i0 + j < total; ++j) out[i0 + j] = (uint8_t)(v[j >> 2] >> (8 * (j & 3)));
  }
}

template <typename T>
struct DevBuf {
  T *p = nullptr;
  ~DevBuf() { (void)hipFree(p); }
};

}  // namespace

extern "C" int lz4jpeg_rand_rgba_device(unsigned seed, uint64_t first_pixel, size_t npix,
                                        void *d_rgba, void *stream) {
  if (!d_rgba || (reinterpret_cast<uintptr_t>(d_rgba) & 3)) return -1;
  if (npix == 0) return 0;
  hipStream_t s = static_cast<hipStream_t>(stream);
  const size_t runs = (npix + kRunPix - 1) / kRunPix;
  uint32_t *h = static_cast<uint32_t *>(malloc(runs * kDeg * sizeof(uint32_t)));
  if (!h) return -1;
  lz4jpeg_rand_states(seed, 3 * first_pixel, 3 * (uint64_t)kRunPix, runs, h);
  DevBuf<uint32_t> st;
  int rc = 0;
  if (hipMalloc(&st.p, runs * kDeg * sizeof(uint32_t)) != hipSuccess ||
      hipMemcpyAsync(st.p, h, runs * kDeg * sizeof(uint32_t), hipMemcpyHostToDevice, s) !=
          hipSuccess)
    rc = -4;
  if (rc == 0) {
    hipLaunchKernelGGL(rand_rgba_chunks, dim3((unsigned)((runs + 255) / 256)), dim3(256), 0, s,
                       st.p, (uint64_t)npix, static_cast<uint32_t *>(d_rgba));
    if (hipGetLastError() != hipSuccess || hipStreamSynchronize(s) != hipSuccess) rc = -4;
  }
  free(h);
  return rc;
}

extern "C" int lz4jpeg_random_passages_device(const uint8_t *src_host, size_t src_len,
                                              unsigned seed, size_t length, uint64_t first,
                                              size_t total, void *d_out, void *stream) {
  if (!src_host || !d_out || length == 0 || src_len <= length ||
      (reinterpret_cast<uintptr_t>(d_out) & 15))
    return -1;
  if (total == 0) return 0;
  hipStream_t s = static_cast<hipStream_t>(stream);
  const uint64_t k0 = first / length, k1 = (first + total - 1) / length;
  const size_t count = (size_t)(k1 - k0 + 1);
  uint32_t *h = static_cast<uint32_t *>(malloc(count * sizeof(uint32_t)));
  if (!h) return -1;
  if (lz4jpeg_passage_starts(src_len, seed, length, k0, count, h) != count) {
    free(h);
    return -1;
  }
  DevBuf<uint32_t> st;
  DevBuf<uint8_t> src;
  int rc = 0;
  if (hipMalloc(&st.p, count * sizeof(uint32_t)) != hipSuccess ||
      hipMalloc(&src.p, src_len) != hipSuccess ||
      hipMemcpyAsync(st.p, h, count * sizeof(uint32_t), hipMemcpyHostToDevice, s) != hipSuccess ||
      hipMemcpyAsync(src.p, src_host, src_len, hipMemcpyHostToDevice, s) != hipSuccess)
    rc = -4;
  // launches of at most 2^34 bytes (2^30 work-items: under HIP's 2^32 grid limit)
  constexpr uint64_t kPiece = uint64_t(1) << 34;
  for (uint64_t o = 0; rc == 0 && o < total; o += kPiece) {
    const uint64_t len = total - o < kPiece ? total - o : kPiece;
    const uint64_t threads = (len + 15) / 16;
    hipLaunchKernelGGL(passages_kernel, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0, s,
                       src.p, st.p + (size_t)((first + o) / length - k0), (uint64_t)length,
                       first + o, len, static_cast<uint8_t *>(d_out) + o);
    if (hipGetLastError() != hipSuccess) rc = -4;
  }
  if (rc == 0 && hipStreamSynchronize(s) != hipSuccess) rc = -4;
  free(h);
  return rc;
}
