// store_rate.hip -- tools only: cost of the scattered, byte-aligned global
// stores a lane-per-sequence LZ4 emission would issue, against the aligned
// 16-B stores of an LDS-image emission, on the same ~1.1 GB output.
// Each wave writes a contiguous 1,280-B range; in the scattered form lane l
// owns 20 bytes at 20 l and writes them as an 8-B, an overlapping 8-B, a
// 4-B, a 2-B and a 1-B store at byte offsets (the header / trailer / short
// literal pieces), in the 16-B form the same range leaves as 80 aligned
// chunks.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

typedef uint64_t u64u __attribute__((aligned(1)));
typedef uint32_t u32u __attribute__((aligned(1)));
typedef uint16_t u16u __attribute__((aligned(1)));
typedef uint4 u128u __attribute__((aligned(1)));

__global__ __launch_bounds__(256) void scattered(uint8_t *out, size_t nw, int mode) {
  const size_t w = (size_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (w >= nw) return;
  const int lane = threadIdx.x & 63;
  uint8_t *p = out + w * 1280 + 20 * lane;
  const uint32_t v = 0x01010101u * (uint32_t)lane;
  if (mode == 0) {          // five pieces per lane
    *reinterpret_cast<u64u *>(p) = (uint64_t)v << 32 | v;
    *reinterpret_cast<u64u *>(p + 5) = (uint64_t)v << 32 | v;
    *reinterpret_cast<u32u *>(p + 13) = v;
    *reinterpret_cast<u16u *>(p + 17) = (uint16_t)v;
    p[19] = (uint8_t)v;
  } else if (mode == 1) {   // a 16-B piece + a 4-B piece per lane
    *reinterpret_cast<u128u *>(p) = make_uint4(v, v, v, v);
    *reinterpret_cast<u32u *>(p + 16) = v;
  } else {                  // aligned 16-B chunks of the wave's range
    uint4 *q = reinterpret_cast<uint4 *>(out + w * 1280);
    q[lane] = make_uint4(v, v, v, v);
    if (lane < 16) q[64 + lane] = make_uint4(v, v, v, v);
  }
}

int main() {
  const size_t nw = 900000;                    // 1.15 GB
  uint8_t *out;
  if (hipMalloc(&out, nw * 1280 + 64) != hipSuccess) return 1;
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  const char *names[3] = {"five byte-aligned pieces per lane", "16-B + 4-B unaligned per lane",
                          "aligned 16-B chunks"};
  for (int mode = 0; mode < 3; ++mode) {
    for (int i = 0; i < 20; ++i)
      hipLaunchKernelGGL(scattered, dim3((unsigned)((nw + 3) / 4)), dim3(256), 0, 0, out, nw, mode);
    hipEventRecord(a);
    const int reps = 50;
    for (int i = 0; i < reps; ++i)
      hipLaunchKernelGGL(scattered, dim3((unsigned)((nw + 3) / 4)), dim3(256), 0, 0, out, nw, mode);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    ms /= reps;
    printf("%-36s %.3f ms  %.1f GB/s\n", names[mode], ms, nw * 1280.0 / ms / 1e6);
  }
  return hipGetLastError() == hipSuccess ? 0 : 1;
}
