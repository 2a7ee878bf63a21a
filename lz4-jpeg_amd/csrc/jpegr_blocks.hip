// jpegr_blocks.hip -- the reference's per-block JPEG functions as batched
// gfx950 kernels, bit-exact, for the in-process compatibility layer
// (include/lz4jpeg_compat.h) and the JPEG_seq executable.
//
//   jpegr_planes_device      build_luminance_matrix / build_r/bChrominance_matrix
//                            (JPEG.c:114-185): full-resolution Y, Cr, Cb planes
//   jpegr_dct_blocks_device  discrete_cosine_transform (JPEG.c:451-494) on a
//                            batch of planar uint8 blocks, width 8 or 4, height 8
//   jpegr_quantize_device    Quantize (JPEG.c:621-629): c = (int)(c / table[i])
//   jpegr_zigzag_device      zigzag_pattern (JPEG.c:693-728): permutation
//
// The fused image kernel (jpegr.hip) is the hot path; these exist so that
// code written against the reference's function-level API runs on the GPU
// with the same results.  Arithmetic follows jpegr.hip: fp64, no contraction,
// reference summation order, baked correctly-rounded cos / alpha constants.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "jpeg_tables.h"
#include "../../include/jpegr.h"

#pragma clang fp contract(off)

namespace {

__constant__ double bC8[8][8];
__constant__ double bC4[4][4];
__constant__ double bAA88[8][8];
__constant__ double bAA84[8][4];

__device__ __forceinline__ int clamp_u8(int v) {       // JPEG.c:132-139
  return v < 0 ? 0 : (v > 255 ? 255 : v);
}

__global__ void planes_kernel(const uint8_t *__restrict__ rgba, size_t npx,
                              uint8_t *__restrict__ yp, uint8_t *__restrict__ crp,
                              uint8_t *__restrict__ cbp) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= npx) return;
  const uint32_t p = reinterpret_cast<const uint32_t *>(rgba)[i];
  const double R = (double)(p & 255u), G = (double)((p >> 8) & 255u),
               B = (double)((p >> 16) & 255u);
  const double y = 0.299 * R + 0.587 * G + 0.114 * B;                       // JPEG.c:127
  yp[i] = (uint8_t)(unsigned)y;
  crp[i] = (uint8_t)clamp_u8((int)(0.439 * R - 0.368 * G - 0.071 * B + 128.0));  // :157
  cbp[i] = (uint8_t)clamp_u8((int)(-0.148 * R - 0.291 * G + 0.439 * B + 128.0)); // :180
}

// one thread per coefficient (u, v) of one block; blockDim = 8 * W
template <int W>
__global__ void dct_blocks_kernel(const uint8_t *__restrict__ in, int nblocks,
                                  double *__restrict__ out) {
  const int b = blockIdx.x;
  const int t = threadIdx.x;
  if (b >= nblocks) return;
  const int u = t / W, v = t % W;
  const uint8_t *blk = in + (size_t)b * 8 * W;
  double s = 0.0;
#pragma unroll
  for (int x = 0; x < 8; ++x) {
    const double cx = bC8[x][u];
#pragma unroll
    for (int y = 0; y < W; ++y) {
      const double cy = (W == 8) ? bC8[y][v] : bC4[y][v];
      s = s + ((double)((int)blk[x * W + y] - 128) * cx) * cy;       // JPEG.c:483
    }
  }
  out[(size_t)b * 8 * W + t] = ((W == 8) ? bAA88[u][v] : bAA84[u][v]) * s;   // :489
}

__global__ void quantize_kernel(double *__restrict__ c, const double *__restrict__ table,
                                int size, size_t n) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  c[i] = (double)(int)(c[i] / table[i % size]);                         // JPEG.c:626-627
}

__global__ void permute_kernel(const double *__restrict__ in, double *__restrict__ out,
                               const int *__restrict__ perm, int size, size_t n) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const size_t blk = i / size;
  out[i] = in[blk * size + perm[i % size]];
}

bool g_ready[64] = {false};

hipError_t upload() {
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return e;
  if (dev >= 0 && dev < 64 && g_ready[dev]) return hipSuccess;
  using namespace jpegr_tables;
  if ((e = hipMemcpyToSymbol(HIP_SYMBOL(bC8), C8, sizeof(C8))) != hipSuccess) return e;
  if ((e = hipMemcpyToSymbol(HIP_SYMBOL(bC4), C4, sizeof(C4))) != hipSuccess) return e;
  if ((e = hipMemcpyToSymbol(HIP_SYMBOL(bAA88), AA88, sizeof(AA88))) != hipSuccess) return e;
  if ((e = hipMemcpyToSymbol(HIP_SYMBOL(bAA84), AA84, sizeof(AA84))) != hipSuccess) return e;
  if (dev >= 0 && dev < 64) g_ready[dev] = true;
  return hipSuccess;
}

unsigned grid_for(size_t n, unsigned bs) { return (unsigned)((n + bs - 1) / bs); }

}  // namespace

extern "C" {

int jpegr_planes_device(const void *d_rgba, int w, int h, void *d_y, void *d_cr, void *d_cb,
                        void *stream) {
  if (!d_rgba || !d_y || !d_cr || !d_cb || w <= 0 || h <= 0) return JPEGR_ERR_ARG;
  const size_t npx = (size_t)w * (size_t)h;
  if (npx / 256 + 1 > 0x7fffffffULL) return JPEGR_ERR_ARG;
  hipLaunchKernelGGL(planes_kernel, dim3(grid_for(npx, 256)), dim3(256), 0,
                     static_cast<hipStream_t>(stream), static_cast<const uint8_t *>(d_rgba),
                     npx, static_cast<uint8_t *>(d_y), static_cast<uint8_t *>(d_cr),
                     static_cast<uint8_t *>(d_cb));
  return hipGetLastError() == hipSuccess ? JPEGR_OK : JPEGR_ERR_HIP;
}

int jpegr_dct_blocks_device(const void *d_blocks, int width, int height, int nblocks,
                            void *d_out_f64, void *stream) {
  if (!d_blocks || !d_out_f64 || height != 8 || (width != 8 && width != 4) || nblocks <= 0)
    return JPEGR_ERR_ARG;
  if (upload() != hipSuccess) return JPEGR_ERR_HIP;
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (width == 8)
    hipLaunchKernelGGL(dct_blocks_kernel<8>, dim3((unsigned)nblocks), dim3(64), 0, s,
                       static_cast<const uint8_t *>(d_blocks), nblocks,
                       static_cast<double *>(d_out_f64));
  else
    hipLaunchKernelGGL(dct_blocks_kernel<4>, dim3((unsigned)nblocks), dim3(32), 0, s,
                       static_cast<const uint8_t *>(d_blocks), nblocks,
                       static_cast<double *>(d_out_f64));
  return hipGetLastError() == hipSuccess ? JPEGR_OK : JPEGR_ERR_HIP;
}

int jpegr_quantize_device(void *d_coef_f64, const void *d_table_f64, int size, size_t n,
                          void *stream) {
  if (!d_coef_f64 || !d_table_f64 || size <= 0 || n == 0) return JPEGR_ERR_ARG;
  if (n / 256 + 1 > 0x7fffffffULL) return JPEGR_ERR_ARG;
  hipLaunchKernelGGL(quantize_kernel, dim3(grid_for(n, 256)), dim3(256), 0,
                     static_cast<hipStream_t>(stream), static_cast<double *>(d_coef_f64),
                     static_cast<const double *>(d_table_f64), size, n);
  return hipGetLastError() == hipSuccess ? JPEGR_OK : JPEGR_ERR_HIP;
}

int jpegr_permute_device(const void *d_in_f64, void *d_out_f64, const void *d_perm_i32,
                         int size, size_t n, void *stream) {
  if (!d_in_f64 || !d_out_f64 || !d_perm_i32 || size <= 0 || n == 0) return JPEGR_ERR_ARG;
  if (n / 256 + 1 > 0x7fffffffULL) return JPEGR_ERR_ARG;
  hipLaunchKernelGGL(permute_kernel, dim3(grid_for(n, 256)), dim3(256), 0,
                     static_cast<hipStream_t>(stream), static_cast<const double *>(d_in_f64),
                     static_cast<double *>(d_out_f64), static_cast<const int *>(d_perm_i32),
                     size, n);
  return hipGetLastError() == hipSuccess ? JPEGR_OK : JPEGR_ERR_HIP;
}

}  // extern "C"
