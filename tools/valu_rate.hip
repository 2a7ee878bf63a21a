// Micro-benchmark: wave64 issue rate of integer VALU / SALU / DPP on gfx950
// with 8 waves per SIMD (the lz4_tiles occupancy).  Prints cycles per
// wave-instruction per SIMD, using the in-kernel clock (s_memtime vs
// s_memrealtime at 100 MHz) to convert wall time into cycles.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

#define REP 4096

template <int KIND>
__global__ __launch_bounds__(64) void body(uint32_t *out, uint64_t *clk) {
  uint32_t a = threadIdx.x, b = a * 3u, c = a * 5u, d = a * 7u;
  uint32_t s0 = blockIdx.x, s1 = s0 * 3u;
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
  const uint64_t r0 = __builtin_amdgcn_s_memrealtime();
  for (int i = 0; i < REP; ++i) {
    if (KIND == 0) {   // 8 independent v_add_u32
      asm volatile(
          "v_add_u32 %0, %0, %1\n\tv_add_u32 %1, %1, %2\n\tv_add_u32 %2, %2, %3\n\t"
          "v_add_u32 %3, %3, %0\n\tv_xor_b32 %0, %0, %2\n\tv_xor_b32 %1, %1, %3\n\t"
          "v_and_b32 %2, %2, %0\n\tv_or_b32 %3, %3, %1\n\t"
          : "+v"(a), "+v"(b), "+v"(c), "+v"(d));
    } else if (KIND == 1) {  // 8 v_max_u32_dpp row_shr
      asm volatile(
          "v_max_u32_dpp %0, %0, %0 row_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
          "v_max_u32_dpp %1, %1, %1 row_shr:2 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
          "v_max_u32_dpp %2, %2, %2 row_shr:4 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
          "v_max_u32_dpp %3, %3, %3 row_shr:8 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
          "v_max_u32_dpp %0, %0, %0 row_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
          "v_max_u32_dpp %1, %1, %1 row_shr:2 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
          "v_max_u32_dpp %2, %2, %2 row_shr:4 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
          "v_max_u32_dpp %3, %3, %3 row_shr:8 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
          : "+v"(a), "+v"(b), "+v"(c), "+v"(d));
    } else if (KIND == 2) {  // 8 s_add_u32
      asm volatile(
          "s_add_u32 %0, %0, %1\n\ts_add_u32 %1, %1, %0\n\ts_add_u32 %0, %0, %1\n\t"
          "s_add_u32 %1, %1, %0\n\ts_xor_b32 %0, %0, %1\n\ts_xor_b32 %1, %1, %0\n\t"
          "s_and_b32 %0, %0, %1\n\ts_or_b32 %1, %1, %0\n\t"
          : "+s"(s0), "+s"(s1) : : "scc");
    } else if (KIND == 3) {  // 8 v_mul_lo_u32
      asm volatile(
          "v_mul_lo_u32 %0, %0, %1\n\tv_mul_lo_u32 %1, %1, %2\n\tv_mul_lo_u32 %2, %2, %3\n\t"
          "v_mul_lo_u32 %3, %3, %0\n\tv_mul_lo_u32 %0, %0, %2\n\tv_mul_lo_u32 %1, %1, %3\n\t"
          "v_mul_lo_u32 %2, %2, %0\n\tv_mul_lo_u32 %3, %3, %1\n\t"
          : "+v"(a), "+v"(b), "+v"(c), "+v"(d));
    } else {                 // 4 VALU + 4 SALU interleaved
      asm volatile(
          "v_add_u32 %0, %0, %1\n\ts_add_u32 %4, %4, %5\n\tv_add_u32 %1, %1, %2\n\t"
          "s_add_u32 %5, %5, %4\n\tv_add_u32 %2, %2, %3\n\ts_xor_b32 %4, %4, %5\n\t"
          "v_add_u32 %3, %3, %0\n\ts_xor_b32 %5, %5, %4\n\t"
          : "+v"(a), "+v"(b), "+v"(c), "+v"(d), "+s"(s0), "+s"(s1) : : "scc");
    }
  }
  const uint64_t t1 = __builtin_amdgcn_s_memtime();
  const uint64_t r1 = __builtin_amdgcn_s_memrealtime();
  out[blockIdx.x * 64 + threadIdx.x] = a ^ b ^ c ^ d ^ s0 ^ s1;
  if (threadIdx.x == 0) {
    clk[blockIdx.x * 2] = t1 - t0;
    clk[blockIdx.x * 2 + 1] = r1 - r0;
  }
}

template <int K>
void run(const char *name, int grid, uint32_t *out, uint64_t *clk) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipLaunchKernelGGL(body<K>, dim3(grid), dim3(64), 0, 0, out, clk);
  hipEventRecord(e0, 0);
  hipLaunchKernelGGL(body<K>, dim3(grid), dim3(64), 0, 0, out, clk);
  hipEventRecord(e1, 0);
  hipEventSynchronize(e1);
  float ms = 0;
  hipEventElapsedTime(&ms, e0, e1);
  uint64_t h[2];
  hipMemcpy(h, clk, 16, hipMemcpyDeviceToHost);
  const double ghz = (double)h[0] / ((double)h[1] * 10.0);   // memrealtime 100 MHz
  const double instr_per_simd = (double)grid / 1024.0 * REP * 8.0;
  const double cyc = ms * 1e-3 * ghz * 1e9;
  printf("%-22s grid %6d  %.3f ms  clk %.2f GHz  cycles per wave-instr per SIMD %.2f\n", name,
         grid, ms, ghz, cyc / instr_per_simd);
}

int main() {
  uint32_t *out;
  uint64_t *clk;
  const int grid = 256 * 4 * 8;
  hipMalloc(&out, grid * 64 * 4);
  hipMalloc(&clk, grid * 16);
  for (int g : {256 * 4, 256 * 4 * 2, grid}) {
    run<0>("v_add/xor/and/or", g, out, clk);
    run<1>("v_max_u32_dpp", g, out, clk);
    run<2>("s_add/xor", g, out, clk);
    run<3>("v_mul_lo_u32", g, out, clk);
    run<4>("4 valu + 4 salu", g, out, clk);
  }
  return 0;
}
