// Micro-benchmark: LDS cost per wave-instruction on gfx950 at the lz4_tiles
// occupancy (one-wave workgroups, ~5 KB of LDS each -> 8 waves per SIMD), for
// aligned and misaligned ds_read/ds_write of 1..8 bytes.  Prints CU cycles
// per wave-instruction (wall time x clock / instructions per CU).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define REP 1024

// 8 accesses per asm block at base + 0, 64*W, 128*W ... (no two lanes of one
// instruction share a dword unless STRIDE says so)
#define R8(op, O1, O2, O3, O4, O5, O6, O7)                                              \
  asm volatile(op " %0, %8\n\t" op " %1, %8 offset:" O1 "\n\t" op " %2, %8 offset:" O2    \
               "\n\t" op " %3, %8 offset:" O3 "\n\t" op " %4, %8 offset:" O4 "\n\t" op      \
               " %5, %8 offset:" O5 "\n\t" op " %6, %8 offset:" O6 "\n\t" op " %7, %8 offset:" \
               O7 "\n\ts_waitcnt lgkmcnt(0)"                                                 \
               : "=v"(r[0]), "=v"(r[1]), "=v"(r[2]), "=v"(r[3]), "=v"(r[4]), "=v"(r[5]),    \
                 "=v"(r[6]), "=v"(r[7])                                                       \
               : "v"(adr)                                                                    \
               : "memory")
#define W8(op, O1, O2, O3, O4, O5, O6, O7)                                              \
  asm volatile(op " %0, %1\n\t" op " %0, %1 offset:" O1 "\n\t" op " %0, %1 offset:" O2    \
               "\n\t" op " %0, %1 offset:" O3 "\n\t" op " %0, %1 offset:" O4 "\n\t" op      \
               " %0, %1 offset:" O5 "\n\t" op " %0, %1 offset:" O6 "\n\t" op " %0, %1 offset:" \
               O7 "\n\ts_waitcnt lgkmcnt(0)"                                                 \
               :                                                                             \
               : "v"(adr), "v"(val)                                                          \
               : "memory")

template <int K>
__global__ __launch_bounds__(64) void body(uint32_t *out, uint64_t *clk) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[5056];
  const int lane = threadIdx.x;
  for (int i = lane; i < 5056 / 4; i += 64) reinterpret_cast<uint32_t *>(lds)[i] = i * 2654435761u;
  __syncthreads();
  typedef __attribute__((address_space(3))) uint8_t lu8;
  const uint32_t b0 = (uint32_t)(uintptr_t)(lu8 *)lds;
  // K: 0 rd b32 al, 1 rd b32 +1, 2 rd b64 al, 3 rd b64 +4, 4 rd b64 +1,
  //    5 wr b32 al, 6 wr b32 +1, 7 wr b64 al, 8 wr b64 +1, 9 wr b16 al, 10 wr b8,
  //    11 rd b64 +(5*lane) (lz4 lcp-like), 12 wr b64 +(5*lane)
  uint32_t adr;
  switch (K) {
    case 0: case 5: adr = b0 + 4 * lane; break;
    case 1: case 6: adr = b0 + 4 * lane + 1; break;
    case 2: case 7: adr = b0 + 8 * lane; break;
    case 3: adr = b0 + 8 * lane + 4; break;
    case 4: case 8: adr = b0 + 8 * lane + 1; break;
    case 9: adr = b0 + 2 * lane; break;
    case 10: adr = b0 + lane; break;
    default: adr = b0 + 5 * lane; break;
  }
  uint32_t acc = 0;
  uint32_t r[8];
  uint64_t r64[8];
  const uint32_t val = lane * 3u;
  const uint64_t val64 = lane * 7ull;
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
  const uint64_t q0 = __builtin_amdgcn_s_memrealtime();
  for (int i = 0; i < REP; ++i) {
    if (K == 0 || K == 1) {
      R8("ds_read_b32", "512", "1024", "1536", "2048", "2560", "3072", "3584");
      acc ^= r[0] ^ r[1] ^ r[2] ^ r[3] ^ r[4] ^ r[5] ^ r[6] ^ r[7];
    } else if (K == 2 || K == 3 || K == 4 || K == 11) {
      asm volatile(
          "ds_read_b64 %0, %8\n\tds_read_b64 %1, %8 offset:512\n\tds_read_b64 %2, %8 offset:1024\n\t"
          "ds_read_b64 %3, %8 offset:1536\n\tds_read_b64 %4, %8 offset:2048\n\t"
          "ds_read_b64 %5, %8 offset:2560\n\tds_read_b64 %6, %8 offset:3072\n\t"
          "ds_read_b64 %7, %8 offset:3584\n\ts_waitcnt lgkmcnt(0)"
          : "=v"(r64[0]), "=v"(r64[1]), "=v"(r64[2]), "=v"(r64[3]), "=v"(r64[4]), "=v"(r64[5]),
            "=v"(r64[6]), "=v"(r64[7])
          : "v"(adr)
          : "memory");
      acc ^= (uint32_t)(r64[0] ^ r64[1] ^ r64[2] ^ r64[3] ^ r64[4] ^ r64[5] ^ r64[6] ^ r64[7]);
    } else if (K == 5 || K == 6) {
      W8("ds_write_b32", "512", "1024", "1536", "2048", "2560", "3072", "3584");
    } else if (K == 7 || K == 8 || K == 12) {
      asm volatile(
          "ds_write_b64 %0, %1\n\tds_write_b64 %0, %1 offset:512\n\tds_write_b64 %0, %1 offset:1024\n\t"
          "ds_write_b64 %0, %1 offset:1536\n\tds_write_b64 %0, %1 offset:2048\n\t"
          "ds_write_b64 %0, %1 offset:2560\n\tds_write_b64 %0, %1 offset:3072\n\t"
          "ds_write_b64 %0, %1 offset:3584\n\ts_waitcnt lgkmcnt(0)"
          :
          : "v"(adr), "v"(val64)
          : "memory");
    } else if (K == 9) {
      W8("ds_write_b16", "512", "1024", "1536", "2048", "2560", "3072", "3584");
    } else {
      W8("ds_write_b8", "512", "1024", "1536", "2048", "2560", "3072", "3584");
    }
  }
  const uint64_t t1 = __builtin_amdgcn_s_memtime();
  const uint64_t q1 = __builtin_amdgcn_s_memrealtime();
  out[blockIdx.x * 64 + lane] = acc ^ lds[lane];
  if (lane == 0) {
    clk[blockIdx.x * 2] = t1 - t0;
    clk[blockIdx.x * 2 + 1] = q1 - q0;
  }
}

template <int K>
void run(const char *name, int grid, uint32_t *out, uint64_t *clk, int cus) {
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
  const double ghz = (double)h[0] / ((double)h[1] * 10.0);
  const double instr_per_cu = (double)grid / cus * REP * 8.0;
  const double cyc = ms * 1e-3 * ghz * 1e9;
  printf("%-26s %6.2f CU cycles per wave-instruction  (%.3f ms, %.2f GHz)\n", name,
         cyc / instr_per_cu, ms, ghz);
}

int main() {
  int cus = 0;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  const int grid = cus * 32 * 4;   // 32 resident one-wave workgroups per CU, 4 rounds
  uint32_t *out;
  uint64_t *clk;
  hipMalloc(&out, (size_t)grid * 64 * 4);
  hipMalloc(&clk, (size_t)grid * 16);
  run<0>("ds_read_b32 aligned", grid, out, clk, cus);
  run<1>("ds_read_b32 +1", grid, out, clk, cus);
  run<2>("ds_read_b64 aligned", grid, out, clk, cus);
  run<3>("ds_read_b64 +4", grid, out, clk, cus);
  run<4>("ds_read_b64 +1", grid, out, clk, cus);
  run<11>("ds_read_b64 5*lane", grid, out, clk, cus);
  run<5>("ds_write_b32 aligned", grid, out, clk, cus);
  run<6>("ds_write_b32 +1", grid, out, clk, cus);
  run<7>("ds_write_b64 aligned", grid, out, clk, cus);
  run<8>("ds_write_b64 +1", grid, out, clk, cus);
  run<12>("ds_write_b64 5*lane", grid, out, clk, cus);
  run<9>("ds_write_b16 aligned", grid, out, clk, cus);
  run<10>("ds_write_b8", grid, out, clk, cus);
  return 0;
}
