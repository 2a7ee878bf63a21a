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
  if (KIND == 35 || KIND == 36)
    asm volatile("s_mov_b64 vcc, %0" : : "s"((uint64_t)s0 * 0x9E3779B97F4A7C15ull) : "vcc");
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
    } else if (KIND == 5) {  // 8 v_lshlrev_b64 (4 chains of 64-bit pairs)
      uint64_t x = ((uint64_t)a << 32) | b, y = ((uint64_t)c << 32) | d;
      asm volatile(
          "v_lshlrev_b64 %0, %2, %0\n\tv_lshrrev_b64 %1, %3, %1\n\t"
          "v_lshlrev_b64 %0, %3, %0\n\tv_lshrrev_b64 %1, %2, %1\n\t"
          "v_lshlrev_b64 %0, %2, %0\n\tv_lshrrev_b64 %1, %3, %1\n\t"
          "v_lshlrev_b64 %0, %3, %0\n\tv_lshrrev_b64 %1, %2, %1\n\t"
          : "+v"(x), "+v"(y) : "v"(a & 7u), "v"(c & 7u));
      a = (uint32_t)x; b = (uint32_t)(x >> 32); c = (uint32_t)y; d = (uint32_t)(y >> 32);
    } else if (KIND == 6) {  // 8 v_alignbyte_b32
      asm volatile(
          "v_alignbyte_b32 %0, %1, %0, %2\n\tv_alignbyte_b32 %1, %2, %1, %3\n\t"
          "v_alignbyte_b32 %2, %3, %2, %0\n\tv_alignbyte_b32 %3, %0, %3, %1\n\t"
          "v_alignbyte_b32 %0, %1, %0, %2\n\tv_alignbyte_b32 %1, %2, %1, %3\n\t"
          "v_alignbyte_b32 %2, %3, %2, %0\n\tv_alignbyte_b32 %3, %0, %3, %1\n\t"
          : "+v"(a), "+v"(b), "+v"(c), "+v"(d));
    } else if (KIND == 7) {  // 8 v_cndmask_b32 on vcc-free SGPR masks
      asm volatile(
          "v_cndmask_b32_e64 %0, %0, %1, %4\n\tv_cndmask_b32_e64 %1, %1, %2, %5\n\t"
          "v_cndmask_b32_e64 %2, %2, %3, %4\n\tv_cndmask_b32_e64 %3, %3, %0, %5\n\t"
          "v_cndmask_b32_e64 %0, %0, %1, %5\n\tv_cndmask_b32_e64 %1, %1, %2, %4\n\t"
          "v_cndmask_b32_e64 %2, %2, %3, %5\n\tv_cndmask_b32_e64 %3, %3, %0, %4\n\t"
          : "+v"(a), "+v"(b), "+v"(c), "+v"(d)
          : "s"((uint64_t)s0 * 0x9E3779B97F4A7C15ull), "s"((uint64_t)s1 * 0xC2B2AE3D27D4EB4Full));
    } else if (KIND == 8) {  // 8 v_add3_u32 / v_lshl_add_u32 (VOP3 three-operand)
      asm volatile(
          "v_add3_u32 %0, %0, %1, %2\n\tv_lshl_add_u32 %1, %1, 2, %2\n\t"
          "v_add3_u32 %2, %2, %3, %0\n\tv_lshl_add_u32 %3, %3, 3, %0\n\t"
          "v_add3_u32 %0, %0, %1, %2\n\tv_lshl_add_u32 %1, %1, 2, %3\n\t"
          "v_add3_u32 %2, %2, %3, %1\n\tv_lshl_add_u32 %3, %3, 3, %2\n\t"
          : "+v"(a), "+v"(b), "+v"(c), "+v"(d));
    } else if (KIND == 9) {  // 8 v_mbcnt_lo/hi
      asm volatile(
          "v_mbcnt_lo_u32_b32 %0, %4, %0\n\tv_mbcnt_hi_u32_b32 %1, %4, %1\n\t"
          "v_mbcnt_lo_u32_b32 %2, %4, %2\n\tv_mbcnt_hi_u32_b32 %3, %4, %3\n\t"
          "v_mbcnt_lo_u32_b32 %0, %4, %0\n\tv_mbcnt_hi_u32_b32 %1, %4, %1\n\t"
          "v_mbcnt_lo_u32_b32 %2, %4, %2\n\tv_mbcnt_hi_u32_b32 %3, %4, %3\n\t"
          : "+v"(a), "+v"(b), "+v"(c), "+v"(d) : "s"(s0));
    } else if (KIND == 10) { // 8 v_perm_b32
      asm volatile(
          "v_perm_b32 %0, %1, %0, %4\n\tv_perm_b32 %1, %2, %1, %4\n\t"
          "v_perm_b32 %2, %3, %2, %4\n\tv_perm_b32 %3, %0, %3, %4\n\t"
          "v_perm_b32 %0, %1, %0, %4\n\tv_perm_b32 %1, %2, %1, %4\n\t"
          "v_perm_b32 %2, %3, %2, %4\n\tv_perm_b32 %3, %0, %3, %4\n\t"
          : "+v"(a), "+v"(b), "+v"(c), "+v"(d) : "s"(0x05040100u));
    } else if (KIND == 11) { // 8 v_mov_b32_dpp wave_shr:1
      asm volatile(
          "v_mov_b32_dpp %0, %1 wave_shr:1 row_mask:0xf bank_mask:0xf\n\t"
          "v_mov_b32_dpp %1, %2 wave_shr:1 row_mask:0xf bank_mask:0xf\n\t"
          "v_mov_b32_dpp %2, %3 wave_shr:1 row_mask:0xf bank_mask:0xf\n\t"
          "v_mov_b32_dpp %3, %0 wave_shr:1 row_mask:0xf bank_mask:0xf\n\t"
          "v_mov_b32_dpp %0, %1 wave_shr:1 row_mask:0xf bank_mask:0xf\n\t"
          "v_mov_b32_dpp %1, %2 wave_shr:1 row_mask:0xf bank_mask:0xf\n\t"
          "v_mov_b32_dpp %2, %3 wave_shr:1 row_mask:0xf bank_mask:0xf\n\t"
          "v_mov_b32_dpp %3, %0 wave_shr:1 row_mask:0xf bank_mask:0xf\n\t"
          : "+v"(a), "+v"(b), "+v"(c), "+v"(d));
    } else if (KIND == 12) { // 8 v_bfe_u32 / v_and_or_b32
      asm volatile(
          "v_bfe_u32 %0, %1, 3, 9\n\tv_and_or_b32 %1, %2, %0, %3\n\t"
          "v_bfe_u32 %2, %3, 5, 7\n\tv_and_or_b32 %3, %0, %2, %1\n\t"
          "v_bfe_u32 %0, %1, 3, 9\n\tv_and_or_b32 %1, %2, %0, %3\n\t"
          "v_bfe_u32 %2, %3, 5, 7\n\tv_and_or_b32 %3, %0, %2, %1\n\t"
          : "+v"(a), "+v"(b), "+v"(c), "+v"(d));
    } else if (KIND == 13) { // 8 v_cmp_lt_u32 -> SGPR pairs
      uint64_t m0 = 0, m1 = 0;
      asm volatile(
          "v_cmp_lt_u32_e64 %4, %0, %1\n\tv_cmp_lt_u32_e64 %5, %2, %3\n\t"
          "v_cmp_lt_u32_e64 %4, %1, %2\n\tv_cmp_lt_u32_e64 %5, %3, %0\n\t"
          "v_cmp_lt_u32_e64 %4, %0, %2\n\tv_cmp_lt_u32_e64 %5, %1, %3\n\t"
          "v_cmp_lt_u32_e64 %4, %2, %1\n\tv_cmp_lt_u32_e64 %5, %3, %1\n\t"
          : "+v"(a), "+v"(b), "+v"(c), "+v"(d), "=s"(m0), "=s"(m1));
      s0 ^= (uint32_t)m0;
      s1 ^= (uint32_t)(m1 >> 32);
    } else if (KIND == 14) { // 8 v_cndmask_b32_e32 (mask in vcc)
      asm volatile(
          "s_mov_b64 vcc, %4\n\t"
          "v_cndmask_b32_e32 %0, %0, %1, vcc\n\tv_cndmask_b32_e32 %1, %1, %2, vcc\n\t"
          "v_cndmask_b32_e32 %2, %2, %3, vcc\n\tv_cndmask_b32_e32 %3, %3, %0, vcc\n\t"
          "v_cndmask_b32_e32 %0, %0, %1, vcc\n\tv_cndmask_b32_e32 %1, %1, %2, vcc\n\t"
          "v_cndmask_b32_e32 %2, %2, %3, vcc\n\tv_cndmask_b32_e32 %3, %3, %0, vcc\n\t"
          : "+v"(a), "+v"(b), "+v"(c), "+v"(d)
          : "s"((uint64_t)s0 * 0x9E3779B97F4A7C15ull) : "vcc");
    } else if (KIND == 15) { // 8 VOP2 with a 32-bit literal
      asm volatile(
          "v_and_b32_e32 %0, 0x7ff0f, %0\n\tv_add_u32_e32 %1, 0x12345, %1\n\t"
          "v_xor_b32_e32 %2, 0x55aa55, %2\n\tv_or_b32_e32 %3, 0x8000, %3\n\t"
          "v_and_b32_e32 %0, 0x7ff0f, %0\n\tv_add_u32_e32 %1, 0x12345, %1\n\t"
          "v_xor_b32_e32 %2, 0x55aa55, %2\n\tv_or_b32_e32 %3, 0x8000, %3\n\t"
          : "+v"(a), "+v"(b), "+v"(c), "+v"(d));
    } else if (KIND == 16) { // 8 v_lshlrev_b32_e32 / v_lshrrev_b32_e32 / v_max_u32_e32 / v_sub_u32_e32
      asm volatile(
          "v_lshlrev_b32_e32 %0, 3, %0\n\tv_lshrrev_b32_e32 %1, 2, %1\n\t"
          "v_max_u32_e32 %2, %2, %3\n\tv_sub_u32_e32 %3, %3, %0\n\t"
          "v_lshlrev_b32_e32 %0, %1, %0\n\tv_lshrrev_b32_e32 %1, %2, %1\n\t"
          "v_min_u32_e32 %2, %2, %0\n\tv_sub_u32_e32 %3, %3, %1\n\t"
          : "+v"(a), "+v"(b), "+v"(c), "+v"(d));
    } else if (KIND == 17) { // 8 v_cmp_*_e32 -> vcc (VOPC)
      asm volatile(
          "v_cmp_lt_u32_e32 vcc, %0, %1\n\tv_cmp_lt_u32_e32 vcc, %2, %3\n\t"
          "v_cmp_lt_u32_e32 vcc, %1, %2\n\tv_cmp_lt_u32_e32 vcc, %3, %0\n\t"
          "v_cmp_lt_u32_e32 vcc, %0, %2\n\tv_cmp_lt_u32_e32 vcc, %1, %3\n\t"
          "v_cmp_lt_u32_e32 vcc, %2, %1\n\tv_cmp_lt_u32_e32 vcc, %3, %1\n\t"
          "v_cndmask_b32_e32 %0, %0, %1, vcc\n\t"
          : "+v"(a), "+v"(b), "+v"(c), "+v"(d) : : "vcc");
    } else if (KIND == 18) { // 8 v_mul_u32_u24_e32 (VOP2) / v_mad_u32_u24 (VOP3)
      asm volatile(
          "v_mul_u32_u24_e32 %0, %1, %0\n\tv_mul_u32_u24_e32 %1, %2, %1\n\t"
          "v_mul_u32_u24_e32 %2, %3, %2\n\tv_mul_u32_u24_e32 %3, %0, %3\n\t"
          "v_mul_u32_u24_e32 %0, %1, %0\n\tv_mul_u32_u24_e32 %1, %2, %1\n\t"
          "v_mul_u32_u24_e32 %2, %3, %2\n\tv_mul_u32_u24_e32 %3, %0, %3\n\t"
          : "+v"(a), "+v"(b), "+v"(c), "+v"(d));
    } else if (KIND == 19) { // 8 VOP1: v_mov_b32 / v_not_b32 / v_ffbl_b32 / v_bfrev_b32
      asm volatile(
          "v_not_b32_e32 %0, %1\n\tv_ffbl_b32_e32 %1, %2\n\t"
          "v_bfrev_b32_e32 %2, %3\n\tv_not_b32_e32 %3, %0\n\t"
          "v_ffbl_b32_e32 %0, %1\n\tv_bfrev_b32_e32 %1, %2\n\t"
          "v_not_b32_e32 %2, %3\n\tv_ffbl_b32_e32 %3, %0\n\t"
          : "+v"(a), "+v"(b), "+v"(c), "+v"(d));
    } else if (KIND == 20) { // 8 VOP2 with an SGPR operand
      asm volatile(
          "v_add_u32_e32 %0, %4, %0\n\tv_and_b32_e32 %1, %4, %1\n\t"
          "v_xor_b32_e32 %2, %4, %2\n\tv_or_b32_e32 %3, %4, %3\n\t"
          "v_add_u32_e32 %0, %4, %0\n\tv_and_b32_e32 %1, %4, %1\n\t"
          "v_xor_b32_e32 %2, %4, %2\n\tv_or_b32_e32 %3, %4, %3\n\t"
          : "+v"(a), "+v"(b), "+v"(c), "+v"(d) : "s"(s0));
    } else if (KIND == 21) { // 8 v_add_u32_e64 (VOP2 op, VOP3 encoding)
      asm volatile(
          "v_add_u32_e64 %0, %0, %1\n\tv_add_u32_e64 %1, %1, %2\n\t"
          "v_add_u32_e64 %2, %2, %3\n\tv_add_u32_e64 %3, %3, %0\n\t"
          "v_xor_b32_e64 %0, %0, %2\n\tv_xor_b32_e64 %1, %1, %3\n\t"
          "v_and_b32_e64 %2, %2, %0\n\tv_or_b32_e64 %3, %3, %1\n\t"
          : "+v"(a), "+v"(b), "+v"(c), "+v"(d));
    } else if (KIND == 22) { // 8 v_readfirstlane / v_readlane (VALU -> SGPR)
      uint32_t t0, t1;
      asm volatile(
          "v_readfirstlane_b32 %4, %0\n\tv_readlane_b32 %5, %1, 63\n\t"
          "v_readfirstlane_b32 %4, %2\n\tv_readlane_b32 %5, %3, 63\n\t"
          "v_readfirstlane_b32 %4, %1\n\tv_readlane_b32 %5, %0, 63\n\t"
          "v_readfirstlane_b32 %4, %3\n\tv_readlane_b32 %5, %2, 63\n\t"
          : "+v"(a), "+v"(b), "+v"(c), "+v"(d), "=s"(t0), "=s"(t1));
      s0 ^= t0;
      s1 ^= t1;
    } else if (KIND == 23) { // 8 v_mov_b32_e32 (VOP1 copy)
      asm volatile(
          "v_mov_b32_e32 %0, %1\n\tv_mov_b32_e32 %1, %2\n\tv_mov_b32_e32 %2, %3\n\t"
          "v_mov_b32_e32 %3, %0\n\tv_mov_b32_e32 %0, %2\n\tv_mov_b32_e32 %1, %3\n\t"
          "v_mov_b32_e32 %2, %0\n\tv_mov_b32_e32 %3, %1\n\t"
          : "+v"(a), "+v"(b), "+v"(c), "+v"(d));
    } else if (KIND == 24) { // 8 v_sub_u32_e32
      asm volatile(
          "v_sub_u32_e32 %0, %0, %1\n\tv_sub_u32_e32 %1, %1, %2\n\tv_sub_u32_e32 %2, %2, %3\n\t"
          "v_sub_u32_e32 %3, %3, %0\n\tv_sub_u32_e32 %0, %0, %2\n\tv_sub_u32_e32 %1, %1, %3\n\t"
          "v_sub_u32_e32 %2, %2, %0\n\tv_sub_u32_e32 %3, %3, %1\n\t"
          : "+v"(a), "+v"(b), "+v"(c), "+v"(d));
    } else if (KIND == 25) { // 8 v_lshlrev_b32_e32 / v_lshrrev_b32_e32 (VGPR shift)
      asm volatile(
          "v_lshlrev_b32_e32 %0, %1, %0\n\tv_lshrrev_b32_e32 %1, %2, %1\n\t"
          "v_lshlrev_b32_e32 %2, %3, %2\n\tv_lshrrev_b32_e32 %3, %0, %3\n\t"
          "v_lshlrev_b32_e32 %0, 3, %0\n\tv_lshrrev_b32_e32 %1, 2, %1\n\t"
          "v_lshlrev_b32_e32 %2, 5, %2\n\tv_lshrrev_b32_e32 %3, 7, %3\n\t"
          : "+v"(a), "+v"(b), "+v"(c), "+v"(d));
    } else if (KIND == 26) { // 8 v_max_u32_e32 / v_min_u32_e32
      asm volatile(
          "v_max_u32_e32 %0, %0, %1\n\tv_min_u32_e32 %1, %1, %2\n\tv_max_u32_e32 %2, %2, %3\n\t"
          "v_min_u32_e32 %3, %3, %0\n\tv_max_u32_e32 %0, %0, %2\n\tv_min_u32_e32 %1, %1, %3\n\t"
          "v_max_u32_e32 %2, %2, %0\n\tv_min_u32_e32 %3, %3, %1\n\t"
          : "+v"(a), "+v"(b), "+v"(c), "+v"(d));
    } else if (KIND == 27) { // 8 v_lshl_add_u64 (64-bit address arithmetic)
      uint64_t x = ((uint64_t)a << 32) | b, y = ((uint64_t)c << 32) | d;
      asm volatile(
          "v_lshl_add_u64 %0, %0, 2, %1\n\tv_lshl_add_u64 %1, %1, 1, %0\n\t"
          "v_lshl_add_u64 %0, %0, 0, %1\n\tv_lshl_add_u64 %1, %1, 3, %0\n\t"
          "v_lshl_add_u64 %0, %0, 2, %1\n\tv_lshl_add_u64 %1, %1, 1, %0\n\t"
          "v_lshl_add_u64 %0, %0, 0, %1\n\tv_lshl_add_u64 %1, %1, 3, %0\n\t"
          : "+v"(x), "+v"(y));
      a = (uint32_t)x; b = (uint32_t)(x >> 32); c = (uint32_t)y; d = (uint32_t)(y >> 32);
    } else if (KIND == 28) { // 8 s_nop 0
      asm volatile("s_nop 0\n\ts_nop 0\n\ts_nop 0\n\ts_nop 0\n\ts_nop 0\n\ts_nop 0\n\ts_nop 0\n\ts_nop 0");
    } else if (KIND == 29) { // 8 v_bfi_b32 / v_xad_u32 / v_min3_u32 / v_max3_i32
      asm volatile(
          "v_bfi_b32 %0, %1, %2, %3\n\tv_xad_u32 %1, %2, %3, %0\n\t"
          "v_min3_u32 %2, %3, %0, %1\n\tv_max3_i32 %3, %0, %1, %2\n\t"
          "v_bfi_b32 %0, %1, %2, %3\n\tv_xad_u32 %1, %2, %3, %0\n\t"
          "v_min3_u32 %2, %3, %0, %1\n\tv_max3_i32 %3, %0, %1, %2\n\t"
          : "+v"(a), "+v"(b), "+v"(c), "+v"(d));
    } else if (KIND == 30) { // 8 v_cndmask_b32_e32 on a VCC written by VALU (v_cmp_e32)
      asm volatile(
          "v_cmp_lt_u32_e32 vcc, %0, %1\n\t"
          "v_cndmask_b32_e32 %0, %0, %1, vcc\n\tv_cndmask_b32_e32 %1, %1, %2, vcc\n\t"
          "v_cndmask_b32_e32 %2, %2, %3, vcc\n\tv_cndmask_b32_e32 %3, %3, %0, vcc\n\t"
          "v_cndmask_b32_e32 %0, %0, %1, vcc\n\tv_cndmask_b32_e32 %1, %1, %2, vcc\n\t"
          "v_cndmask_b32_e32 %2, %2, %3, vcc\n\t"
          : "+v"(a), "+v"(b), "+v"(c), "+v"(d) : : "vcc");
    } else if (KIND == 31) { // 4 s_and_b64 mask -> v_cndmask_b32_e64 at once (SALU -> VALU lane mask)
      uint64_t m = 0;
      asm volatile(
          "s_and_b64 %4, %5, %6\n\tv_cndmask_b32_e64 %0, %0, %1, %4\n\t"
          "s_xor_b64 %4, %4, %6\n\tv_cndmask_b32_e64 %1, %1, %2, %4\n\t"
          "s_and_b64 %4, %4, %5\n\tv_cndmask_b32_e64 %2, %2, %3, %4\n\t"
          "s_or_b64 %4, %4, %6\n\tv_cndmask_b32_e64 %3, %3, %0, %4\n\t"
          : "+v"(a), "+v"(b), "+v"(c), "+v"(d), "=&s"(m)
          : "s"((uint64_t)s0 * 0x9E3779B97F4A7C15ull), "s"((uint64_t)s1 * 0xC2B2AE3D27D4EB4Full)
          : "scc");
      s0 ^= (uint32_t)m;
    } else if (KIND == 32) { // 4 v_cmp_e64 -> s_and_saveexec-free: ballot then s_bcnt1 (VALU -> SALU)
      uint64_t m = 0;
      uint32_t cnt = 0;
      asm volatile(
          "v_cmp_lt_u32_e64 %4, %0, %1\n\ts_bcnt1_i32_b64 %5, %4\n\t"
          "v_cmp_lt_u32_e64 %4, %2, %3\n\ts_bcnt1_i32_b64 %5, %4\n\t"
          "v_cmp_lt_u32_e64 %4, %1, %2\n\ts_bcnt1_i32_b64 %5, %4\n\t"
          "v_cmp_lt_u32_e64 %4, %3, %0\n\ts_bcnt1_i32_b64 %5, %4\n\t"
          : "+v"(a), "+v"(b), "+v"(c), "+v"(d), "=&s"(m), "=&s"(cnt) : : "scc");
      s0 ^= cnt;
    } else if (KIND == 33) { // 8 v_writelane_b32 (SGPR lane select)
      asm volatile(
          "v_writelane_b32 %0, %4, 3\n\tv_writelane_b32 %1, %4, 7\n\t"
          "v_writelane_b32 %2, %4, 11\n\tv_writelane_b32 %3, %4, 13\n\t"
          "v_writelane_b32 %0, %4, 17\n\tv_writelane_b32 %1, %4, 19\n\t"
          "v_writelane_b32 %2, %4, 23\n\tv_writelane_b32 %3, %4, 29\n\t"
          : "+v"(a), "+v"(b), "+v"(c), "+v"(d) : "s"(s0));
    } else if (KIND == 34) { // 8 v_ffbl_b32 alone
      asm volatile(
          "v_ffbl_b32_e32 %0, %1\n\tv_ffbl_b32_e32 %1, %2\n\tv_ffbl_b32_e32 %2, %3\n\t"
          "v_ffbl_b32_e32 %3, %0\n\tv_ffbl_b32_e32 %0, %2\n\tv_ffbl_b32_e32 %1, %3\n\t"
          "v_ffbl_b32_e32 %2, %0\n\tv_ffbl_b32_e32 %3, %1\n\t"
          : "+v"(a), "+v"(b), "+v"(c), "+v"(d));
    } else if (KIND == 35) { // 8 v_cndmask_b32_e32 on a VCC set once before the loop
      asm volatile(
          "v_cndmask_b32_e32 %0, %0, %1, vcc\n\tv_cndmask_b32_e32 %1, %1, %2, vcc\n\t"
          "v_cndmask_b32_e32 %2, %2, %3, vcc\n\tv_cndmask_b32_e32 %3, %3, %0, vcc\n\t"
          "v_cndmask_b32_e32 %0, %0, %1, vcc\n\tv_cndmask_b32_e32 %1, %1, %2, vcc\n\t"
          "v_cndmask_b32_e32 %2, %2, %3, vcc\n\tv_cndmask_b32_e32 %3, %3, %0, vcc\n\t"
          : "+v"(a), "+v"(b), "+v"(c), "+v"(d) : : );
    } else if (KIND == 36) { // 8 v_cndmask_b32_e64 reading vcc (set once before the loop)
      asm volatile(
          "v_cndmask_b32_e64 %0, %0, %1, vcc\n\tv_cndmask_b32_e64 %1, %1, %2, vcc\n\t"
          "v_cndmask_b32_e64 %2, %2, %3, vcc\n\tv_cndmask_b32_e64 %3, %3, %0, vcc\n\t"
          "v_cndmask_b32_e64 %0, %0, %1, vcc\n\tv_cndmask_b32_e64 %1, %1, %2, vcc\n\t"
          "v_cndmask_b32_e64 %2, %2, %3, vcc\n\tv_cndmask_b32_e64 %3, %3, %0, vcc\n\t"
          : "+v"(a), "+v"(b), "+v"(c), "+v"(d) : : );
    } else if (KIND == 37) { // 4 x (v_cmp_e64 -> SGPR pair, v_cndmask_b32_e64 on it at once)
      uint64_t m = 0;
      asm volatile(
          "v_cmp_lt_u32_e64 %4, %0, %1\n\tv_cndmask_b32_e64 %1, %1, %2, %4\n\t"
          "v_cmp_lt_u32_e64 %4, %2, %3\n\tv_cndmask_b32_e64 %3, %3, %0, %4\n\t"
          "v_cmp_lt_u32_e64 %4, %1, %2\n\tv_cndmask_b32_e64 %0, %0, %1, %4\n\t"
          "v_cmp_lt_u32_e64 %4, %3, %0\n\tv_cndmask_b32_e64 %2, %2, %3, %4\n\t"
          : "+v"(a), "+v"(b), "+v"(c), "+v"(d), "=&s"(m));
    } else if (KIND == 38) { // 4 x (v_cmp_e32 -> vcc, v_cndmask_b32_e32 on it at once)
      asm volatile(
          "v_cmp_lt_u32_e32 vcc, %0, %1\n\tv_cndmask_b32_e32 %1, %1, %2, vcc\n\t"
          "v_cmp_lt_u32_e32 vcc, %2, %3\n\tv_cndmask_b32_e32 %3, %3, %0, vcc\n\t"
          "v_cmp_lt_u32_e32 vcc, %1, %2\n\tv_cndmask_b32_e32 %0, %0, %1, vcc\n\t"
          "v_cmp_lt_u32_e32 vcc, %3, %0\n\tv_cndmask_b32_e32 %2, %2, %3, vcc\n\t"
          : "+v"(a), "+v"(b), "+v"(c), "+v"(d) : : "vcc");
    } else if (KIND == 39) { // 8 v_cndmask_b32_e64 with an inline-constant operand (0 / 1)
      asm volatile(
          "v_cndmask_b32_e64 %0, 0, %1, %4\n\tv_cndmask_b32_e64 %1, %2, 1, %5\n\t"
          "v_cndmask_b32_e64 %2, 0, %3, %4\n\tv_cndmask_b32_e64 %3, %0, 1, %5\n\t"
          "v_cndmask_b32_e64 %0, 0, %1, %5\n\tv_cndmask_b32_e64 %1, %2, 1, %4\n\t"
          "v_cndmask_b32_e64 %2, 0, %3, %5\n\tv_cndmask_b32_e64 %3, %0, 1, %4\n\t"
          : "+v"(a), "+v"(b), "+v"(c), "+v"(d)
          : "s"((uint64_t)s0 * 0x9E3779B97F4A7C15ull), "s"((uint64_t)s1 * 0xC2B2AE3D27D4EB4Full));
    } else if (KIND == 40) { // 8 v_mov_b32_e32 from an SGPR
      asm volatile(
          "v_mov_b32_e32 %0, %4\n\tv_mov_b32_e32 %1, %5\n\tv_mov_b32_e32 %2, %4\n\t"
          "v_mov_b32_e32 %3, %5\n\tv_mov_b32_e32 %0, %5\n\tv_mov_b32_e32 %1, %4\n\t"
          "v_mov_b32_e32 %2, %5\n\tv_mov_b32_e32 %3, %4\n\t"
          : "+v"(a), "+v"(b), "+v"(c), "+v"(d) : "s"(s0), "s"(s1));
    } else if (KIND == 41) { // 8 v_lshl_or_b32 / v_add_lshl_u32 / v_lshl_add_u32
      asm volatile(
          "v_lshl_or_b32 %0, %1, 3, %2\n\tv_add_lshl_u32 %1, %2, %3, 2\n\t"
          "v_lshl_add_u32 %2, %3, 1, %0\n\tv_lshl_or_b32 %3, %0, 5, %1\n\t"
          "v_lshl_or_b32 %0, %1, 3, %2\n\tv_add_lshl_u32 %1, %2, %3, 2\n\t"
          "v_lshl_add_u32 %2, %3, 1, %0\n\tv_lshl_or_b32 %3, %0, 5, %1\n\t"
          : "+v"(a), "+v"(b), "+v"(c), "+v"(d));
    } else if (KIND == 42) { // 8 v_and_b32 with an SGPR operand (as the compiler emits for 64-bit masks)
      asm volatile(
          "v_and_b32_e32 %0, %4, %0\n\tv_and_b32_e32 %1, %5, %1\n\t"
          "v_and_b32_e32 %2, %4, %2\n\tv_and_b32_e32 %3, %5, %3\n\t"
          "v_and_b32_e32 %0, %5, %0\n\tv_and_b32_e32 %1, %4, %1\n\t"
          "v_and_b32_e32 %2, %5, %2\n\tv_and_b32_e32 %3, %4, %3\n\t"
          : "+v"(a), "+v"(b), "+v"(c), "+v"(d) : "s"(s0), "s"(s1));
    } else if (KIND == 43) { // 4 v_perm_b32 + 4 v_add_u32 interleaved (is the cost additive?)
      asm volatile(
          "v_perm_b32 %0, %1, %0, %4\n\tv_add_u32 %1, %1, %2\n\t"
          "v_perm_b32 %2, %3, %2, %4\n\tv_add_u32 %3, %3, %0\n\t"
          "v_perm_b32 %0, %1, %0, %4\n\tv_add_u32 %1, %1, %2\n\t"
          "v_perm_b32 %2, %3, %2, %4\n\tv_add_u32 %3, %3, %0\n\t"
          : "+v"(a), "+v"(b), "+v"(c), "+v"(d) : "s"(0x05040100u));
    } else if (KIND == 44) { // 4 v_cndmask_b32_e64 + 4 v_add_u32 interleaved
      asm volatile(
          "v_cndmask_b32_e64 %0, %0, %1, %4\n\tv_add_u32 %1, %1, %2\n\t"
          "v_cndmask_b32_e64 %2, %2, %3, %5\n\tv_add_u32 %3, %3, %0\n\t"
          "v_cndmask_b32_e64 %0, %0, %1, %5\n\tv_add_u32 %1, %1, %2\n\t"
          "v_cndmask_b32_e64 %2, %2, %3, %4\n\tv_add_u32 %3, %3, %0\n\t"
          : "+v"(a), "+v"(b), "+v"(c), "+v"(d)
          : "s"((uint64_t)s0 * 0x9E3779B97F4A7C15ull), "s"((uint64_t)s1 * 0xC2B2AE3D27D4EB4Full));
    } else if (KIND == 45) { // 4 v_max_u32_dpp + 4 v_add_u32 interleaved
      asm volatile(
          "v_max_u32_dpp %0, %0, %0 row_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\tv_add_u32 %1, %1, %2\n\t"
          "v_max_u32_dpp %2, %2, %2 row_shr:2 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\tv_add_u32 %3, %3, %0\n\t"
          "v_max_u32_dpp %0, %0, %0 row_shr:4 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\tv_add_u32 %1, %1, %2\n\t"
          "v_max_u32_dpp %2, %2, %2 row_shr:8 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\tv_add_u32 %3, %3, %0\n\t"
          : "+v"(a), "+v"(b), "+v"(c), "+v"(d));
    } else if (KIND == 46) { // 4 v_lshrrev_b32 + 4 v_add_u32 interleaved
      asm volatile(
          "v_lshrrev_b32 %0, 3, %0\n\tv_add_u32 %1, %1, %2\n\t"
          "v_lshrrev_b32 %2, 5, %2\n\tv_add_u32 %3, %3, %0\n\t"
          "v_lshrrev_b32 %0, 7, %0\n\tv_add_u32 %1, %1, %2\n\t"
          "v_lshrrev_b32 %2, 2, %2\n\tv_add_u32 %3, %3, %0\n\t"
          : "+v"(a), "+v"(b), "+v"(c), "+v"(d));
    } else if (KIND == 47) { // 4 v_perm_b32 + 4 v_cndmask_b32_e64 interleaved (two slow classes)
      asm volatile(
          "v_perm_b32 %0, %1, %0, %6\n\tv_cndmask_b32_e64 %1, %1, %2, %4\n\t"
          "v_perm_b32 %2, %3, %2, %6\n\tv_cndmask_b32_e64 %3, %3, %0, %5\n\t"
          "v_perm_b32 %0, %1, %0, %6\n\tv_cndmask_b32_e64 %1, %1, %2, %5\n\t"
          "v_perm_b32 %2, %3, %2, %6\n\tv_cndmask_b32_e64 %3, %3, %0, %4\n\t"
          : "+v"(a), "+v"(b), "+v"(c), "+v"(d)
          : "s"((uint64_t)s0 * 0x9E3779B97F4A7C15ull), "s"((uint64_t)s1 * 0xC2B2AE3D27D4EB4Full),
            "s"(0x05040100u));
    } else if (KIND == 48) { // 4 v_perm_b32 + 4 s_add (slow VALU beside SALU)
      asm volatile(
          "v_perm_b32 %0, %1, %0, %6\n\ts_add_u32 %4, %4, %5\n\t"
          "v_perm_b32 %2, %3, %2, %6\n\ts_add_u32 %5, %5, %4\n\t"
          "v_perm_b32 %0, %1, %0, %6\n\ts_xor_b32 %4, %4, %5\n\t"
          "v_perm_b32 %2, %3, %2, %6\n\ts_xor_b32 %5, %5, %4\n\t"
          : "+v"(a), "+v"(b), "+v"(c), "+v"(d), "+s"(s0), "+s"(s1) : "s"(0x05040100u) : "scc");
    } else if (KIND == 50) { // 4 v_mbcnt + 4 v_add_u32 interleaved
      uint32_t t5 = 0;
      uint64_t m6 = 0;
      asm volatile(
          "v_mbcnt_lo_u32_b32 %0, %4, %0\n\tv_add_u32 %1, %1, %3\n\t"
          "v_mbcnt_hi_u32_b32 %2, %4, %2\n\tv_add_u32 %3, %3, %1\n\t"
          "v_mbcnt_lo_u32_b32 %0, %4, %0\n\tv_add_u32 %1, %1, %3\n\t"
          "v_mbcnt_hi_u32_b32 %2, %4, %2\n\tv_add_u32 %3, %3, %1\n\t"
          : "+v"(a), "+v"(b), "+v"(c), "+v"(d), "+s"(s0), "=&s"(t5), "=&s"(m6));
      s1 ^= t5 ^ (uint32_t)m6;
    } else if (KIND == 51) { // 4 v_readlane + 4 v_add_u32 interleaved
      uint32_t t5 = 0;
      uint64_t m6 = 0;
      asm volatile(
          "v_readlane_b32 %5, %0, 63\n\tv_add_u32 %1, %1, %3\n\t"
          "v_readfirstlane_b32 %5, %2\n\tv_add_u32 %3, %3, %1\n\t"
          "v_readlane_b32 %5, %0, 63\n\tv_add_u32 %1, %1, %3\n\t"
          "v_readfirstlane_b32 %5, %2\n\tv_add_u32 %3, %3, %1\n\t"
          : "+v"(a), "+v"(b), "+v"(c), "+v"(d), "+s"(s0), "=&s"(t5), "=&s"(m6));
      s1 ^= t5 ^ (uint32_t)m6;
    } else if (KIND == 52) { // 4 v_writelane + 4 v_add_u32 interleaved
      uint32_t t5 = 0;
      uint64_t m6 = 0;
      asm volatile(
          "v_writelane_b32 %0, %4, 5\n\tv_add_u32 %1, %1, %3\n\t"
          "v_writelane_b32 %2, %4, 9\n\tv_add_u32 %3, %3, %1\n\t"
          "v_writelane_b32 %0, %4, 5\n\tv_add_u32 %1, %1, %3\n\t"
          "v_writelane_b32 %2, %4, 9\n\tv_add_u32 %3, %3, %1\n\t"
          : "+v"(a), "+v"(b), "+v"(c), "+v"(d), "+s"(s0), "=&s"(t5), "=&s"(m6));
      s1 ^= t5 ^ (uint32_t)m6;
    } else if (KIND == 53) { // 4 v_alignbyte + 4 v_add_u32 interleaved
      uint32_t t5 = 0;
      uint64_t m6 = 0;
      asm volatile(
          "v_alignbyte_b32 %0, %1, %0, %3\n\tv_add_u32 %1, %1, %3\n\t"
          "v_alignbyte_b32 %2, %3, %2, %1\n\tv_add_u32 %3, %3, %1\n\t"
          "v_alignbyte_b32 %0, %1, %0, %3\n\tv_add_u32 %1, %1, %3\n\t"
          "v_alignbyte_b32 %2, %3, %2, %1\n\tv_add_u32 %3, %3, %1\n\t"
          : "+v"(a), "+v"(b), "+v"(c), "+v"(d), "+s"(s0), "=&s"(t5), "=&s"(m6));
      s1 ^= t5 ^ (uint32_t)m6;
    } else if (KIND == 54) { // 4 v_mul_lo_u32 + 4 v_add_u32 interleaved
      uint32_t t5 = 0;
      uint64_t m6 = 0;
      asm volatile(
          "v_mul_lo_u32 %0, %0, %1\n\tv_add_u32 %1, %1, %3\n\t"
          "v_mul_lo_u32 %2, %2, %3\n\tv_add_u32 %3, %3, %1\n\t"
          "v_mul_lo_u32 %0, %0, %1\n\tv_add_u32 %1, %1, %3\n\t"
          "v_mul_lo_u32 %2, %2, %3\n\tv_add_u32 %3, %3, %1\n\t"
          : "+v"(a), "+v"(b), "+v"(c), "+v"(d), "+s"(s0), "=&s"(t5), "=&s"(m6));
      s1 ^= t5 ^ (uint32_t)m6;
    } else if (KIND == 55) { // 4 v_bfe/bfi + 4 v_add_u32 interleaved
      uint32_t t5 = 0;
      uint64_t m6 = 0;
      asm volatile(
          "v_bfe_u32 %0, %1, 3, 9\n\tv_add_u32 %1, %1, %3\n\t"
          "v_bfi_b32 %2, %3, %1, %2\n\tv_add_u32 %3, %3, %1\n\t"
          "v_bfe_u32 %0, %1, 3, 9\n\tv_add_u32 %1, %1, %3\n\t"
          "v_bfi_b32 %2, %3, %1, %2\n\tv_add_u32 %3, %3, %1\n\t"
          : "+v"(a), "+v"(b), "+v"(c), "+v"(d), "+s"(s0), "=&s"(t5), "=&s"(m6));
      s1 ^= t5 ^ (uint32_t)m6;
    } else if (KIND == 56) { // 4 v_add3/lshl_add + 4 v_add_u32 interleaved
      uint32_t t5 = 0;
      uint64_t m6 = 0;
      asm volatile(
          "v_add3_u32 %0, %0, %1, %3\n\tv_add_u32 %1, %1, %3\n\t"
          "v_lshl_add_u32 %2, %3, 2, %2\n\tv_add_u32 %3, %3, %1\n\t"
          "v_add3_u32 %0, %0, %1, %3\n\tv_add_u32 %1, %1, %3\n\t"
          "v_lshl_add_u32 %2, %3, 2, %2\n\tv_add_u32 %3, %3, %1\n\t"
          : "+v"(a), "+v"(b), "+v"(c), "+v"(d), "+s"(s0), "=&s"(t5), "=&s"(m6));
      s1 ^= t5 ^ (uint32_t)m6;
    } else if (KIND == 57) { // 4 v_cmp_e64 + 4 v_add_u32 interleaved
      uint32_t t5 = 0;
      uint64_t m6 = 0;
      asm volatile(
          "v_cmp_lt_u32_e64 %6, %0, %1\n\tv_add_u32 %1, %1, %3\n\t"
          "v_cmp_lt_u32_e64 %6, %2, %3\n\tv_add_u32 %3, %3, %1\n\t"
          "v_cmp_lt_u32_e64 %6, %0, %1\n\tv_add_u32 %1, %1, %3\n\t"
          "v_cmp_lt_u32_e64 %6, %2, %3\n\tv_add_u32 %3, %3, %1\n\t"
          : "+v"(a), "+v"(b), "+v"(c), "+v"(d), "+s"(s0), "=&s"(t5), "=&s"(m6));
      s1 ^= t5 ^ (uint32_t)m6;
    } else if (KIND == 58) { // 4 v_ffbl + 4 v_add_u32 interleaved
      uint32_t t5 = 0;
      uint64_t m6 = 0;
      asm volatile(
          "v_ffbl_b32_e32 %0, %1\n\tv_add_u32 %1, %1, %3\n\t"
          "v_ffbl_b32_e32 %2, %3\n\tv_add_u32 %3, %3, %1\n\t"
          "v_ffbl_b32_e32 %0, %1\n\tv_add_u32 %1, %1, %3\n\t"
          "v_ffbl_b32_e32 %2, %3\n\tv_add_u32 %3, %3, %1\n\t"
          : "+v"(a), "+v"(b), "+v"(c), "+v"(d), "+s"(s0), "=&s"(t5), "=&s"(m6));
      s1 ^= t5 ^ (uint32_t)m6;
    } else if (KIND == 59) { // 4 v_max/min + 4 v_add_u32 interleaved
      uint32_t t5 = 0;
      uint64_t m6 = 0;
      asm volatile(
          "v_max_u32_e32 %0, %0, %1\n\tv_add_u32 %1, %1, %3\n\t"
          "v_min_u32_e32 %2, %2, %3\n\tv_add_u32 %3, %3, %1\n\t"
          "v_max_u32_e32 %0, %0, %1\n\tv_add_u32 %1, %1, %3\n\t"
          "v_min_u32_e32 %2, %2, %3\n\tv_add_u32 %3, %3, %1\n\t"
          : "+v"(a), "+v"(b), "+v"(c), "+v"(d), "+s"(s0), "=&s"(t5), "=&s"(m6));
      s1 ^= t5 ^ (uint32_t)m6;
    } else if (KIND == 60) { // 4 v_lshl_add_u64 + 4 v_add_u32 interleaved
      uint64_t x = ((uint64_t)a << 32) | b;
      asm volatile(
          "v_lshl_add_u64 %0, %0, 2, %0\n\tv_add_u32 %1, %1, %2\n\t"
          "v_lshl_add_u64 %0, %0, 1, %0\n\tv_add_u32 %2, %2, %1\n\t"
          "v_lshl_add_u64 %0, %0, 2, %0\n\tv_add_u32 %1, %1, %2\n\t"
          "v_lshl_add_u64 %0, %0, 1, %0\n\tv_add_u32 %2, %2, %1\n\t"
          : "+v"(x), "+v"(c), "+v"(d));
      a = (uint32_t)x; b = (uint32_t)(x >> 32);
    } else if (KIND == 61) { // 4 v_add sgpr + 4 v_add_u32 interleaved
      uint32_t t5 = 0;
      uint64_t m6 = 0;
      asm volatile(
          "v_add_u32_e32 %0, %4, %0\n\tv_add_u32 %1, %1, %3\n\t"
          "v_and_b32_e32 %2, %4, %2\n\tv_add_u32 %3, %3, %1\n\t"
          "v_add_u32_e32 %0, %4, %0\n\tv_add_u32 %1, %1, %3\n\t"
          "v_and_b32_e32 %2, %4, %2\n\tv_add_u32 %3, %3, %1\n\t"
          : "+v"(a), "+v"(b), "+v"(c), "+v"(d), "+s"(s0), "=&s"(t5), "=&s"(m6));
      s1 ^= t5 ^ (uint32_t)m6;
    } else if (KIND == 62) { // 4 v_mov from sgpr + 4 v_add_u32 interleaved
      uint32_t t5 = 0;
      uint64_t m6 = 0;
      asm volatile(
          "v_mov_b32_e32 %0, %4\n\tv_add_u32 %1, %1, %3\n\t"
          "v_mov_b32_e32 %2, %4\n\tv_add_u32 %3, %3, %1\n\t"
          "v_mov_b32_e32 %0, %4\n\tv_add_u32 %1, %1, %3\n\t"
          "v_mov_b32_e32 %2, %4\n\tv_add_u32 %3, %3, %1\n\t"
          : "+v"(a), "+v"(b), "+v"(c), "+v"(d), "+s"(s0), "=&s"(t5), "=&s"(m6));
      s1 ^= t5 ^ (uint32_t)m6;
    } else if (KIND == 63) { // 4 v_perm/xad + 4 v_add_u32 interleaved
      uint32_t t5 = 0;
      uint64_t m6 = 0;
      asm volatile(
          "v_xad_u32 %0, %1, %3, %0\n\tv_add_u32 %1, %1, %3\n\t"
          "v_and_or_b32 %2, %3, %1, %2\n\tv_add_u32 %3, %3, %1\n\t"
          "v_xad_u32 %0, %1, %3, %0\n\tv_add_u32 %1, %1, %3\n\t"
          "v_and_or_b32 %2, %3, %1, %2\n\tv_add_u32 %3, %3, %1\n\t"
          : "+v"(a), "+v"(b), "+v"(c), "+v"(d), "+s"(s0), "=&s"(t5), "=&s"(m6));
      s1 ^= t5 ^ (uint32_t)m6;
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
  // the other VALU forms the compressor uses, at 8 waves per SIMD
  run<5>("v_lshl/lshrrev_b64", grid, out, clk);
  run<6>("v_alignbyte_b32", grid, out, clk);
  run<7>("v_cndmask_b32_e64", grid, out, clk);
  run<8>("v_add3 / v_lshl_add", grid, out, clk);
  run<9>("v_mbcnt_lo/hi", grid, out, clk);
  run<10>("v_perm_b32", grid, out, clk);
  run<11>("v_mov_b32_dpp wave_shr", grid, out, clk);
  run<12>("v_bfe / v_and_or", grid, out, clk);
  run<13>("v_cmp_e64 -> sgpr", grid, out, clk);
  run<14>("v_cndmask_b32_e32 vcc", grid, out, clk);
  run<15>("VOP2 + literal", grid, out, clk);
  run<16>("VOP2 shifts/max/sub", grid, out, clk);
  run<17>("v_cmp_e32 -> vcc", grid, out, clk);
  run<18>("v_mul_u32_u24_e32", grid, out, clk);
  run<19>("VOP1 not/ffbl/bfrev", grid, out, clk);
  run<20>("VOP2 + sgpr", grid, out, clk);
  run<21>("v_add/xor_e64 (VOP3 enc)", grid, out, clk);
  run<22>("v_readfirstlane/readlane", grid, out, clk);
  run<23>("v_mov_b32_e32", grid, out, clk);
  run<24>("v_sub_u32_e32", grid, out, clk);
  run<25>("v_lshl/lshrrev_b32_e32", grid, out, clk);
  run<26>("v_max/min_u32_e32", grid, out, clk);
  run<27>("v_lshl_add_u64", grid, out, clk);
  run<28>("s_nop 0", grid, out, clk);
  run<29>("v_bfi/xad/min3/max3", grid, out, clk);
  run<30>("v_cndmask_e32 vcc<-valu", grid, out, clk);
  run<31>("salu mask->v_cndmask (8)", grid, out, clk);
  run<32>("v_cmp->s_bcnt1 (8)", grid, out, clk);
  run<33>("v_writelane_b32", grid, out, clk);
  run<34>("v_ffbl_b32_e32", grid, out, clk);
  run<35>("v_cndmask_e32 vcc const", grid, out, clk);
  run<36>("v_cndmask_e64 vcc const", grid, out, clk);
  run<37>("v_cmp_e64->cndmask (8)", grid, out, clk);
  run<38>("v_cmp_e32->cndmask_e32 (8)", grid, out, clk);
  run<39>("v_cndmask_e64 inline k", grid, out, clk);
  run<40>("v_mov_b32 from sgpr", grid, out, clk);
  run<41>("v_lshl_or/add_lshl/lshl_add", grid, out, clk);
  run<42>("v_and_b32 sgpr (vop2)", grid, out, clk);
  run<43>("4 v_perm + 4 v_add", grid, out, clk);
  run<44>("4 v_cndmask + 4 v_add", grid, out, clk);
  run<45>("4 dpp + 4 v_add", grid, out, clk);
  run<46>("4 v_lshrrev + 4 v_add", grid, out, clk);
  run<47>("4 v_perm + 4 v_cndmask", grid, out, clk);
  run<48>("4 v_perm + 4 s_add", grid, out, clk);
  run<50>("4 v_mbcnt + 4 v_add", grid, out, clk);
  run<51>("4 v_readlane + 4 v_add", grid, out, clk);
  run<52>("4 v_writelane + 4 v_add", grid, out, clk);
  run<53>("4 v_alignbyte + 4 v_add", grid, out, clk);
  run<54>("4 v_mul_lo_u32 + 4 v_add", grid, out, clk);
  run<55>("4 v_bfe/bfi + 4 v_add", grid, out, clk);
  run<56>("4 v_add3/lshl_add + 4 v_add", grid, out, clk);
  run<57>("4 v_cmp_e64 + 4 v_add", grid, out, clk);
  run<58>("4 v_ffbl + 4 v_add", grid, out, clk);
  run<59>("4 v_max/min + 4 v_add", grid, out, clk);
  run<60>("4 v_lshl_add_u64 + 4 v_add", grid, out, clk);
  run<61>("4 v_add sgpr + 4 v_add", grid, out, clk);
  run<62>("4 v_mov from sgpr + 4 v_add", grid, out, clk);
  run<63>("4 v_perm/xad + 4 v_add", grid, out, clk);
  return 0;
}
