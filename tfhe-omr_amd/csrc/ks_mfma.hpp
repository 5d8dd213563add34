// LWE key switch on the matrix cores (NonPowOf2LweKeySwitchingKey::key_switch, detector.rs:560-563,
// with the modulus switch :571-575 and offset :577-594).
//
// The key switch is a binary-by-integer matrix product:
//   acc[m][col] = sum_i sum_j bit_j(x[m][i]) * KSK[i][j][col]      (i < 1024, j < 27, col <= 670)
// so it runs as an int8 GEMM: A[m][32 i + j] = bit_j(x[m][i]) (0/1, j < 27, zero for j >= 27),
// B_l[32 i + j][col] = the l-th 7-bit limb of KSK[i][j][col] (l = 0..3, 28 bits >= 27), one
// v_mfma_i32_32x32x32_i8 per (32 messages x 32 columns x 32 digits x limb). Per limb the int32
// sums stay below 27648 * 127 < 2^22; acc = sum_l C_l 2^(7 l) < 2^43 is exact in int64 and then
// reduced mod q1 like the oracle's u64 sum, so the output is bit-identical.
#pragma once

#include "kernels.hpp"

namespace omr {

constexpr int KSM_COLS = 672;  // NI + 1 = 671 output columns, padded to 21 tiles of 32
constexpr int KSM_LIMBS = 4;
constexpr size_t KSKB_WORDS = (size_t)N1 * KSM_LIMBS * KSM_COLS * 8;  // 32 int8 per (i, l, col)

typedef int omr_v4i __attribute__((ext_vector_type(4)));
typedef int omr_v16i __attribute__((ext_vector_type(16)));

// KSK u32 [1024][27][671] -> int8 limbs [1024][4][672][32] (packed 4 per u32 word, byte b of word
// w = digit 4 w + b), zero for digits >= 27 and column 671.
__global__ void ksk_to_i8_kernel(const uint32_t *__restrict__ ksk, uint32_t *__restrict__ out) {
  const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= KSKB_WORDS) return;
  const int w = (int)(t & 7);
  const size_t rest = t >> 3;
  const int col = (int)(rest % KSM_COLS);
  const size_t il = rest / KSM_COLS;
  const int limb = (int)(il & 3), i = (int)(il >> 2);
  uint32_t word = 0;
#pragma unroll
  for (int b = 0; b < 4; ++b) {
    const int j = 4 * w + b;
    uint32_t v = 0;
    if (j < KS_DIGITS && col <= NI) v = (ksk[((size_t)i * KS_DIGITS + j) * (NI + 1) + col] >> (7 * limb)) & 127u;
    word |= v << (8 * b);
  }
  out[t] = word;
}

// Output column `col` of one message from the exact key-switch sum (detector.rs:560-594):
// b' = b - sum (columns < 670: -sum), modulus switch q1 -> 4096 (round half up), and the
// offset b += 7 * 128 on the body.
__device__ __forceinline__ uint32_t ks_epilogue(uint64_t sum, uint64_t bq, int col) {
  const uint64_t s = sum % Q1;
  uint64_t v = col < NI ? (Q1 - s) % Q1 : (bq + Q1 - s) % Q1;
  v = ((2ull * QI * v + Q1) / (2ull * Q1)) % QI;
  if (col == NI) v = (v + CLUES * (QI / TI)) % QI;
  return (uint32_t)v;
}

// 0/1 bytes of the 16 bits of x starting at bit `base` (A fragment: 16 int8 per lane): each
// nibble n spreads to four bytes as (n * 0x204081) & 0x01010101 (shifted copies 0, 7, 14, 21
// never overlap).
__device__ __forceinline__ omr_v4i bit_bytes16(uint32_t x, int base) {
  omr_v4i a;
#pragma unroll
  for (int v = 0; v < 4; ++v) a[v] = (int)((((x >> (base + 4 * v)) & 15u) * 0x204081u) & 0x01010101u);
  return a;
}

// grid (ceil(B / 64), 21), 64 threads: one wave computes messages m0 .. m0 + 63 (two 32-row
// tiles) x columns c0 .. c0 + 31 for the 4 limbs. Operand maps of v_mfma_i32_32x32x32_i8 (as the
// bf16 32x32x16 form, 16 elements per lane): lane l (r = l & 31, h = l >> 5) holds A[row r][k = 16 h
// + e] and B[k = 16 h + e][col r]; D: col = l & 31, row = (reg & 3) + 8 (reg >> 2) + 4 h.
__global__ __launch_bounds__(64, 2) void ks_mfma_kernel(const uint32_t *__restrict__ lwe1t,
                                                     const uint32_t *__restrict__ kskb,
                                                     uint32_t *__restrict__ lwe_int, int B) {
  const int lane = threadIdx.x, r = lane & 31, h = lane >> 5;
  const int m0 = blockIdx.x * 64, c0 = blockIdx.y * 32;
  omr_v16i acc[2][KSM_LIMBS];
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int l = 0; l < KSM_LIMBS; ++l) acc[t][l] = omr_v16i{};
  const bool live0 = m0 + r < B, live1 = m0 + 32 + r < B;
  const omr_v4i *bbase = reinterpret_cast<const omr_v4i *>(kskb) + (size_t)(c0 + r) * 2 + h;
#pragma unroll 1
  for (int i = 0; i < N1; ++i) {
    const uint32_t x0 = live0 ? lwe1t[(size_t)i * B + m0 + r] : 0u;
    const uint32_t x1 = live1 ? lwe1t[(size_t)i * B + m0 + 32 + r] : 0u;
    const omr_v4i a0 = bit_bytes16(x0, 16 * h), a1 = bit_bytes16(x1, 16 * h);
#pragma unroll
    for (int l = 0; l < KSM_LIMBS; ++l) {
      const omr_v4i b = bbase[((size_t)i * KSM_LIMBS + l) * KSM_COLS * 2];
      acc[0][l] = __builtin_amdgcn_mfma_i32_32x32x32_i8(a0, b, acc[0][l], 0, 0, 0);
      acc[1][l] = __builtin_amdgcn_mfma_i32_32x32x32_i8(a1, b, acc[1][l], 0, 0, 0);
    }
  }
  const int col = c0 + r;
  if (col > NI) return;
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int reg = 0; reg < 16; ++reg) {
      const int m = m0 + 32 * t + (reg & 3) + 8 * (reg >> 2) + 4 * h;
      if (m >= B) continue;
      const uint64_t sum = (uint64_t)acc[t][0][reg] + ((uint64_t)acc[t][1][reg] << 7) +
                           ((uint64_t)acc[t][2][reg] << 14) + ((uint64_t)acc[t][3][reg] << 21);
      lwe_int[(size_t)m * (NI + 1) + col] = ks_epilogue(sum, lwe1t[(size_t)N1 * B + m], col);
    }
}

}  // namespace omr
