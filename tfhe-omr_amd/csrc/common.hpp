// Shared constants and small host/device helpers for libomr_gpu.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <string>

#include "../../include/omr_gpu.h"

#define OMR_HD __host__ __device__ __forceinline__

namespace omr {

// Parameter set (omr_core/src/parameters/mod.rs:39-105).
constexpr int N0 = OMR_N0;           // clue LWE dimension
constexpr int Q0 = OMR_Q0;           // clue modulus
constexpr int CLUES = OMR_CLUE_COUNT;
constexpr uint64_t Q1 = OMR_Q1;      // FirstLevelField
constexpr int N1 = OMR_N1;
constexpr int LOGB1 = 5, D1 = 4, DROP1 = 7;
constexpr int KS_DIGITS = OMR_KS_DIGITS;
constexpr int NI = OMR_NI;
constexpr int QI = OMR_QI, TI = 32;
constexpr uint64_t Q2 = OMR_Q2;      // SecondLevelField
constexpr int N2 = OMR_N2;
constexpr int LOGB2 = 7, D2 = 6, DROP2 = 8;
constexpr int LOGBT = 2, DT = OMR_TRACE_DIGITS, TRACE_STEPS = OMR_TRACE_STEPS;
constexpr int P = OMR_P;
constexpr int PAYLOAD_LEN = OMR_PAYLOAD_LEN;
constexpr int BUCKETS = 130;         // key_gen/secret.rs:189-209
constexpr int SEGMENTS = 25;

// Noise standard deviations (parameters/mod.rs).
constexpr double SIGMA_CLUE = 0.8293;
constexpr double SIGMA_BR1 = 3.1859;
constexpr double SIGMA_KS = 2.0329 * 1024.0;
constexpr double SIGMA_BR2 = 0.3908;
constexpr double SIGMA_TRACE = 0.3908;

// Key sizes (elements) in the boundary layout of include/omr_gpu.h.
constexpr size_t BSK1_ELEMS = (size_t)N0 * 2 * D1 * 2 * N1;
constexpr size_t KSK_ELEMS = (size_t)N1 * KS_DIGITS * (NI + 1);
constexpr size_t BSK2_ELEMS = (size_t)NI * 2 * D2 * 2 * N2;
constexpr size_t TK_ELEMS = (size_t)TRACE_STEPS * DT * 2 * N2;

// ChaCha block (djb layout: 64-bit counter in words 12-13, 64-bit stream id in 14-15).
OMR_HD uint32_t rotl32(uint32_t v, int n) { return (v << n) | (v >> (32 - n)); }
OMR_HD void chacha_block(int rounds, const uint32_t key[8], uint64_t counter, uint64_t stream,
                         uint32_t out[16]) {
  uint32_t in[16] = {0x61707865u, 0x3320646eu, 0x79622d32u, 0x6b206574u, key[0], key[1],
                     key[2],      key[3],      key[4],      key[5],      key[6], key[7],
                     (uint32_t)counter, (uint32_t)(counter >> 32), (uint32_t)stream,
                     (uint32_t)(stream >> 32)};
  uint32_t x[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) x[i] = in[i];
#define OMR_QR(a, b, c, d)                                                                   \
  x[a] += x[b]; x[d] = rotl32(x[d] ^ x[a], 16); x[c] += x[d]; x[b] = rotl32(x[b] ^ x[c], 12); \
  x[a] += x[b]; x[d] = rotl32(x[d] ^ x[a], 8);  x[c] += x[d]; x[b] = rotl32(x[b] ^ x[c], 7);
  for (int r = 0; r < rounds; r += 2) {
    OMR_QR(0, 4, 8, 12) OMR_QR(1, 5, 9, 13) OMR_QR(2, 6, 10, 14) OMR_QR(3, 7, 11, 15)
    OMR_QR(0, 5, 10, 15) OMR_QR(1, 6, 11, 12) OMR_QR(2, 7, 8, 13) OMR_QR(3, 4, 9, 14)
  }
#undef OMR_QR
#pragma unroll
  for (int i = 0; i < 16; ++i) out[i] = x[i] + in[i];
}

// Bucket choice for encode_pertinent_indices: ChaCha12 keyed by (seed, ct), block counter = the
// global message index, word s = segment. Replaces thread_rng + Uniform(0,130) (detector.rs:262,278)
// with a stream every shard can evaluate independently.
OMR_HD void bucket_words(uint64_t seed, uint32_t ct, uint64_t gi, uint32_t out[16]) {
  const uint32_t key[8] = {(uint32_t)seed, (uint32_t)(seed >> 32), 0x6f6d7262u, ct, 0, 0, 0, 0};
  chacha_block(12, key, gi, 0x62756b74u, out);
}
OMR_HD uint32_t bucket_of(uint32_t word) { return (uint32_t)(((uint64_t)word * BUCKETS) >> 32); }

// Error reporting (thread-local message behind omr_last_error()).
omr_status set_error(omr_status st, const std::string &msg);

}  // namespace omr
