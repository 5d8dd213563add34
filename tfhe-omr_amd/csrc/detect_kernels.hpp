// Detect-path kernels: level-1 blind rotation (x7 per message), 7-clue sum + sample extract,
// LWE key switch + modulus switch, level-2 blind rotation fused with the homomorphic trace.
#pragma once

#include <type_traits>

#include "kernels.hpp"

namespace omr {

// Level-2 gadget digits (logB 7, d 6, drop 8) in closed form: y = floor((v + 2^7) / 2^8) has
// balanced base-128 digits d_k in [-64, 63] (k < 5) and a top digit d_5 in [-64, 64]; with the
// bias 64 (1 + 128 + ... + 128^5), y' = y + bias is exact in FP64 (0 <= y' < 2^43) and splits
// exactly into lo = y' mod 2^21 (fields 0-2) and hi = floor(y' / 2^21) (fields 3-5). Field k holds
// d_k + 64: 7 bits at 7 (k mod 3) in word k / 3, the top field 8 bits (bit 21 of lo is zero, so
// the (offset, width) of field j of either word is (7 j, j == 2 ? 8 : 7)). Same digits as the
// recursive NonPowOf2ApproxSignedBasis decomposition of the oracle (gadget convention in
// include/omr_gpu.h; tests/test_digit_forms.py checks every boundary).
struct Digits2 {
  static constexpr int DW = 2;
  static_assert(LOGB2 == 7 && D2 == 6 && DROP2 == 8, "closed form written for the level-2 basis");
  __device__ static __forceinline__ void pack(double v, uint32_t (&pk)[DW]) {
    const double y = floor(__fma_rn(v, 1.0 / 256.0, 0.5)) + 2216338399296.0;  // + 17315143744 + 64 * 2^35
    const double hi = floor(y * (1.0 / 2097152.0));
    const double lo = __fma_rn(-hi, 2097152.0, y);
    pk[0] = (uint32_t)(int)lo;
    pk[1] = (uint32_t)(int)hi;
  }
  // d_{j + 3 h} + 64 (the word is chosen at compile time, the offset may be a run-time uniform)
  template <int H>
  __device__ static __forceinline__ int field(const uint32_t (&pk)[DW], int j) {
    return (int)__builtin_amdgcn_ubfe(pk[H], 7 * j, j == 2 ? 8 : 7);
  }
  __device__ static __forceinline__ int get_int(const uint32_t (&pk)[DW], int k) {
    return (k < 3 ? field<0>(pk, k) : field<1>(pk, k - 3)) - 64;
  }
};
// Trace basis (q2, 2, None): 25 balanced base-4 digits (24 in [-2, 1], the top one in [-2, 3]).
struct DigitsTrace {
  static constexpr int DW = 2;
  static_assert(DT == 25, "closed form written for the trace basis");
  // Closed form of the recursive balanced base-4 decomposition (d = y - 4 floor(y / 4 + 1/2), 24
  // times, then the rest; round 5): y' = v + 2 (1 + 4 + ... + 4^23) has field k (bits 2k, 2k + 1)
  // = d_k + 2 for k < 24 and y' >> 48 = d_24. Y = y' + 1.5 * 2^52 is exact (|v| < 2^49) and the low
  // 51 bits of its mantissa are y' in two's complement, so the words are Y's two dwords, each field
  // XORed with 2 (a two's-complement 2-bit digit: one v_bfe_i32): 1 FP64 add and 2 XORs per
  // coefficient instead of 24 floor / fma / conversion rounds (tests/test_lvl1_offset_model.py).
  __device__ static __forceinline__ void pack(double v, uint32_t (&pk)[DW]) {
    const uint64_t b = __builtin_bit_cast(uint64_t, v + (187649984473770.0 + 6755399441055744.0));
    pk[0] = (uint32_t)b ^ 0xAAAAAAAAu;      // digits 0..15
    pk[1] = (uint32_t)(b >> 32) ^ 0xAAAAu;  // digits 16..23 in bits 0..15, d_24 in bits 16..18
  }
  __device__ static __forceinline__ int get_int(const uint32_t (&pk)[DW], int k) {
    const uint32_t w = k < 16 ? pk[0] : pk[1];
    return (int)__builtin_amdgcn_sbfe(w, k < 16 ? 2 * k : 2 * (k - 16), k == DT - 1 ? 3 : 2);
  }
  __device__ static __forceinline__ double get(const uint32_t (&pk)[DW], int k) { return (double)get_int(pk, k); }
};

// (X^r * p)[j] for p in LDS, r in [0, 2N): sign-corrected read.
template <int N>
__device__ __forceinline__ double rot_read(const double *p, int j, int r) {
  int t = j - r;
  double s = 1.0;
  if (t < 0) {
    t += N;
    s = -1.0;
  }
  if (t < 0) {
    t += N;
    s = 1.0;
  }
  return s * p[t];
}

// (X^r * p)[j] for p in LDS as t = (j - r) mod 2N: p[t] for t < N, -p[t - N] above (the sign
// flipped by one xor of bit 63 instead of compare/select pairs and a multiply).
template <int N>
__device__ __forceinline__ double rot_read_lds(const double *p, int j, int r) {
  static_assert((N & (N - 1)) == 0 && N <= (1 << 20), "power-of-two ring degree");
  const uint32_t t = (uint32_t)(j - r) & (2 * N - 1);
  const double v = p[t & (N - 1)];
  const uint32_t hi = (uint32_t)(__builtin_bit_cast(uint64_t, v) >> 32) ^ ((t & N) << (31 - ilog2(N)));
  return __builtin_bit_cast(double, (__builtin_bit_cast(uint64_t, v) & 0xffffffffull) | ((uint64_t)hi << 32));
}

}  // namespace omr

#include "br1_fft.hpp"

namespace omr {

// One key row of the level-2 GGSW (NTT domain, [2][N]: A and B components), E residues per thread.
template <typename KeyT, int E>
struct KeyRow {
  KeyT a[E], b[E];
  __device__ __forceinline__ void load(const KeyT *__restrict__ row, int N, int off) {
#pragma unroll
    for (int e = 0; e < E; ++e) {
      a[e] = row[off + e];
      b[e] = row[N + off + e];
    }
  }
};

// Sum of the 7 extracted LWEs mod q1 (detector.rs:556), transposed to [N1+1][B] for the key
// switch (lanes = messages).
__global__ void sum7_kernel(const uint32_t *__restrict__ ext, uint32_t *__restrict__ lwe1t,
                            int B) {
  const size_t idx = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (size_t)B * (N1 + 1)) return;
  const size_t m = idx % B, i = idx / B;
  uint32_t s = 0;
#pragma unroll
  for (int c = 0; c < CLUES; ++c) s += ext[(m * CLUES + c) * (N1 + 1) + i];
  lwe1t[i * B + m] = s % (uint32_t)Q1;
}

}  // namespace omr

#include "ks_mfma.hpp"

namespace omr {

// hom_trace (detector.rs:626-639) of the level-2 accumulator (coefficient layout tid + e*T,
// canonical) and store of NTT(c) as NttRlweCiphertext u64 [2][N2] at o. tw/itw: NTT twiddles in
// LDS; xch: N2 doubles of LDS.
__device__ __forceinline__ void hom_trace_store(double (&acc0)[BR2_E], double (&acc1)[BR2_E],
                                                double *xch, const double *tw, const double *itw,
                                                const double *__restrict__ tk, const DeviceTables &tb,
                                                uint64_t *__restrict__ o, int tid) {
  using M = Mod<2>;
  constexpr int T = BR2_T, E = BR2_E, N = N2;
  using NTT = WgNtt<M, T, E>;
  // ---- hom_trace: c *= N^-1; for k: c += KS_k(sigma_g(c)); output NTT(c) ----
  // The mask stays in the coefficient domain (ca, layout tid + e*T); the body moves to the NTT
  // domain (cb, layout tid*E + e) where sigma_g is an index permutation.
  constexpr double NINV = -549755813880.0;  // 2048^-1 mod q2 = 1125350151012361, centred (secret.rs:167-168)
  double ca[E], cb[E];
#pragma unroll
  for (int e = 0; e < E; ++e) {
    ca[e] = canon<M>(mm<M>(acc0[e], NINV));
    cb[e] = canon<M>(mm<M>(acc1[e], NINV));
  }
  NTT::fwd(cb, xch, tw, tid);
#pragma unroll
  for (int e = 0; e < E; ++e) cb[e] = canon<M>(cb[e]);
#pragma unroll 1
  for (int k = 0; k < TRACE_STEPS; ++k) {
    const uint16_t *src = tb.trace_src + k * N;
    const uint16_t *perm = tb.trace_perm + k * N;
    uint32_t pk[E][DigitsTrace::DW];
#pragma unroll
    for (int e = 0; e < E; ++e) xch[tid + e * T] = ca[e];
    __syncthreads();
#pragma unroll
    for (int e = 0; e < E; ++e) {
      const int s = src[tid + e * T];
      DigitsTrace::pack(s < N ? xch[s] : -xch[s - N], pk[e]);  // sigma_g(a)
    }
    __syncthreads();
    double accA[E], accB[E];
#pragma unroll
    for (int e = 0; e < E; ++e) accA[e] = accB[e] = 0.0;
    const double *key = tk + (size_t)k * DT * 2 * N;
#pragma unroll 1
    for (int d = 0; d < DT; ++d) {
      const double *ka = key + (size_t)(d * 2) * N + tid * E;  // alpha (pre-scaled by N^-1)
      const double *kb = ka + N;                                 // beta (unscaled)
      double kra[E], krb[E];
#pragma unroll
      for (int e = 0; e < E; ++e) {
        kra[e] = ka[e];
        krb[e] = kb[e];
      }
      double x[E];
#pragma unroll
      for (int e = 0; e < E; ++e) x[e] = DigitsTrace::get(pk[e], d);
      NTT::fwd(x, xch, tw, tid);
#pragma unroll
      for (int e = 0; e < E; ++e) {
        accA[e] += mm<M>(x[e], kra[e]);
        accB[e] += mm<M>(x[e], krb[e]);
      }
      if ((d % 3) == 2) {
#pragma unroll
        for (int e = 0; e < E; ++e) {
          accA[e] = red<M>(accA[e]);
          accB[e] = red<M>(accB[e]);
        }
      }
    }
    // b_ntt += sigma_g(b)_ntt + B
#pragma unroll
    for (int e = 0; e < E; ++e) xch[tid * E + e] = cb[e];
    __syncthreads();
#pragma unroll
    for (int e = 0; e < E; ++e) cb[e] = canon<M>(cb[e] + xch[perm[tid * E + e]] + red<M>(accB[e]));
    __syncthreads();
    // a += INTT(A)
#pragma unroll
    for (int e = 0; e < E; ++e) accA[e] = red<M>(accA[e]);
    NTT::inv(accA, xch, itw, tid);
#pragma unroll
    for (int e = 0; e < E; ++e) ca[e] = canon<M>(ca[e] + accA[e]);
  }
  NTT::fwd(ca, xch, tw, tid);
#pragma unroll
  for (int e = 0; e < E; ++e) {
    const int t = tid * E + e;
    o[t] = to_u64<M>(canon<M>(ca[e]));
    o[N + t] = to_u64<M>(cb[e]);
  }
}

}  // namespace omr

