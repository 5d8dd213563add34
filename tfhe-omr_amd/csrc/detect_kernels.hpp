// Detect-path kernels: level-1 blind rotation (x7 per message), 7-clue sum + sample extract,
// LWE key switch + modulus switch, level-2 blind rotation fused with the homomorphic trace.
#pragma once

#include "kernels.hpp"

namespace omr {

// ------------------------------------------------------------------------------------------
// Gadget decomposition into packed signed 8-bit digits (NonPowOf2ApproxSignedBasis,
// parameters/mod.rs:55,81; convention in include/omr_gpu.h). v is a canonical centred residue.
// ------------------------------------------------------------------------------------------
template <int LOGB, int D, int DROP>
struct Digits8 {
  static constexpr int DW = (D + 3) / 4;
  __device__ static __forceinline__ void pack(double v, uint32_t (&pk)[DW]) {
    double y = DROP ? floor(__fma_rn(v, 1.0 / (double)(1 << DROP), 0.5)) : v;
    constexpr double B = (double)(1 << LOGB), IB = 1.0 / (double)(1 << LOGB);
#pragma unroll
    for (int w = 0; w < DW; ++w) pk[w] = 0;
#pragma unroll
    for (int k = 0; k < D; ++k) {
      double d;
      if (k < D - 1) {
        const double c = floor(__fma_rn(y, IB, 0.5));
        d = __fma_rn(-c, B, y);
        y = c;
      } else {
        d = y;
      }
      pk[k / 4] |= ((uint32_t)(int)d & 0xffu) << (8 * (k % 4));
    }
  }
  __device__ static __forceinline__ double get(const uint32_t (&pk)[DW], int k) {
    uint32_t w = pk[0];
#pragma unroll
    for (int i = 1; i < DW; ++i) w = (k >> 2) == i ? pk[i] : w;
    const int s = 24 - 8 * (k & 3);
    return (double)((int32_t)(w << s) >> 24);
  }
};

// Trace basis (q2, 2, None): 25 digits in [-2, 2], 3 bits each (value + 2), 10 per dword.
struct DigitsTrace {
  static constexpr int DW = 3;
  __device__ static __forceinline__ void pack(double v, uint32_t (&pk)[DW]) {
    double y = v;
    pk[0] = pk[1] = pk[2] = 0;
#pragma unroll
    for (int k = 0; k < DT; ++k) {
      double d;
      if (k < DT - 1) {
        const double c = floor(__fma_rn(y, 0.25, 0.5));
        d = __fma_rn(-c, 4.0, y);
        y = c;
      } else {
        d = y;
      }
      pk[k / 10] |= (uint32_t)((int)d + 2) << (3 * (k % 10));
    }
  }
  __device__ static __forceinline__ double get(const uint32_t (&pk)[DW], int k) {
    const int wi = k / 10;
    const uint32_t w = wi == 0 ? pk[0] : (wi == 1 ? pk[1] : pk[2]);
    return (double)((int)((w >> (3 * (k - 10 * wi))) & 7u) - 2);
  }
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

// ------------------------------------------------------------------------------------------
// One CMUX step of the binary blind rotation (BlindRotationKey::blind_rotate):
//   ACC += ((X^a - 1) * ACC) [x] GGSW_i
// acc_a/acc_b: coefficient domain, canonical, in LDS. ggsw: NTT-domain rows [2D][2][N],
// pre-scaled by N^-1. All threads of the workgroup participate.
// ------------------------------------------------------------------------------------------
template <int LEVEL, int T, int E, int LOGB, int D, int DROP>
__device__ __forceinline__ void cmux_step(double *acc_a, double *acc_b, double *xch, int a,
                                          const double *__restrict__ ggsw,
                                          const double *__restrict__ tw,
                                          const double *__restrict__ itw, int tid) {
  using M = Mod<LEVEL>;
  using NTT = WgNtt<M, T, E>;
  using DG = Digits8<LOGB, D, DROP>;
  constexpr int N = M::N;
  double accA[E], accB[E];
#pragma unroll
  for (int e = 0; e < E; ++e) accA[e] = accB[e] = 0.0;
#pragma unroll 1
  for (int p = 0; p < 2; ++p) {
    const double *src = p ? acc_b : acc_a;
    uint32_t pk[E][DG::DW];
#pragma unroll
    for (int e = 0; e < E; ++e) {
      const int j = tid + e * T;
      const double v = canon_small<M>(rot_read<N>(src, j, a) - src[j]);
      DG::pack(v, pk[e]);
    }
#pragma unroll 1
    for (int k = 0; k < D; ++k) {
      double x[E];
#pragma unroll
      for (int e = 0; e < E; ++e) x[e] = DG::get(pk[e], k);
      NTT::fwd(x, xch, tw, tid);
      const double *ka = ggsw + (size_t)((p * D + k) * 2) * N + tid * E;
      const double *kb = ka + N;
#pragma unroll
      for (int e = 0; e < E; ++e) {
        accA[e] += mm<M>(x[e], ka[e]);
        accB[e] += mm<M>(x[e], kb[e]);
      }
      if (LEVEL == 2 && (k % 3) == 2) {
#pragma unroll
        for (int e = 0; e < E; ++e) {
          accA[e] = red<M>(accA[e]);
          accB[e] = red<M>(accB[e]);
        }
      }
    }
  }
#pragma unroll
  for (int e = 0; e < E; ++e) {
    accA[e] = red<M>(accA[e]);
    accB[e] = red<M>(accB[e]);
  }
  NTT::inv(accA, xch, itw, tid);
#pragma unroll
  for (int e = 0; e < E; ++e) {
    const int j = tid + e * T;
    acc_a[j] = canon<M>(acc_a[j] + accA[e]);
  }
  NTT::inv(accB, xch, itw, tid);
#pragma unroll
  for (int e = 0; e < E; ++e) {
    const int j = tid + e * T;
    acc_b[j] = canon<M>(acc_b[j] + accB[e]);
  }
  __syncthreads();
}

// ACC = (0, X^{-b} * LUT)
template <int LEVEL, int T, int E>
__device__ __forceinline__ void br_init(double *acc_a, double *acc_b, const double *lut, int b,
                                        int tid) {
  constexpr int N = Mod<LEVEL>::N;
  const int r = (2 * N - (b % (2 * N))) % (2 * N);
#pragma unroll
  for (int e = 0; e < E; ++e) {
    const int j = tid + e * T;
    acc_a[j] = 0.0;
    acc_b[j] = canon_small<Mod<LEVEL>>(rot_read<N>(lut, j, r));
  }
  __syncthreads();
}

// ------------------------------------------------------------------------------------------
// Level 1 (first_level_bootstrapping, detector.rs:533-597): one workgroup per (message, clue).
// mode 0: write the sample-extracted LWE (coefficient 0) as u32 [wg][N1+1];
// mode 1: write the full RLWE (a, b) as u64 [wg][2][N1] (stage test).
// Input is either a clue (lwe_a == nullptr: extract clue wg%7 of message wg/7, detector.rs:514)
// or an explicit LWE (lwe_a [wg][512], lwe_b [wg]).
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(BR1_T) void br1_kernel(const uint16_t *__restrict__ clue_a,
                                                   const uint16_t *__restrict__ clue_b,
                                                   const uint16_t *__restrict__ lwe_a,
                                                   const uint16_t *__restrict__ lwe_b,
                                                   const double *__restrict__ bsk1, DeviceTables tb,
                                                   uint32_t *__restrict__ ext,
                                                   uint64_t *__restrict__ rlwe_out, int mode) {
  using M = Mod<1>;
  constexpr int T = BR1_T, E = BR1_E, N = N1;
  __shared__ double acc[2][N];
  __shared__ double xch[WgNtt<M, T, E>::LDS_DOUBLES];
  __shared__ uint16_t la[N0];
  const int tid = threadIdx.x;
  const size_t wg = blockIdx.x;
  int b;
  if (lwe_a == nullptr) {
    const size_t m = wg / CLUES;
    const int c = (int)(wg % CLUES);
    const uint16_t *A = clue_a + m * N0;
    for (int i = tid; i < N0; i += T)
      la[i] = i <= c ? (uint16_t)(A[c - i] & (Q0 - 1)) : (uint16_t)((Q0 - A[N0 + c - i]) & (Q0 - 1));
    b = clue_b[m * CLUES + c] & (Q0 - 1);
  } else {
    for (int i = tid; i < N0; i += T) la[i] = lwe_a[wg * N0 + i] & (Q0 - 1);
    b = lwe_b[wg] & (Q0 - 1);
  }
  br_init<1, T, E>(acc[0], acc[1], tb.lut1, b, tid);
#pragma unroll 1
  for (int i = 0; i < N0; ++i) {
    const int a = __builtin_amdgcn_readfirstlane(la[i]);
    if (a == 0) continue;  // (X^0 - 1) * ACC = 0
    cmux_step<1, T, E, LOGB1, D1, DROP1>(acc[0], acc[1], xch, a,
                                         bsk1 + (size_t)i * (2 * D1 * 2 * N), tb.tw1, tb.itw1, tid);
  }
  if (mode == 0) {
    uint32_t *o = ext + wg * (N + 1);
    for (int j = tid; j < N; j += T) {
      const double v = j == 0 ? acc[0][0] : -acc[0][N - j];  // extract_lwe_locally, :561
      o[j] = (uint32_t)to_u64<M>(v);
    }
    if (tid == 0) o[N] = (uint32_t)to_u64<M>(acc[1][0]);
  } else {
    uint64_t *o = rlwe_out + wg * 2 * N;
    for (int j = tid; j < N; j += T) {
      o[j] = to_u64<M>(acc[0][j]);
      o[N + j] = to_u64<M>(acc[1][j]);
    }
  }
}

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

// LWE key switch 1024 -> 670 with 27 binary digits (NonPowOf2LweKeySwitchingKey::key_switch,
// detector.rs:560-563) + modulus switch q1 -> 4096 (:571-575) + b += 7*128 (:577-594).
// One wave per workgroup: lanes = 64 messages, the wave walks KS_COLS columns; KSK values are
// wave-uniform (scalar loads), each lane masks them with its own digit bits.
template <int CT>
__global__ __launch_bounds__(64) void ks_kernel(const uint32_t *__restrict__ lwe1t,
                                               const uint32_t *__restrict__ ksk,
                                               uint32_t *__restrict__ lwe_int, int B) {
  const int lane = threadIdx.x;
  const int m = blockIdx.x * 64 + lane;
  const int c0 = blockIdx.y * CT;
  const bool live = m < B;
  uint64_t acc[CT];
#pragma unroll
  for (int c = 0; c < CT; ++c) acc[c] = 0;
#pragma unroll 1
  for (int i = 0; i < N1; ++i) {
    const uint32_t x = live ? lwe1t[(size_t)i * B + m] : 0u;
    // Rows are read CT columns wide; the last tile reads into the next row / the 64-element
    // tail padding of the KSK allocation and those columns are never written.
    const uint32_t *row = ksk + (size_t)i * KS_DIGITS * (NI + 1) + c0;
    uint32_t part[CT];
#pragma unroll
    for (int c = 0; c < CT; ++c) part[c] = 0;
#pragma unroll 1
    for (int j = 0; j < KS_DIGITS; ++j) {
      const uint32_t mask = 0u - ((x >> j) & 1u);
      const uint32_t *r = row + (size_t)j * (NI + 1);
#pragma unroll
      for (int c = 0; c < CT; ++c) part[c] += r[c] & mask;  // 27 * 2^27 < 2^32
    }
#pragma unroll
    for (int c = 0; c < CT; ++c) acc[c] += part[c];
  }
  if (!live) return;
  const uint32_t b = lwe1t[(size_t)N1 * B + m];
#pragma unroll
  for (int c = 0; c < CT; ++c) {
    const int col = c0 + c;
    if (col > NI) break;
    const uint64_t s = acc[c] % Q1;
    uint64_t v = col < NI ? (Q1 - s) % Q1 : (b + Q1 - s) % Q1;
    v = ((2ull * QI * v + Q1) / (2ull * Q1)) % QI;
    if (col == NI) v = (v + CLUES * (QI / TI)) % QI;
    lwe_int[(size_t)m * (NI + 1) + col] = (uint32_t)v;
  }
}
constexpr int KS_CT = 16;

// ------------------------------------------------------------------------------------------
// Level 2 (second_level_bootstrapping, detector.rs:599-624) fused with hom_trace (:626-639):
// one workgroup per message. mode 0: trace + NTT output u64 [wg][2][N2] (NttRlweCiphertext);
// mode 1: blind rotation only, coefficient-domain output (stage test).
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(BR2_T) void br2_trace_kernel(const uint32_t *__restrict__ lwe_int,
                                                         const double *__restrict__ bsk2,
                                                         const double *__restrict__ tk,
                                                         DeviceTables tb,
                                                         uint64_t *__restrict__ out, int mode) {
  using M = Mod<2>;
  constexpr int T = BR2_T, E = BR2_E, N = N2;
  using NTT = WgNtt<M, T, E>;
  __shared__ double acc[2][N];
  __shared__ double xch[NTT::LDS_DOUBLES];
  const int tid = threadIdx.x;
  const size_t wg = blockIdx.x;
  const uint32_t *lwe = lwe_int + wg * (NI + 1);
  br_init<2, T, E>(acc[0], acc[1], tb.lut2, (int)lwe[NI], tid);
#pragma unroll 1
  for (int i = 0; i < NI; ++i) {
    const int a = (int)__builtin_amdgcn_readfirstlane(lwe[i]) & (2 * N - 1);
    if (a == 0) continue;
    cmux_step<2, T, E, LOGB2, D2, DROP2>(acc[0], acc[1], xch, a, bsk2 + (size_t)i * (2 * D2 * 2 * N),
                                         tb.tw2, tb.itw2, tid);
  }
  uint64_t *o = out + wg * 2 * N;
  if (mode == 1) {
    for (int j = tid; j < N; j += T) {
      o[j] = to_u64<M>(acc[0][j]);
      o[N + j] = to_u64<M>(acc[1][j]);
    }
    return;
  }
  // ---- hom_trace: c *= N^-1; for k: c += KS_k(sigma_g(c)); output NTT(c) ----
  // a stays in the coefficient domain (acc[0]); b moves to the NTT domain (acc[1], index order).
  constexpr double NINV = -549755813880.0;  // 2048^-1 mod q2 = 1125350151012361, centred (secret.rs:167-168)
  {
    double x[E];
#pragma unroll
    for (int e = 0; e < E; ++e) {
      const int j = tid + e * T;
      acc[0][j] = canon<M>(mm<M>(acc[0][j], NINV));
      x[e] = canon<M>(mm<M>(acc[1][j], NINV));
    }
    NTT::fwd(x, xch, tb.tw2, tid);
#pragma unroll
    for (int e = 0; e < E; ++e) acc[1][tid * E + e] = canon<M>(x[e]);
    __syncthreads();
  }
#pragma unroll 1
  for (int k = 0; k < TRACE_STEPS; ++k) {
    const uint16_t *src = tb.trace_src + k * N;
    const uint16_t *perm = tb.trace_perm + k * N;
    uint32_t pk[E][DigitsTrace::DW];
#pragma unroll
    for (int e = 0; e < E; ++e) {
      const int j = tid + e * T;
      const int s = src[j];
      const double v = s < N ? acc[0][s] : -acc[0][s - N];  // sigma_g(a)
      DigitsTrace::pack(v, pk[e]);
    }
    double accA[E], accB[E];
#pragma unroll
    for (int e = 0; e < E; ++e) accA[e] = accB[e] = 0.0;
    const double *key = tk + (size_t)k * DT * 2 * N;
#pragma unroll 1
    for (int d = 0; d < DT; ++d) {
      double x[E];
#pragma unroll
      for (int e = 0; e < E; ++e) x[e] = DigitsTrace::get(pk[e], d);
      NTT::fwd(x, xch, tb.tw2, tid);
      const double *ka = key + (size_t)(d * 2) * N + tid * E;  // alpha (pre-scaled by N^-1)
      const double *kb = ka + N;                                 // beta (unscaled)
#pragma unroll
      for (int e = 0; e < E; ++e) {
        accA[e] += mm<M>(x[e], ka[e]);
        accB[e] += mm<M>(x[e], kb[e]);
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
    double nb[E];
#pragma unroll
    for (int e = 0; e < E; ++e) {
      const int t = tid * E + e;
      nb[e] = acc[1][t] + acc[1][perm[t]] + red<M>(accB[e]);
    }
    __syncthreads();
#pragma unroll
    for (int e = 0; e < E; ++e) acc[1][tid * E + e] = canon<M>(nb[e]);
    // a += INTT(A)
#pragma unroll
    for (int e = 0; e < E; ++e) accA[e] = red<M>(accA[e]);
    NTT::inv(accA, xch, tb.itw2, tid);
#pragma unroll
    for (int e = 0; e < E; ++e) {
      const int j = tid + e * T;
      acc[0][j] = canon<M>(acc[0][j] + accA[e]);
    }
    __syncthreads();
  }
  {
    double x[E];
#pragma unroll
    for (int e = 0; e < E; ++e) x[e] = acc[0][tid + e * T];
    NTT::fwd(x, xch, tb.tw2, tid);
#pragma unroll
    for (int e = 0; e < E; ++e) {
      const int t = tid * E + e;
      o[t] = to_u64<M>(canon<M>(x[e]));
      o[N + t] = to_u64<M>(acc[1][t]);
    }
  }
}

}  // namespace omr
