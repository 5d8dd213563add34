// Detect-path kernels: level-1 blind rotation (x7 per message), 7-clue sum + sample extract,
// LWE key switch + modulus switch, level-2 blind rotation fused with the homomorphic trace.
#pragma once

#include <type_traits>

#include "kernels.hpp"

#ifndef OMR_DIGITS2_CLOSED
#define OMR_DIGITS2_CLOSED 1  // level-2 digits in closed form (Digits2; -1 % on the three-buffer step)
#endif

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
  __device__ static __forceinline__ int get_int(const uint32_t (&pk)[DW], int k) {
    uint32_t w = pk[0];
#pragma unroll
    for (int i = 1; i < DW; ++i) w = (k >> 2) == i ? pk[i] : w;
    const int s = 24 - 8 * (k & 3);
    return (int32_t)(w << s) >> 24;
  }
  __device__ static __forceinline__ double get(const uint32_t (&pk)[DW], int k) { return (double)get_int(pk, k); }
};

// Level-2 gadget digits (logB 7, d 6, drop 8) in closed form: y = floor((v + 2^7) / 2^8) has
// balanced base-128 digits d_k in [-64, 63] (k < 5) and a top digit; with the bias
// 64 (1 + 128 + ... + 128^4), y' = y + bias is exact in FP64 (|y'| < 2^42) and splits exactly into
// lo = y' mod 2^21 (digits 0-2) and hi = floor(y' / 2^21) (digits 3-4, top = hi >> 14). Same
// digits as Digits8<7, 6, 8> (tools check: every boundary and 2.6 M random residues).
struct Digits2 {
  static constexpr int DW = 2;
  static_assert(LOGB2 == 7 && D2 == 6 && DROP2 == 8, "closed form written for the level-2 basis");
  __device__ static __forceinline__ void pack(double v, uint32_t (&pk)[DW]) {
    const double y = floor(__fma_rn(v, 1.0 / 256.0, 0.5)) + 17315143744.0;
    const double hi = floor(y * (1.0 / 2097152.0));
    const double lo = __fma_rn(-hi, 2097152.0, y);
    pk[0] = (uint32_t)(int)lo;
    pk[1] = (uint32_t)(int)hi;
  }
  __device__ static __forceinline__ int get_int(const uint32_t (&pk)[DW], int k) {
    if (k == D2 - 1) return (int)pk[1] >> 14;
    const uint32_t w = k < 3 ? pk[0] : pk[1];
    const int sh = 7 * (k < 3 ? k : k - 3);
    return (int)((w >> sh) & 127u) - 64;
  }
  __device__ static __forceinline__ double get(const uint32_t (&pk)[DW], int k) { return (double)get_int(pk, k); }
};
template <int LEVEL, int LOGB, int D, int DROP>
using DigitsFor = std::conditional_t<LEVEL == 2 && OMR_DIGITS2_CLOSED, Digits2, Digits8<LOGB, D, DROP>>;

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
  __device__ static __forceinline__ int get_int(const uint32_t (&pk)[DW], int k) {
    const int wi = k / 10;
    const uint32_t w = wi == 0 ? pk[0] : (wi == 1 ? pk[1] : pk[2]);
    return (int)((w >> (3 * (k - 10 * wi))) & 7u) - 2;
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

}  // namespace omr

#include "br1_fft.hpp"

namespace omr {

// ------------------------------------------------------------------------------------------
// One CMUX step of the binary blind rotation (BlindRotationKey::blind_rotate):
//   ACC += ((X^a - 1) * ACC) [x] GGSW_i
// acc[p][e]: accumulator poly p (0 = mask, 1 = body), coefficient tid + e*T, canonical, held in
// registers. xch: the workgroup's LDS buffer (N doubles) used for the rotation gather and the
// NTT exchanges. tw/itw: twiddle tables (LDS copies). ggsw: NTT-domain rows [2D][2][N] of KeyT,
// pre-scaled by N^-1. Digit rows are walked in one loop (row r = p*D + k) and key rows are
// prefetched DEPTH rows ahead so their L2/MALL latency hides behind the transforms.
// ------------------------------------------------------------------------------------------
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

// Stage poly `src` (registers, coefficient layout) into LDS and gather (X^a - 1) * src.
template <class M, int T, int E>
__device__ __forceinline__ void rotate_diff(const double (&src)[E], double *xch, int a, int tid,
                                            double (&out)[E]) {
  constexpr int N = M::N;
#pragma unroll
  for (int e = 0; e < E; ++e) xch[tid + e * T] = src[e];
  __syncthreads();
#pragma unroll
  for (int e = 0; e < E; ++e) out[e] = canon_small<M>(rot_read<N>(xch, tid + e * T, a) - src[e]);
  __syncthreads();
}

template <int LEVEL, int T, int E, int LOGB, int D, int DROP, typename KeyT, int DEPTH, bool G = false>
__device__ __forceinline__ void cmux_step(double (&acc0)[E], double (&acc1)[E], double *xch, int a,
                                          const KeyT *__restrict__ ggsw, const double *tw,
                                          const double *itw, int tid,
                                          const double *__restrict__ gtw = nullptr,
                                          const double *__restrict__ gitw = nullptr) {
  using M = Mod<LEVEL>;
  using NTT = WgNtt<M, T, E>;
  using DG = DigitsFor<LEVEL, LOGB, D, DROP>;
  constexpr int N = M::N;
  double accA[E], accB[E];
#pragma unroll
  for (int e = 0; e < E; ++e) accA[e] = accB[e] = 0.0;
  KeyRow<KeyT, E> cur, nxt;
  cur.load(ggsw, N, tid * E);
  uint32_t pk[E][DG::DW];
#pragma unroll 1
  for (int r = 0; r < 2 * D; ++r) {
    if (DEPTH > 1 && r + 1 < 2 * D) nxt.load(ggsw + (size_t)(r + 1) * 2 * N, N, tid * E);
    const int k = r < D ? r : r - D;
    if (k == 0) {  // digits of (X^a - 1) * ACC_p, p = r / D
      double src[E], v[E];
#pragma unroll
      for (int e = 0; e < E; ++e) src[e] = r == 0 ? acc0[e] : acc1[e];
      rotate_diff<M, T, E>(src, xch, a, tid, v);
#pragma unroll
      for (int e = 0; e < E; ++e) DG::pack(v[e], pk[e]);
    }
    double x[E];
#pragma unroll
    for (int e = 0; e < E; ++e) x[e] = DG::get(pk[e], k);
    if constexpr (G)
      NTT::fwd_g(x, xch, tw, gtw, tid);
    else
      NTT::fwd(x, xch, tw, tid);
#pragma unroll
    for (int e = 0; e < E; ++e) {
      accA[e] += mm<M>(x[e], (double)cur.a[e]);
      accB[e] += mm<M>(x[e], (double)cur.b[e]);
    }
    if (LEVEL == 2 && (k % 3) == 2) {
#pragma unroll
      for (int e = 0; e < E; ++e) {
        accA[e] = red<M>(accA[e]);
        accB[e] = red<M>(accB[e]);
      }
    }
    if (r + 1 < 2 * D) {
      if (DEPTH > 1)
        cur = nxt;
      else
        cur.load(ggsw + (size_t)(r + 1) * 2 * N, N, tid * E);
    }
  }
#pragma unroll
  for (int e = 0; e < E; ++e) {
    accA[e] = red<M>(accA[e]);
    accB[e] = red<M>(accB[e]);
  }
  if constexpr (G)
    NTT::inv_g(accA, xch, itw, gitw, tid);
  else
    NTT::inv(accA, xch, itw, tid);
#pragma unroll
  for (int e = 0; e < E; ++e) acc0[e] = canon<M>(acc0[e] + accA[e]);
  if constexpr (G)
    NTT::inv_g(accB, xch, itw, gitw, tid);
  else
    NTT::inv(accB, xch, itw, tid);
#pragma unroll
  for (int e = 0; e < E; ++e) acc1[e] = canon<M>(acc1[e] + accB[e]);
}

// Level-2 CMUX step on three-buffer exchanges (OMR_XBUF3; xch holds WgNtt::LDS3_DOUBLES).
// Cross-wave uses of the LDS per step, in order: staging of the mask in X1, the 6 mask-digit
// NTTs on X0, X1, X0, X1, X0, X1, staging of the body in X0, the 6 body-digit NTTs on X1, X0,
// ..., X0, the inverse A on X1 and B on X0; the step starts on X1 and ends on X0. Consecutive
// cross-wave uses always alternate, so each writes a buffer whose last readers have passed the
// other buffer's barrier: no transform and no staging needs a trailing barrier, 16 workgroup
// barriers per step (one per cross-wave use) instead of 32.
template <int T, int E, typename KeyT>
__device__ __forceinline__ void cmux_step3(double (&acc0)[E], double (&acc1)[E], double *xch, int a,
                                           const KeyT *__restrict__ ggsw, const double *tw,
                                           const double *itw, int tid, const double *t0 = nullptr) {
  using M = Mod<2>;
  using NTT = WgNtt<M, T, E>;
  using DG = DigitsFor<2, LOGB2, D2, DROP2>;
  constexpr int N = M::N;
  static_assert(D2 % 2 == 0, "digit loop unrolled by two (alternating cross-wave buffers)");
  double accA[E], accB[E];
#pragma unroll
  for (int e = 0; e < E; ++e) accA[e] = accB[e] = 0.0;
  KeyRow<KeyT, E> cur;
  cur.load(ggsw, N, tid * E);
  uint32_t pk[E][DG::DW];
#pragma unroll
  for (int p = 0; p < 2; ++p) {
    {  // digits of (X^a - 1) * ACC_p, staged in X1 (mask) / X0 (body)
      double *st = xch + (p == 0 ? N : 0);
#pragma unroll
      for (int e = 0; e < E; ++e) st[tid + e * T] = p == 0 ? acc0[e] : acc1[e];
      __syncthreads();
#pragma unroll
      for (int e = 0; e < E; ++e)
        DG::pack(canon_small<M>(rot_read<N>(st, tid + e * T, a) - (p == 0 ? acc0[e] : acc1[e])), pk[e]);
      __builtin_amdgcn_wave_barrier();
      __atomic_signal_fence(__ATOMIC_SEQ_CST);
    }
#pragma unroll 1
    for (int k2 = 0; k2 < D2; k2 += 2) {
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int k = k2 + h, r = p * D2 + k;
        double x[E];
        if (OMR_NTT_SMALL0) {
          int d[E];
#pragma unroll
          for (int e = 0; e < E; ++e) d[e] = DG::get_int(pk[e], k);
          if ((h ^ p) == 0)  // mask digits on X0, X1, ...; body digits on X1, X0, ...
            NTT::template fwd3_small<0>(d, t0, x, xch, tw, tid);
          else
            NTT::template fwd3_small<1>(d, t0, x, xch, tw, tid);
        } else {
#pragma unroll
          for (int e = 0; e < E; ++e) x[e] = DG::get(pk[e], k);
          if ((h ^ p) == 0)
            NTT::template fwd3<0>(x, xch, tw, tid);
          else
            NTT::template fwd3<1>(x, xch, tw, tid);
        }
#pragma unroll
        for (int e = 0; e < E; ++e) {
          accA[e] += mm<M>(x[e], (double)cur.a[e]);
          accB[e] += mm<M>(x[e], (double)cur.b[e]);
        }
        // |x| <= 4.96q after the transform, so |mm(x, key)| <= 1.49q: four products on a
        // reduced sum stay below 6.5q < 2^53 (OMR_MAC_RED4); three with the per-row rule
        if (OMR_MAC_RED4 ? ((r % 4) == 3 && r + 1 < 2 * D2) : (k % 3) == 2) {
#pragma unroll
          for (int e = 0; e < E; ++e) {
            accA[e] = red<M>(accA[e]);
            accB[e] = red<M>(accB[e]);
          }
        }
        if (r + 1 < 2 * D2) cur.load(ggsw + (size_t)(r + 1) * 2 * N, N, tid * E);
      }
    }
  }
#pragma unroll
  for (int e = 0; e < E; ++e) {
    accA[e] = red<M>(accA[e]);
    accB[e] = red<M>(accB[e]);
  }
  if (OMR_NTT_SMALL0)
    NTT::template inv3m<1>(accA, xch, tw, tid);
  else
    NTT::template inv3<1>(accA, xch, itw, tid);
#pragma unroll
  for (int e = 0; e < E; ++e) acc0[e] = canon<M>(acc0[e] + accA[e]);
  if (OMR_NTT_SMALL0)
    NTT::template inv3m<0>(accB, xch, tw, tid);
  else
    NTT::template inv3<0>(accB, xch, itw, tid);
#pragma unroll
  for (int e = 0; e < E; ++e) acc1[e] = canon<M>(acc1[e] + accB[e]);
}

// Paired variant: digit k of the mask and digit k of the body are transformed together
// (two interleaved NTTs sharing every barrier), and the two inverse transforms likewise.
// xch holds 2N doubles. MAC_EXACT (level 1 only): the transformed digit is reduced to
// |x| <= q/2 + 2, so x*k is exact in FP64 (|x*k| < 2^52 for |k| <= (q1-1)/2) and two
// products plus the running sum stay below 2^53; one reduction per two products.
template <int LEVEL, int T, int E, int LOGB, int D, int DROP, typename KeyT, int DEPTH, bool MAC_EXACT>
__device__ __forceinline__ void cmux_step_pair(double (&acc0)[E], double (&acc1)[E], double *xch,
                                               int a, const KeyT *__restrict__ ggsw,
                                               const double *tw, const double *itw, int tid) {
  using M = Mod<LEVEL>;
  using NTT = WgNtt<M, T, E>;
  using DG = DigitsFor<LEVEL, LOGB, D, DROP>;
  constexpr int N = M::N;
  static_assert(!MAC_EXACT || LEVEL == 1, "exact-product MAC needs q < 2^27");
  double acc[2][E];  // [0] = mask accumulator A, [1] = body accumulator B (NTT domain)
#pragma unroll
  for (int e = 0; e < E; ++e) acc[0][e] = acc[1][e] = 0.0;
  uint32_t pk[2][E][DG::DW];
  {  // digits of (X^a - 1) * ACC for both polys: one staging round trip
#pragma unroll
    for (int e = 0; e < E; ++e) {
      xch[tid + e * T] = acc0[e];
      xch[N + tid + e * T] = acc1[e];
    }
    __syncthreads();
#pragma unroll
    for (int e = 0; e < E; ++e) {
      const int j = tid + e * T;
      DG::pack(canon_small<M>(rot_read<N>(xch, j, a) - acc0[e]), pk[0][e]);
      DG::pack(canon_small<M>(rot_read<N>(xch + N, j, a) - acc1[e]), pk[1][e]);
    }
    __syncthreads();
  }
  // key rows: row k (mask digit k) and row D+k (body digit k), each [2][N] (A, B components)
  KeyRow<KeyT, E> c0, c1, n0, n1;
  c0.load(ggsw, N, tid * E);
  c1.load(ggsw + (size_t)D * 2 * N, N, tid * E);
#pragma unroll 1
  for (int k = 0; k < D; ++k) {
    if (DEPTH > 1 && k + 1 < D) {
      n0.load(ggsw + (size_t)(k + 1) * 2 * N, N, tid * E);
      n1.load(ggsw + (size_t)(D + k + 1) * 2 * N, N, tid * E);
    }
    double x[2][E];
#pragma unroll
    for (int e = 0; e < E; ++e) {
      x[0][e] = DG::get(pk[0][e], k);
      x[1][e] = DG::get(pk[1][e], k);
    }
    NTT::template fwdC<2>(x, xch, tw, tid);
#pragma unroll
    for (int e = 0; e < E; ++e) {
      if constexpr (MAC_EXACT) {
        const double x0 = red<M>(x[0][e]), x1 = red<M>(x[1][e]);
        acc[0][e] = red<M>(__fma_rn(x1, (double)c1.a[e], __fma_rn(x0, (double)c0.a[e], acc[0][e])));
        acc[1][e] = red<M>(__fma_rn(x1, (double)c1.b[e], __fma_rn(x0, (double)c0.b[e], acc[1][e])));
      } else {
        acc[0][e] += mm<M>(x[0][e], (double)c0.a[e]) + mm<M>(x[1][e], (double)c1.a[e]);
        acc[1][e] += mm<M>(x[0][e], (double)c0.b[e]) + mm<M>(x[1][e], (double)c1.b[e]);
        if (LEVEL == 2) {
          acc[0][e] = red<M>(acc[0][e]);
          acc[1][e] = red<M>(acc[1][e]);
        }
      }
    }
    if (k + 1 < D) {
      if (DEPTH > 1) {
        c0 = n0;
        c1 = n1;
      } else {
        c0.load(ggsw + (size_t)(k + 1) * 2 * N, N, tid * E);
        c1.load(ggsw + (size_t)(D + k + 1) * 2 * N, N, tid * E);
      }
    }
  }
#pragma unroll
  for (int e = 0; e < E; ++e) {
    acc[0][e] = red<M>(acc[0][e]);
    acc[1][e] = red<M>(acc[1][e]);
  }
  NTT::template invC<2>(acc, xch, itw, tid);
#pragma unroll
  for (int e = 0; e < E; ++e) {
    acc0[e] = canon<M>(acc0[e] + acc[0][e]);
    acc1[e] = canon<M>(acc1[e] + acc[1][e]);
  }
}

// ACC = (0, X^{-b} * LUT) in registers; copies the twiddle tables into LDS.
template <int LEVEL, int T, int E>
__device__ __forceinline__ void br_init(double (&acc0)[E], double (&acc1)[E], const double *lut,
                                        int b, double *tws, const double *tw, const double *itw,
                                        int tid) {
  constexpr int N = Mod<LEVEL>::N;
  const int r = (2 * N - (b % (2 * N))) % (2 * N);
#pragma unroll
  for (int e = 0; e < E; ++e) {
    const int j = tid + e * T;
    acc0[e] = 0.0;
    acc1[e] = canon_small<Mod<LEVEL>>(rot_read<N>(lut, j, r));
    tws[j] = tw[j];
    tws[N + j] = itw[j];
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
__global__ __launch_bounds__(BR1_T, BR1_WAVES) void br1_kernel(const uint16_t *__restrict__ clue_a,
                                                   const uint16_t *__restrict__ clue_b,
                                                   const uint16_t *__restrict__ lwe_a,
                                                   const uint16_t *__restrict__ lwe_b,
                                                   const Key1T *__restrict__ bsk1, DeviceTables tb,
                                                   uint32_t *__restrict__ ext,
                                                   uint64_t *__restrict__ rlwe_out, int mode) {
  using M = Mod<1>;
  constexpr int T = BR1_T, E = BR1_E, N = N1;
  __shared__ double xch[(OMR_PAIR1 ? 2 : 1) * WgNtt<M, T, E>::LDS_DOUBLES];
  __shared__ double tws[2 * N];
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
  double acc0[E], acc1[E];
  br_init<1, T, E>(acc0, acc1, tb.lut1, b, tws, tb.tw1, tb.itw1, tid);
#pragma unroll 1
  for (int i = 0; i < N0; ++i) {
    const int a = __builtin_amdgcn_readfirstlane(la[i]);
    if (a == 0) continue;  // (X^0 - 1) * ACC = 0
#if OMR_PAIR1
    cmux_step_pair<1, T, E, LOGB1, D1, DROP1, Key1T, OMR_KEY_DEPTH1, OMR_MAC_EXACT1 != 0>(
        acc0, acc1, xch, a, bsk1 + (size_t)i * (2 * D1 * 2 * N), tws, tws + N, tid);
#else
    cmux_step<1, T, E, LOGB1, D1, DROP1, Key1T, OMR_KEY_DEPTH1>(
        acc0, acc1, xch, a, bsk1 + (size_t)i * (2 * D1 * 2 * N), tws, tws + N, tid);
#endif
  }
  if (mode == 0) {  // extract_lwe_locally (coefficient 0), detector.rs:561
#pragma unroll
    for (int e = 0; e < E; ++e) xch[tid + e * T] = acc0[e];
    __syncthreads();
    uint32_t *o = ext + wg * (N + 1);
#pragma unroll
    for (int e = 0; e < E; ++e) {
      const int j = tid + e * T;
      o[j] = (uint32_t)to_u64<M>(j == 0 ? xch[0] : -xch[N - j]);
    }
    if (tid == 0) o[N] = (uint32_t)to_u64<M>(acc1[0]);
  } else {
    uint64_t *o = rlwe_out + wg * 2 * N;
#pragma unroll
    for (int e = 0; e < E; ++e) {
      o[tid + e * T] = to_u64<M>(acc0[e]);
      o[N + tid + e * T] = to_u64<M>(acc1[e]);
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

// One trace digit d on the three-buffer NTT (cross-wave buffer XB): forward transform of the
// small digits (|d| <= 2, stage tables t0) and multiply-accumulate with the key row.
template <int XB>
__device__ __forceinline__ void trace_digit3(const uint32_t (&pk)[BR2_E][DigitsTrace::DW], int d,
                                             const double *__restrict__ key, double (&accA)[BR2_E],
                                             double (&accB)[BR2_E], double *xch, const double *tw,
                                             const double *t0, int tid) {
  using M = Mod<2>;
  constexpr int T = BR2_T, E = BR2_E, N = N2;
  using NTT = WgNtt<M, T, E>;
  const double *ka = key + (size_t)(d * 2) * N + tid * E;  // alpha (pre-scaled by N^-1)
  const double *kb = ka + N;                                 // beta (unscaled)
  double kra[E], krb[E];
#pragma unroll
  for (int e = 0; e < E; ++e) {
    kra[e] = ka[e];
    krb[e] = kb[e];
  }
  int dg[E];
#pragma unroll
  for (int e = 0; e < E; ++e) dg[e] = DigitsTrace::get_int(pk[e], d);
  double x[E];
  NTT::template fwd3_small<XB>(dg, t0, x, xch, tw, tid);
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

// hom_trace_store on the three-buffer exchanges (OMR_TRACE3; xch holds 3N doubles, tw the
// forward table, t0 the small-digit tables). Per automorphism step: staging of sigma_g(a)
// through X0 (trailing barrier), the 25 digit transforms on X1, X0, ..., X1 (no trailing
// barriers: consecutive cross-wave uses alternate), the body permutation through X0 (its last
// use, digit 23, is behind digit 24's barrier; trailing barrier), the inverse on X1 with the
// mirrored forward table (X1's last use, digit 24, is behind the permutation's barriers). The
// next step's staging writes X0, whose last use had a trailing barrier.
__device__ __forceinline__ void hom_trace_store3(double (&acc0)[BR2_E], double (&acc1)[BR2_E],
                                                 double *xch, const double *tw, const double *t0,
                                                 const double *__restrict__ tk, const DeviceTables &tb,
                                                 uint64_t *__restrict__ o, int tid) {
  using M = Mod<2>;
  constexpr int T = BR2_T, E = BR2_E, N = N2;
  using NTT = WgNtt<M, T, E>;
  static_assert(DT % 2 == 1, "digit pairs on X1, X0 and a last digit on X1");
  constexpr double NINV = -549755813880.0;  // 2048^-1 mod q2, centred (secret.rs:167-168)
  double ca[E], cb[E];
#pragma unroll
  for (int e = 0; e < E; ++e) {
    ca[e] = canon<M>(mm<M>(acc0[e], NINV));
    cb[e] = canon<M>(mm<M>(acc1[e], NINV));
  }
  NTT::fwd(cb, xch, tw, tid);  // X0, X1 (double-buffered), trailing barrier
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
    for (int d = 0; d < DT - 1; d += 2) {
      trace_digit3<1>(pk, d, key, accA, accB, xch, tw, t0, tid);
      trace_digit3<0>(pk, d + 1, key, accA, accB, xch, tw, t0, tid);
    }
    trace_digit3<1>(pk, DT - 1, key, accA, accB, xch, tw, t0, tid);
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
    NTT::template inv3m<1>(accA, xch, tw, tid);
#pragma unroll
    for (int e = 0; e < E; ++e) ca[e] = canon<M>(ca[e] + accA[e]);
  }
  __syncthreads();  // the last inverse's cross-wave reads of X1 are done everywhere
  NTT::fwd(ca, xch, tw, tid);
#pragma unroll
  for (int e = 0; e < E; ++e) {
    const int t = tid * E + e;
    o[t] = to_u64<M>(canon<M>(ca[e]));
    o[N + t] = to_u64<M>(cb[e]);
  }
}

// ------------------------------------------------------------------------------------------
// Level 2 (second_level_bootstrapping, detector.rs:599-624) fused with hom_trace (:626-639):
// one workgroup per message. mode 0: trace + NTT output u64 [wg][2][N2] (NttRlweCiphertext);
// mode 1: blind rotation only, coefficient-domain output (stage test).
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(BR2_T, BR2_WAVES) void br2_trace_kernel(const uint32_t *__restrict__ lwe_int,
                                                         const Key2T *__restrict__ bsk2,
                                                         const double *__restrict__ tk,
                                                         DeviceTables tb,
                                                         uint64_t *__restrict__ out, int mode) {
  using M = Mod<2>;
  constexpr int T = BR2_T, E = BR2_E, N = N2;
  using NTT = WgNtt<M, T, E>;
  __shared__ double xch[OMR_XBUF3 ? NTT::LDS3_DOUBLES : (OMR_PAIR2 ? 2 : 1) * NTT::LDS_DOUBLES];
  // tw (N) + itw (N), or with OMR_NTT_SMALL0 tw (N) + the 129-entry stage-0 table
  constexpr int TWS = (OMR_XBUF3 && OMR_NTT_SMALL0) ? N + 136 * OMR_NTT_T0_TABLES : 2 * N;
  __shared__ double tws[TWS];
  const int tid = threadIdx.x;
  const size_t wg = blockIdx.x;
  const uint32_t *lwe = lwe_int + wg * (NI + 1);
  double acc0[E], acc1[E];
  const double *tw = tws, *itw = tws + N, *t0 = tws + N;
  if (OMR_XBUF3 && OMR_NTT_SMALL0) {
    const int b = (int)lwe[NI];
    const int rr = (2 * N - (b % (2 * N))) % (2 * N);
#pragma unroll
    for (int e = 0; e < E; ++e) {
      const int j = tid + e * T;
      acc0[e] = 0.0;
      acc1[e] = canon_small<M>(rot_read<N>(tb.lut2, j, rr));
      tws[j] = tb.tw2[j];
    }
    if (tid <= 128) {  // table k: d * c_k, d = tid - 64 (c = tw1 [, tw2, tw1 tw2, tw3, tw1 tw3])
      const double w1 = tb.tw2[1], w2 = tb.tw2[2], w3 = tb.tw2[3];
      const double c[5] = {w1, w2, canon<M>(mm<M>(w1, w2)), w3, canon<M>(mm<M>(w1, w3))};
#pragma unroll
      for (int k = 0; k < OMR_NTT_T0_TABLES; ++k) tws[N + 136 * k + tid] = canon<M>(mm<M>((double)(tid - 64), c[k]));
    }
    __syncthreads();
  } else {
    br_init<2, T, E>(acc0, acc1, tb.lut2, (int)lwe[NI], tws, tb.tw2, tb.itw2, tid);
  }
#pragma unroll 1
  for (int i = 0; i < NI; ++i) {
    const int a = (int)__builtin_amdgcn_readfirstlane(lwe[i]) & (2 * N - 1);
    if (a == 0) continue;
#if OMR_XBUF3
    cmux_step3<T, E, Key2T>(acc0, acc1, xch, a, bsk2 + (size_t)OMR_KEYROW2(i) * (2 * D2 * 2 * N), tw,
                            itw, tid, t0);
#elif OMR_PAIR2
    cmux_step_pair<2, T, E, LOGB2, D2, DROP2, Key2T, OMR_KEY_DEPTH2, false>(
        acc0, acc1, xch, a, bsk2 + (size_t)OMR_KEYROW2(i) * (2 * D2 * 2 * N), tw, itw, tid);
#else
    cmux_step<2, T, E, LOGB2, D2, DROP2, Key2T, OMR_KEY_DEPTH2, OMR_NTT_GTW != 0>(
        acc0, acc1, xch, a, bsk2 + (size_t)OMR_KEYROW2(i) * (2 * D2 * 2 * N), tw, itw, tid, tb.tw2,
        tb.itw2);
#endif
  }
  uint64_t *o = out + wg * 2 * N;
#ifdef OMR_EXPT_NO_TRACE  // timing experiment only (wrong results): blind rotation without the trace
  mode = 1;
#endif
  if (mode == 1) {
#pragma unroll
    for (int e = 0; e < E; ++e) {
      o[tid + e * T] = to_u64<M>(acc0[e]);
      o[N + tid + e * T] = to_u64<M>(acc1[e]);
    }
    return;
  }
  if (OMR_XBUF3) __syncthreads();  // the last inverse's cross-wave reads of X0 are done everywhere
  if (OMR_XBUF3 && OMR_NTT_SMALL0 && OMR_TRACE3) {
    hom_trace_store3(acc0, acc1, xch, tw, t0, tk, tb, o, tid);
  } else if (OMR_XBUF3 && OMR_NTT_SMALL0) {  // the trace's inverse table goes to the W buffer
    double *itw_t = xch + 2 * N;
#pragma unroll
    for (int e = 0; e < E; ++e) itw_t[tid + e * T] = tb.itw2[tid + e * T];
    __syncthreads();
    hom_trace_store(acc0, acc1, xch, tw, itw_t, tk, tb, o, tid);
  } else {
    hom_trace_store(acc0, acc1, xch, tw, itw, tk, tb, o, tid);
  }
}

}  // namespace omr

#include "br2_fft.hpp"
#include "br2_sliced.hpp"
