// Workgroup complex FFTs for the external products (gfx950).
//
// Exactness: the external product only ever multiplies small gadget digits by key residues, so
// every coefficient of sum_r digit_r * key_r is an integer well inside FP64's 53 bits and an FP64
// FFT product rounds to it exactly:
//   level 1: |d| <= 17, |k| <= 2^26, 8 rows, N = 1024: |coef| < 2^43; worst error of a lane-exact
//            model with adversarial digits 1.8e-3 (tools/fft_exactness.py), rigorous bound < 0.15;
// Replacing the modular NTTs by half-length complex FFTs removes ~45 % of the level-1 FP64 work,
// with bit-identical results.
//
// Ring map: R[X]/(X^2n + 1) -> C[X]/(X^n - i), p -> z with z_j = p_j + i p_{j+n}, n = 2^L.
// X^n - i splits over the roots w^(1+4k) (w = exp(i pi / 2n)); the forward transform is a
// Cooley-Tukey tree on that factorisation (the twist is folded into the twiddles), the inverse a
// Gentleman-Sande tree with conjugate twiddles, unscaled (the 1/n is folded into the keys).
// Node i of stage s uses w^(eps(s, i) / 2), eps(0, 0) = n, eps(s+1, 2i) = eps(s, i) / 2,
// eps(s+1, 2i+1) = eps(s, i) / 2 + 2n (mod 4n); table layout in twiddle_index.
//
// T lanes hold E complex values each (N = T E), log2(E) radix-2 stages per pass, an LDS exchange
// between passes (XOR swizzle found by tools/fft_lds_banks.py: no bank conflicts for
// ds_write_b128 / ds_read_b128), C independent transforms interleaved. One wave per transform.
//   forward: in  x[e] = coefficient (lane + T e)    out x[e] = transform index (E lane + e)
//   inverse: in  x[e] = transform index (E lane + e) out x[e] = coefficient (lane + T e)
#pragma once

#include <utility>

#include "device_ntt.hpp"

namespace omr {

// LDS visibility within one wave: this wave's LDS writes have landed, and the compiler moves no
// memory operation across (waves of a workgroup stay independent).
__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0)
  __builtin_amdgcn_wave_barrier();
  __atomic_signal_fence(__ATOMIC_SEQ_CST);
}
// Compiler-only ordering of one wave's LDS accesses (its LDS operations complete in order).
__device__ __forceinline__ void wave_lds_fence() {
  __builtin_amdgcn_wave_barrier();
  __atomic_signal_fence(__ATOMIC_SEQ_CST);
}
// XOR swizzle of the LDS exchange slots, slot(j) = j ^ f(j), f linear over GF(2): no bank
// conflicts for any exchange of the geometry (tools/fft_lds_banks.py 64 8 9).
template <int T, int E, int L>
struct FftSwizzle;
template <>
struct FftSwizzle<64, 8, 9> {
  static constexpr int M[6] = {4, 9, 15, 14, 0, 8};
};

template <int T_, int E_, int L_>
struct WgFft {
  static constexpr int T = T_, E = E_, L = L_, N = T * E, R = ilog2(E), NPASS = (L + R - 1) / R;
  static_assert(N == (1 << L), "FFT geometry");
  static_assert(T == 64, "one transform per wave (wave-level LDS synchronisation)");
  // stages in pass p (the last pass may be shorter)
  static constexpr int stages(int p) { return (L - p * R) < R ? (L - p * R) : R; }

  // element index of register e in pass p (the WgNtt scheme, partial last pass included)
  __device__ static __forceinline__ int index(int p, int lane, int e) {
    const int s0 = p * R, r = stages(p), lb = L - s0 - r;
    const int F = (lane << (R - r)) | (e >> r);
    return ((F >> lb) << (L - s0)) | ((e & ((1 << r) - 1)) << lb) | (F & ((1 << lb) - 1));
  }
  // bank-conflict-free XOR swizzle (linear over GF(2); folds to constants per unrolled e)
  template <int... B>
  __device__ static __forceinline__ int swz_bits(int j, std::integer_sequence<int, B...>) {
    return (0 ^ ... ^ (((j >> (3 + B)) & 1) * FftSwizzle<T, E, L>::M[B]));
  }
  __device__ static __forceinline__ int swz(int j) {
    return j ^ swz_bits(j, std::make_integer_sequence<int, L - 3>{});
  }
  static constexpr int BUF = N;  // LDS slots (double2) per transform
  // slot of register e of `lane` in pass p
  __device__ static __forceinline__ int slot(int p, int lane, int e) { return swz(index(p, lane, e)); }
  // Node twiddle of stage P*R + k for register e. The last pass's stages are stored lane-minor
  // (entry (1 << s) + j * T + lane holds node (lane << k) + j) so a wave reads consecutive
  // entries; in earlier passes lanes of a group share (broadcast) entries.
  template <int P>
  __device__ static __forceinline__ int twiddle_index(int k, int e, int lane) {
    constexpr int s0 = P * R, r = stages(P), lb = L - s0 - r;
    const int F = (lane << (R - r)) | (e >> r);
    const int node = ((F >> lb) << k) | ((e & ((1 << r) - 1)) >> (r - k));
    if constexpr (P == NPASS - 1) {  // lane-minor: node = (lane << q) | j  ->  (1 << s) + j T + lane
      const int q = R - r + k;
      return (1 << (s0 + k)) + (node & ((1 << q) - 1)) * T + lane;
    }
    return (1 << (s0 + k)) + node;
  }

  // Exchange between passes PF and PT through the wave's LDS buffer (C transforms).
  template <int C, int PF, int PT>
  __device__ static __forceinline__ void exchange(double (&xr)[C][E], double (&xi)[C][E],
                                                  double2 *lds, int lane) {
#pragma unroll
    for (int c = 0; c < C; ++c)
#pragma unroll
      for (int e = 0; e < E; ++e)
        lds[c * BUF + slot(PF, lane, e)] = make_double2(xr[c][e], xi[c][e]);
    wave_lds_sync();
#pragma unroll
    for (int c = 0; c < C; ++c)
#pragma unroll
      for (int e = 0; e < E; ++e) {
        const double2 v = lds[c * BUF + slot(PT, lane, e)];
        xr[c][e] = v.x;
        xi[c][e] = v.y;
      }
    // the next exchange's writes must not move above these reads: a compiler fence suffices
    // (one wave's LDS operations complete in order; waiting for the reads here is 1.1 % slower)
    wave_lds_fence();
  }

  // Pass 0's node index does not depend on the lane (lane >> (L - R) == 0), so its twiddles
  // are read from the global table with uniform addresses (scalar loads kept in SGPRs) when
  // gtw is given; later passes read the LDS copy.
  template <int P, bool G>
  __device__ static __forceinline__ double2 twiddle(const double2 *tws, const double2 *__restrict__ gtw,
                                                    int k, int e, int lane) {
    if constexpr (P == 0 && G) return gtw[(1 << k) + ((e & ((1 << stages(0)) - 1)) >> (stages(0) - k))];
    return tws[twiddle_index<P>(k, e, lane)];
  }

  // K0: first stage of the pass (a caller that computed stage 0 itself passes 1)
  template <int P, int C, bool G = false, int K0 = 0>
  __device__ static __forceinline__ void fwd_pass(double (&xr)[C][E], double (&xi)[C][E],
                                                  const double2 *tws, int lane,
                                                  const double2 *__restrict__ gtw = nullptr) {
    constexpr int r = stages(P);
#pragma unroll
    for (int k = K0; k < r; ++k) {
      const int half = 1 << (r - 1 - k);
#pragma unroll
      for (int e = 0; e < E; ++e) {
        if (e & half) continue;
        // sibling nodes 2j, 2j + 1 have twiddles w and i w (half-angles of eps and eps + 2n):
        // odd nodes reuse the even twiddle and apply the factor i by swapping parts (fewer LDS
        // twiddle reads, no extra arithmetic)
        const int pb = k >= 1 ? (1 << (r - k)) : 0;
        const bool odd = (e & pb) != 0;
        const double2 w = twiddle<P, G>(tws, gtw, k, odd ? (e & ~pb) : e, lane);
#pragma unroll
        for (int c = 0; c < C; ++c) {
          const double vr = __fma_rn(xr[c][e + half], w.x, -xi[c][e + half] * w.y);
          const double vi = __fma_rn(xr[c][e + half], w.y, xi[c][e + half] * w.x);
          const double ur = xr[c][e], ui = xi[c][e];
          xr[c][e] = odd ? ur - vi : ur + vr;  // u + i v  |  u + v
          xi[c][e] = odd ? ui + vr : ui + vi;
          xr[c][e + half] = odd ? ur + vi : ur - vr;
          xi[c][e + half] = odd ? ui - vr : ui - vi;
        }
      }
    }
  }
  template <int P, int C, bool G = false>
  __device__ static __forceinline__ void inv_pass(double (&xr)[C][E], double (&xi)[C][E],
                                                  const double2 *tws, int lane,
                                                  const double2 *__restrict__ gtw = nullptr) {
    constexpr int r = stages(P);
#pragma unroll
    for (int k = r - 1; k >= 0; --k) {
      const int half = 1 << (r - 1 - k);
#pragma unroll
      for (int e = 0; e < E; ++e) {
        if (e & half) continue;
        const int pb = k >= 1 ? (1 << (r - k)) : 0;  // see fwd_pass
        const bool odd = (e & pb) != 0;
        const double2 w = twiddle<P, G>(tws, gtw, k, odd ? (e & ~pb) : e, lane);
#pragma unroll
        for (int c = 0; c < C; ++c) {
          const double ur = xr[c][e], ui = xi[c][e];
          const double dr = ur - xr[c][e + half], di = ui - xi[c][e + half];
          xr[c][e] = ur + xr[c][e + half];
          xi[c][e] = ui + xi[c][e + half];
          // (dr + i di) * conj(w); odd node: conj(i w) = -i conj(w)
          const double tr = __fma_rn(dr, w.x, di * w.y), ti = __fma_rn(di, w.x, -dr * w.y);
          xr[c][e + half] = odd ? ti : tr;
          xi[c][e + half] = odd ? -tr : ti;
        }
      }
    }
  }
  // C transforms at once (lds holds C * BUF complex)
  // G: pass-0 twiddles from the global table gtw (must be non-null)
  template <int C, bool G = false, int K0 = 0>
  __device__ static __forceinline__ void fwd(double (&xr)[C][E], double (&xi)[C][E], double2 *lds,
                                             const double2 *tws, int lane,
                                             const double2 *__restrict__ gtw = nullptr) {
    static_assert(NPASS <= 5, "unrolled for up to 5 passes");
    fwd_pass<0, C, G, K0>(xr, xi, tws, lane, gtw);
#define OMR_FFT_FWD_STEP(P)                                                                   \
  if constexpr (NPASS > P) {                                                                  \
    constexpr int Q = NPASS > P ? P : 1;                                                      \
    exchange<C, Q - 1, Q>(xr, xi, lds, lane);                                                 \
    fwd_pass<(NPASS > P ? P : 0), C>(xr, xi, tws, lane);                                      \
  }
    OMR_FFT_FWD_STEP(1)
    OMR_FFT_FWD_STEP(2)
    OMR_FFT_FWD_STEP(3)
    OMR_FFT_FWD_STEP(4)
#undef OMR_FFT_FWD_STEP
  }
  template <int C, bool G = false>
  __device__ static __forceinline__ void inv(double (&xr)[C][E], double (&xi)[C][E], double2 *lds,
                                             const double2 *tws, int lane,
                                             const double2 *__restrict__ gtw = nullptr) {
    static_assert(NPASS <= 5, "unrolled for up to 5 passes");
#define OMR_FFT_INV_STEP(P)                                                                   \
  if constexpr (NPASS > P) {                                                                  \
    constexpr int Q = NPASS > P ? P : 1;                                                      \
    inv_pass<(NPASS > P ? P : 0), C>(xr, xi, tws, lane);                                      \
    exchange<C, Q, Q - 1>(xr, xi, lds, lane);                                                 \
  }
    OMR_FFT_INV_STEP(4)
    OMR_FFT_INV_STEP(3)
    OMR_FFT_INV_STEP(2)
    OMR_FFT_INV_STEP(1)
#undef OMR_FFT_INV_STEP
    inv_pass<0, C, G>(xr, xi, tws, lane, gtw);
  }
  __device__ static __forceinline__ void fwd(double (&xr)[E], double (&xi)[E], double2 *lds,
                                             const double2 *tws, int lane,
                                             const double2 *__restrict__ gtw = nullptr) {
    fwd<1>(reinterpret_cast<double(&)[1][E]>(xr), reinterpret_cast<double(&)[1][E]>(xi), lds, tws, lane);
  }
  __device__ static __forceinline__ void inv(double (&xr)[E], double (&xi)[E], double2 *lds,
                                             const double2 *tws, int lane,
                                             const double2 *__restrict__ gtw = nullptr) {
    inv<1>(reinterpret_cast<double(&)[1][E]>(xr), reinterpret_cast<double(&)[1][E]>(xi), lds, tws, lane);
  }
};

using Fft512 = WgFft<64, 8, 9>;  // level 1: N1 = 1024, one wave

}  // namespace omr
