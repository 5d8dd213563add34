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
// eps(s+1, 2i+1) = eps(s, i) / 2 + 2n (mod 4n). Passes are radix-8 blocks of that tree (WgFft::fwd_pass).
//
// T lanes hold E complex values each (N = T E), log2(E) = 3 stages per pass, an LDS exchange
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
  // Radix-8 passes. Pass P of a lane works on one block of the twiddle tree: the stage-s0 node
  // hi = F >> lb with twiddle A, its children (B, i B) and grandchildren (C, i C, w8 C, i w8 C),
  // w8 = exp(i pi / 4) (node 4 hi + 2 is the even child of node 2 hi + 1: eps / 4 + n). Three radix-2
  // stages on registers e (pairs (e, e + 4) with A; (e, e + 2) with B / i B; (e, e + 1) with C, i C,
  // w8 C, i w8 C) equal "multiply x_e by T_e, then a constant 8-point network" with
  // T = (1, C, B, BC, A, AC, AB, ABC): 7 complex products + 24 complex additions, the factors i
  // free and w8 folded into FMAs -- 80 FP64 operations instead of 96
  // (tools/fft_exactness.py checks both forms against the exact product).
  // Table: entry t * 8^P - 1 + hi holds T_t of block hi of pass P (t = 1..7; 511 entries), so a
  // pass-2 read is lane-contiguous and pass-0 reads are wave-uniform.
  static_assert(R == 3 && L % R == 0, "radix-8 passes: every pass has three stages");
  __device__ static __forceinline__ constexpr int tw_base(int p) { return (1 << (3 * p)) - 1; }
  template <int P>
  __device__ static __forceinline__ int block_of(int lane) { return lane >> (L - P * R - R); }
  template <int P, bool G>
  __device__ static __forceinline__ double2 block_twiddle(const double2 *tws, const double2 *__restrict__ gtw,
                                                          int t, int hi) {
    const int idx = t * (1 << (3 * P)) - 1 + hi;
    if constexpr (P == 0 && G) return gtw[idx];  // hi == 0: uniform, scalar loads
    return tws[idx];
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

  static constexpr double S8 = 0.70710678118654752440;  // 1 / sqrt(2), w8 = S8 (1 + i)

  template <int P, int C, bool G = false>
  __device__ static __forceinline__ void fwd_pass(double (&xr)[C][E], double (&xi)[C][E],
                                                  const double2 *tws, int lane,
                                                  const double2 *__restrict__ gtw = nullptr) {
    const int hi = block_of<P>(lane);
#pragma unroll
    for (int t = 1; t < 8; ++t) {  // x_t *= T_t
      const double2 w = block_twiddle<P, G>(tws, gtw, t, hi);
#pragma unroll
      for (int c = 0; c < C; ++c) {
        const double r = __fma_rn(xr[c][t], w.x, -xi[c][t] * w.y);
        const double i = __fma_rn(xr[c][t], w.y, xi[c][t] * w.x);
        xr[c][t] = r;
        xi[c][t] = i;
      }
    }
#pragma unroll
    for (int c = 0; c < C; ++c) {
      double ar[4], ai[4], br[4], bi[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        ar[e] = xr[c][e] + xr[c][e + 4];
        ai[e] = xi[c][e] + xi[c][e + 4];
        br[e] = xr[c][e] - xr[c][e + 4];
        bi[e] = xi[c][e] - xi[c][e + 4];
      }
      // c = a0 +- a2, a1 +- a3; d = b0 +- i b2, b1 +- i b3
      const double c0r = ar[0] + ar[2], c0i = ai[0] + ai[2], c2r = ar[0] - ar[2], c2i = ai[0] - ai[2];
      const double c1r = ar[1] + ar[3], c1i = ai[1] + ai[3], c3r = ar[1] - ar[3], c3i = ai[1] - ai[3];
      const double d0r = br[0] - bi[2], d0i = bi[0] + br[2], d2r = br[0] + bi[2], d2i = bi[0] - br[2];
      const double d1r = br[1] - bi[3], d1i = bi[1] + br[3], d3r = br[1] + bi[3], d3i = bi[1] - br[3];
      xr[c][0] = c0r + c1r;
      xi[c][0] = c0i + c1i;
      xr[c][1] = c0r - c1r;
      xi[c][1] = c0i - c1i;
      xr[c][2] = c2r - c3i;  // c2 + i c3
      xi[c][2] = c2i + c3r;
      xr[c][3] = c2r + c3i;  // c2 - i c3
      xi[c][3] = c2i - c3r;
      const double u = d1r - d1i, v = d1r + d1i;  // w8 d1 = S8 (u + i v)
      xr[c][4] = __fma_rn(S8, u, d0r);
      xi[c][4] = __fma_rn(S8, v, d0i);
      xr[c][5] = __fma_rn(-S8, u, d0r);
      xi[c][5] = __fma_rn(-S8, v, d0i);
      const double u3 = d3r + d3i, v3 = d3r - d3i;  // i w8 d3 = S8 (-u3 + i v3)
      xr[c][6] = __fma_rn(-S8, u3, d2r);
      xi[c][6] = __fma_rn(S8, v3, d2i);
      xr[c][7] = __fma_rn(S8, u3, d2r);
      xi[c][7] = __fma_rn(-S8, v3, d2i);
    }
  }
  // Unscaled inverse of fwd_pass (8 x its inverse): the adjoint network, then x_e *= conj(T_e).
  template <int P, int C, bool G = false>
  __device__ static __forceinline__ void inv_pass(double (&xr)[C][E], double (&xi)[C][E],
                                                  const double2 *tws, int lane,
                                                  const double2 *__restrict__ gtw = nullptr) {
    const int hi = block_of<P>(lane);
#pragma unroll
    for (int c = 0; c < C; ++c) {
      const double *o_r = xr[c], *o_i = xi[c];
      const double c0r = o_r[0] + o_r[1], c0i = o_i[0] + o_i[1], c1r = o_r[0] - o_r[1], c1i = o_i[0] - o_i[1];
      const double c2r = o_r[2] + o_r[3], c2i = o_i[2] + o_i[3];
      const double c3r = o_i[2] - o_i[3], c3i = o_r[3] - o_r[2];  // -i (o2 - o3)
      const double d0r = o_r[4] + o_r[5], d0i = o_i[4] + o_i[5];
      const double ur = o_r[4] - o_r[5], ui = o_i[4] - o_i[5];
      const double d1r = ur + ui, d1i = ui - ur;  // (1 - i) (o4 - o5) = sqrt 2 conj(w8) (o4 - o5)
      const double d2r = o_r[6] + o_r[7], d2i = o_i[6] + o_i[7];
      const double vr = o_r[6] - o_r[7], vi = o_i[6] - o_i[7];
      const double d3r = vi - vr, d3i = -vr - vi;  // (-1 - i) (o6 - o7) = sqrt 2 conj(i w8) (o6 - o7)
      const double a0r = c0r + c2r, a0i = c0i + c2i, a2r = c0r - c2r, a2i = c0i - c2i;
      const double a1r = c1r + c3r, a1i = c1i + c3i, a3r = c1r - c3r, a3i = c1i - c3i;
      const double b0r = d0r + d2r, b0i = d0i + d2i;
      const double b2r = d0i - d2i, b2i = d2r - d0r;  // -i (d0 - d2)
      const double b1r = d1r + d3r, b1i = d1i + d3i;
      const double b3r = d1i - d3i, b3i = d3r - d1r;  // -i (d1 - d3)
      xr[c][0] = a0r + b0r;
      xi[c][0] = a0i + b0i;
      xr[c][4] = a0r - b0r;
      xi[c][4] = a0i - b0i;
      xr[c][2] = a2r + b2r;
      xi[c][2] = a2i + b2i;
      xr[c][6] = a2r - b2r;
      xi[c][6] = a2i - b2i;
      xr[c][1] = __fma_rn(S8, b1r, a1r);
      xi[c][1] = __fma_rn(S8, b1i, a1i);
      xr[c][5] = __fma_rn(-S8, b1r, a1r);
      xi[c][5] = __fma_rn(-S8, b1i, a1i);
      xr[c][3] = __fma_rn(S8, b3r, a3r);
      xi[c][3] = __fma_rn(S8, b3i, a3i);
      xr[c][7] = __fma_rn(-S8, b3r, a3r);
      xi[c][7] = __fma_rn(-S8, b3i, a3i);
    }
#pragma unroll
    for (int t = 1; t < 8; ++t) {  // x_t *= conj(T_t)
      const double2 w = block_twiddle<P, G>(tws, gtw, t, hi);
#pragma unroll
      for (int c = 0; c < C; ++c) {
        const double r = __fma_rn(xr[c][t], w.x, xi[c][t] * w.y);
        const double i = __fma_rn(xi[c][t], w.x, -xr[c][t] * w.y);
        xr[c][t] = r;
        xi[c][t] = i;
      }
    }
  }
  // C transforms at once (lds holds C * BUF complex)
  // G: pass-0 twiddles from the global table gtw (must be non-null)
  template <int C, bool G = false>
  __device__ static __forceinline__ void fwd(double (&xr)[C][E], double (&xi)[C][E], double2 *lds,
                                             const double2 *tws, int lane,
                                             const double2 *__restrict__ gtw = nullptr) {
    static_assert(NPASS <= 5, "unrolled for up to 5 passes");
    fwd_pass<0, C, G>(xr, xi, tws, lane, gtw);
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
