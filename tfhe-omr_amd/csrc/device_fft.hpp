// Wave-level 512-point complex FFT for the level-1 external product (gfx950).
//
// Level-1 residues are small: gadget digits satisfy |d| <= 17 and key coefficients |k| <= 2^26,
// so every coefficient of sum_r d_r * k_r over the 8 GGSW rows is an integer below 2^43 and an
// FP64 FFT product rounds to it exactly (worst error of a lane-exact model of this transform
// with adversarial digits: 1.8e-3, tools/fft_exactness.py; rigorous FFT product bounds < 0.15). The transform
// therefore replaces the 1024-point NTT mod q1 with a 512-point complex transform at ~45 % of
// its FP64 work, and the results stay bit-identical to the modular computation.
//
// Ring map: R[X]/(X^1024 + 1) -> C[X]/(X^512 - i), p -> z with z_j = p_j + i p_{j+512}.
// X^512 - i splits over the roots w^(1+4k) (w = exp(i pi / 1024)); the forward transform is a
// Cooley-Tukey tree on that factorisation (the twist is folded into the twiddles), the inverse a
// Gentleman-Sande tree with conjugate twiddles, unscaled (the 1/512 is folded into the keys).
//
// One wave (64 lanes) owns a transform (or C interleaved ones), 8 complex values per lane, 3
// radix-2 stages per pass, 2 LDS exchanges per transform (wave-private 8 KB buffer, XOR swizzle found by
// tools/fft_lds_banks.py: no bank conflicts for ds_write_b128 / ds_read_b128).
//   forward: in  x[e] = coefficient (lane + 64 e)    out x[e] = transform index (8 lane + e)
//   inverse: in  x[e] = transform index (8 lane + e)  out x[e] = coefficient (lane + 64 e)
// Twiddles: node i of stage s uses w^(eps(s, i) / 2) with eps(0, 0) = 512,
// eps(s+1, 2i) = eps(s, i) / 2, eps(s+1, 2i+1) = eps(s, i) / 2 + 1024 (mod 2048); table layout in
// twiddle_index (stages 0-5 at (1 << s) + i, stages 6-8 lane-minor).
#pragma once

#include "device_ntt.hpp"

namespace omr {

struct Fft512 {
  static constexpr int T = 64, E = 8, N = 512, L = 9, R = 3, NPASS = 3;

  // element index of register e in pass p (the WgNtt scheme with r == R in every pass)
  __device__ static __forceinline__ int index(int p, int lane, int e) {
    const int lb = L - (p + 1) * R;
    return ((lane >> lb) << (L - p * R)) | (e << lb) | (lane & ((1 << lb) - 1));
  }
  // bank-conflict-free XOR swizzle (linear over GF(2), so swz(a ^ b) == swz(a) ^ swz(b))
  __device__ static __forceinline__ int swz(int j) {
    return j ^ (((j >> 3) & 1) * 4) ^ (((j >> 4) & 1) * 9) ^ (((j >> 5) & 1) * 15) ^
           (((j >> 6) & 1) * 14) ^ (((j >> 8) & 1) * 8);
  }

  // Node twiddle of stage P*R + k for register e. The last pass's stages (6, 7, 8) are stored
  // lane-minor (entry (1 << s) + j * 64 + lane holds node (lane << k) + j) so that a wave's
  // ds_read_b128 hits 64 consecutive entries (no bank conflicts); earlier passes broadcast.
  template <int P>
  __device__ static __forceinline__ int twiddle_index(int k, int e, int lane) {
    constexpr int s0 = P * R, lb = L - s0 - R;
    if constexpr (P == NPASS - 1) return (1 << (s0 + k)) + ((e >> (R - k)) << 6) + lane;
    return (1 << (s0 + k)) + (((lane >> lb) << k) | (e >> (R - k)));
  }

  // C independent transforms interleaved (C x 8 complex per lane, C LDS buffers of 512)
  template <int C>
  __device__ static __forceinline__ void exchange(double (&xr)[C][E], double (&xi)[C][E],
                                                  double2 *lds, int lane, int p_from, int p_to) {
#pragma unroll
    for (int c = 0; c < C; ++c)
#pragma unroll
      for (int e = 0; e < E; ++e)
        lds[c * N + swz(index(p_from, lane, e))] = make_double2(xr[c][e], xi[c][e]);
    __syncthreads();
#pragma unroll
    for (int c = 0; c < C; ++c)
#pragma unroll
      for (int e = 0; e < E; ++e) {
        const double2 v = lds[c * N + swz(index(p_to, lane, e))];
        xr[c][e] = v.x;
        xi[c][e] = v.y;
      }
    __syncthreads();
  }

  template <int P, int C>
  __device__ static __forceinline__ void fwd_pass(double (&xr)[C][E], double (&xi)[C][E],
                                                  const double2 *tws, int lane) {
    constexpr int s0 = P * R, lb = L - s0 - R;
#pragma unroll
    for (int k = 0; k < R; ++k) {
      const int half = 1 << (R - 1 - k);
#pragma unroll
      for (int e = 0; e < E; ++e) {
        if (e & half) continue;
        const double2 w = tws[twiddle_index<P>(k, e, lane)];
#pragma unroll
        for (int c = 0; c < C; ++c) {
          const double vr = __fma_rn(xr[c][e + half], w.x, -xi[c][e + half] * w.y);
          const double vi = __fma_rn(xr[c][e + half], w.y, xi[c][e + half] * w.x);
          const double ur = xr[c][e], ui = xi[c][e];
          xr[c][e] = ur + vr;
          xi[c][e] = ui + vi;
          xr[c][e + half] = ur - vr;
          xi[c][e + half] = ui - vi;
        }
      }
    }
  }
  template <int P, int C>
  __device__ static __forceinline__ void inv_pass(double (&xr)[C][E], double (&xi)[C][E],
                                                  const double2 *tws, int lane) {
    constexpr int s0 = P * R, lb = L - s0 - R;
#pragma unroll
    for (int k = R - 1; k >= 0; --k) {
      const int half = 1 << (R - 1 - k);
#pragma unroll
      for (int e = 0; e < E; ++e) {
        if (e & half) continue;
        const double2 w = tws[twiddle_index<P>(k, e, lane)];
#pragma unroll
        for (int c = 0; c < C; ++c) {
          const double ur = xr[c][e], ui = xi[c][e];
          const double dr = ur - xr[c][e + half], di = ui - xi[c][e + half];
          xr[c][e] = ur + xr[c][e + half];
          xi[c][e] = ui + xi[c][e + half];
          // (dr + i di) * conj(w)
          xr[c][e + half] = __fma_rn(dr, w.x, di * w.y);
          xi[c][e + half] = __fma_rn(di, w.x, -dr * w.y);
        }
      }
    }
  }

  template <int C>
  __device__ static __forceinline__ void fwd(double (&xr)[C][E], double (&xi)[C][E], double2 *lds,
                                             const double2 *tws, int lane) {
    fwd_pass<0, C>(xr, xi, tws, lane);
    exchange<C>(xr, xi, lds, lane, 0, 1);
    fwd_pass<1, C>(xr, xi, tws, lane);
    exchange<C>(xr, xi, lds, lane, 1, 2);
    fwd_pass<2, C>(xr, xi, tws, lane);
  }
  template <int C>
  __device__ static __forceinline__ void inv(double (&xr)[C][E], double (&xi)[C][E], double2 *lds,
                                             const double2 *tws, int lane) {
    inv_pass<2, C>(xr, xi, tws, lane);
    exchange<C>(xr, xi, lds, lane, 2, 1);
    inv_pass<1, C>(xr, xi, tws, lane);
    exchange<C>(xr, xi, lds, lane, 1, 0);
    inv_pass<0, C>(xr, xi, tws, lane);
  }
  // single transform
  __device__ static __forceinline__ void fwd(double (&xr)[E], double (&xi)[E], double2 *lds,
                                             const double2 *tws, int lane) {
    fwd<1>(reinterpret_cast<double(&)[1][E]>(xr), reinterpret_cast<double(&)[1][E]>(xi), lds, tws, lane);
  }
  __device__ static __forceinline__ void inv(double (&xr)[E], double (&xi)[E], double2 *lds,
                                             const double2 *tws, int lane) {
    inv<1>(reinterpret_cast<double(&)[1][E]>(xr), reinterpret_cast<double(&)[1][E]>(xi), lds, tws, lane);
  }
};

}  // namespace omr
