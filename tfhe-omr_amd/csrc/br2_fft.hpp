// Level-2 blind rotation with the FFT external product (second_level_bootstrapping,
// detector.rs:599-624) fused with hom_trace (:626-639): one 256-thread workgroup per message.
//
// q2 has 50 bits, so each BSK2 coefficient is split into two 25-bit limbs,
// k = k1 * 2^25 + k0 with k0 in [-2^24, 2^24): every product sum_r digit_r * limb_r is then an
// integer below 2^44.6 and the FP64 FFT returns it exactly (device_fft.hpp). Per CMUX step:
//   digits of (X^a - 1) * ACC (Digits8, 6 signed 7-bit digits per coefficient and poly)
//   -> 12 forward 1024-point FFTs, each multiplied into 4 accumulators (A/B output x limb) with
//   the pre-transformed key limbs -> 4 inverse FFTs -> round, out = red(P0) + 2^25 red(P1) mod
//   q2, added into ACC (coefficient domain, canonical, layout tid + 256 e as the NTT trace uses).
// Registers per thread: ACC 16 doubles, digits 16 u32, one transform 8 doubles, accumulators 32
// doubles, one key row 32 doubles. LDS: 32 KB exchange + 32 KB twiddles (FFT during the blind
// rotation, NTT tables during the trace).
#pragma once

#include "device_fft.hpp"

namespace omr {

#ifndef BR2F_PAIR
#define BR2F_PAIR 0       // transform mask and body digit k together (more spills: slower)
#endif
#ifndef BR2F_KEY_SPLIT
#define BR2F_KEY_SPLIT 1  // (unpaired) load the B-output key limbs after the transform
#endif

constexpr double LIMB2 = 33554432.0;  // 2^25

#ifdef OMR_BR2_GEOM_DEFAULT
__device__ __forceinline__ void br2f_step(double (&acc0)[BR2_E], double (&acc1)[BR2_E], double2 *xch,
                                          const double2 *tws, int a, const double2 *__restrict__ ggsw,
                                          int tid) {
  using F = Fft1024;
  using M = Mod<2>;
  using DG = DigitsFor<2, LOGB2, D2, DROP2>;
  constexpr int T = BR2_T, NF = F::N;
  static_assert(T == F::T && BR2_E == 2 * F::E, "level-2 FFT geometry must match the ACC layout");
  double *xd = reinterpret_cast<double *>(xch);
  uint32_t pk[2][BR2_E][DG::DW];
  {
    double v[BR2_E];
    rotate_diff<M, T, BR2_E>(acc0, xd, a, tid, v);
#pragma unroll
    for (int e = 0; e < BR2_E; ++e) DG::pack(v[e], pk[0][e]);
    rotate_diff<M, T, BR2_E>(acc1, xd, a, tid, v);
#pragma unroll
    for (int e = 0; e < BR2_E; ++e) DG::pack(v[e], pk[1][e]);
  }
  double outr[2][2][4], outi[2][2][4];  // [output A/B][limb][point]
#pragma unroll
  for (int o = 0; o < 2; ++o)
#pragma unroll
    for (int l = 0; l < 2; ++l)
#pragma unroll
      for (int e = 0; e < 4; ++e) outr[o][l][e] = outi[o][l][e] = 0.0;
#if BR2F_PAIR
  // mask digit k and body digit k transformed together (shared exchanges / barriers)
#pragma unroll 1
  for (int k = 0; k < D2; ++k) {
    const double2 *kr0 = ggsw + (size_t)k * 4 * NF + tid * 4;         // row k (mask digit)
    const double2 *kr1 = ggsw + (size_t)(D2 + k) * 4 * NF + tid * 4;  // row D2 + k (body digit)
    double2 key[2][2][4];  // [row][limb][point], A output first
#pragma unroll
    for (int l = 0; l < 2; ++l)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        key[0][l][e] = kr0[l * NF + e];
        key[1][l][e] = kr1[l * NF + e];
      }
    double xr[2][4], xi[2][4];
#pragma unroll
    for (int p = 0; p < 2; ++p)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        xr[p][e] = DG::get(pk[p][e], k);
        xi[p][e] = DG::get(pk[p][e + 4], k);
      }
    F::fwd<2>(xr, xi, xch, tws, tid);
#pragma unroll
    for (int o = 0; o < 2; ++o) {
      if (o == 1) {  // B-output limbs, loaded after the transform
#pragma unroll
        for (int l = 0; l < 2; ++l)
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            key[0][l][e] = kr0[(2 + l) * NF + e];
            key[1][l][e] = kr1[(2 + l) * NF + e];
          }
      }
#pragma unroll
      for (int p = 0; p < 2; ++p)
#pragma unroll
        for (int l = 0; l < 2; ++l)
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const double2 kk = key[p][l][e];
            outr[o][l][e] = __fma_rn(xr[p][e], kk.x, __fma_rn(-xi[p][e], kk.y, outr[o][l][e]));
            outi[o][l][e] = __fma_rn(xr[p][e], kk.y, __fma_rn(xi[p][e], kk.x, outi[o][l][e]));
          }
    }
  }
#else
#pragma unroll
  for (int p = 0; p < 2; ++p) {
#pragma unroll 1
    for (int k = 0; k < D2; ++k) {
      // GGSW row p*D2 + k: [A/B][limb][1024] complex, thread's 4 points contiguous
      const double2 *kr = ggsw + (size_t)(p * D2 + k) * 4 * NF + tid * 4;
      double2 key[4][4];
#pragma unroll
      for (int q = 0; q < (BR2F_KEY_SPLIT ? 2 : 4); ++q)
#pragma unroll
        for (int e = 0; e < 4; ++e) key[q][e] = kr[q * NF + e];
      double xr[4], xi[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        xr[e] = DG::get(pk[p][e], k);      // coefficient tid + 256 e
        xi[e] = DG::get(pk[p][e + 4], k);  // coefficient tid + 256 e + 1024
      }
      F::fwd(xr, xi, xch, tws, tid);
      if (BR2F_KEY_SPLIT) {
#pragma unroll
        for (int q = 2; q < 4; ++q)
#pragma unroll
          for (int e = 0; e < 4; ++e) key[q][e] = kr[q * NF + e];
      }
#pragma unroll
      for (int o = 0; o < 2; ++o)
#pragma unroll
        for (int l = 0; l < 2; ++l)
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const double2 kk = key[o * 2 + l][e];
            outr[o][l][e] = __fma_rn(xr[e], kk.x, __fma_rn(-xi[e], kk.y, outr[o][l][e]));
            outi[o][l][e] = __fma_rn(xr[e], kk.y, __fma_rn(xi[e], kk.x, outi[o][l][e]));
          }
    }
  }
#endif
#pragma unroll
  for (int o = 0; o < 2; ++o) {
    F::inv<2>(outr[o], outi[o], xch, tws, tid);
#pragma unroll
    for (int e = 0; e < BR2_E; ++e) {
      const int h = e >> 2, ee = e & 3;
      const double p0 = rint(h ? outi[o][0][ee] : outr[o][0][ee]);  // exact (< 2^44.6)
      const double p1 = rint(h ? outi[o][1][ee] : outr[o][1][ee]);
      const double t = red<M>(p0) + mm<M>(red<M>(p1), LIMB2);
      if (o == 0)
        acc0[e] = canon<M>(acc0[e] + t);
      else
        acc1[e] = canon<M>(acc1[e] + t);
    }
  }
}

// mode 0: trace + NTT output u64 [wg][2][N2] (NttRlweCiphertext); mode 1: blind rotation only,
// coefficient-domain output (stage test).
__global__ __launch_bounds__(BR2_T, BR2_WAVES) void br2f_trace_kernel(
    const uint32_t *__restrict__ lwe_int, const double2 *__restrict__ bskf,
    const double *__restrict__ tk, DeviceTables tb, uint64_t *__restrict__ out, int mode) {
  using M = Mod<2>;
  constexpr int T = BR2_T, E = BR2_E, N = N2, NF = Fft1024::N;
  __shared__ double2 xch[2 * NF];   // FFT exchange (2 transforms); N2-double staging; trace xch
  __shared__ double tabs[2 * N];    // FFT twiddles (blind rotation), then NTT tw / itw (trace)
  double2 *ftw = reinterpret_cast<double2 *>(tabs);
  const int tid = threadIdx.x;
  const size_t wg = blockIdx.x;
  const uint32_t *lwe = lwe_int + wg * (NI + 1);
  // ACC = (0, X^{-b} * LUT2)
  double acc0[E], acc1[E];
  {
    const int b = (int)lwe[NI];
    const int r = (2 * N - (b % (2 * N))) % (2 * N);
#pragma unroll
    for (int e = 0; e < E; ++e) {
      acc0[e] = 0.0;
      acc1[e] = canon_small<M>(rot_read<N>(tb.lut2, tid + e * T, r));
    }
#pragma unroll
    for (int e = 0; e < NF / T; ++e) ftw[tid + e * T] = tb.fft2[tid + e * T];
    __syncthreads();
  }
#pragma unroll 1
  for (int i = 0; i < NI; ++i) {
    const int a = (int)__builtin_amdgcn_readfirstlane(lwe[i]) & (2 * N - 1);
    if (a == 0) continue;
    br2f_step(acc0, acc1, xch, ftw, a, bskf + (size_t)OMR_KEYROW2(i) * (2 * D2 * 4 * NF), tid);
  }
  uint64_t *o = out + wg * 2 * N;
  if (mode == 1) {
#pragma unroll
    for (int e = 0; e < E; ++e) {
      o[tid + e * T] = to_u64<M>(acc0[e]);
      o[N + tid + e * T] = to_u64<M>(acc1[e]);
    }
    return;
  }
  __syncthreads();  // all FFT twiddle reads done before the NTT tables replace them
#pragma unroll
  for (int e = 0; e < E; ++e) {
    tabs[tid + e * T] = tb.tw2[tid + e * T];
    tabs[N + tid + e * T] = tb.itw2[tid + e * T];
  }
  __syncthreads();
  hom_trace_store(acc0, acc1, reinterpret_cast<double *>(xch), tabs, tabs + N, tk, tb, o, tid);
}

#endif  // OMR_BR2_GEOM_DEFAULT

// Coefficient-domain canonical u64 key polynomials -> two 25-bit limbs, each FFT-transformed and
// scaled by 1/1024, stored [poly][limb][1024] complex in transform-index order.
__global__ __launch_bounds__(256) void key_to_fft2_kernel(const uint64_t *__restrict__ in,
                                                          double2 *__restrict__ out, size_t npoly,
                                                          const double2 *__restrict__ tw) {
  using F = Fft1024;
  __shared__ double2 xch[2 * F::N];
  __shared__ double2 tws[F::N];
  const int tid = threadIdx.x;
  const size_t poly = blockIdx.x;
  if (poly >= npoly) return;
  const uint64_t *src = in + poly * N2;
  double xr[2][4], xi[2][4];
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    tws[tid + e * 256] = tw[tid + e * 256];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const double v = from_u64<Mod<2>>(src[tid + e * 256 + h * F::N]);
      const double hi = floor(__fma_rn(v, 1.0 / LIMB2, 0.5));  // v = hi 2^25 + lo, lo in [-2^24, 2^24)
      const double lo = __fma_rn(-hi, LIMB2, v);
      (h ? xi : xr)[0][e] = lo;
      (h ? xi : xr)[1][e] = hi;
    }
  }
  __syncthreads();
  F::fwd<2>(xr, xi, xch, tws, tid);
#pragma unroll
  for (int l = 0; l < 2; ++l)
#pragma unroll
    for (int e = 0; e < 4; ++e)
      out[(poly * 2 + l) * F::N + tid * 4 + e] = make_double2(xr[l][e] * (1.0 / F::N), xi[l][e] * (1.0 / F::N));
}

}  // namespace omr
