// Level-2 blind rotation on the exact 2-limb FFT, "sliced" across the workgroup
// (second_level_bootstrapping, detector.rs:599-624, fused with hom_trace :626-639): one 256-thread
// workgroup (4 waves) per message, 1 wave per SIMD (the whole register file per wave).
//
// Per CMUX step:
//   * the accumulator (coefficient layout tid + 256 e, canonical FP64) is staged in LDS; waves
//     0-1 decompose the mask, waves 2-3 the body ((X^a - 1) * ACC, closed-form Digits2 words),
//     each wave keeping the 3 digits it will transform;
//   * 3 rounds: each wave runs one 1024-point complex FFT (Fft1024W, wave-local: 16 points per
//     lane, no workgroup barrier inside) and publishes it in its slot; after one barrier each wave
//     multiply-accumulates ITS quarter of the 1024 frequencies for all 4 published digits into
//     the 4 accumulators (A/B output x 25-bit key limb) — keys come straight from L2, prefetched
//     during the transform;
//   * the accumulators are gathered so that wave q owns accumulator q, inverted wave-locally,
//     rounded (exact integers < 2^44.6) and reduced mod q2; out = P_0 + 2^25 P_1 per output is
//     added into the accumulator.
// 11 workgroup barriers per step instead of the NTT kernel's ~30, and ~40 % of its FP64 work.
// Keys: br2_fft.hpp's FFT-domain limbs (same transform order for both FFT geometries:
// tools/fft_exactness.py --level 2).
#pragma once

#include "br2_fft.hpp"

namespace omr {

// XOR swizzle of the 1024-slot publication buffers: conflict free for the transform-order writes
// (t = 16 lane + e) and the frequency-slice reads (t = 256 w + 4 lane + m) of ds_*_b128
// (searched like tools/fft_lds_banks.py).
__device__ __forceinline__ int slot_swz(int t) {
  return t ^ (((t >> 3) & 1) * 1) ^ (((t >> 4) & 1) * 10) ^ (((t >> 5) & 1) * 5) ^ (((t >> 6) & 1) * 4) ^
         (((t >> 7) & 1) * 13) ^ (((t >> 9) & 1) * 1);
}

#ifdef OMR_BR2_GEOM_DEFAULT
__global__ __launch_bounds__(256, 1) void br2s_trace_kernel(const uint32_t *__restrict__ lwe_int,
                                                            const double2 *__restrict__ bskf,
                                                            const double *__restrict__ tk,
                                                            DeviceTables tb, uint64_t *__restrict__ out,
                                                            int mode) {
  using F = Fft1024W;
  using M = Mod<2>;
  constexpr int T = BR2_T, E = BR2_E, N = N2, NF = F::N;
  static_assert(T == 256 && E == 8, "sliced level 2 assumes 256 threads x 8 coefficients");
  __shared__ double2 slots[4][NF];  // per-wave transform buffer / round slot; staging; trace
  __shared__ double2 ftw[NF];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int pw = w >> 1, hw = w & 1;  // this wave's poly and digit half (digits 3 hw .. 3 hw + 2)
  const size_t wg = blockIdx.x;
  const uint32_t *lwe = lwe_int + wg * (NI + 1);
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
    for (int e = 0; e < NF / T; ++e) ftw[tid + e * T] = tb.fft2w[tid + e * T];
    __syncthreads();
  }
  double *stg = reinterpret_cast<double *>(&slots[0][0]);  // 2 x N2 doubles (slots 0-1)
#pragma unroll 1
  for (int i = 0; i < NI; ++i) {
    const int a = (int)__builtin_amdgcn_readfirstlane(lwe[i]) & (2 * N - 1);
    if (a == 0) continue;
    const double2 *kstep = bskf + (size_t)OMR_KEYROW2(i) * (2 * D2 * 4 * NF);
    // ---- stage ACC, decompose this wave's poly over its transform-input coefficients ----
#pragma unroll
    for (int e = 0; e < E; ++e) {
      stg[tid + e * T] = acc0[e];
      stg[N + tid + e * T] = acc1[e];
    }
    __syncthreads();
    uint32_t dw[32];  // lo word (digits 0-2) or hi word (digits 3-5) of the Digits2 split
    {
      const double *sp = stg + pw * N;
#pragma unroll
      for (int j = 0; j < 32; ++j) {
        const int c = lane + 64 * (j & 15) + 1024 * (j >> 4);
        const double v = canon_small<M>(rot_read<N>(sp, c, a) - sp[c]);
        uint32_t pk[2];
        Digits2::pack(v, pk);
        dw[j] = hw ? pk[1] : pk[0];
      }
    }
    __syncthreads();  // staging area is reused by the transforms
    double ar[4][4], ai[4][4];  // accumulators [o * 2 + limb][frequency m], slice 256 w + 4 lane + m
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int m = 0; m < 4; ++m) ar[q][m] = ai[q][m] = 0.0;
#pragma unroll 1
    for (int rho = 0; rho < 3; ++rho) {
      // keys of the 4 digits published this round, for this wave's frequency slice
      double2 key[4][4][4];  // [publishing wave v][o * 2 + limb][m]
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        const int row = (v >> 1) * D2 + 3 * (v & 1) + rho;
        const double2 *kr = kstep + (size_t)row * 4 * NF + 256 * w + 4 * lane;
#pragma unroll
        for (int q = 0; q < 4; ++q)
#pragma unroll
          for (int m = 0; m < 4; ++m) key[v][q][m] = kr[q * NF + m];
      }
      // this wave's digit k = 3 hw + rho of poly pw
      double xr[16], xi[16];
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const uint32_t wr = dw[e], wi = dw[16 + e];  // coefficients lane + 64 e, + 1024
        if (hw == 0 || rho < 2) {
          xr[e] = (double)((int)((wr >> (7 * rho)) & 127u) - 64);
          xi[e] = (double)((int)((wi >> (7 * rho)) & 127u) - 64);
        } else {  // top digit = hi >> 14
          xr[e] = (double)((int)wr >> 14);
          xi[e] = (double)((int)wi >> 14);
        }
      }
      F::fwd(xr, xi, &slots[w][0], ftw, lane);
#pragma unroll
      for (int e = 0; e < 16; ++e) slots[w][slot_swz(16 * lane + e)] = make_double2(xr[e], xi[e]);
      __syncthreads();
#pragma unroll
      for (int v = 0; v < 4; ++v)
#pragma unroll
        for (int m = 0; m < 4; ++m) {
          const double2 x = slots[v][slot_swz(256 * w + 4 * lane + m)];
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const double2 k = key[v][q][m];
            ar[q][m] = __fma_rn(x.x, k.x, __fma_rn(-x.y, k.y, ar[q][m]));
            ai[q][m] = __fma_rn(x.x, k.y, __fma_rn(x.y, k.x, ai[q][m]));
          }
        }
      __syncthreads();  // slots free for the next round
    }
    // ---- gather accumulator q into slot q, invert it in wave q ----
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int m = 0; m < 4; ++m) slots[q][slot_swz(256 * w + 4 * lane + m)] = make_double2(ar[q][m], ai[q][m]);
    __syncthreads();
    {
      double yr[16], yi[16];
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const double2 v = slots[w][slot_swz(16 * lane + e)];
        yr[e] = v.x;
        yi[e] = v.y;
      }
      wave_lds_sync();
      F::inv(yr, yi, &slots[w][0], ftw, lane);
      double *pq = reinterpret_cast<double *>(&slots[w][0]);  // P_w, coefficient order
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        pq[lane + 64 * e] = red<M>(rint(yr[e]));  // exact integers (< 2^44.6) reduced mod q2
        pq[NF + lane + 64 * e] = red<M>(rint(yi[e]));
      }
    }
    __syncthreads();
    {
      const double *p0 = reinterpret_cast<const double *>(&slots[0][0]);
      const double *p1 = reinterpret_cast<const double *>(&slots[1][0]);
      const double *p2 = reinterpret_cast<const double *>(&slots[2][0]);
      const double *p3 = reinterpret_cast<const double *>(&slots[3][0]);
#pragma unroll
      for (int e = 0; e < E; ++e) {
        const int c = tid + e * T;
        acc0[e] = canon<M>(acc0[e] + p0[c] + mm<M>(p1[c], LIMB2));
        acc1[e] = canon<M>(acc1[e] + p2[c] + mm<M>(p3[c], LIMB2));
      }
    }
    __syncthreads();  // slots are restaged by the next step
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
  double *tabs = reinterpret_cast<double *>(&slots[0][0]);  // NTT tw / itw (slots 0-1)
  double *xd = reinterpret_cast<double *>(&slots[2][0]);    // trace exchange (slots 2-3)
#pragma unroll
  for (int e = 0; e < E; ++e) {
    tabs[tid + e * T] = tb.tw2[tid + e * T];
    tabs[N + tid + e * T] = tb.itw2[tid + e * T];
  }
  __syncthreads();
  hom_trace_store(acc0, acc1, xd, tabs, tabs + N, tk, tb, o, tid);
}

#endif  // OMR_BR2_GEOM_DEFAULT

}  // namespace omr
