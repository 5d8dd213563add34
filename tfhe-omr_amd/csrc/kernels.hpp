// Kernels of the detect / encode path (gfx950). Each kernel cites the reference function it
// replaces; the launch code is in context.hip.
#pragma once

#include "device_ntt.hpp"

namespace omr {

// Workgroup geometry per level (T threads x E residues per thread = N).
// Geometry / register targets chosen from measured variants:
// level 1: 256 threads x 4 residues, >= 2 waves/SIMD; level 2: 256 x 8, 2 waves/SIMD.
#ifndef BR1_WAVES
#define BR1_WAVES 2
#endif
#ifndef BR2_WAVES
#define BR2_WAVES 2
#endif
#ifndef BR1_TE
#define BR1_TE 256, 4
#endif
#ifndef BR2_TE
#define BR2_TE 256, 8
#define OMR_BR2_GEOM_DEFAULT 1  // the level-2 FFT / sliced options are written for 256 x 8
#endif
#ifndef OMR_KEY_DEPTH1
#define OMR_KEY_DEPTH1 1  // level-1 key rows prefetched this many digits ahead (1 or 2)
#endif
#ifndef OMR_KEY_DEPTH2
#define OMR_KEY_DEPTH2 1
#endif
#ifndef OMR_PAIR1
#define OMR_PAIR1 1       // level 1: transform mask and body digits as interleaved pairs
#endif
#ifndef OMR_MAC_EXACT1
#define OMR_MAC_EXACT1 1  // level 1: exact-product multiply-accumulate (one reduction per 2)
#endif
#ifndef OMR_PAIR2
#define OMR_PAIR2 0       // level 2: paired mask/body digit transforms
#endif
#ifndef OMR_FFT1
#define OMR_FFT1 1        // level 1: FP64 complex-FFT external product (br1_fft.hpp)
#endif
#ifdef OMR_EXPT_KEYWRAP  // timing experiment only (wrong results): L2-resident key rows
#define OMR_KEYROW2(i) ((i) & 3)
#else
#define OMR_KEYROW2(i) (i)
#endif
#ifndef OMR_FFT2
#define OMR_FFT2 0        // level 2: FP64 complex-FFT external product, 2-limb keys (br2_fft.hpp);
                          // exact and tested, slower than the NTT at this geometry
#endif
#ifndef OMR_BR2_SLICED
#define OMR_BR2_SLICED 0  // level 2: sliced exact-FFT kernel (br2_sliced.hpp); implies FFT-form keys
#endif
#ifndef OMR_KS_MFMA
#define OMR_KS_MFMA 1     // LWE key switch as an int8 GEMM on the matrix cores (ks_mfma.hpp)
#endif
#ifndef OMR_DEFAULT_BATCH
#define OMR_DEFAULT_BATCH 16384  // messages per detect chunk (scratch 36 KiB/msg)
#endif
#ifndef OMR_OVERLAP
#define OMR_OVERLAP 0     // detect: level 2 of chunk c on a second stream beside level 1 of chunk c + 1
#endif
#ifndef OMR_NTT_GTW
#define OMR_NTT_GTW 0     // level 2: pass-0 NTT twiddles (workgroup-uniform) by scalar loads (+1.5 %: off)
#endif
#ifndef OMR_BR2_PERSIST
#define OMR_BR2_PERSIST 0 // level 2: resident-sized grid walking messages with a grid stride
#endif
#ifndef OMR_TRACE3
#define OMR_TRACE3 0      // trace digit transforms on the three-buffer NTT with the small-digit tables
                          // (bit-exact; 128 B/lane of scratch in the fused kernel: br2 +1 %, off)
#endif
#ifndef OMR_MAC_RED4
#define OMR_MAC_RED4 1    // level-2 CMUX: reduce the NTT-domain accumulators every 4 digit products
#endif
#ifndef OMR_KEY_NT
#define OMR_KEY_NT 0
#endif
constexpr int BR1_GEOM[2] = {BR1_TE};
constexpr int BR2_GEOM[2] = {BR2_TE};
constexpr int BR1_T = BR1_GEOM[0], BR1_E = BR1_GEOM[1];  // N1 = 1024
constexpr int BR2_T = BR2_GEOM[0], BR2_E = BR2_GEOM[1];  // N2 = 2048

// Device key element types: level 1 residues fit int32 (|x| <= (q1-1)/2), level 2 need FP64.
#ifndef OMR_KEY1_DOUBLE
#define OMR_KEY1_DOUBLE 0
#endif
#if OMR_KEY1_DOUBLE
typedef double Key1T;
#else
typedef int32_t Key1T;
#endif
typedef double Key2T;
constexpr int KS_MSGS = 64, KS_COLS = 64, KS_THREADS = 256;
constexpr int ENC_T = 128, ENC_E = 16;

struct DeviceTables {
  const double *tw1, *itw1, *tw2, *itw2;  // psi^brv(k), psi^-brv(k) (centred)
  const double *lut1, *lut2;              // LUTs, coefficient domain (centred)
  const uint16_t *trace_perm;             // [11][2048] NTT-domain permutation of sigma_g
  const uint16_t *trace_src;              // [11][2048] coefficient source index of sigma_g (+N: negate)
  const double2 *fft1, *fft2, *fft2w;     // FFT twiddles: level 1, level 2 (256x4), level 2 (64x16)
};

// ---- key conversion: coefficient-domain canonical residues -> NTT-domain centred residues ----
template <int LEVEL, typename IN, typename OUT>
__global__ void key_to_ntt_kernel(const IN *in, OUT *out, size_t npoly, double scale,
                                  const double *tw) {
  using M = Mod<LEVEL>;
  constexpr int T = LEVEL == 1 ? BR1_T : BR2_T, E = LEVEL == 1 ? BR1_E : BR2_E;
  using NTT = WgNtt<M, T, E>;
  __shared__ double lds[NTT::LDS_DOUBLES];
  const size_t poly = blockIdx.x;
  const int tid = threadIdx.x;
  if (poly >= npoly) return;
  const IN *src = in + poly * M::N;
  double x[E];
#pragma unroll
  for (int e = 0; e < E; ++e) x[e] = from_u64<M>((uint64_t)src[tid + e * T]);
  NTT::fwd(x, lds, tw, tid);
  OUT *dst = out + poly * M::N + tid * E;
#pragma unroll
  for (int e = 0; e < E; ++e)
    dst[e] = (OUT)(scale == 1.0 ? canon<M>(x[e]) : canon<M>(mm<M>(canon<M>(x[e]), scale)));
}

// ---- plain NTT of canonical u64 polynomials (tests / omr_ntt) ----
template <int LEVEL>
__global__ void ntt_u64_kernel(uint64_t *polys, size_t npoly, int inverse, double ninv,
                               const double *tw, const double *itw) {
  using M = Mod<LEVEL>;
  constexpr int T = LEVEL == 1 ? BR1_T : BR2_T, E = LEVEL == 1 ? BR1_E : BR2_E;
  using NTT = WgNtt<M, T, E>;
  __shared__ double lds[NTT::LDS_DOUBLES];
  const size_t poly = blockIdx.x;
  const int tid = threadIdx.x;
  if (poly >= npoly) return;
  uint64_t *p = polys + poly * M::N;
  double x[E];
  if (!inverse) {
#pragma unroll
    for (int e = 0; e < E; ++e) x[e] = from_u64<M>(p[tid + e * T]);
    NTT::fwd(x, lds, tw, tid);
    __syncthreads();
#pragma unroll
    for (int e = 0; e < E; ++e) p[tid * E + e] = to_u64<M>(canon<M>(x[e]));
  } else {
#pragma unroll
    for (int e = 0; e < E; ++e) x[e] = from_u64<M>(p[tid * E + e]);
    NTT::inv(x, lds, itw, tid);
    __syncthreads();
#pragma unroll
    for (int e = 0; e < E; ++e) p[tid + e * T] = to_u64<M>(canon<M>(mm<M>(canon<M>(x[e]), ninv)));
  }
}

}  // namespace omr
