// Kernels of the detect / encode path (gfx950). Each kernel cites the reference function it
// replaces; the launch code is in context.hip.
#pragma once

#include "device_ntt.hpp"

namespace omr {

// Workgroup geometry per level (T threads x E residues per thread = N) of the modular NTTs.
// Level 2 (latency blind rotations, trace, encode, key conversion): 256 threads x 8 residues.
// Both throughput blind rotations run on exact complex FFTs (br1_fft.hpp, br2_fft.hpp); level 1
// needs the NTT only for omr_ntt (tests).
constexpr int BR1_T = 256, BR1_E = 4;  // N1 = 1024
constexpr int BR2_T = 256, BR2_E = 8;  // N2 = 2048
constexpr int ENC_T = 128, ENC_E = 16;
constexpr size_t OMR_DEFAULT_BATCH = 16384;  // messages per detect chunk (scratch 36 KiB/msg)
constexpr size_t OMR_ENC_MAX_CHUNKS = 4096;   // default chunk partials per encode ciphertext

struct DeviceTables {
  const double *tw1, *itw1, *tw2, *itw2;  // psi^brv(k), psi^-brv(k) (centred)
  const double *tw2c;                     // tw2 with stages 9, 10 permuted for CmuxNtt
  const double *lut1, *lut2;              // LUTs, coefficient domain (centred)
  const uint16_t *trace_perm;             // [11][2048] NTT-domain permutation of sigma_g
  const uint16_t *trace_src;              // [11][2048] coefficient source index of sigma_g (+N: negate)
  const double2 *fft1;                    // level-1 FFT twiddles
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
