// Level-1 blind rotation with the FFT external product (first_level_bootstrapping,
// detector.rs:533-597; BlindRotationKey::blind_rotate with a binary LWE secret): one wave per
// (message, clue). Exact by construction: see device_fft.hpp for why the rounded FFT product is
// the integer product, and DESIGN.md §3.
//
// Per CMUX step (a_i != 0):
//   stage ACC in LDS -> digits of (X^a - 1) * ACC (int32 arithmetic, 4 signed digits packed per
//   coefficient) -> 8 forward FFTs (4 mask digits, 4 body digits) each multiplied into the two
//   output accumulators with the GGSW row (pre-transformed, pre-scaled by 1/512) -> 2 inverse
//   FFTs -> round, reduce mod q1, add into ACC.
// Registers per lane: ACC 2 x 16 int32, digits 2 x 16 u32, one transform 16 doubles, output
// accumulators 32 doubles, one key row 32 doubles. LDS: 8 KB exchange/staging + 8 KB twiddles.
#pragma once

#include "device_fft.hpp"
#include "kernels.hpp"

namespace omr {

#ifndef BR1F_WAVES
#define BR1F_WAVES 2  // waves per SIMD the register allocation targets (256 VGPRs)
#endif
#ifndef BR1F_KEY_SPLIT
#define BR1F_KEY_SPLIT 1  // load the B component of a key row after the transform (32 VGPRs less)
#endif

struct Lvl1Int {
  static constexpr int Q = 134215681, H = 67107840;
  __device__ static __forceinline__ int canon(int x) {  // |x| < q + H -> [-H, H]
    x = x > H ? x - Q : x;
    return x < -H ? x + Q : x;
  }
  __device__ static __forceinline__ uint32_t to_u32(int x) { return (uint32_t)(x < 0 ? x + Q : x); }
  // NonPowOf2ApproxSignedBasis (logB 5, d 4, drop 7) on a canonical residue: the same digits as
  // Digits8<LOGB1, D1, DROP1> (floor((v + 2^6) / 2^7), balanced base-32 digits, top unbounded),
  // packed as signed bytes.
  __device__ static __forceinline__ uint32_t digits(int v) {
    int y = (v + (1 << (DROP1 - 1))) >> DROP1;  // arithmetic shift = floor division
    uint32_t pk = 0;
#pragma unroll
    for (int k = 0; k < D1 - 1; ++k) {
      const int c = (y + (1 << (LOGB1 - 1))) >> LOGB1;
      pk |= ((uint32_t)(y - c * (1 << LOGB1)) & 0xffu) << (8 * k);
      y = c;
    }
    return pk | (((uint32_t)y & 0xffu) << (8 * (D1 - 1)));
  }
  // signed digit k of a packed word
  __device__ static __forceinline__ double digit(uint32_t pk, int k) {
    return (double)((int)(pk << (24 - 8 * k)) >> 24);
  }
  // (X^r * p)[j] for p staged in LDS, r in [0, 2N)
  __device__ static __forceinline__ int rot_read(const int *p, int j, int r) {
    const int t = j - r;
    int u = t < 0 ? t + N1 : t;
    const bool neg = (t < 0) != (u < 0);  // wrapped exactly once: X^N = -1
    u = u < 0 ? u + N1 : u;
    const int v = p[u];
    return neg ? -v : v;
  }
};

// ACC layout: ac[p][h * 8 + e] = coefficient lane + 64 e + 512 h of poly p (0 mask, 1 body).
__device__ __forceinline__ int acc_coef(int lane, int i) { return lane + 64 * (i & 7) + 512 * (i >> 3); }

// digits of (X^a - 1) * ACC for both polys (ACC staged through LDS)
__device__ __forceinline__ void br1f_digits(const int (&ac)[2][16], double2 *xch, int a, int lane,
                                            uint32_t (&pk)[2][16]) {
  int *st = reinterpret_cast<int *>(xch);  // [2][N1] int32 staging (8 KB)
#pragma unroll
  for (int p = 0; p < 2; ++p)
#pragma unroll
    for (int i = 0; i < 16; ++i) st[p * N1 + acc_coef(lane, i)] = ac[p][i];
  __syncthreads();
#pragma unroll
  for (int p = 0; p < 2; ++p)
#pragma unroll
    for (int i = 0; i < 16; ++i)
      pk[p][i] = Lvl1Int::digits(
          Lvl1Int::canon(Lvl1Int::rot_read(st + p * N1, acc_coef(lane, i), a) - ac[p][i]));
  __syncthreads();
}

__device__ __forceinline__ void br1f_step(int (&ac)[2][16], double2 *xch, const double2 *tws, int a,
                                          const double2 *__restrict__ ggsw, int lane) {
  using F = Fft512;
  constexpr int NF = F::N;
  uint32_t pk[2][16];
  br1f_digits(ac, xch, a, lane, pk);

  double outr[2][8], outi[2][8];
#pragma unroll
  for (int o = 0; o < 2; ++o)
#pragma unroll
    for (int e = 0; e < 8; ++e) outr[o][e] = outi[o][e] = 0.0;
#pragma unroll
  for (int p = 0; p < 2; ++p) {
#pragma unroll 1
    for (int k = 0; k < D1; ++k) {
      // GGSW row p*D1 + k: [2][512] complex (A, B), lane's 8 values contiguous
      const double2 *kr = ggsw + (size_t)(p * D1 + k) * 2 * NF + lane * 8;
      double2 ka[8], kb[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        ka[e] = kr[e];
        if (!BR1F_KEY_SPLIT) kb[e] = kr[NF + e];
      }
      double xr[8], xi[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        xr[e] = Lvl1Int::digit(pk[p][e], k);
        xi[e] = Lvl1Int::digit(pk[p][8 + e], k);
      }
      F::fwd(xr, xi, xch, tws, lane);
      if (BR1F_KEY_SPLIT) {
#pragma unroll
        for (int e = 0; e < 8; ++e) kb[e] = kr[NF + e];
      }
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        outr[0][e] = __fma_rn(xr[e], ka[e].x, __fma_rn(-xi[e], ka[e].y, outr[0][e]));
        outi[0][e] = __fma_rn(xr[e], ka[e].y, __fma_rn(xi[e], ka[e].x, outi[0][e]));
        outr[1][e] = __fma_rn(xr[e], kb[e].x, __fma_rn(-xi[e], kb[e].y, outr[1][e]));
        outi[1][e] = __fma_rn(xr[e], kb[e].y, __fma_rn(xi[e], kb[e].x, outi[1][e]));
      }
    }
  }
#pragma unroll
  for (int o = 0; o < 2; ++o) {
    F::inv(outr[o], outi[o], xch, tws, lane);
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const double v = rint(i < 8 ? outr[o][i] : outi[o][i - 8]);  // exact integer (< 2^43)
      ac[o][i] = Lvl1Int::canon(ac[o][i] + (int)red<Mod<1>>(v));
    }
  }
}

__global__ __launch_bounds__(64, BR1F_WAVES) void br1f_kernel(const uint16_t *__restrict__ clue_a,
                                                      const uint16_t *__restrict__ clue_b,
                                                      const uint16_t *__restrict__ lwe_a,
                                                      const uint16_t *__restrict__ lwe_b,
                                                      const double2 *__restrict__ bskf, DeviceTables tb,
                                                      uint32_t *__restrict__ ext,
                                                      uint64_t *__restrict__ rlwe_out, int mode) {
  constexpr int NF = Fft512::N;
  __shared__ double2 xch[NF];
  __shared__ double2 tws[NF];
  __shared__ uint16_t la[N0];
  const int lane = threadIdx.x;
  const size_t wg = blockIdx.x;
  int b;
  if (lwe_a == nullptr) {  // extract clue c of message m (CmLweCiphertext::extract_all, :514)
    const size_t m = wg / CLUES;
    const int c = (int)(wg % CLUES);
    const uint16_t *A = clue_a + m * N0;
    for (int i = lane; i < N0; i += 64)
      la[i] = i <= c ? (uint16_t)(A[c - i] & (Q0 - 1)) : (uint16_t)((Q0 - A[N0 + c - i]) & (Q0 - 1));
    b = clue_b[m * CLUES + c] & (Q0 - 1);
  } else {
    for (int i = lane; i < N0; i += 64) la[i] = lwe_a[wg * N0 + i] & (Q0 - 1);
    b = lwe_b[wg] & (Q0 - 1);
  }
  // ACC = (0, X^{-b} * LUT1)
  int ac[2][16];
  const int r0 = (2 * N1 - (b % (2 * N1))) % (2 * N1);
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    ac[0][i] = 0;
    ac[1][i] = (int)canon_small<Mod<1>>(rot_read<N1>(tb.lut1, acc_coef(lane, i), r0));
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) tws[lane + 64 * e] = tb.fft1[lane + 64 * e];
  __syncthreads();
#pragma unroll 1
  for (int i = 0; i < N0; ++i) {
    const int a = __builtin_amdgcn_readfirstlane(la[i]);
    if (a == 0) continue;  // (X^0 - 1) * ACC = 0
    if (mode == 2) {  // debug: packed digits of the first CMUX step
      uint32_t pk[2][16];
      br1f_digits(ac, xch, a, lane, pk);
#pragma unroll
      for (int p = 0; p < 2; ++p)
#pragma unroll
        for (int j = 0; j < 16; ++j) rlwe_out[wg * 2 * N1 + p * N1 + acc_coef(lane, j)] = pk[p][j];
      return;
    }
    br1f_step(ac, xch, tws, a, bskf + (size_t)i * (2 * D1 * 2 * NF), lane);
  }
  if (mode == 0) {  // extract_lwe_locally (coefficient 0), detector.rs:561
    int *st = reinterpret_cast<int *>(xch);
#pragma unroll
    for (int i = 0; i < 16; ++i) st[acc_coef(lane, i)] = ac[0][i];
    __syncthreads();
    uint32_t *o = ext + wg * (N1 + 1);
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int j = acc_coef(lane, i);
      o[j] = Lvl1Int::to_u32(j == 0 ? st[0] : -st[N1 - j]);
    }
    if (lane == 0) o[N1] = Lvl1Int::to_u32(ac[1][0]);
  } else {
    uint64_t *o = rlwe_out + wg * 2 * N1;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      o[acc_coef(lane, i)] = Lvl1Int::to_u32(ac[0][i]);
      o[N1 + acc_coef(lane, i)] = Lvl1Int::to_u32(ac[1][i]);
    }
  }
}

// Coefficient-domain canonical u32 key polynomials -> FFT domain / 512, transform-index order.
__global__ __launch_bounds__(64) void key_to_fft1_kernel(const uint32_t *__restrict__ in,
                                                         double2 *__restrict__ out, size_t npoly,
                                                         const double2 *__restrict__ tw) {
  using F = Fft512;
  __shared__ double2 xch[F::N];
  __shared__ double2 tws[F::N];
  const int lane = threadIdx.x;
  const size_t poly = blockIdx.x;
  if (poly >= npoly) return;
  const uint32_t *src = in + poly * N1;
  double xr[8], xi[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    tws[lane + 64 * e] = tw[lane + 64 * e];
    xr[e] = from_u64<Mod<1>>(src[lane + 64 * e]);
    xi[e] = from_u64<Mod<1>>(src[lane + 64 * e + 512]);
  }
  __syncthreads();
  F::fwd(xr, xi, xch, tws, lane);
  double2 *dst = out + poly * F::N + lane * 8;
#pragma unroll
  for (int e = 0; e < 8; ++e) dst[e] = make_double2(xr[e] * (1.0 / 512), xi[e] * (1.0 / 512));
}

// Test entry (omr_fft1_mul): out = a * k mod (X^1024 + 1, q1) through the level-1 FFT path,
// for |a| small (digit-sized) and canonical k.
__global__ __launch_bounds__(64) void fft1_mul_kernel(const uint32_t *__restrict__ a,
                                                      const uint32_t *__restrict__ k,
                                                      uint64_t *__restrict__ out,
                                                      const double2 *__restrict__ tw) {
  using F = Fft512;
  __shared__ double2 xch[F::N];
  __shared__ double2 tws[F::N];
  const int lane = threadIdx.x;
  const size_t poly = blockIdx.x;
  double ar[8], ai[8], kr[8], ki[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    tws[lane + 64 * e] = tw[lane + 64 * e];
    ar[e] = from_u64<Mod<1>>(a[poly * N1 + lane + 64 * e]);
    ai[e] = from_u64<Mod<1>>(a[poly * N1 + lane + 64 * e + 512]);
    kr[e] = from_u64<Mod<1>>(k[poly * N1 + lane + 64 * e]);
    ki[e] = from_u64<Mod<1>>(k[poly * N1 + lane + 64 * e + 512]);
  }
  __syncthreads();
  F::fwd(ar, ai, xch, tws, lane);
  F::fwd(kr, ki, xch, tws, lane);
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const double r = (ar[e] * kr[e] - ai[e] * ki[e]) * (1.0 / 512);
    const double i = (ar[e] * ki[e] + ai[e] * kr[e]) * (1.0 / 512);
    ar[e] = r;
    ai[e] = i;
  }
  F::inv(ar, ai, xch, tws, lane);
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    out[poly * N1 + lane + 64 * e] = to_u64<Mod<1>>(canon<Mod<1>>(rint(ar[e])));
    out[poly * N1 + lane + 64 * e + 512] = to_u64<Mod<1>>(canon<Mod<1>>(rint(ai[e])));
  }
}

}  // namespace omr
