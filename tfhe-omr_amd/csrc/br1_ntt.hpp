// Level-1 blind rotation on the exact modular NTT (round 5): BlindRotationKey::blind_rotate with
// concrete-ntt's arithmetic, as the reference runs it (detector.rs:553-557; omr_core/Cargo.toml:38-45).
// Two uses:
//  - the exact fallback of a guarded level-1 launch (context.hip, launch_br1): run after the guarded
//    FFT kernel, every workgroup reads that launch's rounding-margin word and leaves unless it
//    reached the certificate threshold 1 - E1, in which case the launch's rotations are recomputed
//    here and overwrite the FFT outputs -- so a key whose a priori bound does not prove the FFT exact
//    still gets exact outputs, as level 2's breaches do (br2l_fallback_kernel);
//  - omr_ctx_set_exact_level1: every level-1 launch on this kernel, a full-size cross-check of the
//    FFT kernels (both families share the level-1 FFT) against an independent exact arithmetic.
// One 64-thread workgroup (one wave) per rotation: WgNtt<Mod<1>, 64, 16> is wave-private (its
// exchanges need no workgroup barrier), residues are exact integers in FP64 registers
// (device_ntt.hpp), the key rows are read from L2 in the NTT domain x N1^-1 (context.hip, bsk1n:
// [512][2 D1 rows][2 outputs][1024] centred doubles, NTT index order). Per CMUX step: the digits of
// (X^a - 1) * ACC for both polynomials (the same decomposition as br1f: Lvl1Int::digits), 8 forward
// transforms each multiplied into the two output accumulators, 2 inverse transforms, ACC += out.
// Not tuned: a fallback that never runs on a real key, and a test instrument.
#pragma once

#include "detect_kernels.hpp"
#include "br1_fft.hpp"
#include "latency_kernels.hpp"

namespace omr {

using Ntt1W = WgNtt<Mod<1>, 64, 16>;
static_assert(Ntt1W::N == N1 && Ntt1W::LDS_DOUBLES * sizeof(double) >= 2 * N1 * sizeof(int),
              "the exchange buffer also stages [ACC, -ACC]");

// signed digit k of an Lvl1Int::digits word: fields of LOGB1 bits from bit 0, the top digit the
// sign-extended rest
__device__ __forceinline__ double lvl1_digit(uint32_t w, int k) {
  return (double)(int)__builtin_amdgcn_sbfe(w, LOGB1 * k, k < D1 - 1 ? LOGB1 : 32 - LOGB1 * (D1 - 1));
}

// Rotation g: clue g % 7 of message g / 7 (lwe_a == nullptr) or LWE g; the outputs as br1f_body's
// (mode 0: the extracted LWE, mode 1: the full RLWE).
__device__ __forceinline__ void br1n_body(const uint16_t *__restrict__ clue_a, const uint16_t *__restrict__ clue_b,
                                          const uint16_t *__restrict__ lwe_a, const uint16_t *__restrict__ lwe_b,
                                          const double *__restrict__ bsk1n, const DeviceTables &tb,
                                          uint32_t *__restrict__ ext, uint64_t *__restrict__ rlwe_out, int mode,
                                          size_t g) {
  using M = Mod<1>;
  __shared__ double lds[Ntt1W::LDS_DOUBLES];  // the transforms' exchanges; [ACC, -ACC] between them
  __shared__ uint16_t la[N0];
  const int lane = threadIdx.x;
  int b;
  if (lwe_a == nullptr) {  // CmLweCiphertext::extract_all (:514), as br1f_body
    const size_t m = g / CLUES;
    const int c = (int)(g % CLUES);
    const uint16_t *A = clue_a + m * N0;
    for (int i = lane; i < N0; i += 64)
      la[i] = i <= c ? (uint16_t)(A[c - i] & (Q0 - 1)) : (uint16_t)((Q0 - A[N0 + c - i]) & (Q0 - 1));
    b = clue_b[m * CLUES + c] & (Q0 - 1);
  } else {
    for (int i = lane; i < N0; i += 64) la[i] = lwe_a[g * N0 + i] & (Q0 - 1);
    b = lwe_b[g] & (Q0 - 1);
  }
  // ACC = (0, X^{-b} * LUT1); ac[p][e] = coefficient lane + 64 e, canonical centred
  double ac[2][16];
  const int r0 = (2 * N1 - (b % (2 * N1))) % (2 * N1);
#pragma unroll
  for (int e = 0; e < 16; ++e) {
    ac[0][e] = 0.0;
    ac[1][e] = canon_small<M>(rot_read<N1>(tb.lut1, lane + 64 * e, r0));
  }
  __syncthreads();
  int *st = reinterpret_cast<int *>(lds);
#pragma unroll 1
  for (int i = 0; i < N0; ++i) {
    const int a = __builtin_amdgcn_readfirstlane(la[i]);
    uint32_t w[2][16];  // digit words of canon(X^a ACC_p - ACC_p), coefficient lane + 64 e
#pragma unroll
    for (int p = 0; p < 2; ++p) {
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        st[lane + 64 * e] = (int)ac[p][e];
        st[N1 + lane + 64 * e] = -(int)ac[p][e];
      }
      Ntt1W::wave_sync();
#pragma unroll
      for (int e = 0; e < 16; ++e) {  // (X^a ACC)[j] = [ACC, -ACC][(j - a) mod 2N]
        const int x = st[(lane + 64 * e - a) & (2 * N1 - 1)];
        w[p][e] = Lvl1Int::digits(Lvl1Int::canon(x - (int)ac[p][e]));
      }
      Ntt1W::wave_sync();  // the reads are done before the buffer is written again
    }
    double o[2][16];
#pragma unroll
    for (int p = 0; p < 2; ++p)
#pragma unroll 1
      for (int k = 0; k < D1; ++k) {  // GGSW row p D1 + k: digit k of polynomial p
        double x[16];
#pragma unroll
        for (int e = 0; e < 16; ++e) x[e] = lvl1_digit(w[p][e], k);
        Ntt1W::fwd(x, lds, tb.tw1, lane);
        const double *kr = bsk1n + ((size_t)i * 2 * D1 + p * D1 + k) * 2 * N1 + lane * 16;
#pragma unroll
        for (int out = 0; out < 2; ++out)
#pragma unroll
          for (int e = 0; e < 16; ++e) {
            const double v = mm<M>(x[e], kr[out * N1 + e]);
            o[out][e] = p == 0 && k == 0 ? v : o[out][e] + v;
          }
      }
#pragma unroll
    for (int out = 0; out < 2; ++out) {
#pragma unroll
      for (int e = 0; e < 16; ++e) o[out][e] = canon<M>(o[out][e]);
      Ntt1W::inv(o[out], lds, tb.itw1, lane);
#pragma unroll
      for (int e = 0; e < 16; ++e) ac[out][e] = canon<M>(ac[out][e] + o[out][e]);
    }
  }
  if (mode == 0) {  // extract_lwe_locally (coefficient 0), detector.rs:561
#pragma unroll
    for (int e = 0; e < 16; ++e) st[lane + 64 * e] = (int)ac[0][e];
    Ntt1W::wave_sync();
    uint32_t *o = ext + g * (N1 + 1);
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const int j = lane + 64 * e;
      o[j] = Lvl1Int::to_u32(j == 0 ? st[0] : -st[N1 - j]);
    }
    if (lane == 0) o[N1] = Lvl1Int::to_u32((int)ac[1][0]);
  } else {
    uint64_t *o = rlwe_out + g * 2 * N1;
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      o[lane + 64 * e] = Lvl1Int::to_u32((int)ac[0][e]);
      o[N1 + lane + 64 * e] = Lvl1Int::to_u32((int)ac[1][e]);
    }
  }
}

__global__ __launch_bounds__(64) void br1n_kernel(const uint16_t *__restrict__ clue_a,
                                                  const uint16_t *__restrict__ clue_b,
                                                  const uint16_t *__restrict__ lwe_a,
                                                  const uint16_t *__restrict__ lwe_b,
                                                  const double *__restrict__ bsk1n, DeviceTables tb,
                                                  uint32_t *__restrict__ ext, uint64_t *__restrict__ rlwe_out,
                                                  int mode, size_t nrot) {
  if (blockIdx.x >= nrot) return;
  br1n_body(clue_a, clue_b, lwe_a, lwe_b, bsk1n, tb, ext, rlwe_out, mode, blockIdx.x);
}
// The exact fallback of a guarded level-1 launch: runs only when that launch's margin word reached thr.
__global__ __launch_bounds__(64) void br1n_fallback_kernel(const uint16_t *__restrict__ clue_a,
                                                           const uint16_t *__restrict__ clue_b,
                                                           const uint16_t *__restrict__ lwe_a,
                                                           const uint16_t *__restrict__ lwe_b,
                                                           const double *__restrict__ bsk1n, DeviceTables tb,
                                                           uint32_t *__restrict__ ext,
                                                           uint64_t *__restrict__ rlwe_out, int mode, size_t nrot,
                                                           const unsigned long long *lmargin, double thr) {
  if (blockIdx.x >= nrot || !margin_breached(lmargin, thr)) return;
  br1n_body(clue_a, clue_b, lwe_a, lwe_b, bsk1n, tb, ext, rlwe_out, mode, blockIdx.x);
}

}  // namespace omr
