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
#include "exactness.hpp"
#include "kernels.hpp"

namespace omr {

constexpr int BR1F_WPG = 4;  // level-1 waves (rotations) per workgroup, kept in lockstep per CMUX step

struct Lvl1Int {
  static constexpr int Q = 134215681, H = 67107840;
  __device__ static __forceinline__ int canon(int x) {  // |x| < q + H -> [-H, H]
    // unsigned min folds, no VCC (compare/select pairs serialise on VCC with hazard NOPs):
    // y = x + H in [-Q, 2Q); min(y, y + Q) lifts [-Q, 0) into [0, Q), min(y, y - Q) lowers
    // [Q, 2Q) into [0, Q) (the other operand wraps above 2^31 and loses)
    uint32_t y = (uint32_t)(x + H);
    y = min(y, y + (uint32_t)Q);
    y = min(y, y - (uint32_t)Q);
    return (int)y - H;
  }
  __device__ static __forceinline__ uint32_t to_u32(int x) { return (uint32_t)(x < 0 ? x + Q : x); }
  // y = an integer + e (|y| < 2^43, |e| < 0.01: an FFT product output): round(y) mod q, centred,
  // as an int. The quotient is rint(y / q) and r = y - kq keeps the fraction; adding 1.5 * 2^52
  // rounds r to the nearest integer in the low mantissa bits, which are its two's complement
  // (|round(r)| <= H + 1): one FP64 add instead of rint + conversion.
  // With a RoundGuard, |r - round(r)| = |y - rint(y)| (r = y - kq is exact) is recorded.
  template <bool G = false>
  __device__ static __forceinline__ int round_red(double y, RoundGuard<G> *rg = nullptr) {
    const double r = __fma_rn(-rint(y * (1.0 / 134215681.0)), 134215681.0, y);
    const double s = r + 6755399441055744.0;
    if constexpr (G) rg->note(r, s - 6755399441055744.0);
    return (int)(uint32_t)__builtin_bit_cast(uint64_t, s);
  }
  // NonPowOf2ApproxSignedBasis (logB 5, d 4, drop 7) on a canonical residue: y = floor((v + 2^6)
  // / 2^7) has balanced base-32 digits d_k in [-16, 15] (k < 3) and an unbounded top digit; in
  // closed form, with y' = y + 16 (1 + 32 + 32^2): d_k = ((y' >> 5k) & 31) - 16 for k < 3 and
  // d_3 = y' >> 15 (the same digits as the recursive Digits8<LOGB1, D1, DROP1>). The word kept is
  // y' ^ (16 (1 + 32 + 32^2)): field k then holds d_k in two's complement (d_k + 16 = f in
  // [0, 32) and (f - 16) mod 32 = f ^ 16), the top digit is unchanged, and every digit is one
  // signed bit-field extract with wave-uniform offset and width (digit()). Returns that word.
  static constexpr int DIGIT_BIAS = ((1 << (LOGB1 * (D1 - 1))) - 1) / ((1 << LOGB1) - 1) * (1 << (LOGB1 - 1));
  __device__ static __forceinline__ uint32_t digits(int v) {
    return (uint32_t)(((v + (1 << (DROP1 - 1))) >> DROP1) + DIGIT_BIAS) ^ (uint32_t)DIGIT_BIAS;
  }
  // signed digit k of a digits() word: one v_bfe_i32 with wave-uniform offset and width
  // (checked in the listing: v_bfe_i32 + v_cvt_f64_i32; an inline-asm v_bfe_i32 is slower, it
  // constrains the scheduler).
  __device__ static __forceinline__ double digit(uint32_t w, int k) {
    return (double)(int)__builtin_amdgcn_sbfe(w, LOGB1 * k, k < D1 - 1 ? LOGB1 : 32 - LOGB1 * (D1 - 1));
  }
  // the same digit by two shifts (the latency kernel measured 1-2 % faster with these)
  __device__ static __forceinline__ double digit_shifts(uint32_t w, int k) {
    const int s1 = k < D1 - 1 ? 32 - LOGB1 * (k + 1) : 0, s2 = k < D1 - 1 ? 32 - LOGB1 : LOGB1 * (D1 - 1);
    return (double)((int)(w << s1) >> s2);
  }
};

// br1f keeps ACC offset by H: ac' = ac + H in [0, Q) (u32). A value y in (-Q, 2Q) is reduced to
// [0, Q) by one v_min3_u32(y, y + Q, y - Q) (the wrapped operands lose), the digit word of the
// canonical residue y' - H is ((y' - H + 2^6 + 2^7 DIGIT_BIAS) >> 7) ^ DIGIT_BIAS (the bias folded
// in before the shift), and the stored negacyclic extension 2H - ac' is again "value + H": 7
// integer operations per digit word instead of 10, 4 per accumulator update instead of 7.
struct Lvl1Off {
  static constexpr uint32_t Q = (uint32_t)Lvl1Int::Q, H = (uint32_t)Lvl1Int::H;
  __device__ static __forceinline__ uint32_t fold(uint32_t y, uint32_t yq, uint32_t ymq) {  // y, y + Q, y - Q
    return min(min(y, yq), ymq);
  }
  // digit word of canon(x - ac) from x' = x + H (stored) and n = 2H - ac' = H - ac
  __device__ static __forceinline__ uint32_t digits(uint32_t xs, uint32_t n) {
    const uint32_t y = fold(xs + n - H, xs + n + (Q - H), xs + n - (Q + H));
    constexpr uint32_t C = (uint32_t)((1 << (DROP1 - 1)) - Lvl1Int::H + (Lvl1Int::DIGIT_BIAS << DROP1));
    return (uint32_t)((int)(y + C) >> DROP1) ^ (uint32_t)Lvl1Int::DIGIT_BIAS;
  }
  // ac' + r for r in [-H - 1, H + 1], reduced to [0, Q)
  __device__ static __forceinline__ uint32_t add(uint32_t acp, int r) {
    const uint32_t s = acp + (uint32_t)r;
    return fold(s, s + Q, s - Q);
  }
};

// ACC layout: ac[p][h * 8 + e] = coefficient lane + 64 e + 512 h of poly p (0 mask, 1 body).
__device__ __forceinline__ int acc_coef(int lane, int i) { return lane + 64 * (i & 7) + 512 * (i >> 3); }

// digits of (X^a - 1) * ACC for both polys. Each poly is staged with its negacyclic extension
// ext = [ACC, -ACC] (2N int32 = the wave's 8 KB buffer st), so (X^a * ACC)[j] = ext[(j - a) mod 2N]:
// one masked index and no sign fix-up per coefficient.
// (ACC in the Lvl1Off representation: ext = [ac', 2H - ac'], every entry "value + H".)
__device__ __forceinline__ void br1f_digits(const uint32_t (&ac)[2][16], uint32_t *st, int a, int lane,
                                            uint32_t (&pk)[2][16]) {
#pragma unroll
  for (int p = 0; p < 2; ++p) {
    uint32_t n[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      n[i] = 2 * Lvl1Off::H - ac[p][i];
      st[acc_coef(lane, i)] = ac[p][i];
      st[N1 + acc_coef(lane, i)] = n[i];
    }
    wave_lds_sync();
    const int base = lane - a + 2 * N1;
#pragma unroll
    for (int i = 0; i < 16; ++i) pk[p][i] = Lvl1Off::digits(st[(base + acc_coef(0, i)) & (2 * N1 - 1)], n[i]);
    wave_lds_fence();  // the next poly's writes stay below these reads
  }
}

// ---- key rows staged through LDS by LDS-DMA ----------------------------------
// GGSW row q (global row index over the whole key: step * 8 + row) = [A/B][512] complex, 16 KB,
// copied by the workgroup's waves with global_load_lds_dwordx4 into one of two LDS buffers
// (two barriers per row: one barrier per row exposes the row's load latency, 212 vs 199 ms),
// transposed so that slot comp * 512 + e * 64 + lane holds the lane's e-th point (the
// multiply-accumulate then reads consecutive slots: no bank conflicts). Each wave issues
// 16 / BR1F_WPG of the row's 16 one-KiB instructions. Raw s_barrier + counted vmcnt keep the
// next row's copy in flight across the barriers (cdna_hip_programming.md, "Pipelining across
// barriers").
constexpr int KROW_SLOTS = 2 * Fft512::N;  // double2 per staged row

// Storage position of transform point (lane, e) within a BSK1 key polynomial: register-major, so
// that each LDS-DMA instruction of krow_issue copies 1 KB contiguous (lane-major, 16 B per lane at
// a 128 B stride: level 1 1 % slower, profiles/r03q/key_layout_ab.log).
__device__ __forceinline__ int key1_pos(int lane, int e) { return e * 64 + lane; }
constexpr int KROW_INSTR = 16 / BR1F_WPG;  // glds per wave per row

__device__ __forceinline__ void krow_issue(const double2 *__restrict__ row, double2 *buf, int lane,
                                           int wave) {
#pragma unroll
  for (int u = 0; u < KROW_INSTR; ++u) {
    const int ins = wave * KROW_INSTR + u;  // 0..15: comp = ins / 8, point e = ins % 8
    const int comp = ins >> 3, e = ins & 7;
    const double2 *src = row + comp * Fft512::N + key1_pos(lane, e);
    __builtin_amdgcn_global_load_lds(src, buf + comp * Fft512::N + e * 64, 16, 0, 0);
  }
}
__device__ __forceinline__ void vm_wait_row_in_flight() {  // s_waitcnt vmcnt(KROW_INSTR)
  __builtin_amdgcn_s_waitcnt((KROW_INSTR & 0xF) | ((KROW_INSTR >> 4) << 14) | (0x7 << 4) | (0xF << 8));
}
__device__ __forceinline__ void vm_wait_all() {  // s_waitcnt vmcnt(0)
  __builtin_amdgcn_s_waitcnt((0x7 << 4) | (0xF << 8));
}

// One CMUX step with LDS-staged key rows. q0 = first global row of this step; rows q0..q0+7 are
// consumed, the next step's first row is prefetched on the way. xch: the wave's exchange buffer
// (Fft512::BUF).
template <bool G>
__device__ __forceinline__ void br1f_step_lds(uint32_t (&ac)[2][16], double2 *xch, const double2 *tws, int a,
                                              const double2 *__restrict__ bskf, int q0, int qtotal,
                                              double2 *kbuf, int lane, int wave,
                                              const double2 *__restrict__ gtw, RoundGuard<G> &rg) {
  using F = Fft512;
  uint32_t pk[2][16];
  br1f_digits(ac, reinterpret_cast<uint32_t *>(xch), a, lane, pk);
  double outr[2][8], outi[2][8];
#pragma unroll
  for (int o = 0; o < 2; ++o)
#pragma unroll
    for (int e = 0; e < 8; ++e) outr[o][e] = outi[o][e] = 0.0;
#pragma unroll
  for (int p = 0; p < 2; ++p) {
#pragma unroll 1
    for (int k = 0; k < D1; ++k) {
      const int q = q0 + p * D1 + k;
      const bool more = q + 1 < qtotal;
      wg_barrier_lds();  // every wave has finished reading buffer (q + 1) & 1 (row q - 1)
      if (more) krow_issue(bskf + (size_t)(q + 1) * KROW_SLOTS, kbuf + ((q + 1) & 1) * KROW_SLOTS, lane, wave);
      double xr[1][8], xi[1][8];
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        xr[0][e] = Lvl1Int::digit(pk[p][e], k);
        xi[0][e] = Lvl1Int::digit(pk[p][8 + e], k);
      }
      F::fwd<1, true>(xr, xi, xch, tws, lane, gtw);
      if (more)
        vm_wait_row_in_flight();  // row q landed (row q + 1 may stay in flight)
      else
        vm_wait_all();
      wg_barrier_lds();  // ... in every wave's share
      const double2 *kb = kbuf + (q & 1) * KROW_SLOTS;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const double2 ka = kb[e * 64 + lane], kB = kb[F::N + e * 64 + lane];
        outr[0][e] = __fma_rn(xr[0][e], ka.x, __fma_rn(-xi[0][e], ka.y, outr[0][e]));
        outi[0][e] = __fma_rn(xr[0][e], ka.y, __fma_rn(xi[0][e], ka.x, outi[0][e]));
        outr[1][e] = __fma_rn(xr[0][e], kB.x, __fma_rn(-xi[0][e], kB.y, outr[1][e]));
        outi[1][e] = __fma_rn(xr[0][e], kB.y, __fma_rn(xi[0][e], kB.x, outi[1][e]));
      }
    }
  }
  F::inv_pair<true>(outr, outi, xch, tws, lane, gtw);  // both outputs, interleaved
#pragma unroll
  for (int o = 0; o < 2; ++o)
#pragma unroll
    for (int i = 0; i < 16; ++i)
      ac[o][i] = Lvl1Off::add(ac[o][i], Lvl1Int::round_red<G>(i < 8 ? outr[o][i] : outi[o][i - 8], &rg));
}

// Level-1 blind rotations: BR1F_WPG waves per workgroup, one rotation per wave; rotation
// g = wg * BR1F_WPG + wave: clue g % 7 of message g / 7 (lwe_a == nullptr) or LWE g; nrot bounds
// g. The transforms are wave-private (wave-level LDS sync); the waves run the CMUX steps in
// lockstep, sharing each key row staged in LDS and one twiddle table.
// G: the rounding-margin guard (exactness.hpp) publishes the largest |y - rint(y)| to *margin.
template <bool G>
__device__ __forceinline__ void br1f_body(
    const uint16_t *__restrict__ clue_a, const uint16_t *__restrict__ clue_b,
    const uint16_t *__restrict__ lwe_a, const uint16_t *__restrict__ lwe_b,
    const double2 *__restrict__ bskf, DeviceTables tb, uint32_t *__restrict__ ext,
    uint64_t *__restrict__ rlwe_out, int mode, size_t nrot, unsigned long long *margin) {
  constexpr int NF = Fft512::N, W = BR1F_WPG;
  static_assert(16 % W == 0, "LDS key staging: W divides the row's 16 one-KiB pieces");
  __shared__ double2 xch_all[W][Fft512::BUF];
  __shared__ double2 tws[NF];
  __shared__ uint16_t la_all[W][N0];
  __shared__ double2 kbuf[2 * KROW_SLOTS];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  double2 *xch = xch_all[wave];
  uint16_t *la = la_all[wave];
  const size_t g = (size_t)blockIdx.x * W + wave;
  const size_t gi = g < nrot ? g : nrot - 1;  // a tail slot recomputes the last rotation
  int b;
  if (lwe_a == nullptr) {  // extract clue c of message m (CmLweCiphertext::extract_all, :514)
    const size_t m = gi / CLUES;
    const int c = (int)(gi % CLUES);
    const uint16_t *A = clue_a + m * N0;
    for (int i = lane; i < N0; i += 64)
      la[i] = i <= c ? (uint16_t)(A[c - i] & (Q0 - 1)) : (uint16_t)((Q0 - A[N0 + c - i]) & (Q0 - 1));
    b = clue_b[m * CLUES + c] & (Q0 - 1);
  } else {
    for (int i = lane; i < N0; i += 64) la[i] = lwe_a[gi * N0 + i] & (Q0 - 1);
    b = lwe_b[gi] & (Q0 - 1);
  }
  // ACC = (0, X^{-b} * LUT1)
  uint32_t ac[2][16];  // Lvl1Off: ac + H
  const int r0 = (2 * N1 - (b % (2 * N1))) % (2 * N1);
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    ac[0][i] = Lvl1Off::H;
    ac[1][i] = (uint32_t)((int)canon_small<Mod<1>>(rot_read<N1>(tb.lut1, acc_coef(lane, i), r0)) + Lvl1Int::H);
  }
  for (int j = threadIdx.x; j < NF; j += 64 * W) tws[j] = tb.fft1[j];
  __syncthreads();
  // every step runs (a = 0 gives zero digits and leaves ACC unchanged) so the waves share the
  // staged key rows; row 0 is issued before the loop
  krow_issue(bskf, kbuf, lane, wave);
  RoundGuard<G> rg;
#pragma unroll 1
  for (int i = 0; i < N0; ++i) {
    const int a = __builtin_amdgcn_readfirstlane(la[i]);
    br1f_step_lds<G>(ac, xch, tws, a, bskf, i * 2 * D1, N0 * 2 * D1, kbuf, lane, wave, tb.fft1, rg);
  }
  rg.publish(margin);
  __syncthreads();
  if (g >= nrot) return;
  if (mode == 0) {  // extract_lwe_locally (coefficient 0), detector.rs:561
    int *st = reinterpret_cast<int *>(xch);
#pragma unroll
    for (int i = 0; i < 16; ++i) st[acc_coef(lane, i)] = (int)ac[0][i] - Lvl1Int::H;
    wave_lds_sync();
    uint32_t *o = ext + g * (N1 + 1);
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int j = acc_coef(lane, i);
      o[j] = Lvl1Int::to_u32(j == 0 ? st[0] : -st[N1 - j]);
    }
    if (lane == 0) o[N1] = Lvl1Int::to_u32((int)ac[1][0] - Lvl1Int::H);
  } else {
    uint64_t *o = rlwe_out + g * 2 * N1;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      o[acc_coef(lane, i)] = Lvl1Int::to_u32((int)ac[0][i] - Lvl1Int::H);
      o[N1 + acc_coef(lane, i)] = Lvl1Int::to_u32((int)ac[1][i] - Lvl1Int::H);
    }
  }
}

__global__ __launch_bounds__(64 * BR1F_WPG, 2) void br1f_kernel(
    const uint16_t *__restrict__ clue_a, const uint16_t *__restrict__ clue_b,
    const uint16_t *__restrict__ lwe_a, const uint16_t *__restrict__ lwe_b,
    const double2 *__restrict__ bskf, DeviceTables tb, uint32_t *__restrict__ ext,
    uint64_t *__restrict__ rlwe_out, int mode, size_t nrot) {
  br1f_body<false>(clue_a, clue_b, lwe_a, lwe_b, bskf, tb, ext, rlwe_out, mode, nrot, nullptr);
}
__global__ __launch_bounds__(64 * BR1F_WPG, 2) void br1f_guard_kernel(
    const uint16_t *__restrict__ clue_a, const uint16_t *__restrict__ clue_b,
    const uint16_t *__restrict__ lwe_a, const uint16_t *__restrict__ lwe_b,
    const double2 *__restrict__ bskf, DeviceTables tb, uint32_t *__restrict__ ext,
    uint64_t *__restrict__ rlwe_out, int mode, size_t nrot, unsigned long long *margin) {
  br1f_body<true>(clue_a, clue_b, lwe_a, lwe_b, bskf, tb, ext, rlwe_out, mode, nrot, margin);
}

// Test entry (omr_fft1_mul): out = a * k mod (X^1024 + 1, q1) through the level-1 FFT path,
// for |a| small (digit-sized) and canonical k.
__global__ __launch_bounds__(64) void fft1_mul_kernel(const uint32_t *__restrict__ a,
                                                      const uint32_t *__restrict__ k,
                                                      uint64_t *__restrict__ out,
                                                      const double2 *__restrict__ tw) {
  using F = Fft512;
  __shared__ double2 xch[F::BUF];
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
