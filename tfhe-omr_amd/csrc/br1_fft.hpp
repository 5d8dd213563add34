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
#define BR1F_WAVES (BR1F_RW > 1 ? 1 : 2)  // waves per SIMD the register allocation targets
#endif
#ifndef BR1F_WPG
#define BR1F_WPG 4  // level-1 waves (rotations) per workgroup, kept in lockstep per CMUX step
#endif
#ifndef BR1F_KEY_LDS
#define BR1F_KEY_LDS 1  // key rows staged through LDS by LDS-DMA, shared by the workgroup
#endif
#ifndef BR1F_RW
#define BR1F_RW 1  // level-1 rotations per wave (key rows shared, transforms interleaved)
#endif
#ifndef BR1F_GTW
#define BR1F_GTW 1  // pass-0 twiddles (wave-uniform) by scalar loads from the global table (-2.6 %)
#endif
#ifndef BR1F_BARRIERS
#define BR1F_BARRIERS 2  // workgroup barriers per staged key row (1: next row issued after the MAC barrier;
                         // exposes the row latency: 212 vs 199 ms at D = 4,096)
#endif
#ifndef BR1F_DMA_SPREAD
#define BR1F_DMA_SPREAD 0  // next key row's LDS-DMA pieces one per FFT pass instead of back to back (same speed: off)
#endif
#ifndef BR1F_KBUF
#define BR1F_KBUF 2  // staged key-row buffers: 2 (two barriers per row) or 3 (one; needs BR1F_WPG 8 to fit LDS)
#endif
#ifndef BR1F_T0
#define BR1F_T0 0  // stage 0 of the digit FFTs (one uniform twiddle w) from a 33-entry LDS table d * w
                   // (bit-exact; 730 vs 705 ms: the table reads cost more than the VALU saved, off)
#endif
#ifndef BR1F_DIGIT_SBFE
#define BR1F_DIGIT_SBFE 2  // digit words in two's-complement fields; 2: two uniform shifts per digit, 1: v_bfe_i32 (inline asm, slower)
#endif
#ifndef BR1F_ROT_EXT
#define BR1F_ROT_EXT 1  // rotation through a negacyclic extension [ACC, -ACC] per poly
#endif
#ifndef BR1F_CANON_MIN
#define BR1F_CANON_MIN 1  // level-1 int canonicalisation by unsigned min folds (no VCC hazards)
#endif
#ifndef BR1F_KEY_SPLIT
#define BR1F_KEY_SPLIT 1  // load the B component of a key row after the transform (32 VGPRs less)
#endif

struct Lvl1Int {
  static constexpr int Q = 134215681, H = 67107840;
  __device__ static __forceinline__ int canon(int x) {  // |x| < q + H -> [-H, H]
    if (!BR1F_CANON_MIN) {
      x = x > H ? x - Q : x;
      return x < -H ? x + Q : x;
    }
    // unsigned min folds, no VCC (compare/select pairs serialise on VCC with hazard NOPs):
    // y = x + H in [-Q, 2Q); min(y, y + Q) lifts [-Q, 0) into [0, Q), min(y, y - Q) lowers
    // [Q, 2Q) into [0, Q) (the other operand wraps above 2^31 and loses)
    uint32_t y = (uint32_t)(x + H);
    y = min(y, y + (uint32_t)Q);
    y = min(y, y - (uint32_t)Q);
    return (int)y - H;
  }
  __device__ static __forceinline__ uint32_t to_u32(int x) { return (uint32_t)(x < 0 ? x + Q : x); }
  // NonPowOf2ApproxSignedBasis (logB 5, d 4, drop 7) on a canonical residue: y = floor((v + 2^6)
  // / 2^7) has balanced base-32 digits d_k in [-16, 15] (k < 3) and an unbounded top digit; in
  // closed form, with y' = y + 16 (1 + 32 + 32^2): d_k = ((y' >> 5k) & 31) - 16 for k < 3 and
  // d_3 = y' >> 15 (the same digits as the recursive Digits8<LOGB1, D1, DROP1>). The word kept is
  // y' ^ (16 (1 + 32 + 32^2)): field k then holds d_k in two's complement (d_k + 16 = f in
  // [0, 32) and (f - 16) mod 32 = f ^ 16), the top digit is unchanged, and every digit is one
  // signed bit-field extract with wave-uniform offset and width (digit()). Returns that word.
  static constexpr int DIGIT_BIAS = ((1 << (LOGB1 * (D1 - 1))) - 1) / ((1 << LOGB1) - 1) * (1 << (LOGB1 - 1));
  __device__ static __forceinline__ uint32_t digits(int v) {
    return (uint32_t)(((v + (1 << (DROP1 - 1))) >> DROP1) + DIGIT_BIAS) ^
           (BR1F_DIGIT_SBFE ? (uint32_t)DIGIT_BIAS : 0u);
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
  // signed digit k of a digits() word as an int (two-shift form)
  __device__ static __forceinline__ int digit_int(uint32_t w, int k) {
    static_assert(BR1F_DIGIT_SBFE == 2, "integer digits written for the two-shift form");
    const int s1 = k < D1 - 1 ? 32 - LOGB1 * (k + 1) : 0, s2 = k < D1 - 1 ? 32 - LOGB1 : LOGB1 * (D1 - 1);
    return (int)(w << s1) >> s2;
  }
  // signed digit k of a digits() word
  __device__ static __forceinline__ double digit(uint32_t w, int k) {
    if (!BR1F_DIGIT_SBFE)
      return k < D1 - 1 ? (double)((int)((w >> (LOGB1 * k)) & ((1u << LOGB1) - 1)) - (1 << (LOGB1 - 1)))
                        : (double)((int)w >> (LOGB1 * (D1 - 1)));
    if (BR1F_DIGIT_SBFE == 2) {  // two uniform shifts: field to the top, arithmetic shift down
      const int s1 = k < D1 - 1 ? 32 - LOGB1 * (k + 1) : 0, s2 = k < D1 - 1 ? 32 - LOGB1 : LOGB1 * (D1 - 1);
      return (double)((int)(w << s1) >> s2);
    }
    const int off = LOGB1 * k, width = k < D1 - 1 ? LOGB1 : 32 - LOGB1 * (D1 - 1);
    // v_bfe_i32 by inline asm: clang turns (double)__builtin_amdgcn_sbfe(x, off, width) with a
    // non-constant width into v_cvt_f64_u32 (wrong for negative digits; ROCm 7.2)
    int d;
    asm("v_bfe_i32 %0, %1, %2, %3" : "=v"(d) : "v"(w), "s"(off), "v"(width));
    return (double)d;
  }
};

// ACC layout: ac[p][h * 8 + e] = coefficient lane + 64 e + 512 h of poly p (0 mask, 1 body).
__device__ __forceinline__ int acc_coef(int lane, int i) { return lane + 64 * (i & 7) + 512 * (i >> 3); }

// digits of (X^a - 1) * ACC for both polys. Each poly is staged with its negacyclic extension
// ext = [ACC, -ACC] (2N int32 = the wave's 8 KB buffer st), so (X^a * ACC)[j] = ext[(j - a) mod 2N]:
// one masked index and no sign fix-up per coefficient.
__device__ __forceinline__ void br1f_digits(const int (&ac)[2][16], int *st, int a, int lane,
                                            uint32_t (&pk)[2][16]) {
  if (!BR1F_ROT_EXT) {  // both polys staged at once (8 KB), sign-corrected rotated reads
#pragma unroll
    for (int p = 0; p < 2; ++p)
#pragma unroll
      for (int i = 0; i < 16; ++i) st[p * N1 + acc_coef(lane, i)] = ac[p][i];
    wave_lds_sync();
#pragma unroll
    for (int p = 0; p < 2; ++p)
#pragma unroll
      for (int i = 0; i < 16; ++i)
        pk[p][i] = Lvl1Int::digits(
            Lvl1Int::canon(Lvl1Int::rot_read(st + p * N1, acc_coef(lane, i), a) - ac[p][i]));
    wave_lds_sync();
    return;
  }
#pragma unroll
  for (int p = 0; p < 2; ++p) {
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      st[acc_coef(lane, i)] = ac[p][i];
      st[N1 + acc_coef(lane, i)] = -ac[p][i];
    }
    wave_lds_sync();
    const int base = lane - a + 2 * N1;
#pragma unroll
    for (int i = 0; i < 16; ++i)
      pk[p][i] = Lvl1Int::digits(
          Lvl1Int::canon(st[(base + acc_coef(0, i)) & (2 * N1 - 1)] - ac[p][i]));
    if (OMR_FFT_POSTREAD_WAIT)
      wave_lds_sync();
    else
      wave_lds_fence();  // the next poly's writes stay below these reads
  }
}

// One CMUX step for RW rotations held by this wave (all at the same key row i; a[r] may be 0,
// which yields zero digits and leaves that accumulator unchanged). The key row loads are shared
// by the RW rotations and the RW transforms are interleaved (instruction-level parallelism).
template <int RW>
__device__ __forceinline__ void br1f_step(int (&ac)[RW][2][16], double2 *xch, const double2 *tws,
                                          const int (&a)[RW], const double2 *__restrict__ ggsw,
                                          int lane) {
  using F = Fft512;
  constexpr int NF = F::N;
  uint32_t pk[RW][2][16];
#pragma unroll
  for (int r = 0; r < RW; ++r)
    br1f_digits(ac[r], reinterpret_cast<int *>(xch + r * F::BUF), a[r], lane, pk[r]);

  double outr[2][RW][8], outi[2][RW][8];  // [output A/B][rotation][point]
#pragma unroll
  for (int o = 0; o < 2; ++o)
#pragma unroll
    for (int r = 0; r < RW; ++r)
#pragma unroll
      for (int e = 0; e < 8; ++e) outr[o][r][e] = outi[o][r][e] = 0.0;
#pragma unroll
  for (int p = 0; p < 2; ++p) {
#pragma unroll 1
    for (int k = 0; k < D1; ++k) {
      // GGSW row p*D1 + k: [2][512] complex (A, B), lane's 8 values contiguous
      const double2 *kr = ggsw + (size_t)(p * D1 + k) * 2 * NF + lane * 8;
      double2 ka[8], kb[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) {
#ifdef OMR_EXPT_NO_KEY  // timing experiment only (wrong results): no key loads
        ka[e] = make_double2(1.0 + e, 2.0 - k);
        kb[e] = make_double2(3.0 - e, 1.0 + k);
        continue;
#endif
        ka[e] = kr[e];
        if (!BR1F_KEY_SPLIT) kb[e] = kr[NF + e];
      }
      double xr[RW][8], xi[RW][8];
#pragma unroll
      for (int r = 0; r < RW; ++r)
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          xr[r][e] = Lvl1Int::digit(pk[r][p][e], k);
          xi[r][e] = Lvl1Int::digit(pk[r][p][8 + e], k);
        }
      F::fwd<RW>(xr, xi, xch, tws, lane);
#ifndef OMR_EXPT_NO_KEY
      if (BR1F_KEY_SPLIT) {
#pragma unroll
        for (int e = 0; e < 8; ++e) kb[e] = kr[NF + e];
      }
#endif
#pragma unroll
      for (int r = 0; r < RW; ++r)
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          outr[0][r][e] = __fma_rn(xr[r][e], ka[e].x, __fma_rn(-xi[r][e], ka[e].y, outr[0][r][e]));
          outi[0][r][e] = __fma_rn(xr[r][e], ka[e].y, __fma_rn(xi[r][e], ka[e].x, outi[0][r][e]));
          outr[1][r][e] = __fma_rn(xr[r][e], kb[e].x, __fma_rn(-xi[r][e], kb[e].y, outr[1][r][e]));
          outi[1][r][e] = __fma_rn(xr[r][e], kb[e].y, __fma_rn(xi[r][e], kb[e].x, outi[1][r][e]));
        }
    }
  }
#pragma unroll
  for (int o = 0; o < 2; ++o) {
    F::inv<RW>(outr[o], outi[o], xch, tws, lane);
#pragma unroll
    for (int r = 0; r < RW; ++r)
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const double v = rint(i < 8 ? outr[o][r][i] : outi[o][r][i - 8]);  // exact (< 2^43)
        ac[r][o][i] = Lvl1Int::canon(ac[r][o][i] + (int)red<Mod<1>>(v));
      }
  }
}

// ---- key rows staged through LDS by LDS-DMA (BR1F_KEY_LDS) ----------------------------------
// GGSW row q (global row index over the whole key: step * 8 + row) = [A/B][512] complex, 16 KB,
// copied by the workgroup's waves with global_load_lds_dwordx4 into one of two LDS buffers,
// transposed so that slot comp * 512 + e * 64 + lane holds the lane's e-th point (the
// multiply-accumulate then reads consecutive slots: no bank conflicts). Each wave issues
// 16 / BR1F_WPG of the row's 16 one-KiB instructions. Raw s_barrier + counted vmcnt keep the
// next row's copy in flight across the barriers (cdna_hip_programming.md, "Pipelining across
// barriers").
constexpr int KROW_SLOTS = 2 * Fft512::N;  // double2 per staged row
constexpr int KROW_INSTR = 16 / BR1F_WPG;  // glds per wave per row

__device__ __forceinline__ void krow_issue(const double2 *__restrict__ row, double2 *buf, int lane,
                                           int wave) {
#pragma unroll
  for (int u = 0; u < KROW_INSTR; ++u) {
    const int ins = wave * KROW_INSTR + u;  // 0..15: comp = ins / 8, point e = ins % 8
    const int comp = ins >> 3, e = ins & 7;
    const double2 *src = row + comp * Fft512::N + lane * 8 + e;
    __builtin_amdgcn_global_load_lds(src, buf + comp * Fft512::N + e * 64, 16, 0, 0);
  }
}
// one of this wave's KROW_INSTR pieces of a row (u < KROW_INSTR)
__device__ __forceinline__ void krow_issue_piece(const double2 *__restrict__ row, double2 *buf, int lane,
                                                 int wave, int u) {
  const int ins = wave * KROW_INSTR + u;
  const int comp = ins >> 3, e = ins & 7;
  __builtin_amdgcn_global_load_lds(row + comp * Fft512::N + lane * 8 + e, buf + comp * Fft512::N + e * 64, 16,
                                   0, 0);
}
__device__ __forceinline__ void vm_wait_row_in_flight() {  // s_waitcnt vmcnt(KROW_INSTR)
  __builtin_amdgcn_s_waitcnt((KROW_INSTR & 0xF) | ((KROW_INSTR >> 4) << 14) | (0x7 << 4) | (0xF << 8));
}
__device__ __forceinline__ void vm_wait_all() {  // s_waitcnt vmcnt(0)
  __builtin_amdgcn_s_waitcnt((0x7 << 4) | (0xF << 8));
}
__device__ __forceinline__ void wg_barrier_lds() {  // LDS reads/writes done, then s_barrier
  __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0)
  __builtin_amdgcn_s_barrier();
  __atomic_signal_fence(__ATOMIC_SEQ_CST);
}

// One CMUX step with LDS-staged key rows for the RW rotations of this wave (their transforms
// interleaved, each staged key value read once for all of them). q0 = first global row of this
// step; rows q0..q0+7 are consumed, the next step's first row(s) are prefetched on the way.
// xch: RW exchange buffers of Fft512::BUF.
template <int RW>
__device__ __forceinline__ void br1f_step_lds(int (&ac)[RW][2][16], double2 *xch, const double2 *tws,
                                              const int (&a)[RW], const double2 *__restrict__ bskf,
                                              int q0, int qtotal, double2 *kbuf, int lane, int wave,
                                              const double2 *__restrict__ gtw, const double2 *t1) {
  using F = Fft512;
  uint32_t pk[RW][2][16];
#pragma unroll
  for (int r = 0; r < RW; ++r) br1f_digits(ac[r], reinterpret_cast<int *>(xch + r * F::BUF), a[r], lane, pk[r]);
  double outr[2][RW][8], outi[2][RW][8];
#pragma unroll
  for (int o = 0; o < 2; ++o)
#pragma unroll
    for (int r = 0; r < RW; ++r)
#pragma unroll
      for (int e = 0; e < 8; ++e) outr[o][r][e] = outi[o][r][e] = 0.0;
#pragma unroll
  for (int p = 0; p < 2; ++p) {
#pragma unroll 1
    for (int k = 0; k < D1; ++k) {
      const int q = q0 + p * D1 + k;
      const bool more = q + 1 < qtotal;
#if BR1F_BARRIERS == 2 && BR1F_KBUF == 2
#if !defined(OMR_EXPT_NO_KSTAGE) && !defined(OMR_EXPT_KSTAGE_NOBAR)  // timing experiments only
      wg_barrier_lds();  // every wave has finished reading buffer (q + 1) & 1 (row q - 1)
#endif
#ifndef OMR_EXPT_NO_KSTAGE
      if (!BR1F_DMA_SPREAD && more)
        krow_issue(bskf + (size_t)(q + 1) * KROW_SLOTS, kbuf + ((q + 1) & 1) * KROW_SLOTS, lane, wave);
#endif
#endif
      double xr[RW][8], xi[RW][8];
      if (BR1F_T0) {
        // stage 0 pairs (e, e + 4) under the one twiddle w = tw[1]: w * x[e + 4] for the small
        // digits (|d| <= 16) is a sum of table entries t1[d + 16] = (d w.x, d w.y); rounded
        // products instead of an fma, inside the FFT's error budget (tools/fft_exactness.py
        // models unfused complex products everywhere)
#pragma unroll
        for (int r = 0; r < RW; ++r)
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const double2 a = t1[Lvl1Int::digit_int(pk[r][p][e + 4], k) + 16];
            const double2 b = t1[Lvl1Int::digit_int(pk[r][p][8 + e + 4], k) + 16];
            const double vr = a.x - b.y, vi = a.y + b.x;
            const double ur = Lvl1Int::digit(pk[r][p][e], k), ui = Lvl1Int::digit(pk[r][p][8 + e], k);
            xr[r][e] = ur + vr;
            xi[r][e] = ui + vi;
            xr[r][e + 4] = ur - vr;
            xi[r][e + 4] = ui - vi;
          }
      } else {
#pragma unroll
        for (int r = 0; r < RW; ++r)
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            xr[r][e] = Lvl1Int::digit(pk[r][p][e], k);
            xi[r][e] = Lvl1Int::digit(pk[r][p][8 + e], k);
          }
      }
      if (BR1F_DMA_SPREAD && BR1F_KBUF == 2 && BR1F_BARRIERS == 2) {
        // the next row's LDS-DMA pieces go out one per FFT pass, among VALU work (an issue
        // there costs less than four back to back after the barrier); all are issued before
        // the wait for row q below
        const double2 *nrow = bskf + (size_t)(q + 1) * KROW_SLOTS;
        double2 *nbuf = kbuf + ((q + 1) & 1) * KROW_SLOTS;
        if (more) krow_issue_piece(nrow, nbuf, lane, wave, 0);
        F::fwd_hooked<RW, BR1F_GTW != 0>(xr, xi, xch, tws, lane, gtw, [&](int pass) {
          if (more && pass + 1 < KROW_INSTR) krow_issue_piece(nrow, nbuf, lane, wave, pass + 1);
        });
        static_assert(!BR1F_DMA_SPREAD || KROW_INSTR == Fft512::NPASS + 1, "one piece before the FFT, one per pass");
        static_assert(!BR1F_DMA_SPREAD || !BR1F_T0, "the hooked transform starts at stage 0");
      } else {
        F::fwd<RW, BR1F_GTW != 0, BR1F_T0 ? 1 : 0>(xr, xi, xch, tws, lane, gtw);
      }
#if BR1F_KBUF == 3
      // three staged rows, one barrier per row: row q landed (row q + 1 may stay in flight) in
      // every wave's share, and every wave is past its multiply-accumulate of row q - 1, so
      // buffer (q + 2) % 3 = (q - 1) % 3 is free for row q + 2
      if (more)
        vm_wait_row_in_flight();
      else
        vm_wait_all();
      wg_barrier_lds();
      if (q + 2 < qtotal)
        krow_issue(bskf + (size_t)(q + 2) * KROW_SLOTS, kbuf + ((q + 2) % 3) * KROW_SLOTS, lane, wave);
#elif BR1F_BARRIERS == 2
#ifndef OMR_EXPT_NO_KSTAGE
      if (more)
        vm_wait_row_in_flight();  // row q landed (row q + 1 may stay in flight)
      else
        vm_wait_all();
#endif
#if !defined(OMR_EXPT_NO_KSTAGE) && !defined(OMR_EXPT_KSTAGE_NOBAR)
      wg_barrier_lds();  // ... in every wave's share
#endif
#else
      vm_wait_all();     // this wave's share of row q landed (the only copy in flight)
      wg_barrier_lds();  // row q complete, and every wave is done with row q - 1 (its buffer)
      if (more) krow_issue(bskf + (size_t)(q + 1) * KROW_SLOTS, kbuf + ((q + 1) & 1) * KROW_SLOTS, lane, wave);
#endif
      const double2 *kb = kbuf + (BR1F_KBUF == 3 ? q % 3 : q & 1) * KROW_SLOTS;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const double2 ka = kb[e * 64 + lane], kB = kb[F::N + e * 64 + lane];
#pragma unroll
        for (int r = 0; r < RW; ++r) {
          outr[0][r][e] = __fma_rn(xr[r][e], ka.x, __fma_rn(-xi[r][e], ka.y, outr[0][r][e]));
          outi[0][r][e] = __fma_rn(xr[r][e], ka.y, __fma_rn(xi[r][e], ka.x, outi[0][r][e]));
          outr[1][r][e] = __fma_rn(xr[r][e], kB.x, __fma_rn(-xi[r][e], kB.y, outr[1][r][e]));
          outi[1][r][e] = __fma_rn(xr[r][e], kB.y, __fma_rn(xi[r][e], kB.x, outi[1][r][e]));
        }
      }
    }
  }
#pragma unroll
  for (int o = 0; o < 2; ++o) {
    F::inv<RW, BR1F_GTW != 0>(outr[o], outi[o], xch, tws, lane, gtw);
#pragma unroll
    for (int r = 0; r < RW; ++r)
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const double v = rint(i < 8 ? outr[o][r][i] : outi[o][r][i - 8]);  // exact (< 2^43)
        ac[r][o][i] = Lvl1Int::canon(ac[r][o][i] + (int)red<Mod<1>>(v));
      }
  }
}

// Level-1 blind rotations: BR1F_WPG waves per workgroup, RW rotations per wave; rotation
// g = (wg * BR1F_WPG + wave) * RW + r: clue g % 7 of message g / 7 (lwe_a == nullptr) or LWE g;
// nrot bounds g. The transforms are wave-private (wave-level LDS sync); one workgroup barrier
// per CMUX step keeps the waves in lockstep so they read each key row together (L1/L2 hits)
// and share one twiddle table.
template <int RW>
__global__ __launch_bounds__(64 * BR1F_WPG, BR1F_WAVES) void br1f_kernel(
    const uint16_t *__restrict__ clue_a, const uint16_t *__restrict__ clue_b,
    const uint16_t *__restrict__ lwe_a, const uint16_t *__restrict__ lwe_b,
    const double2 *__restrict__ bskf, DeviceTables tb, uint32_t *__restrict__ ext,
    uint64_t *__restrict__ rlwe_out, int mode, size_t nrot) {
  constexpr int NF = Fft512::N, W = BR1F_WPG;
  __shared__ double2 xch_all[W][RW * Fft512::BUF];
  __shared__ double2 tws[NF];
  __shared__ double2 t1tab[BR1F_T0 ? 33 : 1];
  __shared__ uint16_t la_all[W][RW][N0];
#if BR1F_KEY_LDS
  static_assert(16 % W == 0, "LDS key staging: W divides the row's 16 one-KiB pieces");
  __shared__ double2 kbuf[BR1F_KBUF * KROW_SLOTS];
#endif
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  double2 *xch = xch_all[wave];
  uint16_t(*la)[N0] = la_all[wave];
  int b[RW];
  size_t g[RW];
#pragma unroll
  for (int r = 0; r < RW; ++r) {
    g[r] = ((size_t)blockIdx.x * W + wave) * RW + r;
    const size_t gi = g[r] < nrot ? g[r] : nrot - 1;  // a tail slot recomputes the last rotation
    if (lwe_a == nullptr) {  // extract clue c of message m (CmLweCiphertext::extract_all, :514)
      const size_t m = gi / CLUES;
      const int c = (int)(gi % CLUES);
      const uint16_t *A = clue_a + m * N0;
      for (int i = lane; i < N0; i += 64)
        la[r][i] = i <= c ? (uint16_t)(A[c - i] & (Q0 - 1)) : (uint16_t)((Q0 - A[N0 + c - i]) & (Q0 - 1));
      b[r] = clue_b[m * CLUES + c] & (Q0 - 1);
    } else {
      for (int i = lane; i < N0; i += 64) la[r][i] = lwe_a[gi * N0 + i] & (Q0 - 1);
      b[r] = lwe_b[gi] & (Q0 - 1);
    }
  }
  // ACC = (0, X^{-b} * LUT1)
  int ac[RW][2][16];
#pragma unroll
  for (int r = 0; r < RW; ++r) {
    const int r0 = (2 * N1 - (b[r] % (2 * N1))) % (2 * N1);
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      ac[r][0][i] = 0;
      ac[r][1][i] = (int)canon_small<Mod<1>>(rot_read<N1>(tb.lut1, acc_coef(lane, i), r0));
    }
  }
  for (int j = threadIdx.x; j < NF; j += 64 * W) tws[j] = tb.fft1[j];
  if (BR1F_T0 && threadIdx.x < 33) {  // d * w for d = -16 .. 16, w = the stage-0 twiddle
    const double2 w = tb.fft1[1];
    const double d = (double)((int)threadIdx.x - 16);
    t1tab[threadIdx.x] = make_double2(d * w.x, d * w.y);
  }
  __syncthreads();
#if BR1F_KEY_LDS
  // every step runs (a = 0 gives zero digits and leaves ACC unchanged) so the waves share the
  // staged key rows; row 0 is issued before the loop
  krow_issue(bskf, kbuf, lane, wave);
  if (BR1F_KBUF == 3) krow_issue(bskf + KROW_SLOTS, kbuf + KROW_SLOTS, lane, wave);
#pragma unroll 1
  for (int i = 0; i < N0; ++i) {
    int a[RW];
#pragma unroll
    for (int r = 0; r < RW; ++r) a[r] = __builtin_amdgcn_readfirstlane(la[r][i]);
    br1f_step_lds<RW>(ac, xch, tws, a, bskf, i * 2 * D1, N0 * 2 * D1, kbuf, lane, wave, tb.fft1, t1tab);
  }
  __syncthreads();
#else
#pragma unroll 1
  for (int i = 0; i < N0; ++i) {
    if (W > 1) __syncthreads();  // lockstep: the waves read key row i together
    int a[RW], any = 0;
#pragma unroll
    for (int r = 0; r < RW; ++r) {
      a[r] = __builtin_amdgcn_readfirstlane(la[r][i]);
      any |= a[r];
    }
    if (any == 0) continue;  // (X^0 - 1) * ACC = 0
#ifdef OMR_EXPT_KEYWRAP  // timing experiment only: every step reads one of 4 L2-resident key rows
    br1f_step<RW>(ac, xch, tws, a, bskf + (size_t)(i & 3) * (2 * D1 * 2 * NF), lane);
#else
    br1f_step<RW>(ac, xch, tws, a, bskf + (size_t)i * (2 * D1 * 2 * NF), lane);
#endif
  }
#endif
#pragma unroll
  for (int r = 0; r < RW; ++r) {
    if (g[r] >= nrot) break;
    if (mode == 0) {  // extract_lwe_locally (coefficient 0), detector.rs:561
      int *st = reinterpret_cast<int *>(xch + r * Fft512::BUF);
#pragma unroll
      for (int i = 0; i < 16; ++i) st[acc_coef(lane, i)] = ac[r][0][i];
      wave_lds_sync();
      uint32_t *o = ext + g[r] * (N1 + 1);
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int j = acc_coef(lane, i);
        o[j] = Lvl1Int::to_u32(j == 0 ? st[0] : -st[N1 - j]);
      }
      if (lane == 0) o[N1] = Lvl1Int::to_u32(ac[r][1][0]);
    } else if (mode == 1) {
      uint64_t *o = rlwe_out + g[r] * 2 * N1;
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        o[acc_coef(lane, i)] = Lvl1Int::to_u32(ac[r][0][i]);
        o[N1 + acc_coef(lane, i)] = Lvl1Int::to_u32(ac[r][1][i]);
      }
    }
  }
}

// Coefficient-domain canonical u32 key polynomials -> FFT domain / 512, transform-index order.
__global__ __launch_bounds__(64) void key_to_fft1_kernel(const uint32_t *__restrict__ in,
                                                         double2 *__restrict__ out, size_t npoly,
                                                         const double2 *__restrict__ tw) {
  using F = Fft512;
  __shared__ double2 xch[F::BUF];
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
