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
  // y = an integer + e (|y| < 2^43, |e| < 0.1: an FFT product output): round(y) mod q in [0, q], as
  // a u32. The quotient is floor(y / q) (as computed: it may exceed the true floor only when y is
  // within 2^-37 q of a multiple of q, and then r rounds to 0; it may fall one short only when the
  // rounded result is q), r = y - kq keeps the fraction, and adding 1.5 * 2^52 rounds r to the
  // nearest integer in the low mantissa bits: one FP64 add instead of rint + conversion. The result
  // q (= 0 mod q) is allowed: Lvl1Off::add folds it. With a RoundGuard, |r - round(r)| =
  // |y - rint(y)| (r = y - kq is exact) is recorded.
  template <bool G = false>
  __device__ static __forceinline__ uint32_t round_mod(double y, RoundGuard<G> *rg = nullptr) {
    const double r = __fma_rn(-floor(y * (1.0 / 134215681.0)), 134215681.0, y);
    const double s = r + 6755399441055744.0;
    if constexpr (G) rg->note(r, s - 6755399441055744.0);
    return (uint32_t)__builtin_bit_cast(uint64_t, s);
  }
  // NonPowOf2ApproxSignedBasis (logB 5, d 4, drop 7) on a canonical residue: y = floor((v + 2^6)
  // / 2^7) has balanced base-32 digits d_k in [-16, 15] (k < 3) and an unbounded top digit; in
  // closed form, with y' = y + 16 (1 + 32 + 32^2): d_k = ((y' >> 5k) & 31) - 16 for k < 3 and
  // d_3 = y' >> 15 (the same digits as the recursive Digits8<LOGB1, D1, DROP1>). The word kept is
  // y' ^ (16 (1 + 32 + 32^2)): field k then holds d_k in two's complement (d_k + 16 = f in
  // [0, 32) and (f - 16) mod 32 = f ^ 16), the top digit is unchanged, and every digit is one
  // signed bit-field extract with wave-uniform offset and width (Lvl1Off::digit_u). Returns that word.
  static constexpr int DIGIT_BIAS = ((1 << (LOGB1 * (D1 - 1))) - 1) / ((1 << LOGB1) - 1) * (1 << (LOGB1 - 1));
  __device__ static __forceinline__ uint32_t digits(int v) {
    return (uint32_t)(((v + (1 << (DROP1 - 1))) >> DROP1) + DIGIT_BIAS) ^ (uint32_t)DIGIT_BIAS;
  }
};

// br1f keeps ACC offset by H/2: ac'' in [0, Q) with ac'' = ac + H/2 (mod Q). The stored negacyclic
// extension n = H - ac'' = -ac + H/2 is then in the same representation (as a signed u32, in
// [-H, H]) and is also the operand of the digit word: for a rotated entry x'' (either half),
// t = x'' + n = (x - ac) + H (mod Q) with t in (-Q, 2Q), so one v_min3_u32(t, t + Q, t - Q) (the
// wrapped operands lose) is canon(x - ac) + H in [0, Q), and the digit word of the canonical
// residue y - H is ((y - H + 2^6 + 2^7 DIGIT_BIAS) >> 7) ^ DIGIT_BIAS (the bias folded in before
// the shift; the shift itself folds into the extraction offsets, digits_u): 5 integer operations
// per word. The accumulator update adds a
// rounded product in [0, Q] (Lvl1Int::round_mod): s in [0, 2Q), min(s, s - Q), 3 operations.
struct Lvl1Off {
  static constexpr uint32_t Q = (uint32_t)Lvl1Int::Q, H = (uint32_t)Lvl1Int::H, OFF = H / 2;
  static_assert(H % 2 == 0, "H/2 offset");
  __device__ static __forceinline__ uint32_t fold(uint32_t y, uint32_t yq, uint32_t ymq) {  // y, y + Q, y - Q
    return min(min(y, yq), ymq);
  }
  // centred value v in [-H, H] -> ac''
  __device__ static __forceinline__ uint32_t enc(int v) {
    const uint32_t y = (uint32_t)(v + (int)OFF);
    return min(y, y + Q);
  }
  // ac'' -> centred value in [-H, H]
  __device__ static __forceinline__ int dec(uint32_t acpp) { return Lvl1Int::canon((int)acpp - (int)OFF); }
  // the stored negacyclic half "-ac + H/2" and the digit operand
  __device__ static __forceinline__ uint32_t neg(uint32_t acpp) { return H - acpp; }
  // digit word of canon(x - ac) from a stored entry x'' and n = neg(ac''): t = x - ac + H; the
  // Lvl1Int::digits word before its shift by DROP1 (bits 7.. hold the fields, bits 0..6 the dropped
  // remainder, never read): the shift folds into the extraction offsets (digit_u / digit_shifts_u),
  // one operation fewer per word. Both br1l and br1f use it (br1f since round 5: at 248 VGPRs it no
  // longer spills; same speed, profiles/r05n/bench_variants.log).
  __device__ static __forceinline__ uint32_t digits_u(uint32_t xs, uint32_t n) {
    const uint32_t t = xs + n;
    const uint32_t y = fold(t, t + Q, t - Q);
    constexpr uint32_t C = (uint32_t)((1 << (DROP1 - 1)) - Lvl1Int::H + (Lvl1Int::DIGIT_BIAS << DROP1));
    return (y + C) ^ ((uint32_t)Lvl1Int::DIGIT_BIAS << DROP1);
  }
  // signed digit k of a digits_u() word: one v_bfe_i32 at offset DROP1 + 5 k (the top digit: the
  // word's sign-extended rest)
  __device__ static __forceinline__ double digit_u(uint32_t w, int k) {
    return (double)(int)__builtin_amdgcn_sbfe(w, DROP1 + LOGB1 * k, k < D1 - 1 ? LOGB1 : 32 - DROP1 - LOGB1 * (D1 - 1));
  }
  // signed digit k of a digits_u() word by two shifts
  __device__ static __forceinline__ double digit_shifts_u(uint32_t w, int k) {
    const int s1 = k < D1 - 1 ? 32 - DROP1 - LOGB1 * (k + 1) : 0;
    const int s2 = k < D1 - 1 ? 32 - LOGB1 : DROP1 + LOGB1 * (D1 - 1);
    return (double)((int)(w << s1) >> s2);
  }
  // ac'' + r for r in [0, Q], reduced to [0, Q)
  __device__ static __forceinline__ uint32_t add(uint32_t acpp, uint32_t r) {
    const uint32_t s = acpp + r;
    return min(s, s - Q);
  }
  template <bool G>
  __device__ static __forceinline__ uint32_t round(double y, RoundGuard<G> *rg) { return Lvl1Int::round_mod<G>(y, rg); }
};

// ACC layout: ac[p][h * 8 + e] = coefficient lane + 64 e + 512 h of poly p (0 mask, 1 body).
__device__ __forceinline__ int acc_coef(int lane, int i) { return lane + 64 * (i & 7) + 512 * (i >> 3); }

// digits of (X^a - 1) * ACC for both polys. Each poly is staged with its negacyclic extension
// ext = [ACC, -ACC] (2N int32 = the wave's 8 KB buffer st), so (X^a * ACC)[j] = ext[(j - a) mod 2N]:
// no sign fix-up per coefficient. st is 8 KB-aligned (br1f_body), so the LDS byte address of
// entry (j - a) mod 2N is st | ((4 (lane - a) + 256 i) & 8191) for coefficient j = lane + 64 i:
// one add and one v_and_or_b32 per read.
// (ACC in the Lvl1Off representation: ext = [ac'', H - ac''], every entry "value + H/2".)
typedef __attribute__((address_space(3))) uint32_t lds_u32;
__device__ __forceinline__ void br1f_digits(const uint32_t (&ac)[2][16], uint32_t *st, int a, int lane,
                                            uint32_t (&pk)[2][16]) {
  const uint32_t sbase = (uint32_t)(size_t)(lds_u32 *)st;
  const uint32_t b4 = (uint32_t)(lane - a) * 4u;
  const uint32_t kWrap = 8u * N1 - 1;  // 8 KB - 1 (no VOP3 literals on gfx9: an SGPR operand)
#pragma unroll
  for (int p = 0; p < 2; ++p) {
    uint32_t n[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      n[i] = Lvl1Off::neg(ac[p][i]);
      st[acc_coef(lane, i)] = ac[p][i];
      st[N1 + acc_coef(lane, i)] = n[i];
    }
    wave_lds_sync();
#pragma unroll
    for (int i = 0; i < 16; ++i) {  // acc_coef(0, i) = 64 i
      uint32_t addr;  // ((b4 + 256 i) & 8191) | sbase in one v_and_or_b32 (not formed by the compiler)
      asm("v_and_or_b32 %0, %1, %2, %3" : "=v"(addr) : "v"(b4 + 256u * i), "s"(kWrap), "v"(sbase));  // one SGPR per VOP3 on gfx9
      pk[p][i] = Lvl1Off::digits_u(*(const lds_u32 *)(size_t)addr, n[i]);
    }
    wave_lds_fence();  // the next poly's writes stay below these reads
  }
}

// ---- key rows staged through LDS by LDS-DMA ----------------------------------
// GGSW row q (global row index over the whole key: step * 8 + row) = [A/B][512] complex, 16 KB,
// copied by the workgroup's waves with LDS-DMA (buffer_load_dwordx4 ... lds) into one of two LDS buffers
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

// The key is read through a buffer descriptor (wave-uniform, SGPRs): each DMA instruction is
// buffer_load_dwordx4 ... offen lds with the lane's byte offset (lane * 16, one VGPR for the whole
// kernel) and the row / piece offset in soffset, so issuing a row costs no VALU address arithmetic.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t bsk1_rsrc(const double2 *bskf) {
  constexpr uint32_t bytes = (uint32_t)((size_t)N0 * 2 * D1 * KROW_SLOTS * sizeof(double2));
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<double2 *>(bskf), 0, bytes, 0x00020000);
}
__device__ __forceinline__ void krow_issue(__amdgpu_buffer_rsrc_t rsrc, int q,
                                           double2 *buf, uint32_t lane16, int wave) {
#pragma unroll
  for (int u = 0; u < KROW_INSTR; ++u) {
    const int ins = wave * KROW_INSTR + u;  // 0..15: comp = ins / 8, point e = ins % 8
    const int comp = ins >> 3, e = ins & 7;
    // key1_pos(lane, e) = e * 64 + lane: the piece starts at slot comp * 512 + e * 64
    const int piece = comp * Fft512::N + e * 64;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(
        rsrc, (__attribute__((address_space(3))) void *)(buf + piece), 16, lane16,
        (int)((uint32_t)q * (uint32_t)(KROW_SLOTS * sizeof(double2)) + (uint32_t)(piece * sizeof(double2))), 0, 0);
  }
}
__device__ __forceinline__ void vm_wait_row_in_flight() {  // s_waitcnt vmcnt(KROW_INSTR)
  __builtin_amdgcn_s_waitcnt((KROW_INSTR & 0xF) | ((KROW_INSTR >> 4) << 14) | (0x7 << 4) | (0xF << 8));
}
__device__ __forceinline__ void vm_wait_all() {  // s_waitcnt vmcnt(0)
  __builtin_amdgcn_s_waitcnt((0x7 << 4) | (0xF << 8));
}

// One GGSW row q = q0 + p D1 + k of a CMUX step: digit k of poly p, forward transform,
// multiply-accumulate with the staged row. FIRST (the step's row 0) writes the products instead
// of accumulating, so the accumulators need no zeroing. (A function, not a lambda: a lambda's
// by-reference captures drop __restrict__, and the pass-0 twiddles were then re-read with vector
// loads in every row instead of being kept in registers: 3 % slower.)
template <bool FIRST>
__device__ __forceinline__ void br1f_row(const uint32_t (&pk)[16], int k, int q, int qtotal, double (&outr)[2][8],
                                         double (&outi)[2][8], double2 *xch, const double2 *tws,
                                         __amdgpu_buffer_rsrc_t rsrc, double2 *kbuf, int lane, uint32_t lane16,
                                         int wave, const double2 *__restrict__ gtw, const double2 *w3,
                                         const Tw1Reg &tr) {
  using F = Fft512;
  const bool more = q + 1 < qtotal;
  wg_barrier_lds();  // every wave has finished reading buffer (q + 1) & 1 (row q - 1)
  if (more) krow_issue(rsrc, q + 1, kbuf + ((q + 1) & 1) * KROW_SLOTS, lane16, wave);
  double xr[1][8], xi[1][8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    xr[0][e] = Lvl1Off::digit_u(pk[e], k);
    xi[0][e] = Lvl1Off::digit_u(pk[8 + e], k);
  }
  F::fwd<1, true, true>(xr, xi, xch, tws, lane, gtw, w3, tr);
  if (more)
    vm_wait_row_in_flight();  // row q landed (row q + 1 may stay in flight)
  else
    vm_wait_all();
  wg_barrier_lds();  // ... in every wave's share
  const double2 *kb = kbuf + (q & 1) * KROW_SLOTS;
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const double2 ka = kb[e * 64 + lane], kB = kb[F::N + e * 64 + lane];
    if constexpr (FIRST) {
      outr[0][e] = __fma_rn(xr[0][e], ka.x, -xi[0][e] * ka.y);
      outi[0][e] = __fma_rn(xr[0][e], ka.y, xi[0][e] * ka.x);
      outr[1][e] = __fma_rn(xr[0][e], kB.x, -xi[0][e] * kB.y);
      outi[1][e] = __fma_rn(xr[0][e], kB.y, xi[0][e] * kB.x);
    } else {
      outr[0][e] = __fma_rn(xr[0][e], ka.x, __fma_rn(-xi[0][e], ka.y, outr[0][e]));
      outi[0][e] = __fma_rn(xr[0][e], ka.y, __fma_rn(xi[0][e], ka.x, outi[0][e]));
      outr[1][e] = __fma_rn(xr[0][e], kB.x, __fma_rn(-xi[0][e], kB.y, outr[1][e]));
      outi[1][e] = __fma_rn(xr[0][e], kB.y, __fma_rn(xi[0][e], kB.x, outi[1][e]));
    }
  }
}

// One CMUX step with LDS-staged key rows. q0 = first global row of this step; rows q0..q0+7 are
// consumed, the next step's first row is prefetched on the way. xch: the wave's exchange buffer
// (Fft512::BUF).
template <bool G>
__device__ __forceinline__ void br1f_step_lds(uint32_t (&ac)[2][16], double2 *xch, const double2 *tws, int a,
                                              __amdgpu_buffer_rsrc_t rsrc, int q0, int qtotal, double2 *kbuf,
                                              int lane, uint32_t lane16, int wave,
                                              const double2 *__restrict__ gtw, const double2 *w3,
                                              RoundGuard<G> &rg, const Tw1Reg &tr) {
  using F = Fft512;
  uint32_t pk[2][16];
  br1f_digits(ac, reinterpret_cast<uint32_t *>(xch), a, lane, pk);
  double outr[2][8], outi[2][8];
  br1f_row<true>(pk[0], 0, q0, qtotal, outr, outi, xch, tws, rsrc, kbuf, lane, lane16, wave, gtw, w3, tr);
#pragma unroll 1
  for (int k = 1; k < D1; ++k)
    br1f_row<false>(pk[0], k, q0 + k, qtotal, outr, outi, xch, tws, rsrc, kbuf, lane, lane16, wave, gtw, w3, tr);
#pragma unroll 1
  for (int k = 0; k < D1; ++k)
    br1f_row<false>(pk[1], k, q0 + D1 + k, qtotal, outr, outi, xch, tws, rsrc, kbuf, lane, lane16, wave, gtw, w3,
                    tr);
  F::inv_pair<true, true>(outr, outi, xch, tws, lane, gtw, w3, tr);  // both outputs, interleaved
#pragma unroll
  for (int o = 0; o < 2; ++o)
#pragma unroll
    for (int i = 0; i < 16; ++i)
      ac[o][i] = Lvl1Off::add(ac[o][i], Lvl1Off::round<G>(i < 8 ? outr[o][i] : outi[o][i - 8], &rg));
}

// Level-1 blind rotations: BR1F_WPG waves per workgroup, one rotation per wave; rotation
// g = wg * BR1F_WPG + wave: clue g % 7 of message g / 7 (lwe_a == nullptr) or LWE g; nrot bounds
// g. The transforms are wave-private (wave-level LDS sync); the waves run the CMUX steps in
// lockstep, sharing each key row staged in LDS and one twiddle table.
// G: the rounding-margin guard (exactness.hpp) publishes the largest |y - rint(y)| to *margin.
// LDS of br1f_body, carved from one pool:
// the exchange buffers (8 KB-aligned: br1f_digits' addressing), the twiddles, the LWE masks, the two
// staged key rows: 76 KB.
constexpr size_t BR1_LDS_XCH = 0, BR1_LDS_TWS = BR1_LDS_XCH + (size_t)BR1F_WPG * Fft512::BUF * sizeof(double2),
                 BR1_LDS_LA = BR1_LDS_TWS + (size_t)Fft512::N * sizeof(double2),
                 BR1_LDS_KBUF = BR1_LDS_LA + (size_t)BR1F_WPG * N0 * sizeof(uint16_t),
                 BR1_LDS_BYTES = BR1_LDS_KBUF + 2 * (size_t)KROW_SLOTS * sizeof(double2);

template <bool G>
__device__ __forceinline__ void br1f_body(
    const uint16_t *__restrict__ clue_a, const uint16_t *__restrict__ clue_b,
    const uint16_t *__restrict__ lwe_a, const uint16_t *__restrict__ lwe_b,
    const double2 *__restrict__ bskf, DeviceTables tb, uint32_t *__restrict__ ext,
    uint64_t *__restrict__ rlwe_out, int mode, size_t nrot, unsigned long long *margin, char *pool, size_t item) {
  constexpr int NF = Fft512::N, W = BR1F_WPG;
  static_assert(16 % W == 0, "LDS key staging: W divides the row's 16 one-KiB pieces");
  static_assert(Fft512::BUF * sizeof(double2) == 8192, "one 8 KB buffer per wave");
  double2(&xch_all)[W][Fft512::BUF] = *reinterpret_cast<double2(*)[W][Fft512::BUF]>(pool + BR1_LDS_XCH);
  double2 *tws = reinterpret_cast<double2 *>(pool + BR1_LDS_TWS);
  uint16_t(&la_all)[W][N0] = *reinterpret_cast<uint16_t(*)[W][N0]>(pool + BR1_LDS_LA);
  double2 *kbuf = reinterpret_cast<double2 *>(pool + BR1_LDS_KBUF);
  // the wave index is wave-uniform: readfirstlane keeps it (and every key-row DMA address and M0
  // value derived from it) in SGPRs instead of per-lane VALU arithmetic
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  double2 *xch = xch_all[wave];
  uint16_t *la = la_all[wave];
  const size_t g = item * W + wave;
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
  uint32_t ac[2][16];  // Lvl1Off: ac + OFF
  const int r0 = (2 * N1 - (b % (2 * N1))) % (2 * N1);
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    ac[0][i] = Lvl1Off::enc(0);
    ac[1][i] = Lvl1Off::enc((int)canon_small<Mod<1>>(rot_read<N1>(tb.lut1, acc_coef(lane, i), r0)));
  }
  for (int j = threadIdx.x; j < NF; j += 64 * W) tws[j] = tb.fft1[j];
  __syncthreads();
  // pass 3's two lane twiddles in registers for the whole rotation: 2 KB of LDS reads fewer per
  // transform (LDS runs at ~60 % of its bandwidth here; 595 -> 591 ms per 16,384 messages,
  // profiles/r04/br1f_w3_ab.log)
  const double2 w3[2] = {tws[Fft512::TW_P3 + lane], tws[Fft512::TW_P3 + 64 + lane]};
  // the forward's pass-0 (c, t) and pass-1 (c, t) in registers for the whole rotation (Tw1Reg)
  Tw1Reg tr;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const double2 v = tws[Fft512::TW_P0F + k];
    tr.f0c[k] = v.x;
    const uint64_t y = __builtin_bit_cast(uint64_t, v.y);  // wave-uniform: readfirstlane keeps it in SGPRs
    tr.f0t[k] = __builtin_bit_cast(double, (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)y) |
                                               ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(y >> 32)) << 32));
  }
#pragma unroll
  for (int e0 = 0; e0 < 2; ++e0) {
    tr.p1[2 * e0] = tws[Fft512::tw4_index(lane, e0, 0)];
    tr.p1[2 * e0 + 1] = tws[Fft512::tw4_index(lane, e0, 1)];
  }
  // every step runs (a = 0 gives zero digits and leaves ACC unchanged) so the waves share the
  // staged key rows; row 0 is issued before the loop
  const __amdgpu_buffer_rsrc_t rsrc = bsk1_rsrc(bskf);
  const uint32_t lane16 = (uint32_t)lane * 16u;
  krow_issue(rsrc, 0, kbuf, lane16, wave);
  RoundGuard<G> rg;
#pragma unroll 1
  for (int i = 0; i < N0; ++i) {
    const int a = __builtin_amdgcn_readfirstlane(la[i]);
    br1f_step_lds<G>(ac, xch, tws, a, rsrc, i * 2 * D1, N0 * 2 * D1, kbuf, lane, lane16, wave, tb.fft1, w3, rg, tr);
  }
  rg.publish(margin);
  __syncthreads();
  if (g >= nrot) return;
  if (mode == 0) {  // extract_lwe_locally (coefficient 0), detector.rs:561
    int *st = reinterpret_cast<int *>(xch);
#pragma unroll
    for (int i = 0; i < 16; ++i) st[acc_coef(lane, i)] = Lvl1Off::dec(ac[0][i]);
    wave_lds_sync();
    uint32_t *o = ext + g * (N1 + 1);
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int j = acc_coef(lane, i);
      o[j] = Lvl1Int::to_u32(j == 0 ? st[0] : -st[N1 - j]);
    }
    if (lane == 0) o[N1] = Lvl1Int::to_u32(Lvl1Off::dec(ac[1][0]));
  } else {
    uint64_t *o = rlwe_out + g * 2 * N1;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      o[acc_coef(lane, i)] = Lvl1Int::to_u32(Lvl1Off::dec(ac[0][i]));
      o[N1 + acc_coef(lane, i)] = Lvl1Int::to_u32(Lvl1Off::dec(ac[1][i]));
    }
  }
}

__global__ __launch_bounds__(64 * BR1F_WPG, 2) void br1f_kernel(
    const uint16_t *__restrict__ clue_a, const uint16_t *__restrict__ clue_b,
    const uint16_t *__restrict__ lwe_a, const uint16_t *__restrict__ lwe_b,
    const double2 *__restrict__ bskf, DeviceTables tb, uint32_t *__restrict__ ext,
    uint64_t *__restrict__ rlwe_out, int mode, size_t nrot) {
  __shared__ __attribute__((aligned(8192))) char pool[BR1_LDS_BYTES];
  br1f_body<false>(clue_a, clue_b, lwe_a, lwe_b, bskf, tb, ext, rlwe_out, mode, nrot, nullptr, pool, blockIdx.x);
}
__global__ __launch_bounds__(64 * BR1F_WPG, 2) void br1f_guard_kernel(
    const uint16_t *__restrict__ clue_a, const uint16_t *__restrict__ clue_b,
    const uint16_t *__restrict__ lwe_a, const uint16_t *__restrict__ lwe_b,
    const double2 *__restrict__ bskf, DeviceTables tb, uint32_t *__restrict__ ext,
    uint64_t *__restrict__ rlwe_out, int mode, size_t nrot, unsigned long long *margin) {
  __shared__ __attribute__((aligned(8192))) char pool[BR1_LDS_BYTES];
  br1f_body<true>(clue_a, clue_b, lwe_a, lwe_b, bskf, tb, ext, rlwe_out, mode, nrot, margin, pool, blockIdx.x);
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
