// Level-2 blind rotation on the exact complex FFT (second_level_bootstrapping, detector.rs:599-624).
//
// The external product only multiplies gadget digits (|d| <= 64) by key residues, so with the
// key split into two 25-bit limbs, k = k_lo + 2^25 k_hi (|k_lo|, |k_hi| <= 2^24), every coefficient
// of sum_r d_r * k_r,limb over the 12 GGSW rows is an integer below 12 * 2048 * 64 * 2^24 < 2^44.6,
// and an FP64 FFT product rounds to it exactly (tests/fft2_model.py: worst error ~1e-2 with
// adversarial digits; tests/test_fft2_layout.py). The limb products are recombined mod q2 as
// red(P_hi * 2^25) + P_lo (2^25 P_hi is an exact double). Same digits and rows as the NTT kernels,
// so the output is bit-identical to them.
//
// Transform (Fft1024): R[X]/(X^2048 + 1) -> C[X]/(X^1024 - i), z_j = p_j + i p_{j+1024}; 1,024
// complex points on 256 threads x 4 registers, five radix-4 passes of the twiddle tree of
// device_fft.hpp (n = 1024). Index bits j9..j0, pass P holds bits (9 - 2P, 8 - 2P) in registers
// e = (e1, e0); layouts (position bits e1 e0 | lane l5..l0 | wave w1 w0 -> index bits):
//   P0: 9 8 | 7 6 3 2 1 0 | 5 4    (input: coefficient pairs (j, j + 1024) of point j)
//   P1: 7 6 | 9 8 3 2 1 0 | 5 4    P0 -> P1: register bits 1, 0 <-> lane bits 5, 4 (permlane swaps)
//   P2: 5 4 | 3 2 1 0 9 8 | 7 6    P1 -> P2: cross-wave LDS exchange (X0 / X1)
//   P3: 3 2 | 5 4 1 0 9 8 | 7 6    P2 -> P3: permlane swaps
//   P4: 1 0 | 5 4 3 2 9 8 | 7 6    P3 -> P4: wave-local LDS exchange (W); the multiply-accumulate
//                                  layout: thread t holds points 4t..4t+3 of the key's storage order
// Each exchange has its own XOR swizzle, conflict-free for the ds_write_b128 8-lane and
// ds_read_b128 16-lane groups in its direction (tests/test_fft2_layout.py models the banks).
// Per CMUX step: 12 forward transforms, 48 complex multiply-accumulates per point, 4 inverse
// transforms (2 outputs x 2 limbs) instead of the NTT kernel's 12 + 2 modular transforms.
#pragma once

#include "latency_kernels.hpp"

namespace omr {

struct Fft1024 {
  static constexpr int T = 256, E = 4, n = 1024, L = 10;
  static constexpr int TW_LEN = 3 * (4 + 16 + 64 + 256);  // passes 1..4: (B, A, AB) per block (inverse)
  OMR_HD static constexpr int tw_off(int p) { return p == 1 ? 0 : p == 2 ? 12 : p == 3 ? 60 : 252; }
  // the forward passes' tangent forms (cos, tan) of (A, B) per block follow in the global table:
  // TW_LEN + ct_off(p) + 2 b + k (k: 0 A, 1 B); each thread holds its four blocks' in registers
  static constexpr int CT_LEN = 2 * (4 + 16 + 64 + 256);
  OMR_HD static constexpr int ct_off(int p) { return p == 1 ? 0 : p == 2 ? 8 : p == 3 ? 40 : 168; }

  // index bit of each position bit (e1, e0, l5, l4, l3, l2, l1, l0, w1, w0), per pass layout
  OMR_HD static constexpr int lay(int p, int k) {
    constexpr int tab[5][10] = {{9, 8, 7, 6, 3, 2, 1, 0, 5, 4},
                                {7, 6, 9, 8, 3, 2, 1, 0, 5, 4},
                                {5, 4, 3, 2, 1, 0, 9, 8, 7, 6},
                                {3, 2, 5, 4, 1, 0, 9, 8, 7, 6},
                                {1, 0, 5, 4, 3, 2, 9, 8, 7, 6}};
    return tab[p][k];
  }
  // point index held by register e of thread t in pass layout p
  OMR_HD static constexpr int idx(int p, int t, int e) {
    const int pos[10] = {(e >> 1) & 1, e & 1, (t >> 5) & 1, (t >> 4) & 1, (t >> 3) & 1, (t >> 2) & 1,
                         (t >> 1) & 1, t & 1, (t >> 7) & 1, (t >> 6) & 1};
    int j = 0;
    for (int k = 0; k < 10; ++k) j |= pos[k] << lay(p, k);
    return j;
  }
  OMR_HD static constexpr int bit(int j, int b) { return (j >> b) & 1; }
  // exchange swizzles: slot bits s0..s9 as XORs of index bits (tests/fft2_model.py SWIZZLES)
  OMR_HD static constexpr int slot_xf(int j) {  // P1 -> P2
    return bit(j, 0) | bit(j, 1) << 1 | (bit(j, 2) ^ bit(j, 8)) << 2 | bit(j, 9) << 3 | bit(j, 8) << 4 |
           bit(j, 3) << 5 | ((j >> 4) & 15) << 6;
  }
  OMR_HD static constexpr int slot_xi(int j) {  // P2 -> P1
    return bit(j, 0) | (bit(j, 1) ^ bit(j, 8)) << 1 | (bit(j, 2) ^ bit(j, 9)) << 2 | bit(j, 3) << 3 |
           bit(j, 8) << 4 | bit(j, 9) << 5 | ((j >> 4) & 15) << 6;
  }
  OMR_HD static constexpr int slot_wf(int j) {  // P3 -> P4 (wave bits j7 j6 -> slot bits 9 8)
    return bit(j, 8) | bit(j, 9) << 1 | (bit(j, 2) ^ bit(j, 0)) << 2 | bit(j, 3) << 3 | bit(j, 0) << 4 |
           bit(j, 1) << 5 | ((j >> 4) & 15) << 6;
  }
  OMR_HD static constexpr int slot_wi(int j) {  // P4 -> P3
    return bit(j, 8) | bit(j, 9) << 1 | (bit(j, 2) ^ bit(j, 0)) << 2 | bit(j, 1) << 3 | bit(j, 0) << 4 |
           bit(j, 3) << 5 | ((j >> 4) & 15) << 6;
  }
  // rotation staging of 2048 real coefficients (doubles): conflict-free ds_write_b64 / ds_read_b64
  OMR_HD static constexpr int slot_stage(int c) { return c ^ (((c >> 6) & 1) << 4); }

  // pass-0 twiddles (block 0): B = w^256 = e^{i pi / 8}, A = w^512 = e^{i pi / 4}, AB = e^{3 i pi / 8};
  // tangent forms A = R2 (1 + i), B = C8 (1 + i T8)
  static constexpr double C8 = 0.92387953251128675613, S8 = 0.38268343236508977173, R2 = 0.70710678118654752440;
  static constexpr double T8 = 0.41421356237309504880;  // tan(pi / 8) = sqrt 2 - 1

  __device__ static __forceinline__ void cmulc(double &xr, double &xi, double wr, double wi) {  // * conj(w)
    const double r = __fma_rn(xr, wr, xi * wi);
    const double i = __fma_rn(xi, wr, -xr * wi);
    xr = r;
    xi = i;
  }
  // adjoint network of "x *= T = (1, B, A, AB), then (a0 + a1, a0 - a1, b0 + i b1, b0 - i b1)"
  // (4 x its inverse): y0 = a0 + b0, y1 = a1 + b1, y2 = a0 - b0, y3 = a1 - b1
  __device__ static __forceinline__ void inet4(double (&xr)[E], double (&xi)[E]) {
    const double a0r = xr[0] + xr[1], a0i = xi[0] + xi[1], a1r = xr[0] - xr[1], a1i = xi[0] - xi[1];
    const double b0r = xr[2] + xr[3], b0i = xi[2] + xi[3];
    const double b1r = xi[2] - xi[3], b1i = xr[3] - xr[2];  // -i (o2 - o3)
    xr[0] = a0r + b0r;
    xi[0] = a0i + b0i;
    xr[2] = a0r - b0r;
    xi[2] = a0i - b0i;
    xr[1] = a1r + b1r;
    xi[1] = a1i + b1i;
    xr[3] = a1r - b1r;
    xi[3] = a1i - b1i;
  }
  template <int P>
  __device__ static __forceinline__ int block(int t) {
    return idx(P, t, 0) >> (L - 2 * P);
  }
  // LDS slot of twiddle k (0 B, 1 A, 2 AB) of block b in pass P. The global table (host order) is
  // tw_off(P) + 3 b + k, whose ds_read_b128 reads conflict 4-way in passes 3 and 4; there each k
  // has its own array with the block XOR-swizzled, conflict-free (tests/test_fft2_layout.py::
  // test_twiddle_read_cycles; level 2 0.8 % faster, profiles/r03q/twiddle_soa_ab.log).
  OMR_HD static constexpr int tw_slot(int P, int b, int k) {
    return P == 3 ? tw_off(3) + k * 64 + (b ^ (((b >> 4) & 3) << 1))
         : P == 4 ? tw_off(4) + k * 256 + (b ^ (((b >> 6) & 3) << 2))
                  : tw_off(P) + 3 * b + k;
  }
  // the global table (host order) into LDS slots
  __device__ static __forceinline__ void load_twiddles(double2 *tws, const double2 *__restrict__ twg, int t) {
    for (int j = t; j < TW_LEN; j += T) {
      const int P = j < tw_off(2) ? 1 : j < tw_off(3) ? 2 : j < tw_off(4) ? 3 : 4;
      const int r = j - tw_off(P);
      tws[tw_slot(P, r / 3, r % 3)] = twg[j];
    }
  }
  template <int P>
  __device__ static __forceinline__ void inv_pass(double (&xr)[E], double (&xi)[E], const double2 *tws, int t) {
    inet4(xr, xi);
    if constexpr (P == 0) {
      cmulc(xr[1], xi[1], C8, S8);
      cmulc(xr[2], xi[2], R2, R2);
      cmulc(xr[3], xi[3], S8, C8);
    } else {
      const int b = block<P>(t);
      const double2 B = tws[tw_slot(P, b, 0)], A = tws[tw_slot(P, b, 1)], AB = tws[tw_slot(P, b, 2)];
      cmulc(xr[1], xi[1], B.x, B.y);
      cmulc(xr[2], xi[2], A.x, A.y);
      cmulc(xr[3], xi[3], AB.x, AB.y);
    }
  }
  // inv_pass with the pass's (B, A, AB) already loaded (w)
  __device__ static __forceinline__ void inv_pass_w(double (&xr)[E], double (&xi)[E], const double2 (&w)[3]) {
    inet4(xr, xi);
    cmulc(xr[1], xi[1], w[0].x, w[0].y);
    cmulc(xr[2], xi[2], w[1].x, w[1].y);
    cmulc(xr[3], xi[3], w[2].x, w[2].y);
  }
  template <int P>
  __device__ static __forceinline__ void inv_tw(double2 (&w)[3], const double2 *tws, int t) {
    const int b = block<P>(t);
#pragma unroll
    for (int k = 0; k < 3; ++k) w[k] = tws[tw_slot(P, b, k)];
  }
  // P0 <-> P1 and P2 <-> P3 (an involution): register bit 1 <-> lane bit 5, register bit 0 <-> lane bit 4
  __device__ static __forceinline__ void perm(double (&xr)[E], double (&xi)[E]) {
    swap_lane_bit<5>(xr[0], xr[2]);
    swap_lane_bit<5>(xi[0], xi[2]);
    swap_lane_bit<5>(xr[1], xr[3]);
    swap_lane_bit<5>(xi[1], xi[3]);
    swap_lane_bit<4>(xr[0], xr[1]);
    swap_lane_bit<4>(xi[0], xi[1]);
    swap_lane_bit<4>(xr[2], xr[3]);
    swap_lane_bit<4>(xi[2], xi[3]);
  }
  OMR_HD static constexpr int swz(int S, int j) {
    return S == 0 ? slot_xf(j) : S == 1 ? slot_xi(j) : S == 2 ? slot_wf(j) : slot_wi(j);
  }
  // Slot of register e of thread t in layout P under swizzle S, as base(t) ^ xk(e) + ak(e): the
  // swizzles and layouts are linear over GF(2), so slot = swz(idx(P, t, 0)) ^ swz(idx(P, 0, e));
  // the bits of the second term that base(t) never sets are added as an immediate offset, the
  // rest (at most one distinct value here) is one XOR: two address registers per side.
  OMR_HD static constexpr int base_mask(int S, int P) {
    int m = 0;
    for (int t = 0; t < T; ++t) m |= swz(S, idx(P, t, 0));
    return m;
  }
  template <int S, int P>
  __device__ static __forceinline__ int slot_of(int base, int e) {
    constexpr int M0 = base_mask(S, P);
    const int k = swz(S, idx(P, 0, e));
    return (k & M0 ? base ^ (k & M0) : base) + (k & ~M0);
  }
  // LDS exchange PF -> PT through buf (1024 double2) with swizzle S; CROSS: workgroup barrier
  // between the writes and the reads (a cross-wave exchange), else wave-level ordering
  template <int PF, int PT, int S, bool CROSS>
  __device__ static __forceinline__ void exchange(double (&xr)[E], double (&xi)[E], double2 *buf, int t) {
    const int bw = swz(S, idx(PF, t, 0)), br = swz(S, idx(PT, t, 0));
#pragma unroll
    for (int e = 0; e < E; ++e) buf[slot_of<S, PF>(bw, e)] = make_double2(xr[e], xi[e]);
    if constexpr (CROSS) {
      wg_barrier_lds();  // global loads (the next key blocks) stay in flight
    } else {
      __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0)
      __builtin_amdgcn_wave_barrier();
      __atomic_signal_fence(__ATOMIC_SEQ_CST);
    }
#pragma unroll
    for (int e = 0; e < E; ++e) {
      const double2 v = buf[slot_of<S, PT>(br, e)];
      xr[e] = v.x;
      xi[e] = v.y;
    }
    __builtin_amdgcn_wave_barrier();  // the next writes stay below these reads (in-order LDS per wave)
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
  }
  // forward radix-4 pass in tangent form (device_fft.hpp, bfly): the tree's stage A on the pairs
  // (0, 2), (1, 3), then B on (0, 1) and i B on (2, 3) -- the same map as "T = (1, B, A, AB), then
  // net4" in 24 FMAs instead of 28 operations
  __device__ static __forceinline__ void fwd_pass_t(double (&xr)[E], double (&xi)[E], double2 A, double2 B) {
    bfly<false>(xr[0], xi[0], xr[2], xi[2], A.x, A.y);
    bfly<false>(xr[1], xi[1], xr[3], xi[3], A.x, A.y);
    bfly<false>(xr[0], xi[0], xr[1], xi[1], B.x, B.y);
    bfly<true>(xr[2], xi[2], xr[3], xi[3], B.x, B.y);
  }
  // thread t's (A, B) tangent forms of pass P from the global table (its block is the same for all
  // four registers and all transforms)
  template <int P>
  __device__ static __forceinline__ void block_ct(double2 (&w)[2], const double2 *__restrict__ twg, int t) {
    const int b = block<P>(t);
#pragma unroll
    for (int k = 0; k < 2; ++k) w[k] = twg[TW_LEN + ct_off(P) + 2 * b + k];
  }
  // forward: in P0 layout (point idx(0, t, e)), out P4 layout. X: this transform's cross-wave buffer;
  // the wave-local exchange (P3 -> P4) runs in the wave's own quarter of X (slot bits 9, 8 = wave:
  // tests/test_fft2_layout.py::test_exchange_regions), which after this transform's cross-wave reads
  // no other wave touches until the next-but-one transform writes X behind the next barrier. Every
  // pass in tangent form on the thread's (A, B) held in registers (wc[P - 1]: block_ct<P>).
  struct NoMid {
    __device__ void operator()() const {}
  };
  // mid(): called after the cross-wave exchange (br2f_digit issues key loads there)
  template <typename Mid = NoMid>
  __device__ static __forceinline__ void fwd(double (&xr)[E], double (&xi)[E], double2 *X, int t,
                                             const double2 (&wc)[4][2], Mid mid = Mid()) {
    fwd_pass_t(xr, xi, make_double2(R2, 1.0), make_double2(C8, T8));
    perm(xr, xi);
    fwd_pass_t(xr, xi, wc[0][0], wc[0][1]);
    exchange<1, 2, 0, true>(xr, xi, X, t);
    mid();
    fwd_pass_t(xr, xi, wc[1][0], wc[1][1]);
    perm(xr, xi);
    fwd_pass_t(xr, xi, wc[2][0], wc[2][1]);
    exchange<3, 4, 2, false>(xr, xi, X, t);
    fwd_pass_t(xr, xi, wc[3][0], wc[3][1]);
  }
  // unscaled inverse (x 1024; the keys carry 1/1024): in P4 layout, out P0 layout; the wave-local
  // exchange first, in the wave's own quarter of X (which the previous use of X, two cross-wave
  // uses back, has finished with behind the last barrier), then the cross-wave one (own-quarter
  // writes)
  // Each pass's (B, A, AB) is requested one pass ahead, before the previous pass's arithmetic (round 6:
  // level 2 -0.4 %, profiles/r06f/ab.log), so its LDS round trip is off the pass's critical path.
  __device__ static __forceinline__ void inv(double (&xr)[E], double (&xi)[E], double2 *X, const double2 *tws, int t) {
    double2 w4[3], w3[3], w2[3], w1[3];
    inv_tw<4>(w4, tws, t);
    inv_tw<3>(w3, tws, t);
    inv_pass_w(xr, xi, w4);
    exchange<4, 3, 3, false>(xr, xi, X, t);
    inv_tw<2>(w2, tws, t);
    inv_pass_w(xr, xi, w3);
    perm(xr, xi);
    inv_tw<1>(w1, tws, t);
    inv_pass_w(xr, xi, w2);
    exchange<2, 1, 1, true>(xr, xi, X, t);
    __builtin_amdgcn_s_setprio(2);  // raised past the cross-wave barrier, as in br2f_digit
    inv_pass_w(xr, xi, w1);
    perm(xr, xi);
    inv_pass<0>(xr, xi, tws, t);
    __builtin_amdgcn_s_setprio(0);
  }
};

constexpr double LIMB = 33554432.0;  // 2^25: key = lo + 2^25 hi

// Storage position of point 4 t + e (P4 layout: thread t's register e) within a key block:
// register-major, so that each of a thread's four loads per block is one 1 KB-contiguous wave
// instruction (16 B per lane). The point-major order (4 t + e: 64 B per thread, 16 B per lane at a
// 64 B stride per instruction) ran level 2 8.7 % slower: 667 vs 609 ms per 16,384 messages
// (profiles/r03q/key_layout_ab.log).
__device__ __forceinline__ int key_pos(int t, int e) { return e * Fft1024::T + t; }

// BSK2 rows (canonical u64 [670][12][2][2048]) -> FFT-domain limbs, x 1/1024, as double2
// [670][12][2 out][2 limb][1024], point idx(4, t, e) at key_pos(t, e): key_spectrum_dd_kernel<2>
// (key_spectra.hpp), in double-double.

// Level-2 digit words for br2f: the Digits2 decomposition (NonPowOf2ApproxSignedBasis logB 7,
// d 6, drop 8) with every field a two's-complement digit, so that each digit is one v_bfe_i32
// (Digits2's biased fields need a v_bfe_u32 and a subtraction of 64). Digits 0..4 are biased by 64
// as in Digits2 (so the words have no borrows) and each 7-bit field is then XORed with 64
// ((f - 64) mod 128 = f ^ 64); the top digit d5 is left unbiased, so y >> 21 holds it as a signed
// value in bits 14..29 (sign-extended by the extract; |y| < 2^42, so |d5| < 2^7).
// The words come out of the FP64 bit pattern (round 5): Y = y + 1.5 * 2^52 is exact and its low 51
// mantissa bits are y in two's complement, so lo = Y's low dword (fields 0..2 at bits 0..20; the
// bits above are never extracted) and hi = bits 21..52 of Y (one v_alignbit_b32): 3 FP64 + 3
// integer operations per word pair instead of 8 FP64-rate (two floors, two conversions) + 2.
struct Digits2S {
  static constexpr int DW = 2;
  static_assert(LOGB2 == 7 && D2 == 6 && DROP2 == 8, "closed form written for the level-2 basis");
  __device__ static __forceinline__ void pack(double v, uint32_t (&pk)[DW]) {
    // + 64 (1 + 128 + .. + 128^4) + 1.5 * 2^52, an exact double
    const double y = floor(__fma_rn(v, 1.0 / 256.0, 0.5)) + (17315143744.0 + 6755399441055744.0);
    const uint64_t b = __builtin_bit_cast(uint64_t, y);
    const uint32_t lo = (uint32_t)b, hi = (uint32_t)(b >> 32);
    pk[0] = lo ^ 0x102040u;                                   // fields 0, 1, 2
    pk[1] = __builtin_amdgcn_alignbit(hi, lo, 21) ^ 0x2040u;  // fields 3, 4; d5 in bits 14..29
  }
  static constexpr int TOP_WIDTH = 16;  // d5: bits 35..50 of Y
  // digit j + 3 h as a double (h: the word, a compile-time constant)
  template <int H>
  __device__ static __forceinline__ double digit(const uint32_t (&pk)[DW], int j) {
    return (double)(int)__builtin_amdgcn_sbfe(pk[H], 7 * j, H == 1 && j == 2 ? TOP_WIDTH : 7);
  }
};

// acc + lo + 2^25 hr, reduced to the exact centred representative mod q2 (acc canonical; lo, hr the
// rounded limb products, |lo|, |hr| < 2^46): x = acc + lo and 2^25 hr are exact, the quotient
// k = rint((2^25 hr + x) / q2) is within 2^-30 of the true one, so fma(-k, q2, 2^25 hr) is the exact
// integer r - x (|r| <= q2 / 2 + 2^21), and one red of r is exact (|r| <= q2 - 1): 12 FP64
// operations with the two limb roundings instead of 14 (red of the high product, then canon).
__device__ __forceinline__ double limb_acc(double acc, double lo, double hr) {
  using M = Mod<2>;
  const double x = acc + lo;
  const double hi = hr * LIMB;
  const double k = rint(__fma_rn(hr, LIMB * M::QINV, x * M::QINV));
  return canon_small<M>(__fma_rn(-k, M::Q, hi) + x);
}

// BSK2 (FFT form) through a buffer descriptor: each key load is buffer_load_dwordx4 with the
// thread's byte offset (t * 16) in voffset and the row / block / register offset in soffset, so a
// digit's 16 loads cost no VALU address arithmetic (64-bit VGPR address adds before).
constexpr int BR2_ROW = 4 * Fft1024::n;  // double2 per GGSW row: [2 out][2 limb][1024]
__device__ __forceinline__ __amdgpu_buffer_rsrc_t bsk2_rsrc(const double2 *bskf) {
  constexpr uint32_t bytes = (uint32_t)((size_t)NI * 2 * D2 * BR2_ROW * sizeof(double2));
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<double2 *>(bskf), 0, bytes, 0x00020000);
}
typedef unsigned br2_v4u __attribute__((ext_vector_type(4)));
// output o's two limb blocks of global row q: thread t's 4 points (key_pos(t, e) = e * 256 + t)
__device__ __forceinline__ void br2f_load_half(double2 (&k)[2][Fft1024::E], __amdgpu_buffer_rsrc_t rsrc, int q,
                                               int o, uint32_t t16) {
#pragma unroll
  for (int l = 0; l < 2; ++l)
#pragma unroll
    for (int e = 0; e < Fft1024::E; ++e) {
#ifdef OMR_BR2_KEYABL  // timing-only ablation: every key load from one 4 KB block (L1-resident; wrong output)
      const uint32_t soff = 0;
      (void)q;
#else
      const uint32_t soff = (uint32_t)q * (uint32_t)(BR2_ROW * sizeof(double2)) +
                            (uint32_t)(((o * 2 + l) * Fft1024::n + e * Fft1024::T) * sizeof(double2));
#endif
      k[l][e] = __builtin_bit_cast(double2, __builtin_amdgcn_raw_buffer_load_b128(rsrc, t16, (int)soff, 0));
    }
}

// Digit words of (X^a - 1) * ACC_p from the LDS-resident accumulator (acp: 2048 doubles at
// Fft1024::slot_stage positions): coefficient j and j + 1024 of the thread's P0 points, as the
// Digits2S words (the rotated entry with its negacyclic sign as one xor of bit 63).
__device__ __forceinline__ void br2f_digits(const double *acp, int a, int t,
                                            uint32_t (&pk)[2][Fft1024::E][Digits2S::DW]) {
  using F = Fft1024;
  using M = Mod<2>;
  constexpr int NN = N2;
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int e = 0; e < F::E; ++e) {
      const int c = F::idx(0, t, e) + F::n * h;
      const uint32_t u = (uint32_t)(c - a) & (2 * NN - 1);
      const double v = acp[F::slot_stage(u & (NN - 1))];
      const uint32_t vh = (uint32_t)(__builtin_bit_cast(uint64_t, v) >> 32) ^ ((u & NN) << (31 - 11));
      const double rot = __builtin_bit_cast(double, (__builtin_bit_cast(uint64_t, v) & 0xffffffffull) |
                                                        ((uint64_t)vh << 32));
      Digits2S::pack(canon_small<M>(rot - acp[F::slot_stage(c)]), pk[h][e]);
      // keep the words as integers (not the doubles they come from) across the digit loop
      asm volatile("" : "+v"(pk[h][e][0]), "+v"(pk[h][e][1]));
    }
}

// One digit of a CMUX step: forward transform of digit j + 3 w (W) of the poly whose words are pk,
// then the multiply-accumulate into the four (output, limb) spectra: output A with ka (loaded one
// digit ahead, in flight across the transform), output B with kb (limb 0 loaded mid-transform, limb 1
// after it, in flight across output A's multiply-accumulate); ka is reloaded for the next digit nx
// between the two. (A function, not a lambda: by-reference captures drop __restrict__ / address-space facts.)
template <int W>
__device__ __forceinline__ void br2f_digit(const uint32_t (&pk)[2][Fft1024::E][Digits2S::DW], int j, int q, int nx,
                                           double (&sr)[2][2][Fft1024::E], double (&si)[2][2][Fft1024::E],
                                           double2 (&ka)[2][Fft1024::E], double2 (&kb)[2][Fft1024::E], double2 *X,
                                           __amdgpu_buffer_rsrc_t rsrc, uint32_t t16, int t, const double2 (&wc)[4][2]) {
  using F = Fft1024;
  constexpr int E = F::E;
  double xr[E], xi[E];
#pragma unroll
  for (int e = 0; e < E; ++e) {
    xr[e] = Digits2S::digit<W>(pk[0][e], j);
    xi[e] = Digits2S::digit<W>(pk[1][e], j);
  }
  // output B's limb-0 blocks issued mid-transform (after its cross-wave exchange: 1.3 % faster at
  // level 2 than after the transform; both limbs there spill and run 20-34 % slower,
  // profiles/r05zf/bench_variants.log), limb 1 after it, in flight across output A's products
  auto load_kb = [&](int l) {
#pragma unroll
    for (int e = 0; e < E; ++e) {
#ifdef OMR_BR2_KEYABL
      const uint32_t soff = 0;
#else
      const uint32_t soff = (uint32_t)q * (uint32_t)(BR2_ROW * sizeof(double2)) +
                            (uint32_t)(((1 * 2 + l) * Fft1024::n + e * Fft1024::T) * sizeof(double2));
#endif
      kb[l][e] = __builtin_bit_cast(double2, __builtin_amdgcn_raw_buffer_load_b128(rsrc, t16, (int)soff, 0));
    }
  };
  // Wave priority (s_setprio) raised from the transform's cross-wave barrier to the end of the
  // digit's multiply-accumulates, normal otherwise: of the two workgroups sharing each SIMD, the wave
  // past a barrier issues first, so a workgroup's four waves reach the next barrier closer together
  // (level 2 -3.7 %, stable over 8 alternating runs: profiles/r05zo/; the inverses the same way,
  // Fft1024::inv: profiles/r05zq/). Left raised past the digit
  // (through the inverses and the next digit words) it was as fast in most runs but bimodal, one run
  // in four 50 % slower at level 2 (profiles/r05zn/).
  constexpr int LE = 1;  // limbs issued mid-transform (this form is the measured schedule)
  F::fwd(xr, xi, X, t, wc, [&]() {
    __builtin_amdgcn_s_setprio(2);
#pragma unroll
    for (int l = 0; l < LE; ++l) load_kb(l);
  });
#pragma unroll
  for (int l = LE; l < 2; ++l) load_kb(l);
#pragma unroll
  for (int o = 0; o < 2; ++o) {
#pragma unroll
    for (int l = 0; l < 2; ++l)
#pragma unroll
      for (int e = 0; e < E; ++e) {
        const double2 kv = o ? kb[l][e] : ka[l][e];
        sr[o][l][e] = __fma_rn(xr[e], kv.x, __fma_rn(-xi[e], kv.y, sr[o][l][e]));
        si[o][l][e] = __fma_rn(xr[e], kv.y, __fma_rn(xi[e], kv.x, si[o][l][e]));
      }
    if (o == 0) br2f_load_half(ka, rsrc, nx, 0, t16);
  }
  __builtin_amdgcn_s_setprio(0);
}

// Rounding to the exact limb products, recombination mod q2 and ACC_o += (in place in LDS): thread
// t owns coefficients idx(0, t, e) + 1024 h of ACC_o, which only it reads before the next step.
template <bool G>
__device__ __forceinline__ void br2f_update(double *aco, const double (&sr)[2][Fft1024::E],
                                           const double (&si)[2][Fft1024::E], RoundGuard<G> &rg, int t) {
  using F = Fft1024;
#pragma unroll
  for (int e = 0; e < F::E; ++e)
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const double ylo = h ? si[0][e] : sr[0][e], yhi = h ? si[1][e] : sr[1][e];
      const double lo = rint(ylo), hr = rint(yhi);
      rg.note(ylo, lo);
      rg.note(yhi, hr);
      double &a = aco[F::slot_stage(F::idx(0, t, e) + F::n * h)];
      a = limb_acc(a, lo, hr);
    }
}

// hom_trace (detector.rs:626-639; secret.rs:167-168 for N^-1) on the exact FFT (round 5), in place on
// the LDS-resident accumulator (acs: mask, body at slot_stage positions, canonical): c *= N^-1, then
// for each of the 11 automorphisms sigma_g: c += KS_g(sigma_g(c)), where the key switch decomposes
// sigma_g(a) into 25 balanced base-4 digits (DigitsTrace) and multiply-accumulates them with the
// trace key's rows exactly as a CMUX step does with BSK2's: the same Fft1024 transforms, the key as
// two 25-bit limbs (tkf: [11 * 25 rows][2 out][2 limb][1024], x 1/1024, row q = 11 k + d ... in
// the order k * 25 + d), the four inverses rounded to the exact limb products and recombined mod q2
// (limb_acc). Both halves stay in the coefficient domain, where sigma_g is the signed permutation
// trace_src; A goes to the mask, sigma_g(b) + B to the body. Each digit's products are below
// 2 * 2^24 * 2048 * 25 < 2^42 (|d| <= 2 for 24 of them, 3 for the top one), so the a priori bound
// of this accumulation (apriori_bound level 4) is far below level 2's; the host falls back to the
// NTT trace when it is not below 0.5. 25 transforms of 120 FP64 operations per thread and step
// instead of 25 modular NTTs of ~450.
template <bool G>
__device__ __forceinline__ void br2f_trace(double *acs, const double2 *__restrict__ tkf, double2 (&Xb)[2][Fft1024::n],
                                           const double2 *tws, const double2 *__restrict__ twg, const DeviceTables &tb,
                                           RoundGuard<G> &rg, int t) {
  using F = Fft1024;
  using M = Mod<2>;
  constexpr int E = F::E, NN = N2;
  double2 wc[4][2];  // the forward twiddles again (not kept live across the rotation)
  F::block_ct<1>(wc[0], twg, t);
  F::block_ct<2>(wc[1], twg, t);
  F::block_ct<3>(wc[2], twg, t);
  F::block_ct<4>(wc[3], twg, t);
  constexpr double NINV = -549755813880.0;  // 2048^-1 mod q2 = 1125350151012361, centred
  static_assert(DT == 25 && TRACE_STEPS == 11, "trace geometry");
#pragma unroll
  for (int p = 0; p < 2; ++p)
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int e = 0; e < E; ++e) {
        double &x = acs[p * NN + F::slot_stage(F::idx(0, t, e) + F::n * h)];
        x = canon<M>(mm<M>(x, NINV));
      }
  constexpr uint32_t bytes = (uint32_t)((size_t)TRACE_STEPS * DT * BR2_ROW * sizeof(double2));
  const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc(const_cast<double2 *>(tkf), 0, bytes, 0x00020000);
  const uint32_t t16 = (uint32_t)t * 16u;
#pragma unroll 1
  for (int k = 0; k < TRACE_STEPS; ++k) {
    const uint16_t *src = tb.trace_src + k * NN;
    double2 ka[2][E], kb[2][E];
    br2f_load_half(ka, rsrc, k * DT, 0, t16);
    __syncthreads();  // the previous update (or the scaling) visible
    uint32_t pk[2][E][DigitsTrace::DW];  // sigma_g(a) at the thread's P0 points (coefficients j, j + 1024)
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int e = 0; e < E; ++e) {
        const int sidx = src[F::idx(0, t, e) + F::n * h];
        const double v = sidx < NN ? acs[F::slot_stage(sidx)] : -acs[F::slot_stage(sidx - NN)];
        DigitsTrace::pack(v, pk[h][e]);
        asm volatile("" : "+v"(pk[h][e][0]), "+v"(pk[h][e][1]));
      }
    double sr[2][2][E], si[2][2][E];  // [output A / B][limb]
#pragma unroll
    for (int o = 0; o < 2; ++o)
#pragma unroll
      for (int l = 0; l < 2; ++l)
#pragma unroll
        for (int e = 0; e < E; ++e) sr[o][l][e] = si[o][l][e] = 0.0;
#pragma unroll 1
    for (int d = 0; d < DT; ++d) {
      const int q = k * DT + d;
      double xr[E], xi[E];
#pragma unroll
      for (int e = 0; e < E; ++e) {
        xr[e] = DigitsTrace::get(pk[0][e], d);
        xi[e] = DigitsTrace::get(pk[1][e], d);
      }
      // output B's limb-0 blocks mid-transform, limb 1 after it (as br2f_digit)
      auto load_kb = [&](int l) {
#pragma unroll
        for (int e = 0; e < E; ++e) {
          const uint32_t soff = (uint32_t)q * (uint32_t)(BR2_ROW * sizeof(double2)) +
                                (uint32_t)(((1 * 2 + l) * Fft1024::n + e * Fft1024::T) * sizeof(double2));
          kb[l][e] = __builtin_bit_cast(double2, __builtin_amdgcn_raw_buffer_load_b128(rsrc, t16, (int)soff, 0));
        }
      };
      F::fwd(xr, xi, Xb[d & 1], t, wc, [&]() { load_kb(0); });
      load_kb(1);
#pragma unroll
      for (int o = 0; o < 2; ++o) {
#pragma unroll
        for (int l = 0; l < 2; ++l)
#pragma unroll
          for (int e = 0; e < E; ++e) {
            const double2 kv = o ? kb[l][e] : ka[l][e];
            sr[o][l][e] = __fma_rn(xr[e], kv.x, __fma_rn(-xi[e], kv.y, sr[o][l][e]));
            si[o][l][e] = __fma_rn(xr[e], kv.y, __fma_rn(xi[e], kv.x, si[o][l][e]));
          }
        if (o == 0) br2f_load_half(ka, rsrc, d + 1 < DT ? q + 1 : q, 0, t16);
      }
    }
    // the four inverses on X0, X1, X0, X1 (the digits' last use of X1 was two uses back)
#pragma unroll
    for (int o = 0; o < 2; ++o)
#pragma unroll
      for (int l = 0; l < 2; ++l) F::inv(sr[o][l], si[o][l], Xb[l], tws, t);
    double sb[2][E];  // sigma_g(b) at the thread's coefficients, read before any thread updates acs
    const uint16_t *srcb = src;
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int e = 0; e < E; ++e) {
        const int sidx = srcb[F::idx(0, t, e) + F::n * h];
        sb[h][e] = sidx < NN ? acs[NN + F::slot_stage(sidx)] : -acs[NN + F::slot_stage(sidx - NN)];
      }
    __syncthreads();  // every thread has read sigma_g(a) and sigma_g(b)
#pragma unroll
    for (int e = 0; e < E; ++e)
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int c = F::slot_stage(F::idx(0, t, e) + F::n * h);
        const double alo = h ? si[0][0][e] : sr[0][0][e], ahi = h ? si[0][1][e] : sr[0][1][e];
        const double blo = h ? si[1][0][e] : sr[1][0][e], bhi = h ? si[1][1][e] : sr[1][1][e];
        const double ral = rint(alo), rah = rint(ahi), rbl = rint(blo), rbh = rint(bhi);
        rg.note(alo, ral);
        rg.note(ahi, rah);
        rg.note(blo, rbl);
        rg.note(bhi, rbh);
        acs[c] = limb_acc(acs[c], ral, rah);
        acs[NN + c] = limb_acc(acs[NN + c] + sb[h][e], rbl, rbh);
      }
  }
}

// Level-2 blind rotation (BlindRotationKey::blind_rotate, detector.rs:623) on the exact FFT: one
// 256-thread workgroup per message; output the coefficient-domain rotation (mode 1) or, after
// hom_trace (detector.rs:626-639), the NttRlweCiphertext (mode 0).
// The accumulator lives in LDS (ACC_p at slot_stage positions): each step reads the rotated digits
// of ACC_p straight from it and the update writes it in place, so there is no staging exchange and
// its 32 VGPRs hold the thread's forward twiddles instead (round 5: the tangent forms of passes
// 1..4, the inverse reading the premultiplied (B, A, AB) from LDS). Per CMUX step: for
// each of the 12 digits in issue order (poly p, digit j + 3 w) a forward transform and the
// multiply-accumulate into the four (output, limb) spectra with the key row (output A's blocks
// loaded one digit ahead); then the four inverses, rounding, limb recombination mod q2 and the
// update. Cross-wave uses alternate X0, X1 over the 12 digits and the 4 inverses, and every
// wave-local exchange runs in the wave's own quarter of the current X (Fft1024::fwd / inv), so each
// use rewrites a buffer whose readers have passed a later barrier: 17 workgroup barriers per step
// (one at the step start: the previous update visible to the rotated reads).
// LDS: twiddles 16 KB, X0 / X1 32 KB, ACC 32 KB (80 KB: two workgroups per CU).
// LDS of br2f_body, carved from one pool: the twiddles,
// then X0, X1, ACC (mask, body); the trace's 3 N2 doubles afterwards: 80 KB.
constexpr size_t BR2_LDS_X = 0, BR2_LDS_TWS = 4 * (size_t)Fft1024::n * sizeof(double2),
                 BR2_LDS_BYTES = BR2_LDS_TWS + (size_t)Fft1024::n * sizeof(double2);

template <bool G>
__device__ __forceinline__ void br2f_body(const uint32_t *__restrict__ lwe_int, const double2 *__restrict__ bskf,
                                          const double2 *__restrict__ twg, DeviceTables tb, uint64_t *__restrict__ out,
                                          unsigned long long *margin, double2 *pool, size_t item) {
  using F = Fft1024;
  using M = Mod<2>;
  constexpr int E = F::E, NN = N2;
  static_assert(F::TW_LEN <= F::n, "the twiddle table's LDS doubles as the trace's NTT table");
  double2 *tws = pool + BR2_LDS_TWS / sizeof(double2);
  double2(&lds)[4][F::n] = *reinterpret_cast<double2(*)[4][F::n]>(pool + BR2_LDS_X / sizeof(double2));
  double2(&Xb)[2][F::n] = *reinterpret_cast<double2(*)[2][F::n]>(&lds[0][0]);
  double *acs = reinterpret_cast<double *>(&lds[2][0]);
  const int t = threadIdx.x;
  const uint32_t *lwe = lwe_int + item * (NI + 1);
  F::load_twiddles(tws, twg, t);
  {  // ACC = (0, X^{-b} * LUT2)
    const int b = (int)lwe[NI];
    const int rr = (2 * NN - (b % (2 * NN))) % (2 * NN);
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int e = 0; e < E; ++e) {
        const int c = F::idx(0, t, e) + F::n * h;
        acs[F::slot_stage(c)] = 0.0;
        acs[NN + F::slot_stage(c)] = canon_small<M>(rot_read<NN>(tb.lut2, c, rr));
      }
  }
  __syncthreads();
  double2 wc[4][2];  // this thread's forward twiddles of passes 1..4, for every transform of the rotation
  F::block_ct<1>(wc[0], twg, t);
  F::block_ct<2>(wc[1], twg, t);
  F::block_ct<3>(wc[2], twg, t);
  F::block_ct<4>(wc[3], twg, t);
  double2 ka[2][E], kb[2][E];
  const __amdgpu_buffer_rsrc_t rsrc = bsk2_rsrc(bskf);
  const uint32_t t16 = (uint32_t)t * 16u;
  RoundGuard<G> rg;
  int kq = -1;  // the row whose output-A blocks ka already holds (the previous step's last digit loads them)
#pragma unroll 1
  for (int i = 0; i < NI; ++i) {
    const int a = (int)__builtin_amdgcn_readfirstlane(lwe[i]) & (2 * NN - 1);
    if (a == 0) continue;  // (X^0 - 1) * ACC = 0
    const int q0 = i * 2 * D2;  // the step's first global row
    if (kq != q0) br2f_load_half(ka, rsrc, q0, 0, t16);
    kq = i + 1 < NI ? q0 + 2 * D2 : -1;
    wg_barrier_lds();  // ACC (init or the previous update) visible; the previous inverses' reads done
    double sr[2][2][E], si[2][2][E];  // [output][limb] spectra
#pragma unroll
    for (int p = 0; p < 2; ++p) {
      uint32_t pk[2][E][Digits2S::DW];  // [coefficient j / j + 1024][point] digit words
      br2f_digits(acs + p * NN, a, t, pk);
      // digits in issue order g = 2 j + w: digit j + 3 w sits in word w at field j, so the word is
      // chosen at compile time; its GGSW row is p D2 + j + 3 w. The next digit in issue order: after
      // (j, 0) comes (j, 1), after (j, 1) (j + 1, 0), after the mask's last digit the body's first,
      // after the body's last the next step's first row (in flight across the inverses; kq above;
      // the last step reloads its own row: harmless).
      auto nxt = [&](int j, int w) {
        return q0 + (w == 0 ? p * D2 + j + 3
                            : (j + 1 < D2 / 2 ? p * D2 + j + 1 : (p == 0 ? D2 : (kq >= 0 ? 2 * D2 : 2 * D2 - 1))));
      };
      if (p == 0) {  // (peeling the step's first digit instead measured 10 % slower: 22 spills)
#pragma unroll
        for (int o = 0; o < 2; ++o)
#pragma unroll
          for (int l = 0; l < 2; ++l)
#pragma unroll
            for (int e = 0; e < E; ++e) sr[o][l][e] = si[o][l][e] = 0.0;
      }
#pragma unroll 1
      for (int j = 0; j < D2 / 2; ++j) {
        br2f_digit<0>(pk, j, q0 + p * D2 + j, nxt(j, 0), sr, si, ka, kb, Xb[0], rsrc, t16, t, wc);
        br2f_digit<1>(pk, j, q0 + p * D2 + j + 3, nxt(j, 1), sr, si, ka, kb, Xb[1], rsrc, t16, t, wc);
      }
    }
    // inverses on X0, X1, X0, X1, rounding to the exact limb products, recombination mod q2
    // (pipelining them in barrier stages, the second half of one beside the first half of the next,
    // measured no faster: profiles/r05zd/bench_variants.log, var_kpi; nor reading the accumulator
    // entries ahead of each output's last inverse: profiles/r05zg/, var_upf)
#pragma unroll
    for (int o = 0; o < 2; ++o) {
#pragma unroll
      for (int l = 0; l < 2; ++l) F::inv(sr[o][l], si[o][l], Xb[l], tws, t);
      br2f_update<G>(acs + o * NN, sr[o], si[o], rg, t);
    }
  }
  rg.publish(margin);
  __syncthreads();  // the last updates everywhere
  uint64_t *o = out + item * 2 * NN;
#pragma unroll
  for (int p = 0; p < 2; ++p)
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int e = 0; e < E; ++e) {
        const int c = F::idx(0, t, e) + F::n * h;
        o[p * NN + c] = to_u64<M>(acs[p * NN + F::slot_stage(c)]);
      }
}

// The trace as its own launch on the FFT (trace_fft_kernel, round 5): in place on level 2's
// coefficient-domain output (canonical u64 [2][N2] per message) -> NttRlweCiphertext. br2f_body's
// LDS layout (X0, X1, ACC, twiddles: 80 KB, two workgroups per CU); br2f_trace, then both halves
// to the NTT domain. Its own launch, not fused into br2f_kernel: fused, the trace's live values
// pushed the rotation loop to 37-53 VGPR spills.
template <bool G>
__device__ __forceinline__ void trace_fft_body(uint64_t *__restrict__ io, const double2 *__restrict__ tkf,
                                               const double2 *__restrict__ twg, DeviceTables tb,
                                               unsigned long long *margin) {
  using F = Fft1024;
  using M = Mod<2>;
  constexpr int E = F::E, NN = N2;
  __shared__ double2 pool[BR2_LDS_BYTES / sizeof(double2)];
  double2 *tws = pool + BR2_LDS_TWS / sizeof(double2);
  double2(&lds)[4][F::n] = *reinterpret_cast<double2(*)[4][F::n]>(pool + BR2_LDS_X / sizeof(double2));
  double2(&Xb)[2][F::n] = *reinterpret_cast<double2(*)[2][F::n]>(&lds[0][0]);
  double *acs = reinterpret_cast<double *>(&lds[2][0]);
  const int t = threadIdx.x;
  uint64_t *o = io + (size_t)blockIdx.x * 2 * NN;
  F::load_twiddles(tws, twg, t);
#pragma unroll
  for (int p = 0; p < 2; ++p)
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int e = 0; e < E; ++e) {
        const int c = F::idx(0, t, e) + F::n * h;
        acs[p * NN + F::slot_stage(c)] = from_u64<M>(o[p * NN + c]);
      }
  RoundGuard<G> rg;
  br2f_trace<G>(acs, tkf, Xb, tws, twg, tb, rg, t);
  rg.publish(margin);
  __syncthreads();  // the last updates everywhere
  // to_ntt_rlwe: both halves to the NTT domain (the trace NTTs' coefficient layout t + 256 e)
  using NTT = WgNtt<M, BR2_T, BR2_E>;
  double ca[BR2_E], cb[BR2_E];
#pragma unroll
  for (int e = 0; e < BR2_E; ++e) {
    ca[e] = acs[F::slot_stage(t + e * BR2_T)];
    cb[e] = acs[NN + F::slot_stage(t + e * BR2_T)];
  }
  double *xch = reinterpret_cast<double *>(&lds[0][0]);  // 2 N2 doubles (below the accumulator)
  double *tw = reinterpret_cast<double *>(tws);           // N2 doubles
  static_assert(NTT::LDS_DOUBLES * sizeof(double) <= 2 * F::n * sizeof(double2), "NTT exchange below ACC");
#pragma unroll
  for (int e = 0; e < BR2_E; ++e) tw[t + e * BR2_T] = tb.tw2[t + e * BR2_T];
  __syncthreads();
  NTT::fwd(ca, xch, tw, t);
  NTT::fwd(cb, xch, tw, t);
#pragma unroll
  for (int e = 0; e < BR2_E; ++e) {
    const int j = t * BR2_E + e;
    o[j] = to_u64<M>(canon<M>(ca[e]));
    o[NN + j] = to_u64<M>(canon<M>(cb[e]));
  }
}
__global__ __launch_bounds__(256, 2) void trace_fft_kernel(uint64_t *__restrict__ io, const double2 *__restrict__ tkf,
                                                           const double2 *__restrict__ twg, DeviceTables tb) {
  trace_fft_body<false>(io, tkf, twg, tb, nullptr);
}
__global__ __launch_bounds__(256, 2) void trace_fft_guard_kernel(uint64_t *__restrict__ io,
                                                                 const double2 *__restrict__ tkf,
                                                                 const double2 *__restrict__ twg, DeviceTables tb,
                                                                 unsigned long long *margin) {
  trace_fft_body<true>(io, tkf, twg, tb, margin);
}

__global__ __launch_bounds__(256, 2) void br2f_kernel(const uint32_t *__restrict__ lwe_int,
                                                      const double2 *__restrict__ bskf,
                                                      const double2 *__restrict__ twg, DeviceTables tb,
                                                      uint64_t *__restrict__ out) {
  __shared__ double2 pool[BR2_LDS_BYTES / sizeof(double2)];
  br2f_body<false>(lwe_int, bskf, twg, tb, out, nullptr, pool, blockIdx.x);
}
__global__ __launch_bounds__(256, 2) void br2f_guard_kernel(const uint32_t *__restrict__ lwe_int,
                                                            const double2 *__restrict__ bskf,
                                                            const double2 *__restrict__ twg, DeviceTables tb,
                                                            uint64_t *__restrict__ out, unsigned long long *margin) {
  __shared__ double2 pool[BR2_LDS_BYTES / sizeof(double2)];
  br2f_body<true>(lwe_int, bskf, twg, tb, out, margin, pool, blockIdx.x);
}


// ---- level 2 over two CUs per message on the exact FFT (the latency path) --------------------
// br2x_kernel's division of labour (latency_kernels.hpp) on br2f's arithmetic. Workgroup 2m + r
// owns polynomial r (0 mask, 1 body) of message m and its accumulator ACC_r (LDS, slot_stage
// positions). Its group g (256 threads: one Fft1024 transform) takes word g of the Digits2S
// decomposition of (X^a - 1) ACC_r -- digits 3g + j, GGSW rows r D2 + 3g + j -- and for each digit
// runs the forward transform and multiply-accumulates the four (output, limb) spectra. Group g
// finalises limb g of output r: the groups swap their limb-(1 - g) partials of both outputs through
// LDS; group g keeps limb g of output r and sends limb g of output 1 - r to the partner workgroup
// through global memory under br2x's hand-off rules (sc1 stores, vmcnt(0), a barrier, one flag
// carrying the executed-step count, a bounded poll, sc1 loads; slot = step parity); it adds the
// partner's limb g of output r, runs the inverse, rounds, and the groups swap half of the rounded
// limbs so that each recombines (mod q2) and updates 1,024 of ACC_r's coefficients. Per CU and
// step: three forward transforms per group, one inverse, one hand-off -- br2x's schedule, with
// transforms of 120 / 140 FP64 operations per thread instead of the modular NTT's ~450.
// Key rows: output A's two limb blocks of the next digit are issued after output A's MAC, output
// B's after output B's (in flight across the next transform); the next step's first row is issued
// once the partner's payload has been consumed, so no wait of the hand-off covers it and it stays
// in flight across the inverse, the update and the next step's digit extraction.
// Exact when the a priori bound of this accumulation order (apriori_bound level 3) is below 0.5;
// otherwise, or on a guarded context, the host runs br2x_kernel's exact NTT instead.
// LDS: twiddles 16 KB, X0 / X1 of each group 64 KB, the limb swap 32 KB (+ the groups' X1), ACC_r
// 16 KB: 128 KB, one workgroup per CU.
// Key prefetchers (round 5): a lone message's workgroup streams 384 KB of FFT-form key per step
// from HBM / the Infinity Cache at the per-CU rate of a few outstanding loads (~31 GB/s: 8.3 ms of
// level 2, against 6.1 ms with the key loads skipped, profiles/r05o/); from its XCD's L2 a CU reads
// ~118 GB/s (tools/microbench_l2.hip). So the launch carries BR2Y_H helper workgroups per worker
// on the worker's XCD (workgroups b and b + 8 share one: MI355X_MICROARCH.md, §Workgroup dispatch;
// a placement that differs costs speed, never correctness -- helpers only read the key): helper k
// touches one dword per 64 B of its quarter of the worker's rows of each executed step, at most
// BR2Y_PF executed steps ahead of the worker's hand-off count (its flag), so the rows are L2-resident
// when the worker loads them.
// Same-XCD hand-off (round 5): the hand-off cost 1.2 of br2y's 6.6 ms (profiles/r05t: its payload
// stores, poll and loads removed in a timing-only build) -- an sc1 store writes the line through and
// drops it from L2, so the partner's loads go beyond L2. Both workers of a message are therefore
// placed in one grid column (so on one XCD when the dispatcher deals blocks round-robin), each reads
// its XCD id (HW_REG_XCC_ID) and they swap it through global memory with sc1 accesses once per
// launch. When the ids agree, the payload and the flag are written with plain stores, which stay in
// that XCD's L2 where the partner's sc1 loads (L1 bypassed) find them; otherwise the sc1 protocol
// above runs unchanged. Either way every payload load is an sc1 load, so the choice follows the
// actual placement and changes speed only.
// Grid: w8 = n rounded up to a multiple of 8 columns (message m in column m); row 0 = the mask
// workers, row 1 = the body workers, rows 2 + 2k + r = helper k of worker (m, r); the host launches
// the helper rows only when every workgroup fits on its own CU. flags[2n .. 4n): the XCD ids + 1.
constexpr int BR2Y_T = 2 * Fft1024::T;
constexpr int BR2Y_H = 4, BR2Y_PF = 2;

__device__ __forceinline__ void br2y_prefetch(const uint32_t *__restrict__ lwe_int, const double2 *__restrict__ bskf,
                                              const uint32_t *flags, int wid, int k) {
  constexpr int STEP_LINES = D2 * BR2_ROW * (int)sizeof(double2) / 64;  // 64 B lines of one step's rows
  constexpr int PER_THREAD = STEP_LINES / (BR2Y_H * BR2Y_T);
  static_assert(PER_THREAD * BR2Y_H * BR2Y_T == STEP_LINES, "helpers split a step's rows evenly");
  __shared__ int go;
  const int m = wid >> 1, r = wid & 1;
  const uint32_t *lwe = lwe_int + (size_t)m * (NI + 1);
  uint32_t acc = 0;
  int e = 0;  // executed steps prefetched
#pragma unroll 1
  for (int i = 0; i < NI; ++i) {
    const int a = (int)__builtin_amdgcn_readfirstlane(lwe[i]) & (2 * N2 - 1);
    if (a == 0) continue;
    if (threadIdx.x == 0) {  // the worker has published hand-off e - BR2Y_PF (bounded: a helper may give up)
      int ok = 1, n = 0;
      while ((int)__hip_atomic_load(flags + wid, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < e - BR2Y_PF) {
        if (++n == (1 << 16)) {
          ok = 0;
          break;
        }
        __builtin_amdgcn_s_sleep(2);
      }
      go = ok;
    }
    __syncthreads();
    if (!go) break;
    const char *rows = reinterpret_cast<const char *>(bskf + ((size_t)i * 2 * D2 + (size_t)r * D2) * BR2_ROW);
    uint32_t v[PER_THREAD];
#pragma unroll
    for (int u = 0; u < PER_THREAD; ++u)
      v[u] = *reinterpret_cast<const uint32_t *>(rows + (size_t)((u * BR2Y_H + k) * BR2Y_T + (int)threadIdx.x) * 64);
#pragma unroll
    for (int u = 0; u < PER_THREAD; ++u) acc ^= v[u];
    __syncthreads();  // thread 0's next poll after every load of this step returned
    ++e;
  }
  asm volatile("" ::"v"(acc));  // the loads stay live
}

__global__ __launch_bounds__(BR2Y_T, 1) void br2y_kernel(const uint32_t *__restrict__ lwe_int,
                                                         const double2 *__restrict__ bskf,
                                                         const double2 *__restrict__ twg, DeviceTables tb,
                                                         double *xg, uint32_t *flags, int *err,
                                                         uint64_t *__restrict__ out, int nmsg, int w8,
                                                         int allow_fast) {
  using F = Fft1024;
  using M = Mod<2>;
  constexpr int E = F::E, NN = N2, n = F::n, T = F::T;
  __shared__ double2 tws[n];
  __shared__ double2 xb[2][2][n];  // [group][X0, X1]
  __shared__ double2 px[2][n];     // [group]: its limb-(1 - g) partial of output 1 - r; the rounded halves
  __shared__ double acs[NN];       // ACC_r
  __shared__ int stop, same_xcd;
  const int m = (int)blockIdx.x % w8, row = (int)blockIdx.x / w8;  // uniform
  if (m >= nmsg) return;
  if (row >= 2) {
    br2y_prefetch(lwe_int, bskf, flags, 2 * m + ((row - 2) & 1), (row - 2) >> 1);
    return;
  }
  const int r = row, wid = 2 * m + r;
  const int g = __builtin_amdgcn_readfirstlane((int)threadIdx.x / T), t = (int)threadIdx.x % T;
  const int pslot = __builtin_amdgcn_readfirstlane(wid < 2 ? 8 + 8 * wid + (int)(threadIdx.x >> 6) : -1);
  (void)pslot;
  OMR_PHASE_CLOCK(pslot, 0);
  const uint32_t *lwe = lwe_int + (size_t)m * (NI + 1);
  if (g == 0) F::load_twiddles(tws, twg, t);
  {  // ACC_r = X^{-b} * LUT2 (body) or 0 (mask)
    const int b = (int)lwe[NI];
    const int rr = (2 * NN - (b % (2 * NN))) % (2 * NN);
    for (int c = (int)threadIdx.x; c < NN; c += BR2Y_T)
      acs[F::slot_stage(c)] = r == 1 ? canon_small<M>(rot_read<NN>(tb.lut2, c, rr)) : 0.0;
    if (threadIdx.x == 0) {
      stop = 0;
      // XCD ids through global memory (sc1 both ways); a partner that never answers leaves the
      // sc1 protocol in place (the step loop's bounded poll then reports it)
      uint32_t *xid = flags + 2 * nmsg;
      const uint32_t mine = (uint32_t)__builtin_amdgcn_s_getreg(6164) + 1u;  // hwreg(HW_REG_XCC_ID, 0, 4)
      __hip_atomic_store(xid + wid, mine, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      uint32_t theirs = 0;
      for (int k = 0; k < (1 << 20) && theirs == 0; ++k) {
        theirs = __hip_atomic_load(xid + (wid ^ 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (theirs == 0) __builtin_amdgcn_s_sleep(2);
      }
      same_xcd = allow_fast && theirs == mine;
    }
  }
  double2 wc[4][2];  // this thread's forward twiddles of passes 1..4
  F::block_ct<1>(wc[0], twg, t);
  F::block_ct<2>(wc[1], twg, t);
  F::block_ct<3>(wc[2], twg, t);
  F::block_ct<4>(wc[3], twg, t);
  __syncthreads();  // same_xcd (and the accumulator) visible
  const bool fast = __builtin_amdgcn_readfirstlane(same_xcd) != 0;
  const __amdgpu_buffer_rsrc_t rsrc = bsk2_rsrc(bskf);
  const uint32_t t16 = (uint32_t)t * 16u;
  uint32_t *my_flag = flags + 2 * m + r, *their_flag = flags + 2 * m + (1 - r);
  uint32_t hc = 0;  // hand-offs so far (executed steps)
  double2 ka[2][E], kb[2][E];
  int pre = -1;  // the step whose first row ka / kb hold
#pragma unroll 1
  for (int i = 0; i < NI; ++i) {
    const int a = (int)__builtin_amdgcn_readfirstlane(lwe[i]) & (2 * NN - 1);
    if (a == 0) continue;  // (X^0 - 1) * ACC = 0 (both workgroups of the message skip it)
    OMR_PHASE(pslot, (int)hc, 0);
    const int q0 = i * 2 * D2 + r * D2 + 3 * g;  // the group's first GGSW row of this step
#ifdef OMR_BR2Y_NOKEY
#define br2y_load(...) ((void)0)
    if (i == 0 || pre == -1) {
      br2f_load_half(ka, rsrc, q0, 0, t16);
      br2f_load_half(kb, rsrc, q0, 1, t16);
      pre = -2;
    }
#else
#define br2y_load(...) br2f_load_half(__VA_ARGS__)
    if (pre != i) {
      br2f_load_half(ka, rsrc, q0, 0, t16);
      br2f_load_half(kb, rsrc, q0, 1, t16);
    }
#endif
    wg_barrier_lds();  // ACC_r (init or the previous update) visible; the previous step's LDS reads done
    uint32_t pw[2][E];  // word g of the digits at the thread's P0 points (coefficients j, j + 1024)
    {
      uint32_t pk[2][E][Digits2S::DW];
      br2f_digits(acs, a, t, pk);
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int e = 0; e < E; ++e) pw[h][e] = g ? pk[h][e][1] : pk[h][e][0];
    }
    OMR_PHASE(pslot, (int)hc, 1);
    double sr[2][2][E], si[2][2][E];  // [output][limb] partial spectra of the group's three digits
#pragma unroll
    for (int o = 0; o < 2; ++o)
#pragma unroll
      for (int l = 0; l < 2; ++l)
#pragma unroll
        for (int e = 0; e < E; ++e) sr[o][l][e] = si[o][l][e] = 0.0;
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      const int wd = g == 1 && j == 2 ? Digits2S::TOP_WIDTH : 7;  // the top digit of word 1
      double xr[E], xi[E];
#pragma unroll
      for (int e = 0; e < E; ++e) {
        xr[e] = (double)(int)__builtin_amdgcn_sbfe(pw[0][e], 7 * j, wd);
        xi[e] = (double)(int)__builtin_amdgcn_sbfe(pw[1][e], 7 * j, wd);
      }
      F::fwd(xr, xi, xb[g][j & 1], t, wc);
#pragma unroll
      for (int o = 0; o < 2; ++o) {
#pragma unroll
        for (int l = 0; l < 2; ++l)
#pragma unroll
          for (int e = 0; e < E; ++e) {
            const double2 kv = o ? kb[l][e] : ka[l][e];
            sr[o][l][e] = __fma_rn(xr[e], kv.x, __fma_rn(-xi[e], kv.y, sr[o][l][e]));
            si[o][l][e] = __fma_rn(xr[e], kv.y, __fma_rn(xi[e], kv.x, si[o][l][e]));
          }
        if (j < 2) {
          if (o == 0)
            br2y_load(ka, rsrc, q0 + j + 1, 0, t16);
          else
            br2y_load(kb, rsrc, q0 + j + 1, 1, t16);
        }
      }
    }
    OMR_PHASE(pslot, (int)hc, 2);
    // the four partials by role (r and g are uniform: selects, no dynamic register indexing):
    // [0] output r limb g (kept), [1] output r limb 1 - g, [2] output 1 - r limb g (handed to the
    // partner), [3] output 1 - r limb 1 - g
    double pr4[4][E], pi4[4][E];
#pragma unroll
    for (int e = 0; e < E; ++e) {
      const double rlr = r ? sr[1][0][e] : sr[0][0][e], rhr = r ? sr[1][1][e] : sr[0][1][e];
      const double nlr = r ? sr[0][0][e] : sr[1][0][e], nhr = r ? sr[0][1][e] : sr[1][1][e];
      const double rli = r ? si[1][0][e] : si[0][0][e], rhi = r ? si[1][1][e] : si[0][1][e];
      const double nli = r ? si[0][0][e] : si[1][0][e], nhi = r ? si[0][1][e] : si[1][1][e];
      pr4[0][e] = g ? rhr : rlr;
      pi4[0][e] = g ? rhi : rli;
      pr4[1][e] = g ? rlr : rhr;
      pi4[1][e] = g ? rli : rhi;
      pr4[2][e] = g ? nhr : nlr;
      pi4[2][e] = g ? nhi : nli;
      pr4[3][e] = g ? nlr : nhr;
      pi4[3][e] = g ? nli : nhi;
    }
    // limb swap: group g posts its limb-(1 - g) partials (output r in its X1, free since the third
    // transform's barrier; output 1 - r in px[g]) and takes the other group's limb-g ones
    {
      double2 *pr_ = xb[g][1], *ph = px[g];
#pragma unroll
      for (int e = 0; e < E; ++e) {
        pr_[e * T + t] = make_double2(pr4[1][e], pi4[1][e]);
        ph[e * T + t] = make_double2(pr4[3][e], pi4[3][e]);
      }
    }
    wg_barrier_lds();
    OMR_PHASE(pslot, (int)hc, 3);
    double fr[E], fi[E];  // limb g of output r: this workgroup's six rows, then the partner's six
    {
      const double2 *qr = xb[1 - g][1], *qh = px[1 - g];
      const size_t slot = hc & 1;
      double *dst = xg + ((((size_t)m * 2 + r) * 2 + slot) * 2 + g) * 2 * n;
#pragma unroll
      for (int e = 0; e < E; ++e) {
        const double2 vr = qr[e * T + t], vh = qh[e * T + t];
        fr[e] = pr4[0][e] + vr.x;
        fi[e] = pi4[0][e] + vr.y;
#ifndef OMR_BR2Y_NOHANDOFF  // timing-only ablation: no payload crosses (wrong output)
        if (fast) {  // plain stores: the lines stay in this XCD's L2 for the partner's sc1 loads
          dst[e * T + t] = pr4[2][e] + vh.x;
          dst[n + e * T + t] = pi4[2][e] + vh.y;
        } else {
          st_sc1(dst + e * T + t, pr4[2][e] + vh.x);  // limb g of output 1 - r: the partner's
          st_sc1(dst + n + e * T + t, pi4[2][e] + vh.y);
        }
#else
        (void)dst;
        (void)vh;
        (void)their_flag;
#endif
      }
#ifndef OMR_BR2Y_NOHANDOFF
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#endif
    }
    __syncthreads();
    OMR_PHASE(pslot, (int)hc, 4);
    if (threadIdx.x == 0) {
      if (fast)
        __hip_atomic_store(my_flag, hc + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);  // plain store
      else
        __hip_atomic_store(my_flag, hc + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#ifndef OMR_BR2Y_NOHANDOFF
      int k = 0;
      while (__hip_atomic_load(their_flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < hc + 1) {
        if (++k == BR2X_SPIN) {
          stop = 1;
          atomicExch(err, 1);
          break;
        }
        __builtin_amdgcn_s_sleep(2);
      }
#endif
    }
    __syncthreads();
    OMR_PHASE(pslot, (int)hc, 5);
    if (stop) break;
    {  // the partner's limb g of output r
      const double *src = xg + ((((size_t)m * 2 + (1 - r)) * 2 + (hc & 1)) * 2 + g) * 2 * n;
#pragma unroll
      for (int e = 0; e < E; ++e) {
#ifndef OMR_BR2Y_NOHANDOFF
        fr[e] += ld_sc1(src + e * T + t);
        fi[e] += ld_sc1(src + n + e * T + t);
#else
        (void)src;
#endif
      }
    }
    asm volatile("" : "+v"(fr[0]), "+v"(fr[1]), "+v"(fr[2]), "+v"(fr[3]), "+v"(fi[0]), "+v"(fi[1]), "+v"(fi[2]),
                 "+v"(fi[3])::"memory");  // consumed before the prefetch below is issued
#ifndef OMR_BR2Y_NOKEY
    if (i + 1 < NI) {  // the next step's first row (kept when that step runs next)
      br2f_load_half(ka, rsrc, q0 + 2 * D2, 0, t16);
      br2f_load_half(kb, rsrc, q0 + 2 * D2, 1, t16);
      pre = i + 1;
    }
#endif
    F::inv(fr, fi, xb[g][1], tws, t);  // X1: every reader of the limb swap passed the hand-off barriers
    OMR_PHASE(pslot, (int)hc, 6);
    // round limb g; the groups swap halves: group g recombines the coefficients idx(0, t, e) + 1024 g
    double lv[2][E];  // [h][e]: limb g of coefficient idx(0, t, e) + 1024 h
#pragma unroll
    for (int e = 0; e < E; ++e) {
      lv[0][e] = rint(fr[e]);
      lv[1][e] = rint(fi[e]);
    }
    double *hx = reinterpret_cast<double *>(px[g]);
#pragma unroll
    for (int e = 0; e < E; ++e) hx[e * T + t] = g ? lv[0][e] : lv[1][e];
    wg_barrier_lds();
    const double *ho = reinterpret_cast<const double *>(px[1 - g]);
#pragma unroll
    for (int e = 0; e < E; ++e) {
      const double other = ho[e * T + t];
      const double lo = g == 0 ? lv[0][e] : other, hr = g == 0 ? other : lv[1][e];
      double &acc = acs[F::slot_stage(F::idx(0, t, e) + n * g)];
      acc = limb_acc(acc, lo, hr);
    }
    OMR_PHASE(pslot, (int)hc, 7);
    ++hc;
  }
  OMR_PHASE_CLOCK(pslot, 1);
  __syncthreads();  // the last updates everywhere
  uint64_t *o = out + (size_t)m * 2 * NN + (size_t)r * NN;
  for (int c = (int)threadIdx.x; c < NN; c += BR2Y_T) o[c] = to_u64<M>(acs[F::slot_stage(c)]);
}

}  // namespace omr
