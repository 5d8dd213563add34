// Workgroup complex FFTs for the external products (gfx950).
//
// Exactness: the external product only ever multiplies small gadget digits by key residues, so
// every coefficient of sum_r digit_r * key_r is an integer well inside FP64's 53 bits and an FP64
// FFT product rounds to it exactly:
//   level 1: |d| <= 17, |k| <= 2^26, 8 rows, N = 1024: |coef| < 2^43; worst error of a lane-exact
//            model with adversarial digits 1.8e-3 (tools/fft_exactness.py), rigorous bound < 0.15;
// Replacing the modular NTTs by half-length complex FFTs removes ~45 % of the level-1 FP64 work,
// with bit-identical results.
//
// Ring map: R[X]/(X^2n + 1) -> C[X]/(X^n - i), p -> z with z_j = p_j + i p_{j+n}, n = 2^L.
// X^n - i splits over the roots w^(1+4k) (w = exp(i pi / 2n)); the forward transform is a
// Cooley-Tukey tree on that factorisation (the twist is folded into the twiddles), the inverse a
// Gentleman-Sande tree with conjugate twiddles, unscaled (the 1/n is folded into the keys).
// Node i of stage s uses w^(eps(s, i) / 2), eps(0, 0) = n, eps(s+1, 2i) = eps(s, i) / 2,
// eps(s+1, 2i+1) = eps(s, i) / 2 + 2n (mod 4n). Passes are radix-8 blocks of that tree (WgFft::fwd_pass).
//
// One wave per transform, C independent transforms interleaved (layouts in WgFft below).
//   forward: in  x[e] = coefficient (lane + 64 e)   out x[e] = transform index jidx(3, lane, e)
//   inverse: the reverse (keys are transformed by the same forward, so the pointwise products line up)
#pragma once

#include <utility>

#include "device_ntt.hpp"

namespace omr {

// LDS visibility within one wave: this wave's LDS writes have landed, and the compiler moves no
// memory operation across (waves of a workgroup stay independent).
__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0)
  __builtin_amdgcn_wave_barrier();
  __atomic_signal_fence(__ATOMIC_SEQ_CST);
}
// Compiler-only ordering of one wave's LDS accesses (its LDS operations complete in order).
__device__ __forceinline__ void wave_lds_fence() {
  __builtin_amdgcn_wave_barrier();
  __atomic_signal_fence(__ATOMIC_SEQ_CST);
}
// forward radix-2 butterfly in tangent form: (p, q) <- (p + w q, p - w q), w = c (1 + i t);
// I: the node's twiddle is i w
template <bool I>
__device__ __forceinline__ void bfly(double &pr, double &pi, double &qr, double &qi, double c, double t) {
  const double ur = __fma_rn(-t, qi, qr), ui = __fma_rn(t, qr, qi);  // u = q (1 + i t), w q = c u
  const double ar = pr, ai = pi;
  if constexpr (!I) {
    pr = __fma_rn(c, ur, ar);
    pi = __fma_rn(c, ui, ai);
    qr = __fma_rn(-c, ur, ar);
    qi = __fma_rn(-c, ui, ai);
  } else {  // i c u = c (-ui + i ur)
    pr = __fma_rn(-c, ui, ar);
    pi = __fma_rn(c, ur, ai);
    qr = __fma_rn(c, ui, ar);
    qi = __fma_rn(-c, ur, ai);
  }
}
// its unscaled inverse (Gentleman-Sande): (p, q) <- (p + q, conj(w) (p - q)); conj(i w) = -i conj(w)
template <bool I>
__device__ __forceinline__ void ibfly(double &pr, double &pi, double &qr, double &qi, double c, double t) {
  const double dr = pr - qr, di = pi - qi;
  pr = pr + qr;
  pi = pi + qi;
  const double vr = __fma_rn(t, di, dr), vi = __fma_rn(-t, dr, di);  // v = d (1 - i t), conj(w) d = c v
  if constexpr (!I) {
    qr = c * vr;
    qi = c * vi;
  } else {  // -i c v = c (vi - i vr)
    qr = c * vi;
    qi = -c * vr;
  }
}

// Level-1 transform: 512 complex points, one wave (64 lanes x 8 registers), index bits j8..j0
// (stage s splits on bit 8 - s). Four passes of 3, 2, 3 and 1 stages; jidx(p, lane, e) is the
// index register e of `lane` holds in pass p:
//   P0: e -> j8 j7 j6, lane -> j5..j0                                  (coefficient layout lane + 64 e)
//   P1: e2 -> j5, e1 -> j4, e0 -> j6; lane 5, 4 -> j8, j7, lane 3..0 -> j3..j0
//       (P0 -> P1: register bits 2, 1 <-> lane bits 5, 4 by v_permlane32/16_swap, no LDS)
//   P2: e -> j3 j2 j1, lane 5 -> j0, lane 4..0 -> j8..j4                (the one LDS exchange)
//   P3: e2 -> j0, e1 -> j2, e0 -> j1; lane 5 -> j3, lane 4..0 -> j8..j4
//       (P2 -> P3: register bit 2 <-> lane bit 5, permlane)
// P0 and P2 are radix-8 blocks of the twiddle tree: the block's stage-s0 node (hi) has twiddle A,
// its children B, i B and grandchildren C, i C, w8 C, i w8 C (w8 = exp(i pi / 4)). P1 is two
// radix-4 blocks (register bit 0 = j6 selects the block; A, then B and i B on registers (e0,
// e0 + 2, e0 + 4, e0 + 6)). P3 is one radix-2 stage, odd siblings (register bit 0 = j1) taking i w.
// Forward passes: radix-2 butterflies in tangent form (round 5): a twiddle w = c (1 + i t) stored
// as (c, t = tan), (p, q) -> (p + c u, p - c u) with u = q (1 + i t): 6 FMAs per butterfly instead
// of a complex product and 4 additions (8), and a factor i only permutes the last 4 FMAs' operands,
// so a block needs the (c, t) of A, B, C, w8 C alone. A radix-8 pass is 72 FP64 operations instead
// of the premultiplied form's 80 ("x_e *= T_e, then a constant network", T = (1, C, B, BC, A, AC,
// AB, ABC)), a radix-4 block 24 instead of 28, the radix-2 pass 24 instead of 32: 216 per
// transform instead of 248 (DESIGN.md §3a bounds the error, 4u per stage). Inverse passes: the
// radix-8 ones keep the premultiplied adjoint (80 operations; a Gentleman-Sande butterfly subtracts
// before it multiplies, so the tangent form saves nothing there), P1 and P3 use the (c, t) tree
// (conj(w) d = c (d (1 - i t))), which shares their table with the forward.
// tools/fft_exactness.py (Fft8P, Fft8PT) models both structures against the exact negacyclic
// product. The exchange replaced by the permlane relayouts cost 14 % of the level-1 kernel
// (timing ablation).
// Twiddle table (double2; WgFft::TW_*): [0, 7) T_1..T_7 of P0 (wave-uniform, inverse); [7, 11) (c, t)
// of P0's A, B, C, w8 C; 11 + 2 blk + (A, B) (c, t) of P1's block blk = (j8 j7 j6); 27 + (t - 1) 32
// + hi, hi = j8..j4 = lane & 31, P2's T_t (inverse); 251 + 32 k + hi the (c, t) of P2's A, B, C,
// w8 C; 379 + 64 e1 + lane the (c, t) of P3's stage-8 twiddle of the even sibling.
// Twiddles br1f keeps in registers for its whole loop (round 6): pass 1's (c, t) of A and B of the
// lane's two blocks (p1: 16 VGPRs instead of 4 ds_read_b128 on the critical path of every transform)
// and pass 0's forward (c, t): c per lane (VGPRs, as before), t wave-uniform (SGPRs: the 8 VGPRs that
// make room for p1). Level 1 -1.6 to -2.2 % over six same-box runs (profiles/r06d, r06e).
struct Tw1Reg {
  double f0c[4], f0t[4];
  double2 p1[4];
};

template <int T_, int E_, int L_>
struct WgFft {
  static constexpr int T = T_, E = E_, L = L_, N = T * E;
  static_assert(T == 64 && E == 8 && L == 9, "written for the level-1 geometry: one wave, 64 x 8");
  static constexpr int BUF = N;  // LDS slots (double2) per transform
  // twiddle table offsets (double2 entries; fft_twiddles() in context.hip writes them)
  static constexpr int TW_P0I = 0, TW_P0F = 7, TW_P1 = 11, TW_P2I = 27, TW_P2F = 251, TW_P3 = 379, TW_LEN = 507;
  static_assert(TW_LEN <= N, "the table is copied to an N-entry LDS array");

  __device__ static __forceinline__ int jidx(int p, int lane, int e) {
    const int l5 = (lane >> 5) & 1, l4 = (lane >> 4) & 1;
    if (p == 0) return (e << 6) | lane;
    if (p == 1) return (l5 << 8) | (l4 << 7) | ((e & 1) << 6) | (((e >> 2) & 1) << 5) | (((e >> 1) & 1) << 4) | (lane & 15);
    if (p == 2) return ((lane & 31) << 4) | (e << 1) | l5;
    return ((lane & 31) << 4) | (l5 << 3) | (((e >> 1) & 1) << 2) | ((e & 1) << 1) | ((e >> 2) & 1);
  }
  // bank-conflict-free XOR swizzle of the P1 <-> P2 exchange: j4, j5, j6, j8 into slot bits 0..3
  // (ds_write_b128 8-lane groups and ds_read_b128 16-lane groups, both directions; tests/test_fft1_layout.py)
  __device__ static __forceinline__ int slot(int j) {
    return j ^ ((j >> 4) & 1) ^ (((j >> 5) & 1) << 1) ^ (((j >> 6) & 1) << 2) ^ (((j >> 8) & 1) << 3);
  }

  // P0 <-> P1 and P2 <-> P3 relayouts (involutions)
  template <int C>
  __device__ static __forceinline__ void swap01(double (&xr)[C][E], double (&xi)[C][E]) {
#pragma unroll
    for (int c = 0; c < C; ++c)
#pragma unroll
      for (int e = 0; e < E; ++e) {
        if (!(e & 4)) {
          swap_lane_bit<5>(xr[c][e], xr[c][e + 4]);
          swap_lane_bit<5>(xi[c][e], xi[c][e + 4]);
        }
      }
#pragma unroll
    for (int c = 0; c < C; ++c)
#pragma unroll
      for (int e = 0; e < E; ++e) {
        if (!(e & 2)) {
          swap_lane_bit<4>(xr[c][e], xr[c][e + 2]);
          swap_lane_bit<4>(xi[c][e], xi[c][e + 2]);
        }
      }
  }
  template <int C>
  __device__ static __forceinline__ void swap23(double (&xr)[C][E], double (&xi)[C][E]) {
#pragma unroll
    for (int c = 0; c < C; ++c)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        swap_lane_bit<5>(xr[c][e], xr[c][e + 4]);
        swap_lane_bit<5>(xi[c][e], xi[c][e + 4]);
      }
  }

  // P1 <-> P2 through the wave's LDS buffer (C transforms)
  template <int C, int PF, int PT>
  __device__ static __forceinline__ void exchange(double (&xr)[C][E], double (&xi)[C][E],
                                                  double2 *lds, int lane) {
#pragma unroll
    for (int c = 0; c < C; ++c)
#pragma unroll
      for (int e = 0; e < E; ++e)
        lds[c * BUF + slot(jidx(PF, lane, e))] = make_double2(xr[c][e], xi[c][e]);
    wave_lds_sync();
#pragma unroll
    for (int c = 0; c < C; ++c)
#pragma unroll
      for (int e = 0; e < E; ++e) {
        const double2 v = lds[c * BUF + slot(jidx(PT, lane, e))];
        xr[c][e] = v.x;
        xi[c][e] = v.y;
      }
    // the next exchange's writes must not move above these reads: a compiler fence suffices
    // (one wave's LDS operations complete in order; waiting for the reads here is 1.1 % slower)
    wave_lds_fence();
  }

  static constexpr double S8 = 0.70710678118654752440;  // 1 / sqrt(2), w8 = S8 (1 + i)

  // radix-8 block twiddle T_t (t = 1..7) of pass P in {0, 2} (inverse); pass 0 from the global
  // table with wave-uniform (scalar) loads when G
  template <int P, bool G>
  __device__ static __forceinline__ double2 tw8(const double2 *tws, const double2 *__restrict__ gtw, int t,
                                                int lane) {
    if constexpr (P == 0) return G ? gtw[TW_P0I + t - 1] : tws[TW_P0I + t - 1];
    return tws[TW_P2I + (t - 1) * 32 + (lane & 31)];
  }
  // (c, t) of the radix-8 block's A, B, C, w8 C (k = 0..3), pass P in {0, 2} (forward)
  template <int P, bool G>
  __device__ static __forceinline__ double2 ct8(const double2 *tws, const double2 *__restrict__ gtw, int k,
                                                int lane) {
    if constexpr (P == 0) return G ? gtw[TW_P0F + k] : tws[TW_P0F + k];
    return tws[TW_P2F + k * 32 + (lane & 31)];
  }

  template <int P, int C, bool G = false, bool R = false>
  __device__ static __forceinline__ void fwd8(double (&xr)[C][E], double (&xi)[C][E], const double2 *tws,
                                              int lane, const double2 *__restrict__ gtw = nullptr,
                                              const Tw1Reg &tr = Tw1Reg{}) {
    double2 ct[4];  // (c, t) of A, B, C, w8 C, all requested before the first use (one LDS round trip)
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      if constexpr (P == 0 && R)
        ct[k] = make_double2(tr.f0c[k], tr.f0t[k]);
      else
        ct[k] = ct8<P, G>(tws, gtw, k, lane);
    }
    if constexpr (P != 0) __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int c = 0; c < C; ++c) {
      double *r = xr[c], *i = xi[c];
#pragma unroll
      for (int e = 0; e < 4; ++e) bfly<false>(r[e], i[e], r[e + 4], i[e + 4], ct[0].x, ct[0].y);  // A
      bfly<false>(r[0], i[0], r[2], i[2], ct[1].x, ct[1].y);  // B
      bfly<false>(r[1], i[1], r[3], i[3], ct[1].x, ct[1].y);
      bfly<true>(r[4], i[4], r[6], i[6], ct[1].x, ct[1].y);  // i B
      bfly<true>(r[5], i[5], r[7], i[7], ct[1].x, ct[1].y);
      bfly<false>(r[0], i[0], r[1], i[1], ct[2].x, ct[2].y);  // C
      bfly<true>(r[2], i[2], r[3], i[3], ct[2].x, ct[2].y);   // i C
      bfly<false>(r[4], i[4], r[5], i[5], ct[3].x, ct[3].y);  // w8 C
      bfly<true>(r[6], i[6], r[7], i[7], ct[3].x, ct[3].y);   // i w8 C
    }
  }
  // unscaled inverse of fwd8 (8 x its inverse): the adjoint network, then x_e *= conj(T_e)
  template <int P, int C, bool G = false>
  __device__ static __forceinline__ void inv8(double (&xr)[C][E], double (&xi)[C][E], const double2 *tws,
                                              int lane, const double2 *__restrict__ gtw = nullptr) {
#pragma unroll
    for (int c = 0; c < C; ++c) {
      const double *o_r = xr[c], *o_i = xi[c];
      const double c0r = o_r[0] + o_r[1], c0i = o_i[0] + o_i[1], c1r = o_r[0] - o_r[1], c1i = o_i[0] - o_i[1];
      const double c2r = o_r[2] + o_r[3], c2i = o_i[2] + o_i[3];
      const double c3r = o_i[2] - o_i[3], c3i = o_r[3] - o_r[2];  // -i (o2 - o3)
      const double d0r = o_r[4] + o_r[5], d0i = o_i[4] + o_i[5];
      const double ur = o_r[4] - o_r[5], ui = o_i[4] - o_i[5];
      const double d1r = ur + ui, d1i = ui - ur;  // (1 - i) (o4 - o5) = sqrt 2 conj(w8) (o4 - o5)
      const double d2r = o_r[6] + o_r[7], d2i = o_i[6] + o_i[7];
      const double vr = o_r[6] - o_r[7], vi = o_i[6] - o_i[7];
      const double d3r = vi - vr, d3i = -vr - vi;  // (-1 - i) (o6 - o7) = sqrt 2 conj(i w8) (o6 - o7)
      const double a0r = c0r + c2r, a0i = c0i + c2i, a2r = c0r - c2r, a2i = c0i - c2i;
      const double a1r = c1r + c3r, a1i = c1i + c3i, a3r = c1r - c3r, a3i = c1i - c3i;
      const double b0r = d0r + d2r, b0i = d0i + d2i;
      const double b2r = d0i - d2i, b2i = d2r - d0r;  // -i (d0 - d2)
      const double b1r = d1r + d3r, b1i = d1i + d3i;
      const double b3r = d1i - d3i, b3i = d3r - d1r;  // -i (d1 - d3)
      xr[c][0] = a0r + b0r;
      xi[c][0] = a0i + b0i;
      xr[c][4] = a0r - b0r;
      xi[c][4] = a0i - b0i;
      xr[c][2] = a2r + b2r;
      xi[c][2] = a2i + b2i;
      xr[c][6] = a2r - b2r;
      xi[c][6] = a2i - b2i;
      xr[c][1] = __fma_rn(S8, b1r, a1r);
      xi[c][1] = __fma_rn(S8, b1i, a1i);
      xr[c][5] = __fma_rn(-S8, b1r, a1r);
      xi[c][5] = __fma_rn(-S8, b1i, a1i);
      xr[c][3] = __fma_rn(S8, b3r, a3r);
      xi[c][3] = __fma_rn(S8, b3i, a3i);
      xr[c][7] = __fma_rn(-S8, b3r, a3r);
      xi[c][7] = __fma_rn(-S8, b3i, a3i);
    }
    double2 wt[8];
#pragma unroll
    for (int t = 1; t < 8; ++t) wt[t] = tw8<P, G>(tws, gtw, t, lane);
    if constexpr (P != 0) __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int t = 1; t < 8; ++t) {  // x_t *= conj(T_t)
      const double2 w = wt[t];
#pragma unroll
      for (int c = 0; c < C; ++c) {
        const double r = __fma_rn(xr[c][t], w.x, xi[c][t] * w.y);
        const double i = __fma_rn(xi[c][t], w.x, -xr[c][t] * w.y);
        xr[c][t] = r;
        xi[c][t] = i;
      }
    }
  }

  // P1: two radix-4 blocks, (c, t) of A and B per block
  __device__ static __forceinline__ int tw4_index(int lane, int e0, int k) {  // k: 0 A, 1 B
    return TW_P1 + 2 * ((((lane >> 4) & 3) << 1) | e0) + k;
  }
  template <int C, bool R = false>
  __device__ static __forceinline__ void fwd4(double (&xr)[C][E], double (&xi)[C][E], const double2 *tws, int lane,
                                              const Tw1Reg &tr = Tw1Reg{}) {
#pragma unroll
    for (int e0 = 0; e0 < 2; ++e0) {
      const double2 A = R ? tr.p1[2 * e0] : tws[tw4_index(lane, e0, 0)];
      const double2 B = R ? tr.p1[2 * e0 + 1] : tws[tw4_index(lane, e0, 1)];
      const int r0 = e0, r1 = e0 | 2, r2 = e0 | 4, r3 = e0 | 6;
#pragma unroll
      for (int c = 0; c < C; ++c) {
        double *r = xr[c], *i = xi[c];
        bfly<false>(r[r0], i[r0], r[r2], i[r2], A.x, A.y);
        bfly<false>(r[r1], i[r1], r[r3], i[r3], A.x, A.y);
        bfly<false>(r[r0], i[r0], r[r1], i[r1], B.x, B.y);
        bfly<true>(r[r2], i[r2], r[r3], i[r3], B.x, B.y);
      }
    }
  }
  template <int C, bool R = false>
  __device__ static __forceinline__ void inv4(double (&xr)[C][E], double (&xi)[C][E], const double2 *tws, int lane,
                                              const Tw1Reg &tr = Tw1Reg{}) {
#pragma unroll
    for (int e0 = 0; e0 < 2; ++e0) {
      const double2 A = R ? tr.p1[2 * e0] : tws[tw4_index(lane, e0, 0)];
      const double2 B = R ? tr.p1[2 * e0 + 1] : tws[tw4_index(lane, e0, 1)];
      const int r0 = e0, r1 = e0 | 2, r2 = e0 | 4, r3 = e0 | 6;
#pragma unroll
      for (int c = 0; c < C; ++c) {
        double *r = xr[c], *i = xi[c];
        ibfly<false>(r[r0], i[r0], r[r1], i[r1], B.x, B.y);
        ibfly<true>(r[r2], i[r2], r[r3], i[r3], B.x, B.y);
        ibfly<false>(r[r0], i[r0], r[r2], i[r2], A.x, A.y);
        ibfly<false>(r[r1], i[r1], r[r3], i[r3], A.x, A.y);
      }
    }
  }

  // P3: stage 8, pairs (e, e + 4); register bit 1 selects the even sibling's (c, t), bit 0 the factor i
  template <int C>
  __device__ static __forceinline__ void fwd2(double (&xr)[C][E], double (&xi)[C][E], const double2 *tws, int lane,
                                              const double2 *w3 = nullptr) {
    const double2 W[2] = {w3 ? w3[0] : tws[TW_P3 + lane], w3 ? w3[1] : tws[TW_P3 + 64 + lane]};
#pragma unroll
    for (int c = 0; c < C; ++c)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const double2 w = W[(e >> 1) & 1];
        if (e & 1)
          bfly<true>(xr[c][e], xi[c][e], xr[c][e + 4], xi[c][e + 4], w.x, w.y);
        else
          bfly<false>(xr[c][e], xi[c][e], xr[c][e + 4], xi[c][e + 4], w.x, w.y);
      }
  }
  template <int C>
  __device__ static __forceinline__ void inv2(double (&xr)[C][E], double (&xi)[C][E], const double2 *tws, int lane,
                                              const double2 *w3 = nullptr) {
    const double2 W[2] = {w3 ? w3[0] : tws[TW_P3 + lane], w3 ? w3[1] : tws[TW_P3 + 64 + lane]};
#pragma unroll
    for (int c = 0; c < C; ++c)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const double2 w = W[(e >> 1) & 1];
        if (e & 1)
          ibfly<true>(xr[c][e], xi[c][e], xr[c][e + 4], xi[c][e + 4], w.x, w.y);
        else
          ibfly<false>(xr[c][e], xi[c][e], xr[c][e + 4], xi[c][e + 4], w.x, w.y);
      }
  }

  // C transforms at once (lds holds C * BUF complex)
  // G: pass-0 twiddles from the global table gtw (must be non-null); w3: pass 3's two twiddles of
  // this lane held in registers by the caller (else read from tws)
  template <int C, bool G = false, bool R = false>
  __device__ static __forceinline__ void fwd(double (&xr)[C][E], double (&xi)[C][E], double2 *lds,
                                             const double2 *tws, int lane,
                                             const double2 *__restrict__ gtw = nullptr,
                                             const double2 *w3 = nullptr, const Tw1Reg &tr = Tw1Reg{}) {
    fwd8<0, C, G, R>(xr, xi, tws, lane, gtw, tr);
    swap01<C>(xr, xi);
    fwd4<C, R>(xr, xi, tws, lane, tr);
    exchange<C, 1, 2>(xr, xi, lds, lane);
    fwd8<2, C>(xr, xi, tws, lane);
    swap23<C>(xr, xi);
    fwd2<C>(xr, xi, tws, lane, w3);
  }
  template <int C, bool G = false>
  __device__ static __forceinline__ void inv(double (&xr)[C][E], double (&xi)[C][E], double2 *lds,
                                             const double2 *tws, int lane,
                                             const double2 *__restrict__ gtw = nullptr) {
    inv2<C>(xr, xi, tws, lane);
    swap23<C>(xr, xi);
    inv8<2, C>(xr, xi, tws, lane);
    exchange<C, 2, 1>(xr, xi, lds, lane);
    inv4<C>(xr, xi, tws, lane);
    swap01<C>(xr, xi);
    inv8<0, C, G>(xr, xi, tws, lane, gtw);
  }
  // Two inverses interleaved through ONE transform's exchange buffer: the register passes run on
  // both (C = 2), the LDS exchange of the second follows the first's in the same slots (one
  // wave's LDS operations complete in order; the fence keeps the compiler from hoisting the
  // second's writes above the first's reads).
  template <bool G = false, bool R = false>
  __device__ static __forceinline__ void inv_pair(double (&xr)[2][E], double (&xi)[2][E], double2 *lds,
                                                  const double2 *tws, int lane,
                                                  const double2 *__restrict__ gtw = nullptr,
                                                  const double2 *w3 = nullptr, const Tw1Reg &tr = Tw1Reg{}) {
    inv2<2>(xr, xi, tws, lane, w3);
    swap23<2>(xr, xi);
    inv8<2, 2>(xr, xi, tws, lane);
#pragma unroll
    for (int c = 0; c < 2; ++c)
      exchange<1, 2, 1>(reinterpret_cast<double(&)[1][E]>(xr[c]), reinterpret_cast<double(&)[1][E]>(xi[c]), lds,
                        lane);
    inv4<2, R>(xr, xi, tws, lane, tr);
    swap01<2>(xr, xi);
    inv8<0, 2, G>(xr, xi, tws, lane, gtw);
  }
  __device__ static __forceinline__ void fwd(double (&xr)[E], double (&xi)[E], double2 *lds,
                                             const double2 *tws, int lane,
                                             const double2 *__restrict__ gtw = nullptr) {
    fwd<1>(reinterpret_cast<double(&)[1][E]>(xr), reinterpret_cast<double(&)[1][E]>(xi), lds, tws, lane);
  }
  __device__ static __forceinline__ void inv(double (&xr)[E], double (&xi)[E], double2 *lds,
                                             const double2 *tws, int lane,
                                             const double2 *__restrict__ gtw = nullptr) {
    inv<1>(reinterpret_cast<double(&)[1][E]>(xr), reinterpret_cast<double(&)[1][E]>(xi), lds, tws, lane);
  }
};

using Fft512 = WgFft<64, 8, 9>;  // level 1: N1 = 1024, one wave

}  // namespace omr
