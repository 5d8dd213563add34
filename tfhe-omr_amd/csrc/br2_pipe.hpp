// Level-2 blind rotation on the exact FFT, software-pipelined (second_level_bootstrapping,
// detector.rs:599-624; round 5). Same arithmetic as br2f_kernel (br2_fft.hpp:
// the digits, the Fft1024 passes, the two 25-bit key limbs, the multiply-accumulate order and the
// rounding), so the outputs are bit-identical to it and to the oracle. What changes is the schedule:
//
//  - Two transforms in flight per wave. A transform is cut at its cross-wave exchange into a first
//    half (digit extraction, passes 0, 1) and a second half (passes 2, 3, the wave-local exchange,
//    pass 4, the multiply-accumulate). Between two workgroup barriers a wave runs the second half of
//    transform s and the first half of transform s + 1, which are independent: the LDS round trips
//    of one (its exchange reads, its twiddle reads) overlap the FP64 work of the other. One
//    cross-wave exchange (one barrier) per transform, as before, alternating X0 / X1.
//  - No wave-local buffer W: every exchange direction maps the points of wave w to slots whose
//    bits 9, 8 equal w (tests/test_fft2_layout.py::test_exchange_regions), so the wave-local
//    exchange of transform s runs in wave w's own quarter of X_s, which after the cross-wave reads
//    of transform s no other wave touches until transform s + 2 writes it, behind the barrier of
//    transform s + 1 (forward: cross-wave reads are own-quarter; inverse: cross-wave writes are).
//  - The accumulator lives in LDS (the 16 KB of W plus the 16 KB the rotation staging used): ACC_p
//    at Fft1024::slot_stage positions, read rotated for the digits and updated in place after the
//    inverses, so the step needs no staging exchange and 32 VGPRs are free for the second
//    transform and for output B's key blocks, now loaded at the start of the slot (in flight across
//    the whole slot instead of across output A's multiply-accumulate only).
//  - The four inverses are pipelined the same way (second half of inverse k with the first half of
//    inverse k + 1).
// LDS: twiddles 16 KB, X0 / X1 32 KB, ACC 32 KB = 80 KB (two workgroups per CU, as before).
// Barriers per step: one at the step start (the previous update visible to the rotated reads),
// one per transform (12 + 4): 17 (18 before).
#pragma once

#include "br2_fft.hpp"

namespace omr {

#ifndef OMR_BR2Q_TWR
#define OMR_BR2Q_TWR 0  // br2q: passes 3 and 4 on twiddles held in registers
#endif
#ifndef OMR_BR2Q_KB_AHEAD
#define OMR_BR2Q_KB_AHEAD 0
#endif
#ifndef OMR_BR2P_SERIAL
#define OMR_BR2P_SERIAL 0  // 1: no overlap of the two transforms (B's first half after A's MAC)
#endif
#ifndef OMR_BR2P_KB_EARLY
#define OMR_BR2P_KB_EARLY 0  // output B's key blocks at the slot start (37 VGPR spills) or mid-slot
#endif

struct Br2Pipe {
  using F = Fft1024;
  static constexpr int E = F::E, NN = N2;

  // exchange halves (Fft1024::exchange split at its synchronisation)
  template <int PF, int S>
  __device__ static __forceinline__ void put(const double (&xr)[E], const double (&xi)[E], double2 *buf, int t) {
    const int bw = F::swz(S, F::idx(PF, t, 0));
#pragma unroll
    for (int e = 0; e < E; ++e) buf[F::slot_of<S, PF>(bw, e)] = make_double2(xr[e], xi[e]);
  }
  template <int PT, int S>
  __device__ static __forceinline__ void get(double (&xr)[E], double (&xi)[E], const double2 *buf, int t) {
    const int br = F::swz(S, F::idx(PT, t, 0));
#pragma unroll
    for (int e = 0; e < E; ++e) {
      const double2 v = buf[F::slot_of<S, PT>(br, e)];
      xr[e] = v.x;
      xi[e] = v.y;
    }
  }
  __device__ static __forceinline__ void wave_sync() {  // this wave's LDS writes landed; compiler order
    __builtin_amdgcn_s_waitcnt(0xc07f);                 // lgkmcnt(0)
    __builtin_amdgcn_wave_barrier();
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
  }
  __device__ static __forceinline__ void fence() {
    __builtin_amdgcn_wave_barrier();
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
  }

  // digit words of (X^a - 1) * ACC_p from the resident accumulator (acp: 2048 doubles at slot_stage)
  __device__ static __forceinline__ void digits(const double *acp, int a, int t, uint32_t (&pk)[2][E][Digits2S::DW]) {
    using M = Mod<2>;
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int e = 0; e < E; ++e) {
        const int c = F::idx(0, t, e) + F::n * h;
        const uint32_t u = (uint32_t)(c - a) & (2 * NN - 1);
        const double v = acp[F::slot_stage(u & (NN - 1))];
        const uint32_t vh = (uint32_t)(__builtin_bit_cast(uint64_t, v) >> 32) ^ ((u & NN) << (31 - 11));
        const double rot = __builtin_bit_cast(double, (__builtin_bit_cast(uint64_t, v) & 0xffffffffull) |
                                                          ((uint64_t)vh << 32));
        Digits2S::pack(canon_small<M>(rot - acp[F::slot_stage(c)]), pk[h][e]);
        asm volatile("" : "+v"(pk[h][e][0]), "+v"(pk[h][e][1]));
      }
  }
  // first half of digit transform (j, W): extraction, passes 0, 1 (registers and twiddle reads)
  template <int W>
  __device__ static __forceinline__ void first_half(const uint32_t (&pk)[2][E][Digits2S::DW], int j, double (&xr)[E],
                                                    double (&xi)[E], const double2 *tws, int t) {
#pragma unroll
    for (int e = 0; e < E; ++e) {
      xr[e] = Digits2S::digit<W>(pk[0][e], j);
      xi[e] = Digits2S::digit<W>(pk[1][e], j);
    }
    F::fwd_pass<0>(xr, xi, tws, t);
    F::perm(xr, xi);
    F::fwd_pass<1>(xr, xi, tws, t);
  }
  // multiply-accumulate of a P4 spectrum into the four (output, limb) spectra
  template <bool FIRST>
  __device__ static __forceinline__ void mac(const double (&xr)[E], const double (&xi)[E], const double2 (&k)[2][E],
                                             double (&sr)[2][E], double (&si)[2][E]) {
#pragma unroll
    for (int l = 0; l < 2; ++l)
#pragma unroll
      for (int e = 0; e < E; ++e) {
        const double2 kv = k[l][e];
        if constexpr (FIRST) {
          sr[l][e] = __fma_rn(xr[e], kv.x, -xi[e] * kv.y);
          si[l][e] = __fma_rn(xr[e], kv.y, xi[e] * kv.x);
        } else {
          sr[l][e] = __fma_rn(xr[e], kv.x, __fma_rn(-xi[e], kv.y, sr[l][e]));
          si[l][e] = __fma_rn(xr[e], kv.y, __fma_rn(xi[e], kv.x, si[l][e]));
        }
      }
  }
};

// Global GGSW row of digit transform g (issue order) of a step: poly p = g / 6, digit j + 3 w with
// j = (g % 6) / 2, w = g % 2 (br2f_kernel's order: the MAC order the a priori bound assumes).
__device__ __forceinline__ int br2p_row(int q0, int g) {
  const int p = g >= D2 ? 1 : 0, r = g - p * D2;
  return q0 + p * D2 + (r >> 1) + 3 * (r & 1);
}

// One slot: second half of digit transform A = T_s (its cross-wave data in X_s), multiply-accumulate,
// and (HAS_B) the first half of B = T_{s+1}, whose P1 data then goes to X_{s+1}; ends at the barrier.
// WA / WB: the digit word of A / B (s % 2, (s + 1) % 2). FIRST: s = 0 (writes the spectra).
template <int WA, bool HAS_B, bool FIRST>
__device__ __forceinline__ void br2p_slot(int s, int q0, const uint32_t (&pk)[2][Fft1024::E][Digits2S::DW],
                                          double (&ar)[Fft1024::E], double (&ai)[Fft1024::E],
                                          double (&br)[Fft1024::E], double (&bi)[Fft1024::E],
                                          double (&sr)[2][2][Fft1024::E], double (&si)[2][2][Fft1024::E],
                                          double2 (&ka)[2][Fft1024::E], double2 (&kb)[2][Fft1024::E],
                                          double2 *XA, double2 *XB, const double2 *tws,
                                          __amdgpu_buffer_rsrc_t rsrc, uint32_t t16, int t) {
  using P = Br2Pipe;
  using F = Fft1024;
  constexpr int WB = 1 - WA;
  P::get<2, 0>(ar, ai, XA, t);  // A's cross-wave data (own quarter)
#if OMR_BR2P_KB_EARLY
  br2f_load_half(kb, rsrc, br2p_row(q0, s), 1, t16);  // A's output-B key blocks, in flight all slot
#endif
#if !OMR_BR2P_SERIAL
  if constexpr (HAS_B) {
    const int g = s + 1, r = g >= D2 ? g - D2 : g;
    P::first_half<WB>(pk, r >> 1, br, bi, tws, t);
  }
#endif
  F::fwd_pass<2>(ar, ai, tws, t);
  F::perm(ar, ai);
  F::fwd_pass<3>(ar, ai, tws, t);
#if !OMR_BR2P_KB_EARLY
  br2f_load_half(kb, rsrc, br2p_row(q0, s), 1, t16);  // A's output-B key blocks (in flight across the
#endif                                                 // exchange, pass 4 and output A's MAC)
  P::put<3, 2>(ar, ai, XA, t);  // wave-local exchange in wave w's own quarter of X_s
  P::wave_sync();
  P::get<4, 2>(ar, ai, XA, t);
  P::fence();
  F::fwd_pass<4>(ar, ai, tws, t);
  P::mac<FIRST>(ar, ai, ka, sr[0], si[0]);
  br2f_load_half(ka, rsrc, br2p_row(q0, s + 1 < 2 * D2 ? s + 1 : s), 0, t16);  // next transform's output A
  P::mac<FIRST>(ar, ai, kb, sr[1], si[1]);
  if constexpr (HAS_B) {
#if OMR_BR2P_SERIAL
    const int g = s + 1, r = g >= D2 ? g - D2 : g;
    P::first_half<WB>(pk, r >> 1, br, bi, tws, t);
#endif
    P::put<1, 0>(br, bi, XB, t);
    wg_barrier_lds();
  }
}

// Inverse halves: first = pass 4, the wave-local exchange (own quarter of X), pass 3, perm, pass 2,
// and the cross-wave put (own quarter); second = the cross-wave get, pass 1, perm, pass 0.
__device__ __forceinline__ void br2p_inv_first(double (&xr)[Fft1024::E], double (&xi)[Fft1024::E], double2 *X,
                                               const double2 *tws, int t) {
  using P = Br2Pipe;
  using F = Fft1024;
  F::inv_pass<4>(xr, xi, tws, t);
  P::put<4, 3>(xr, xi, X, t);
  P::wave_sync();
  P::get<3, 3>(xr, xi, X, t);
  P::fence();
  F::inv_pass<3>(xr, xi, tws, t);
  F::perm(xr, xi);
  F::inv_pass<2>(xr, xi, tws, t);
  P::put<2, 1>(xr, xi, X, t);
}
__device__ __forceinline__ void br2p_inv_second(double (&xr)[Fft1024::E], double (&xi)[Fft1024::E], const double2 *X,
                                                const double2 *tws, int t) {
  using P = Br2Pipe;
  using F = Fft1024;
  P::get<1, 1>(xr, xi, X, t);
  F::inv_pass<1>(xr, xi, tws, t);
  F::perm(xr, xi);
  F::inv_pass<0>(xr, xi, tws, t);
}
// rounding to the exact limb products, recombination mod q2 and ACC_o += (in place in LDS)
template <bool G>
__device__ __forceinline__ void br2p_update(double *aco, const double (&sr)[2][Fft1024::E],
                                            const double (&si)[2][Fft1024::E], RoundGuard<G> &rg, int t) {
  using F = Fft1024;
  using M = Mod<2>;
#pragma unroll
  for (int e = 0; e < F::E; ++e)
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const double ylo = h ? si[0][e] : sr[0][e], yhi = h ? si[1][e] : sr[1][e];
      const double lo = rint(ylo), hr = rint(yhi);
      rg.note(ylo, lo);
      rg.note(yhi, hr);
      const double hi = hr * LIMB;  // exact (|P_hi| < 2^45)
      double &a = aco[F::slot_stage(F::idx(0, t, e) + F::n * h)];
      a = canon<M>(a + red<M>(hi) + lo);
    }
}

template <bool G>
__device__ __forceinline__ void br2p_body(const uint32_t *__restrict__ lwe_int, const double2 *__restrict__ bskf,
                                          const double2 *__restrict__ twg, const double *__restrict__ tk,
                                          DeviceTables tb, uint64_t *__restrict__ out, int mode,
                                          unsigned long long *margin) {
  using F = Fft1024;
  using M = Mod<2>;
  constexpr int E = F::E, NN = N2;
  static_assert(F::TW_LEN <= F::n, "the twiddle table's LDS doubles as the trace's NTT table");
  __shared__ double2 tws[F::n];
  __shared__ double2 lds[4][F::n];  // X0, X1, then ACC (mask, body: 2 x 2048 doubles); the trace's 3 N2 doubles
  double2(&Xb)[2][F::n] = *reinterpret_cast<double2(*)[2][F::n]>(&lds[0][0]);
  double *acs = reinterpret_cast<double *>(&lds[2][0]);  // ACC_p at acs + p NN
  const int t = threadIdx.x;
  const uint32_t *lwe = lwe_int + (size_t)blockIdx.x * (NI + 1);
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
  double2 ka[2][E], kb[2][E];
  const __amdgpu_buffer_rsrc_t rsrc = bsk2_rsrc(bskf);
  const uint32_t t16 = (uint32_t)t * 16u;
  RoundGuard<G> rg;
#pragma unroll 1
  for (int i = 0; i < NI; ++i) {
    const int a = (int)__builtin_amdgcn_readfirstlane(lwe[i]) & (2 * NN - 1);
    if (a == 0) continue;  // (X^0 - 1) * ACC = 0
    const int q0 = i * 2 * D2;
    br2f_load_half(ka, rsrc, br2p_row(q0, 0), 0, t16);
    wg_barrier_lds();  // ACC (init or the previous step's update) visible; the previous inverses' reads done
    uint32_t pk[2][E][Digits2S::DW];
    Br2Pipe::digits(acs, a, t, pk);
    double sr[2][2][E], si[2][2][E];  // [output][limb] spectra
    double r0[E], i0[E], r1[E], i1[E];
    // prologue: T_0's first half
    Br2Pipe::first_half<0>(pk, 0, r0, i0, tws, t);
    Br2Pipe::put<1, 0>(r0, i0, Xb[0], t);
    wg_barrier_lds();
    // slots 0 .. 10 in pairs (A in r0 for even s, in r1 for odd s); the body's digits are taken when
    // T_6 (the body's first) starts, in slot 5, where the mask's words are no longer read
    br2p_slot<0, true, true>(0, q0, pk, r0, i0, r1, i1, sr, si, ka, kb, Xb[0], Xb[1], tws, rsrc, t16, t);
    br2p_slot<1, true, false>(1, q0, pk, r1, i1, r0, i0, sr, si, ka, kb, Xb[1], Xb[0], tws, rsrc, t16, t);
#pragma unroll 1
    for (int s = 2; s < 2 * D2 - 2; s += 2) {
      br2p_slot<0, true, false>(s, q0, pk, r0, i0, r1, i1, sr, si, ka, kb, Xb[0], Xb[1], tws, rsrc, t16, t);
      if (s + 1 == D2 - 1) Br2Pipe::digits(acs + NN, a, t, pk);
      br2p_slot<1, true, false>(s + 1, q0, pk, r1, i1, r0, i0, sr, si, ka, kb, Xb[1], Xb[0], tws, rsrc, t16, t);
    }
    br2p_slot<0, true, false>(2 * D2 - 2, q0, pk, r0, i0, r1, i1, sr, si, ka, kb, Xb[0], Xb[1], tws, rsrc, t16, t);
    br2p_slot<1, false, false>(2 * D2 - 1, q0, pk, r1, i1, r0, i0, sr, si, ka, kb, Xb[1], Xb[0], tws, rsrc, t16, t);
    // inverses I_k = (output k / 2, limb k % 2) on X_{k & 1}, pipelined in pairs of halves
    br2p_inv_first(sr[0][0], si[0][0], Xb[0], tws, t);
    wg_barrier_lds();
    br2p_inv_first(sr[0][1], si[0][1], Xb[1], tws, t);
    br2p_inv_second(sr[0][0], si[0][0], Xb[0], tws, t);
    wg_barrier_lds();
    br2p_inv_first(sr[1][0], si[1][0], Xb[0], tws, t);
    br2p_inv_second(sr[0][1], si[0][1], Xb[1], tws, t);
    br2p_update<G>(acs, sr[0], si[0], rg, t);
    wg_barrier_lds();
    br2p_inv_first(sr[1][1], si[1][1], Xb[1], tws, t);
    br2p_inv_second(sr[1][0], si[1][0], Xb[0], tws, t);
    wg_barrier_lds();
    br2p_inv_second(sr[1][1], si[1][1], Xb[1], tws, t);
    br2p_update<G>(acs + NN, sr[1], si[1], rg, t);
  }
  rg.publish(margin);
  __syncthreads();  // the last updates everywhere
  uint64_t *o = out + (size_t)blockIdx.x * 2 * NN;
  if (mode == 1) {
#pragma unroll
    for (int p = 0; p < 2; ++p)
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int e = 0; e < E; ++e) {
          const int c = F::idx(0, t, e) + F::n * h;
          o[p * NN + c] = to_u64<M>(acs[p * NN + F::slot_stage(c)]);
        }
    return;
  }
  // hom_trace on the accumulator in the trace NTTs' coefficient layout (t + 256 e, 8 per thread)
  double acc0[BR2_E], acc1[BR2_E];
#pragma unroll
  for (int e = 0; e < BR2_E; ++e) {
    acc0[e] = acs[F::slot_stage(t + e * BR2_T)];
    acc1[e] = acs[NN + F::slot_stage(t + e * BR2_T)];
  }
  double *xch = reinterpret_cast<double *>(&lds[0][0]);  // 3 N2 doubles
  double *tw = reinterpret_cast<double *>(tws);           // N2 doubles
  __syncthreads();
#pragma unroll
  for (int e = 0; e < BR2_E; ++e) {
    tw[t + e * BR2_T] = tb.tw2[t + e * BR2_T];
    xch[2 * NN + t + e * BR2_T] = tb.itw2[t + e * BR2_T];
  }
  __syncthreads();
  hom_trace_store(acc0, acc1, xch, tw, xch + 2 * NN, tk, tb, o, t);
}

// One digit of br2q with output B's key blocks also loaded one digit ahead (OMR_BR2Q_KB_AHEAD):
// the 32 VGPRs the LDS-resident accumulator frees hold them across the transform.
template <int W>
__device__ __forceinline__ void br2q_digit(const uint32_t (&pk)[2][Fft1024::E][Digits2S::DW], int j, int q, int nx,
                                           double (&sr)[2][2][Fft1024::E], double (&si)[2][2][Fft1024::E],
                                           double2 (&ka)[2][Fft1024::E], double2 (&kb)[2][Fft1024::E], double2 *X,
                                           const double2 *tws, __amdgpu_buffer_rsrc_t rsrc, uint32_t t16, int t,
                                           const double2 (&w3)[3], const double2 (&w4)[3]) {
  using F = Fft1024;
  constexpr int E = F::E;
  double xr[E], xi[E];
#pragma unroll
  for (int e = 0; e < E; ++e) {
    xr[e] = Digits2S::digit<W>(pk[0][e], j);
    xi[e] = Digits2S::digit<W>(pk[1][e], j);
  }
#if OMR_BR2Q_TWR
  F::fwd_r(xr, xi, X, X, tws, t, w3, w4);
#else
  F::fwd(xr, xi, X, X, tws, t);
#endif
#if OMR_BR2Q_KB_AHEAD
  Br2Pipe::mac<false>(xr, xi, ka, sr[0], si[0]);
  br2f_load_half(ka, rsrc, nx, 0, t16);
  Br2Pipe::mac<false>(xr, xi, kb, sr[1], si[1]);
  br2f_load_half(kb, rsrc, nx, 1, t16);
#else
  br2f_load_half(kb, rsrc, q, 1, t16);
  Br2Pipe::mac<false>(xr, xi, ka, sr[0], si[0]);
  br2f_load_half(ka, rsrc, nx, 0, t16);
  Br2Pipe::mac<false>(xr, xi, kb, sr[1], si[1]);
#endif
}

// br2q: br2f_kernel's schedule (one transform at a time) with two of br2p's changes only: the
// accumulator resident in LDS (no staging exchange, 32 VGPRs free) and the wave-local exchanges in
// the wave's own quarter of the cross-wave buffer (no W). The cross-wave uses then alternate
// X0, X1 over the 12 digits (issue order) and the four inverses without the staging uses between.
template <bool G>
__device__ __forceinline__ void br2q_body(const uint32_t *__restrict__ lwe_int, const double2 *__restrict__ bskf,
                                          const double2 *__restrict__ twg, const double *__restrict__ tk,
                                          DeviceTables tb, uint64_t *__restrict__ out, int mode,
                                          unsigned long long *margin) {
  using F = Fft1024;
  using M = Mod<2>;
  constexpr int E = F::E, NN = N2;
  __shared__ double2 tws[F::n];
  __shared__ double2 lds[4][F::n];  // X0, X1, ACC (mask, body); the trace's 3 N2 doubles afterwards
  double2(&Xb)[2][F::n] = *reinterpret_cast<double2(*)[2][F::n]>(&lds[0][0]);
  double *acs = reinterpret_cast<double *>(&lds[2][0]);
  const int t = threadIdx.x;
  const uint32_t *lwe = lwe_int + (size_t)blockIdx.x * (NI + 1);
  F::load_twiddles(tws, twg, t);
  {
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
  double2 ka[2][E], kb[2][E];
  const __amdgpu_buffer_rsrc_t rsrc = bsk2_rsrc(bskf);
  const uint32_t t16 = (uint32_t)t * 16u;
  double2 w3[3], w4[3];  // this thread's pass-3 / pass-4 block twiddles (OMR_BR2Q_TWR)
#if OMR_BR2Q_TWR
  __syncthreads();
  F::block_twiddles<3>(w3, tws, t);
  F::block_twiddles<4>(w4, tws, t);
#endif
  RoundGuard<G> rg;
#pragma unroll 1
  for (int i = 0; i < NI; ++i) {
    const int a = (int)__builtin_amdgcn_readfirstlane(lwe[i]) & (2 * NN - 1);
    if (a == 0) continue;
    const int q0 = i * 2 * D2;
    br2f_load_half(ka, rsrc, q0, 0, t16);
#if OMR_BR2Q_KB_AHEAD
    br2f_load_half(kb, rsrc, q0, 1, t16);
#endif
    wg_barrier_lds();  // ACC visible; the previous step's last inverse reads done
    double sr[2][2][E], si[2][2][E];
#pragma unroll
    for (int p = 0; p < 2; ++p) {
      uint32_t pk[2][E][Digits2S::DW];
      Br2Pipe::digits(acs + p * NN, a, t, pk);
      auto nxt = [&](int j, int w) {
        return q0 + (w == 0 ? p * D2 + j + 3 : (j + 1 < D2 / 2 ? p * D2 + j + 1 : (p == 0 ? D2 : 2 * D2 - 1)));
      };
      if (p == 0) {
#pragma unroll
        for (int o = 0; o < 2; ++o)
#pragma unroll
          for (int l = 0; l < 2; ++l)
#pragma unroll
            for (int e = 0; e < E; ++e) sr[o][l][e] = si[o][l][e] = 0.0;
      }
#pragma unroll 1
      for (int j = 0; j < D2 / 2; ++j) {
        br2q_digit<0>(pk, j, q0 + p * D2 + j, nxt(j, 0), sr, si, ka, kb, Xb[0], tws, rsrc, t16, t, w3, w4);
        br2q_digit<1>(pk, j, q0 + p * D2 + j + 3, nxt(j, 1), sr, si, ka, kb, Xb[1], tws, rsrc, t16, t, w3, w4);
      }
    }
#pragma unroll
    for (int o = 0; o < 2; ++o) {
#pragma unroll
      for (int l = 0; l < 2; ++l) {
#if OMR_BR2Q_TWR
        F::inv_r(sr[o][l], si[o][l], Xb[l], Xb[l], tws, t, w3, w4);
#else
        F::inv(sr[o][l], si[o][l], Xb[l], Xb[l], tws, t);
#endif
      }
      br2p_update<G>(acs + o * NN, sr[o], si[o], rg, t);
    }
  }
  rg.publish(margin);
  __syncthreads();
  uint64_t *o = out + (size_t)blockIdx.x * 2 * NN;
  if (mode == 1) {
#pragma unroll
    for (int p = 0; p < 2; ++p)
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int e = 0; e < E; ++e) {
          const int c = F::idx(0, t, e) + F::n * h;
          o[p * NN + c] = to_u64<M>(acs[p * NN + F::slot_stage(c)]);
        }
    return;
  }
  double acc0[BR2_E], acc1[BR2_E];
#pragma unroll
  for (int e = 0; e < BR2_E; ++e) {
    acc0[e] = acs[F::slot_stage(t + e * BR2_T)];
    acc1[e] = acs[NN + F::slot_stage(t + e * BR2_T)];
  }
  double *xch = reinterpret_cast<double *>(&lds[0][0]);
  double *tw = reinterpret_cast<double *>(tws);
  __syncthreads();
#pragma unroll
  for (int e = 0; e < BR2_E; ++e) {
    tw[t + e * BR2_T] = tb.tw2[t + e * BR2_T];
    xch[2 * NN + t + e * BR2_T] = tb.itw2[t + e * BR2_T];
  }
  __syncthreads();
  hom_trace_store(acc0, acc1, xch, tw, xch + 2 * NN, tk, tb, o, t);
}

__global__ __launch_bounds__(256, 2) void br2q_kernel(const uint32_t *__restrict__ lwe_int,
                                                      const double2 *__restrict__ bskf,
                                                      const double2 *__restrict__ twg, const double *__restrict__ tk,
                                                      DeviceTables tb, uint64_t *__restrict__ out, int mode) {
  br2q_body<false>(lwe_int, bskf, twg, tk, tb, out, mode, nullptr);
}
__global__ __launch_bounds__(256, 2) void br2q_guard_kernel(const uint32_t *__restrict__ lwe_int,
                                                            const double2 *__restrict__ bskf,
                                                            const double2 *__restrict__ twg, const double *__restrict__ tk,
                                                            DeviceTables tb, uint64_t *__restrict__ out, int mode,
                                                            unsigned long long *margin) {
  br2q_body<true>(lwe_int, bskf, twg, tk, tb, out, mode, margin);
}

__global__ __launch_bounds__(256, 2) void br2p_kernel(const uint32_t *__restrict__ lwe_int,
                                                      const double2 *__restrict__ bskf,
                                                      const double2 *__restrict__ twg, const double *__restrict__ tk,
                                                      DeviceTables tb, uint64_t *__restrict__ out, int mode) {
  br2p_body<false>(lwe_int, bskf, twg, tk, tb, out, mode, nullptr);
}
__global__ __launch_bounds__(256, 2) void br2p_guard_kernel(const uint32_t *__restrict__ lwe_int,
                                                            const double2 *__restrict__ bskf,
                                                            const double2 *__restrict__ twg, const double *__restrict__ tk,
                                                            DeviceTables tb, uint64_t *__restrict__ out, int mode,
                                                            unsigned long long *margin) {
  br2p_body<true>(lwe_int, bskf, twg, tk, tb, out, mode, margin);
}

}  // namespace omr
