// Level-2 blind rotation with a hand-pinned two-transform schedule (experiment, OMR_BR2_SCHED=1).
// Same arithmetic, LDS layout and barrier discipline as br2f_kernel (br2_fft.hpp: the accumulator
// in LDS, the wave-local exchange in the wave's own quarter of X, X0 / X1 alternating), so the
// output is bit-identical. Between two barriers ("slot s") a wave runs the second half of digit
// transform A = T_s (from its cross-wave exchange on) and the first half of B = T_{s+1} (up to its
// cross-wave put), and the order is fixed by __builtin_amdgcn_sched_barrier(0) between chunks, so
// that the machine scheduler (which at 256 VGPRs minimises pressure and would serialise the two
// independent streams: br2p_kernel, commit a8ceeaa) keeps the overlap:
//   c1  A: cross-wave get + pass-2/3 twiddle reads issued; output B's key blocks issued;
//       B: digit extraction, pass 0, relayout, pass-1 twiddle reads issued      (covers A's reads)
//   c2  A: pass 2, relayout, pass 3, wave-local put, pass-4 twiddle reads issued
//   c3  B: pass 1, cross-wave put to X_{s+1}                                      (covers A's put)
//   c4  A: wave-local get
//   c5  A: pass 4, multiply-accumulate (output A; next ka issued; output B), barrier
#pragma once

#include "br2_fft.hpp"

namespace omr {

#define OMR_SB() __builtin_amdgcn_sched_barrier(0)
#ifndef OMR_BR2S_KB_LATE
#define OMR_BR2S_KB_LATE 0
#endif

struct Br2S {
  using F = Fft1024;
  static constexpr int E = F::E;
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
  __device__ static __forceinline__ void fence() {
    __builtin_amdgcn_wave_barrier();
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
  }
  template <int W>
  __device__ static __forceinline__ void extract(const uint32_t (&pk)[2][E][Digits2S::DW], int j, double (&xr)[E],
                                                 double (&xi)[E]) {
#pragma unroll
    for (int e = 0; e < E; ++e) {
      xr[e] = Digits2S::digit<W>(pk[0][e], j);
      xi[e] = Digits2S::digit<W>(pk[1][e], j);
    }
  }
  __device__ static __forceinline__ void mac(const double (&xr)[E], const double (&xi)[E], const double2 (&k)[2][E],
                                             double (&sr)[2][E], double (&si)[2][E]) {
#pragma unroll
    for (int l = 0; l < 2; ++l)
#pragma unroll
      for (int e = 0; e < E; ++e) {
        const double2 kv = k[l][e];
        sr[l][e] = __fma_rn(xr[e], kv.x, __fma_rn(-xi[e], kv.y, sr[l][e]));
        si[l][e] = __fma_rn(xr[e], kv.y, __fma_rn(xi[e], kv.x, si[l][e]));
      }
  }
};

// global GGSW row of digit transform g (issue order): poly g / 6, digit j + 3 w, j = (g % 6) / 2, w = g % 2
__device__ __forceinline__ int br2s_row(int q0, int g) {
  const int p = g >= D2 ? 1 : 0, r = g - p * D2;
  return q0 + p * D2 + (r >> 1) + 3 * (r & 1);
}

template <int WA, bool HB>
__device__ __forceinline__ void br2s_slot(int s, int q0, const uint32_t (&pk)[2][Fft1024::E][Digits2S::DW],
                                          double (&ar)[Fft1024::E], double (&ai)[Fft1024::E],
                                          double (&br)[Fft1024::E], double (&bi)[Fft1024::E],
                                          double (&sr)[2][2][Fft1024::E], double (&si)[2][2][Fft1024::E],
                                          double2 (&ka)[2][Fft1024::E], double2 (&kb)[2][Fft1024::E], double2 *XA,
                                          double2 *XB, const double2 *tws, __amdgpu_buffer_rsrc_t rsrc,
                                          uint32_t t16, int t) {
  using F = Fft1024;
  using P = Br2S;
  constexpr int WB = 1 - WA;
  double2 tw2[3], tw3[3], tw1[3], tw4[3];
  // c1
  P::get<2, 0>(ar, ai, XA, t);
  F::block_twiddles<2>(tw2, tws, t);
  F::block_twiddles<3>(tw3, tws, t);
#if !OMR_BR2S_KB_LATE
  br2f_load_half(kb, rsrc, br2s_row(q0, s), 1, t16);
#endif
  if constexpr (HB) {
    const int g = s + 1, r = g >= D2 ? g - D2 : g;
    P::extract<WB>(pk, r >> 1, br, bi);
    F::fwd_pass<0>(br, bi, tws, t);
    F::perm(br, bi);
    F::block_twiddles<1>(tw1, tws, t);
  }
  OMR_SB();
  // c2
  F::fwd_pass_r(ar, ai, tw2);
  F::perm(ar, ai);
  F::fwd_pass_r(ar, ai, tw3);
  P::put<3, 2>(ar, ai, XA, t);  // wave-local exchange in wave w's own quarter of X_s
  F::block_twiddles<4>(tw4, tws, t);
  OMR_SB();
  // c3
  if constexpr (HB) {
    F::fwd_pass_r(br, bi, tw1);
    P::put<1, 0>(br, bi, XB, t);  // X_{s+1}: its last readers (T_{s-1}) passed the slot's opening barrier
  }
  OMR_SB();
  // c4
  __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): this wave's puts landed
  P::fence();
  P::get<4, 2>(ar, ai, XA, t);
  P::fence();
  OMR_SB();
  // c5
#if OMR_BR2S_KB_LATE
  br2f_load_half(kb, rsrc, br2s_row(q0, s), 1, t16);
#endif
  F::fwd_pass_r(ar, ai, tw4);
  P::mac(ar, ai, ka, sr[0], si[0]);
  br2f_load_half(ka, rsrc, br2s_row(q0, s + 1 < 2 * D2 ? s + 1 : s), 0, t16);
  P::mac(ar, ai, kb, sr[1], si[1]);
  if constexpr (HB) wg_barrier_lds();
}

// inverse with every pass's twiddles read from LDS (Fft1024::inv with its own wave-local exchange
// in the wave's own quarter of X; no register twiddles here: the two-transform slots use them)
__device__ __forceinline__ void br2s_inv(double (&xr)[Fft1024::E], double (&xi)[Fft1024::E], double2 *X,
                                         const double2 *tws, int t) {
  using F = Fft1024;
  F::inv_pass<4>(xr, xi, tws, t);
  F::exchange<4, 3, 3, false>(xr, xi, X, t);
  F::inv_pass<3>(xr, xi, tws, t);
  F::perm(xr, xi);
  F::inv_pass<2>(xr, xi, tws, t);
  F::exchange<2, 1, 1, true>(xr, xi, X, t);
  F::inv_pass<1>(xr, xi, tws, t);
  F::perm(xr, xi);
  F::inv_pass<0>(xr, xi, tws, t);
}

template <bool G>
__device__ __forceinline__ void br2s_body(const uint32_t *__restrict__ lwe_int, const double2 *__restrict__ bskf,
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
  RoundGuard<G> rg;
#pragma unroll 1
  for (int i = 0; i < NI; ++i) {
    const int a = (int)__builtin_amdgcn_readfirstlane(lwe[i]) & (2 * NN - 1);
    if (a == 0) continue;
    const int q0 = i * 2 * D2;
    br2f_load_half(ka, rsrc, q0, 0, t16);
    wg_barrier_lds();
    // the digit, inverse and update addresses from an opaque copy of t: recomputed per step instead
    // of hoisted out of the step loop as loop invariants (which spilled them, and every reload
    // waited vmcnt(0), draining the key loads)
    int tt = t;
    asm volatile("" : "+v"(tt));
    uint32_t pk[2][E][Digits2S::DW];
    br2f_digits(acs, a, tt, pk);
    double sr[2][2][E], si[2][2][E];
#pragma unroll
    for (int o = 0; o < 2; ++o)
#pragma unroll
      for (int l = 0; l < 2; ++l)
#pragma unroll
        for (int e = 0; e < E; ++e) sr[o][l][e] = si[o][l][e] = 0.0;
    double r0[E], i0[E], r1[E], i1[E];
    Br2S::extract<0>(pk, 0, r0, i0);  // T_0's first half
    F::fwd_pass<0>(r0, i0, tws, t);
    F::perm(r0, i0);
    F::fwd_pass<1>(r0, i0, tws, t);
    Br2S::put<1, 0>(r0, i0, Xb[0], t);
    wg_barrier_lds();
    // six slot pairs, one loop body: slot 11's "B" is a dummy first half (digit field 3 of the body's
    // words, put to X0 before slot 11's barrier; X0's next use, the first inverse, rewrites its own
    // quarter after that barrier): 1/24 of the step's first halves wasted for a single instantiation
#pragma unroll 1
    for (int s = 0; s < 2 * D2; s += 2) {
      br2s_slot<0, true>(s, q0, pk, r0, i0, r1, i1, sr, si, ka, kb, Xb[0], Xb[1], tws, rsrc, t16, t);
      if (s + 1 == D2 - 1) br2f_digits(acs + NN, a, tt, pk);  // T_6 (the body's first) starts in slot 5
      br2s_slot<1, true>(s + 1, q0, pk, r1, i1, r0, i0, sr, si, ka, kb, Xb[1], Xb[0], tws, rsrc, t16, t);
    }
#pragma unroll
    for (int o = 0; o < 2; ++o) {
#pragma unroll
      for (int l = 0; l < 2; ++l) br2s_inv(sr[o][l], si[o][l], Xb[l], tws, tt);
      br2f_update<G>(acs + o * NN, sr[o], si[o], rg, tt);
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

__global__ __launch_bounds__(256, 2) void br2s_kernel(const uint32_t *__restrict__ lwe_int,
                                                      const double2 *__restrict__ bskf,
                                                      const double2 *__restrict__ twg, const double *__restrict__ tk,
                                                      DeviceTables tb, uint64_t *__restrict__ out, int mode) {
  br2s_body<false>(lwe_int, bskf, twg, tk, tb, out, mode, nullptr);
}
__global__ __launch_bounds__(256, 2) void br2s_guard_kernel(const uint32_t *__restrict__ lwe_int,
                                                            const double2 *__restrict__ bskf,
                                                            const double2 *__restrict__ twg, const double *__restrict__ tk,
                                                            DeviceTables tb, uint64_t *__restrict__ out, int mode,
                                                            unsigned long long *margin) {
  br2s_body<true>(lwe_int, bskf, twg, tk, tb, out, mode, margin);
}

}  // namespace omr
