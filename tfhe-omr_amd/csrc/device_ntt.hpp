// Device-side modular arithmetic and the workgroup negacyclic NTT for gfx950.
//
// Residues are held as exact integers in FP64 registers, centred around 0. A product is
// reduced with the error-free FP64 transform h = a*w, l = fma(a, w, -h) (a*w == h + l exactly)
// and a rounded quotient: r = fma(-rint(h/q), q, h) + l. On MI355X this runs 3.2x faster than a
// 64-bit integer Shoup multiply (profiles/r01_microbench_arith.txt) and needs no carry chains.
// Every operation below is exact as long as |values| < 2^53; the reduction points in the NTT
// keep the bounds (see DESIGN.md "FP64 residue arithmetic").
#pragma once

#include "common.hpp"

namespace omr {

// Exchange register bit r of a pair (a = x[e], b = x[e | 1 << r]) with lane bit LB (5: lanes
// 32..63 of a <-> lanes 0..31 of b, v_permlane32_swap; 4: odd 16-lane rows of a <-> even rows of
// b, v_permlane16_swap): afterwards a holds the lane-bit-0 half and lane bit LB indexes the old
// register bit. One instruction per dword pair.
// Workgroup barrier for LDS traffic only: this wave's LDS reads / writes are done, then s_barrier.
// Unlike __syncthreads() (a workgroup-scope fence: s_waitcnt vmcnt(0) lgkmcnt(0)) it leaves the
// wave's global loads in flight across the barrier (cdna_hip_programming.md, "Pipelining across
// barriers"); callers that hand global data between waves must not use it.
__device__ __forceinline__ void wg_barrier_lds() {
  __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0)
  __builtin_amdgcn_s_barrier();
  __atomic_signal_fence(__ATOMIC_SEQ_CST);
}

template <int LB>
__device__ __forceinline__ void swap_lane_bit(double &a, double &b) {
  static_assert(LB == 4 || LB == 5, "lane bits 4 and 5 have swap instructions");
  const uint64_t ua = __builtin_bit_cast(uint64_t, a), ub = __builtin_bit_cast(uint64_t, b);
  const uint32_t alo = (uint32_t)ua, ahi = (uint32_t)(ua >> 32), blo = (uint32_t)ub, bhi = (uint32_t)(ub >> 32);
  const auto lo = LB == 5 ? __builtin_amdgcn_permlane32_swap(alo, blo, false, false)
                          : __builtin_amdgcn_permlane16_swap(alo, blo, false, false);
  const auto hi = LB == 5 ? __builtin_amdgcn_permlane32_swap(ahi, bhi, false, false)
                          : __builtin_amdgcn_permlane16_swap(ahi, bhi, false, false);
  a = __builtin_bit_cast(double, (uint64_t)lo[0] | ((uint64_t)hi[0] << 32));
  b = __builtin_bit_cast(double, (uint64_t)lo[1] | ((uint64_t)hi[1] << 32));
}

template <int LEVEL>
struct Mod;
template <>
struct Mod<1> {
  static constexpr double Q = 134215681.0;
  static constexpr double QINV = 1.0 / 134215681.0;
  static constexpr double HALF = 67107840.0;  // (q-1)/2
  static constexpr int N = N1, L = 10;
  static constexpr int RED_FWD = 64, RED_INV = 64;  // 2^53 / q1 = 2^26: no reduction inside
};
template <>
struct Mod<2> {
  static constexpr double Q = 1125899906826241.0;
  static constexpr double QINV = 1.0 / 1125899906826241.0;
  static constexpr double HALF = 562949953413120.0;
  static constexpr int N = N2, L = 11;
  // stages between reductions; bounds checked in DESIGN.md §3 (worst intermediate 0.78 * 2^53)
  static constexpr int RED_FWD = 6, RED_INV = 3;
};

// a*w mod q, |result| <= (0.5 + A/5) q for |a| <= A q, |w| <= q/2.
template <class M>
__device__ __forceinline__ double mm(double a, double w) {
  const double h = a * w;
  const double l = __fma_rn(a, w, -h);
  const double qe = rint(h * M::QINV);
  return __fma_rn(-qe, M::Q, h) + l;
}
// x mod q into about [-q/2, q/2] (|x| < 2^53)
template <class M>
__device__ __forceinline__ double red(double x) {
  return __fma_rn(-rint(x * M::QINV), M::Q, x);
}
// For an integer |x| <= q - 1, red(x) is already the exact centred representative: fl(x / q)
// errs by far less than the 2^-52 gap between (q +- 1) / 2q and 1/2, so rint picks the right
// quotient at the +-(q-1)/2 boundaries (checked for both primes). red(red(x)) therefore
// canonicalises any |x| < 2^53 (red leaves |r| <= q/2 + 2) without compare/select pairs, which
// serialise on VCC with hazard NOPs.
// exact centred representative in [-(q-1)/2, (q-1)/2]
template <class M>
__device__ __forceinline__ double canon(double x) {
  return red<M>(red<M>(x));
}
// for |x| <= q - 1 (sum/difference of two canonical values)
template <class M>
__device__ __forceinline__ double canon_small(double x) {
  return red<M>(x);
}
template <class M>
__device__ __forceinline__ uint64_t to_u64(double c) {  // canonical centred -> [0, q)
  const double r = c < 0 ? c + M::Q : c;
  return (uint64_t)r;
}
template <class M>
__device__ __forceinline__ double from_u64(uint64_t v) {  // [0, q) -> centred
  const double r = (double)v;
  return r > M::HALF ? r - M::Q : r;
}

constexpr int ilog2(int x) { return x <= 1 ? 0 : 1 + ilog2(x >> 1); }

// ------------------------------------------------------------------------------------------
// Workgroup NTT over N = T*E points, E elements per thread in registers, log2(E) radix-2
// stages per pass, LDS exchange between passes.
//   forward: in  x[e] = coefficient (tid + e*T)       out x[e] = NTT index (tid*E + e)
//   inverse: in  x[e] = NTT index (tid*E + e)         out x[e] = coefficient (tid + e*T)
// The inverse is unscaled (the caller folds N^-1 into the key). tw[k] = psi^brv(k),
// itw[k] = psi^-brv(k), centred doubles. `lds` holds padded(N) doubles.
// ------------------------------------------------------------------------------------------
template <class M, int T, int E>
struct WgNtt {
  static constexpr int N = T * E;
  static constexpr int L = ilog2(N);
  static constexpr int R = ilog2(E);
  static constexpr int NPASS = (L + R - 1) / R;
  static_assert(N == M::N, "NTT size mismatch");
  // Exchanges alternate between two LDS buffers so only the last exchange of a transform needs
  // the barrier after its reads; lds then holds 2 * C * N doubles.
  static constexpr int LDS_DOUBLES = 2 * N;

  // XOR swizzle of the exchange buffer: bank-conflict free for every (T, E) used here
  // (tools/lds_banks.py models the ds_read_b64 / ds_write_b64 lane groups).
  __device__ static __forceinline__ int pad(int j) { return j ^ ((j >> R) & 31); }

  // Element index of register e in pass p (window of r stages starting at s0).
  __device__ static __forceinline__ int index(int p, int tid, int e) {
    const int s0 = p * R;
    const int r = (L - s0) < R ? (L - s0) : R;
    const int lb = L - s0 - r;
    const int F = (tid << (R - r)) | (e >> r);
    const int ep = e & ((1 << r) - 1);
    return ((F >> lb) << (L - s0)) | (ep << lb) | (F & ((1 << lb) - 1));
  }

  __device__ static __forceinline__ void reduce_all(double (&x)[E]) {
#pragma unroll
    for (int e = 0; e < E; ++e) x[e] = red<M>(x[e]);
  }

  // ---- C independent transforms interleaved (C x E residues per thread, C LDS buffers) ----
  // Thread owning element idx in pass p (inverse of index()).
  static constexpr int thread_of(int p, int idx) {
    const int s0 = p * R;
    const int r = (L - s0) < R ? (L - s0) : R;
    const int lb = L - s0 - r;
    const int F = ((idx >> (L - s0)) << lb) | (idx & ((1 << lb) - 1));
    return F >> (R - r);
  }
  // True when every element stays in the same wave between passes pf and pt: the exchange then
  // needs only wave-level LDS synchronisation (each wave touches its own slots: pad() keeps the
  // high index bits that select the wave).
  static constexpr bool wave_local(int pf, int pt) {
    if (T <= 64) return true;
    for (int idx = 0; idx < N; ++idx)
      if ((thread_of(pf, idx) >> 6) != (thread_of(pt, idx) >> 6)) return false;
    return true;
  }
  __device__ static __forceinline__ void wave_sync() {
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): this wave's LDS writes have landed
    __builtin_amdgcn_wave_barrier();
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
  }

  // Exchange PF -> PT, the ORD-th of its transform; LAST: no further exchange follows (a
  // workgroup barrier then protects the buffers for whatever the caller does next).
  // PREV_WL: the previous exchange of this transform was wave-local, so waves may still be
  // reading their own slots; a cross-wave exchange must then wait for all of them first.
  template <int C, int PF, int PT, int ORD, bool LAST, bool PREV_WL>
  __device__ static __forceinline__ void exchangeC(double (&x)[C][E], double *lds, int tid) {
    constexpr bool WL = wave_local(PF, PT);
    if constexpr (!WL && PREV_WL) __syncthreads();
    double *buf = lds + (ORD & 1) * C * N;
#pragma unroll
    for (int c = 0; c < C; ++c)
#pragma unroll
      for (int e = 0; e < E; ++e) buf[c * N + pad(index(PF, tid, e))] = x[c][e];
    if constexpr (WL)
      wave_sync();
    else
      __syncthreads();
#pragma unroll
    for (int c = 0; c < C; ++c)
#pragma unroll
      for (int e = 0; e < E; ++e) x[c][e] = buf[c * N + pad(index(PT, tid, e))];
    if constexpr (LAST) {
      if constexpr (!LAST && WL)
        wave_sync();
      else
        __syncthreads();
    }
  }

  // K0: first stage of the pass (a caller that computed the earlier stages itself)
  template <int P, int C, int K0 = 0>
  __device__ static __forceinline__ void fwd_passC(double (&x)[C][E], const double *tw, int tid,
                                                   int &since_red) {
    constexpr int s0 = P * R;
    constexpr int r = (L - s0) < R ? (L - s0) : R;
    constexpr int lb = L - s0 - r;
#pragma unroll
    for (int k = K0; k < r; ++k) {
      if (since_red >= M::RED_FWD) {
#pragma unroll
        for (int c = 0; c < C; ++c) reduce_all(x[c]);
        since_red = 0;
      }
      const int s = s0 + k;
      const int half = 1 << (r - 1 - k);
#pragma unroll
      for (int e = 0; e < E; ++e) {
        const int ep = e & ((1 << r) - 1);
        if (ep & half) continue;
        const int F = (tid << (R - r)) | (e >> r);
        const int hi = F >> lb;
        const double w = tw[(1 << s) + ((hi << k) | (ep >> (r - k)))];
#pragma unroll
        for (int c = 0; c < C; ++c) {
          const double u = x[c][e];
          const double v = mm<M>(x[c][e + half], w);
          x[c][e] = u + v;
          x[c][e + half] = u - v;
        }
      }
      ++since_red;
    }
  }

  // MIRROR: itw is the FORWARD table: psi^-brv(2^s + j) = -psi^brv(2^(s+1) - 1 - j) (the node's
  // mirror in its stage), so w = tw[2^(s+1) - 1 - node] and the butterfly multiplies (v - u)
  // instead of (u - v) -- the same exact product, and no inverse table in LDS.
  template <int P, int C, bool MIRROR = false>
  __device__ static __forceinline__ void inv_passC(double (&x)[C][E], const double *itw, int tid,
                                                   int &since_red) {
    constexpr int s0 = P * R;
    constexpr int r = (L - s0) < R ? (L - s0) : R;
    constexpr int lb = L - s0 - r;
#pragma unroll
    for (int k = r - 1; k >= 0; --k) {
      if (since_red >= M::RED_INV) {
#pragma unroll
        for (int c = 0; c < C; ++c) reduce_all(x[c]);
        since_red = 0;
      }
      const int s = s0 + k;
      const int half = 1 << (r - 1 - k);
#pragma unroll
      for (int e = 0; e < E; ++e) {
        const int ep = e & ((1 << r) - 1);
        if (ep & half) continue;
        const int F = (tid << (R - r)) | (e >> r);
        const int hi = F >> lb;
        const int node = (hi << k) | (ep >> (r - k));
        const double w = MIRROR ? itw[(2 << s) - 1 - node] : itw[(1 << s) + node];
#pragma unroll
        for (int c = 0; c < C; ++c) {
          const double u = x[c][e];
          const double v = x[c][e + half];
          x[c][e] = u + v;
          x[c][e + half] = MIRROR ? mm<M>(v - u, w) : mm<M>(u - v, w);
        }
      }
      ++since_red;
    }
  }

  template <int P, int C>
  __device__ static __forceinline__ void fwd_fromC(double (&x)[C][E], double *lds, const double *tw,
                                                   int tid, int &since_red) {
    if constexpr (P < NPASS) {
      if constexpr (P > 0)
        exchangeC<C, P - 1, P, P - 1, P == NPASS - 1, (P >= 2) && wave_local(P - 2, P - 1)>(x, lds, tid);
      fwd_passC<P, C>(x, tw, tid, since_red);
      fwd_fromC<P + 1, C>(x, lds, tw, tid, since_red);
    }
  }
  template <int P, int C>
  __device__ static __forceinline__ void inv_fromC(double (&x)[C][E], double *lds, const double *itw,
                                                   int tid, int &since_red) {
    if constexpr (P >= 0) {
      if constexpr (P < NPASS - 1)
        exchangeC<C, P + 1, P, NPASS - 2 - P, P == 0, (P + 2 <= NPASS - 1) && wave_local(P + 2, P + 1)>(x, lds, tid);
      inv_passC<P, C>(x, itw, tid, since_red);
      inv_fromC<P - 1, C>(x, lds, itw, tid, since_red);
    }
  }

  // C transforms at once; lds holds C * LDS_DOUBLES doubles. Bounds as for the single transforms.
  template <int C>
  __device__ static __forceinline__ void fwdC(double (&x)[C][E], double *lds, const double *tw,
                                              int tid) {
    int since_red = 0;
    fwd_fromC<0, C>(x, lds, tw, tid, since_red);
  }
  template <int C>
  __device__ static __forceinline__ void invC(double (&x)[C][E], double *lds, const double *itw,
                                              int tid) {
    int since_red = 0;
    inv_fromC<NPASS - 1, C>(x, lds, itw, tid, since_red);
  }

  // three exchange buffers of the level-2 CMUX transforms (CmuxNtt) and the trace
  static constexpr int LDS3_DOUBLES = 3 * N;
  // Single-transform API.
  __device__ static __forceinline__ void fwd(double (&x)[E], double *lds, const double *tw, int tid) {
    fwdC<1>(reinterpret_cast<double(&)[1][E]>(x), lds, tw, tid);
  }
  __device__ static __forceinline__ void inv(double (&x)[E], double *lds, const double *itw, int tid) {
    invC<1>(reinterpret_cast<double(&)[1][E]>(x), lds, itw, tid);
  }
};


// ------------------------------------------------------------------------------------------
// Level-2 CMUX transforms (256 threads x 8 residues, N2 = 2048): the digit NTTs, inverse NTTs
// and BSK2 conversion of the blind rotation. Index bits 10..0 (stage s splits on bit 10 - s)
// are processed in four passes; cidx(p, tid, e) is the index register e of thread tid holds:
//   P0: e -> 10..8, tid 7..0 -> 7..0                   (the coefficient layout tid + 256 e)
//   P1: e -> 7..5, tid 7..5 -> 10..8, tid 4..0 -> 4..0 (cross-wave LDS exchange from P0)
//   P2: e -> 4..2, tid 7,6 -> 10,9, tid 3..0 -> 8..5, tid 5 -> 1, tid 4 -> 0 (wave-local LDS)
//   P3: register bits 2,1 <-> lane bits 5,4 of P2 by v_permlane32_swap / v_permlane16_swap
//       (e2 -> 1, e1 -> 0, e0 -> 2, tid 5 -> 4, tid 4 -> 3): no LDS, 16 swaps per transform.
// Stage-9 and -10 twiddles are read lane-contiguously from the permuted table tw2c (a bit
// permutation of each stage's node index, so the mirrored inverse lookup (2 << s) - 1 - pos holds
// unchanged); stages 0..8 of tw2c equal tw2. The forward output (and BSK2) sits at register e of
// thread tid = position tid * 8 + e, NTT index cidx(3, tid, e).
// Exchange buffers (LDS3_DOUBLES): X0 = lds, X1 = lds + N for the cross-wave exchange (the
// caller alternates them, as the staging does), W = lds + 2N for the wave-local one (each wave
// only touches the slots of its own index bits 10, 9).
// ------------------------------------------------------------------------------------------
OMR_HD constexpr int cmux_idx(int p, int tid, int e) {
  return p == 0   ? (e << 8) | tid
         : p == 1 ? ((tid >> 5) << 8) | (e << 5) | (tid & 31)
         : p == 2 ? ((tid >> 6) << 9) | ((tid & 15) << 5) | (e << 2) | (((tid >> 5) & 1) << 1) | ((tid >> 4) & 1)
                  : ((tid >> 6) << 9) | ((tid & 15) << 5) | (((tid >> 5) & 1) << 4) | (((tid >> 4) & 1) << 3) |
                        ((e & 1) << 2) | (((e >> 2) & 1) << 1) | ((e >> 1) & 1);
}
// offset of the stage-s twiddle (within the stage's 2^s entries) of the pair whose lower register
// is e: the node index for s <= 8, the permuted position for s = 9, 10
OMR_HD constexpr int cmux_tw_off(int p, int s, int tid, int e) {
  return s == 9    ? (e & 1) * 256 + tid
         : s == 10 ? ((((e >> 2) & 1) << 1) | (e & 1)) * 256 + tid
                   : cmux_idx(p, tid, e) >> (11 - s);
}

struct CmuxNtt {
  using M = Mod<2>;
  static constexpr int T = 256, E = 8, N = 2048, L = 11;
  using G = WgNtt<M, T, E>;
  static_assert(N == M::N, "level-2 geometry");
  static constexpr int LDS_DOUBLES = 3 * N;
  // register bit holding index bit b in pass p
  static constexpr int rbit(int p, int b) { return p == 0 ? b - 8 : p == 1 ? b - 5 : p == 2 ? b - 2 : (b == 1 ? 2 : 1); }
  // W-buffer swizzle: index bits 5..8 into slot bits 1..4 and bit 8 into bit 0 -- conflict free for
  // ds_write_b64 / ds_read_b64 in both P1 and P2 layouts (tests/test_cmux_layout.py)
  __device__ static __forceinline__ int padw(int j) { return j ^ (((j >> 5) & 15) << 1) ^ ((j >> 8) & 1); }

  // Pass-0 twiddles (stages 0..2) are wave-uniform: with G they come from the global table gt
  // (scalar loads, SGPRs) instead of LDS, whose reads the exchange fences would force again.
  template <int P, int S, bool INV, bool G = false>
  __device__ static __forceinline__ void stage(double (&x)[E], const double *tw, int tid, int &since_red,
                                               const double *__restrict__ gt = nullptr) {
    constexpr int h = 1 << rbit(P, L - 1 - S);
    if (since_red >= (INV ? M::RED_INV : M::RED_FWD)) {
      // forward: only the u operands (x[e], e & h == 0) are reduced; mm takes the v operands as
      // they are (|v| <= 6.3q, |mm| <= 1.7q), which keeps the transform output below 7q
      // (bounds in tests/test_fp64_residues.py)
#pragma unroll
      for (int e = 0; e < E; ++e)
        if (INV || !(e & h)) x[e] = red<M>(x[e]);
      since_red = 0;
    }
#pragma unroll
    for (int e = 0; e < E; ++e) {
      if (e & h) continue;
      // pass 0: the node is e >> (3 - S) for every thread (tid < 256), a wave-uniform index
      const int off = P == 0 ? (e >> (3 - S)) : cmux_tw_off(P, S, tid, e);
      if constexpr (!INV) {
        const double w = (P == 0 && G) ? gt[(1 << S) + off] : tw[(1 << S) + off];
        const double u = x[e], v = mm<M>(x[e + h], w);
        x[e] = u + v;
        x[e + h] = u - v;
      } else {  // psi^-brv(2^s + j) = -psi^brv(2^(s+1) - 1 - j): the forward table mirrored
        const double w = (P == 0 && G) ? gt[(2 << S) - 1 - off] : tw[(2 << S) - 1 - off];
        const double u = x[e], v = x[e + h];
        x[e] = u + v;
        x[e + h] = mm<M>(v - u, w);
      }
    }
    ++since_red;
  }
  template <int P, int S0, int S1, bool G = false>
  __device__ static __forceinline__ void fwd_stages(double (&x)[E], const double *tw, int tid, int &since_red,
                                                    const double *__restrict__ gt = nullptr) {
    if constexpr (S0 < S1) {
      stage<P, S0, false, G>(x, tw, tid, since_red, gt);
      fwd_stages<P, S0 + 1, S1, G>(x, tw, tid, since_red, gt);
    }
  }
  template <int P, int S0, int S1, bool G = false>  // stages S1 - 1 down to S0
  __device__ static __forceinline__ void inv_stages(double (&x)[E], const double *tw, int tid, int &since_red,
                                                    const double *__restrict__ gt = nullptr) {
    if constexpr (S0 < S1) {
      stage<P, S1 - 1, true, G>(x, tw, tid, since_red, gt);
      inv_stages<P, S0, S1 - 1, G>(x, tw, tid, since_red, gt);
    }
  }
  // cross-wave exchange P0 <-> P1 through X0 / X1 (no trailing barrier: see the buffer rule).
  // Unswizzled: consecutive lanes hold consecutive indices in both layouts (P0: tid, P1: tid & 31),
  // so ds_write_b64 16-lane and ds_read_b64 32-lane groups are conflict free, and every address is
  // a per-thread base plus an immediate offset (256 e and 32 e doubles): two address registers.
  template <int PF, int PT, int XB>
  __device__ static __forceinline__ void exchange_x(double (&x)[E], double *lds, int tid) {
    double *buf = lds + XB * N;
#pragma unroll
    for (int e = 0; e < E; ++e) buf[cmux_idx(PF, tid, e)] = x[e];
    wg_barrier_lds();  // LDS only: the caller's key loads stay in flight across the exchange
#pragma unroll
    for (int e = 0; e < E; ++e) x[e] = buf[cmux_idx(PT, tid, e)];
    __builtin_amdgcn_wave_barrier();  // keep the next writes below these reads (in-order LDS)
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
  }
  // wave-local exchange P1 <-> P2 through W
  template <int PF, int PT>
  __device__ static __forceinline__ void exchange_w(double (&x)[E], double *lds, int tid) {
    double *buf = lds + 2 * N;
#pragma unroll
    for (int e = 0; e < E; ++e) buf[padw(cmux_idx(PF, tid, e))] = x[e];
    G::wave_sync();
#pragma unroll
    for (int e = 0; e < E; ++e) x[e] = buf[padw(cmux_idx(PT, tid, e))];
    __builtin_amdgcn_wave_barrier();
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
  }
  // P2 <-> P3: register bit 2 <-> lane bit 5, register bit 1 <-> lane bit 4 (an involution)
  __device__ static __forceinline__ void swap23(double (&x)[E]) {
#pragma unroll
    for (int e = 0; e < E; ++e)
      if (!(e & 4)) swap_lane_bit<5>(x[e], x[e + 4]);
#pragma unroll
    for (int e = 0; e < E; ++e)
      if (!(e & 2)) swap_lane_bit<4>(x[e], x[e + 2]);
  }
  // passes 1..3 of the forward transform after pass 0 (stages 0..2) is done
  template <int XB>
  __device__ static __forceinline__ void fwd_rest(double (&x)[E], double *lds, const double *tw, int tid,
                                                  int &since_red) {
    exchange_x<0, 1, XB>(x, lds, tid);
    fwd_stages<1, 3, 6>(x, tw, tid, since_red);
    exchange_w<1, 2>(x, lds, tid);
    fwd_stages<2, 6, 9>(x, tw, tid, since_red);
    swap23(x);
    fwd_stages<3, 9, 11>(x, tw, tid, since_red);
  }
  // forward transform of arbitrary residues |x| <= q/2 (key conversion)
  template <int XB>
  __device__ static __forceinline__ void fwd(double (&x)[E], double *lds, const double *tw, int tid) {
    int since_red = 0;
    fwd_stages<0, 0, 3>(x, tw, tid, since_red);
    fwd_rest<XB>(x, lds, tw, tid, since_red);
  }
  // Forward transform of a polynomial of small integer digits |d| <= 64, given as fields
  // f = d + 64 in [0, 128]: stages 0 and 1 from
  // five 129-entry LDS tables (t0 + 136 k: d * c_k for c = tw1, tw2, tw1 tw2, tw3, tw1 tw3)
  // instead of modular products. Stage 0 pairs (e, e + 4) under tw[1] for every thread; stage 1
  // pairs (e, e + 2) with tw[2] (e = 0, 1) and tw[3] (e = 4, 5), so tw2 * x[2] = tw2 d2 +
  // tw1 tw2 d6 and tw3 * x[6] = tw3 d2 - tw1 tw3 d6 are table sums. Bound: |x| <= 1.5q + 64 after
  // stage 1, 5.62q before the stage-6 (u-operand) reduction, 6.72q at the output: below 8q < 2^53
  // and inside mm's exact range (replayed in tests/test_fp64_residues.py).
  template <int XB>
  __device__ static __forceinline__ void fwd_small(const int (&f)[E], const double *t0, double (&x)[E],
                                                   double *lds, const double *tw, int tid,
                                                   const double *__restrict__ gt) {
    const double *T1 = t0, *T2 = t0 + 136, *T3 = t0 + 272, *T4 = t0 + 408, *T5 = t0 + 544;
    // the ten table reads (an explicit sched_barrier forcing them all before the first use measured
    // 0.2 % slower)
    double tv[10] = {T1[f[4]], T1[f[5]], T2[f[2]], T3[f[6]], T2[f[3]], T3[f[7]], T4[f[2]], T5[f[6]], T4[f[3]], T5[f[7]]};
    const double a4 = tv[0], a5 = tv[1];
    const double d0 = (double)(f[0] - 64), d1 = (double)(f[1] - 64);
    const double x0 = d0 + a4, x4 = d0 - a4;
    const double x1 = d1 + a5, x5 = d1 - a5;
    const double v0 = tv[2] + tv[3], v1 = tv[4] + tv[5];
    const double v4 = tv[6] - tv[7], v5 = tv[8] - tv[9];
    x[0] = x0 + v0;
    x[2] = x0 - v0;
    x[1] = x1 + v1;
    x[3] = x1 - v1;
    x[4] = x4 + v4;
    x[6] = x4 - v4;
    x[5] = x5 + v5;
    x[7] = x5 - v5;
    int since_red = 2;
    fwd_stages<0, 2, 3, true>(x, tw, tid, since_red, gt);
    fwd_rest<XB>(x, lds, tw, tid, since_red);
  }
  // Two unscaled inverses interleaved (the CMUX step's outputs A and B) for instruction-level
  // parallelism: the wave-local exchanges run one after the other through W; the cross-wave
  // exchanges keep cmux_step3's order and barriers (A through X1, then B through X0: X0 is written
  // only after a barrier that every wave passes after its last X0 read of the body digits).
  __device__ static __forceinline__ void inv2(double (&xa)[E], double (&xb)[E], double *lds, const double *tw,
                                              int tid, const double *__restrict__ gt) {
    int ra = 0, rb = 0;
    inv_stages<3, 9, 11>(xa, tw, tid, ra);
    inv_stages<3, 9, 11>(xb, tw, tid, rb);
    swap23(xa);
    swap23(xb);
    inv_stages<2, 6, 9>(xa, tw, tid, ra);
    inv_stages<2, 6, 9>(xb, tw, tid, rb);
    exchange_w<2, 1>(xa, lds, tid);
    exchange_w<2, 1>(xb, lds, tid);
    inv_stages<1, 3, 6>(xa, tw, tid, ra);
    inv_stages<1, 3, 6>(xb, tw, tid, rb);
    exchange_x<1, 0, 1>(xa, lds, tid);
    exchange_x<1, 0, 0>(xb, lds, tid);
    inv_stages<0, 0, 3, true>(xa, tw, tid, ra, gt);
    inv_stages<0, 0, 3, true>(xb, tw, tid, rb, gt);
  }
  // unscaled inverse (the caller folds N^-1 into the key), tw the forward table (mirrored reads);
  // gt: the same table in global memory (pass-0 twiddles)
  template <int XB>
  __device__ static __forceinline__ void inv(double (&x)[E], double *lds, const double *tw, int tid,
                                             const double *__restrict__ gt) {
    int since_red = 0;
    inv_stages<3, 9, 11>(x, tw, tid, since_red);
    swap23(x);
    inv_stages<2, 6, 9>(x, tw, tid, since_red);
    exchange_w<2, 1>(x, lds, tid);
    inv_stages<1, 3, 6>(x, tw, tid, since_red);
    exchange_x<1, 0, XB>(x, lds, tid);
    inv_stages<0, 0, 3, true>(x, tw, tid, since_red, gt);
  }
};

}  // namespace omr
