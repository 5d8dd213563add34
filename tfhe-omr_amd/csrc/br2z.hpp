// Level 2 of the latency path over four CUs per message on the exact FFT (round 6, br2z_kernel):
// second_level_bootstrapping's blind rotation (detector.rs:599-624) for one message at a time.
//
// br2y_kernel (br2_fft.hpp) gives a polynomial of the accumulator one CU holding two 256-thread
// groups, each transforming three of the polynomial's six digits one after the other, then a limb
// swap between the groups, one hand-off to the partner CU, an inverse per group and a half swap. Here
// every digit word gets a CU of its own: worker w = 2 r + h of message m owns word h of the Digits2S
// decomposition of (X^a - 1) ACC_r -- digits 3 h + j, GGSW rows r D2 + 3 h + j -- and runs it as ONE
// 256-thread group (one wave per SIMD) that transforms its three digits interleaved, pass by pass (three
// independent instruction streams per wave, one barrier for the three cross-wave exchanges), and
// multiply-accumulates all four (output, limb) spectra over them. One all-to-all hand-off per executed
// step then gives each worker the three other workers' partial spectra of output r (both limbs), and
// both workers of polynomial r run the two inverses (interleaved), round, recombine the limbs mod q2
// and update their own copy of ACC_r (identical: the same operations on the same values). Per CU and
// step: one interleaved transform round, one hand-off and one interleaved inverse pair, against br2y's
// three transform rounds, a limb swap, a hand-off and a half swap.
//
// Hand-off (br2x's rules, latency_kernels.hpp): each worker writes its four partial spectra to its
// slot hc & 1 (hc = executed steps so far), drains the stores, and publishes hc + 1 in its flag; it
// then polls the other three flags (bounded: a sticky error flag instead of a hang) and reads the
// six 8 KB halves it needs with sc1 loads. A worker rewrites slot hc & 1 at hand-off hc + 2 only after
// seeing every other flag reach hc + 2, which each worker publishes after its hand-off-hc reads were
// consumed. When all four workers of a message report the same XCD (HW_REG_XCC_ID, swapped once per
// launch with sc1 accesses) the payload and flags use plain stores, which stay in that XCD's L2 where
// the sc1 loads find them (br2y's same-XCD path); otherwise sc1 stores. The grid is co-resident by
// construction (cooperative launch, one workgroup per CU: the host checks the CU count).
// Accumulation order (the exactness bound, context.hip apriori_bound level 5): per (output, limb) the
// worker's three rows in order (two FMAs each), then the three other workers' partials added one by
// one (workers w + 1, w + 2, w + 3 mod 4): row j of any worker carries weight at most 2 (3 - j) + 3.
// The two workers of polynomial r sum in different orders; both results are within the bound of the
// exact integers, so their rounded updates of ACC_r are identical.
// Key prefetchers: BR2Z_H helper workgroups per worker on its XCD touch one dword per 64 B of the
// worker's three rows of each executed step, at most BR2Z_PF executed steps ahead (br2y_prefetch's
// scheme); they only read the key.
// Grid: w8 = n rounded up to a multiple of 8 columns (message m in column m), rows 0..3 the workers,
// rows 4 + BR2Z_H w + k helper k of worker w (launched only when every workgroup gets its own CU).
// flags[0, 4n): hand-off counts [m][w]; flags[4n, 8n): XCD ids + 1. Slots: [m][w][2][4][2][1024].
#pragma once

#include "br2_fft.hpp"

namespace omr {

constexpr int BR2Z_T = Fft1024::T, BR2Z_H = 2, BR2Z_PF = 2;

// C cross-wave / wave-local exchanges of Fft1024 at once: the writes of all C, one barrier (or one
// wave-level wait), the reads of all C (Fft1024::exchange for one transform)
template <int C, int PF, int PT, int S, bool CROSS>
__device__ __forceinline__ void br2z_xchg(double (&xr)[C][Fft1024::E], double (&xi)[C][Fft1024::E],
                                          double2 *const (&X)[C], int t) {
  using F = Fft1024;
  constexpr int E = F::E;
  const int bw = F::swz(S, F::idx(PF, t, 0)), br = F::swz(S, F::idx(PT, t, 0));
#pragma unroll
  for (int c = 0; c < C; ++c)
#pragma unroll
    for (int e = 0; e < E; ++e) X[c][F::slot_of<S, PF>(bw, e)] = make_double2(xr[c][e], xi[c][e]);
  if constexpr (CROSS) {
    wg_barrier_lds();
  } else {
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0)
    __builtin_amdgcn_wave_barrier();
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
  }
#pragma unroll
  for (int c = 0; c < C; ++c)
#pragma unroll
    for (int e = 0; e < E; ++e) {
      const double2 v = X[c][F::slot_of<S, PT>(br, e)];
      xr[c][e] = v.x;
      xi[c][e] = v.y;
    }
  __builtin_amdgcn_wave_barrier();
  __atomic_signal_fence(__ATOMIC_SEQ_CST);
}

// C forward transforms interleaved pass by pass (Fft1024::fwd's passes and exchanges; X[c]: transform
// c's cross-wave buffer, its wave-local exchange in the wave's own quarter of it)
template <int C, typename Mid>
__device__ __forceinline__ void br2z_fwd(double (&xr)[C][Fft1024::E], double (&xi)[C][Fft1024::E],
                                         double2 *const (&X)[C], int t, const double2 (&wc)[4][2], Mid mid) {
  using F = Fft1024;
#pragma unroll
  for (int c = 0; c < C; ++c) {
    F::fwd_pass_t(xr[c], xi[c], make_double2(F::R2, 1.0), make_double2(F::C8, F::T8));
    F::perm(xr[c], xi[c]);
    F::fwd_pass_t(xr[c], xi[c], wc[0][0], wc[0][1]);
  }
  br2z_xchg<C, 1, 2, 0, true>(xr, xi, X, t);
  mid();
#pragma unroll
  for (int c = 0; c < C; ++c) {
    F::fwd_pass_t(xr[c], xi[c], wc[1][0], wc[1][1]);
    F::perm(xr[c], xi[c]);
    F::fwd_pass_t(xr[c], xi[c], wc[2][0], wc[2][1]);
  }
  br2z_xchg<C, 3, 4, 2, false>(xr, xi, X, t);
#pragma unroll
  for (int c = 0; c < C; ++c) F::fwd_pass_t(xr[c], xi[c], wc[3][0], wc[3][1]);
}

// C inverse transforms interleaved (Fft1024::inv: the wave-local exchange first, in the wave's own
// quarter of X[c], then the cross-wave one; twiddles requested one pass ahead, shared by the C)
template <int C>
__device__ __forceinline__ void br2z_inv(double (&xr)[C][Fft1024::E], double (&xi)[C][Fft1024::E],
                                         double2 *const (&X)[C], const double2 *tws, int t) {
  using F = Fft1024;
  double2 w4[3], w3[3], w2[3], w1[3];
  F::inv_tw<4>(w4, tws, t);
  F::inv_tw<3>(w3, tws, t);
#pragma unroll
  for (int c = 0; c < C; ++c) F::inv_pass_w(xr[c], xi[c], w4);
  br2z_xchg<C, 4, 3, 3, false>(xr, xi, X, t);
  F::inv_tw<2>(w2, tws, t);
#pragma unroll
  for (int c = 0; c < C; ++c) {
    F::inv_pass_w(xr[c], xi[c], w3);
    F::perm(xr[c], xi[c]);
  }
  F::inv_tw<1>(w1, tws, t);
#pragma unroll
  for (int c = 0; c < C; ++c) F::inv_pass_w(xr[c], xi[c], w2);
  br2z_xchg<C, 2, 1, 1, true>(xr, xi, X, t);
#pragma unroll
  for (int c = 0; c < C; ++c) {
    F::inv_pass_w(xr[c], xi[c], w1);
    F::perm(xr[c], xi[c]);
    F::inv_pass<0>(xr[c], xi[c], tws, t);
  }
}

// The worker's partial spectra of output o (both limbs) over its three rows, rows in order (k: the
// rows' output-o key blocks), stored to its hand-off slot (dst: [o][l][re / im][1024] at e T + t)
__device__ __forceinline__ void br2z_mac_store(const double (&xr)[3][Fft1024::E], const double (&xi)[3][Fft1024::E],
                                               const double2 (&k)[3][2][Fft1024::E], double (&sr)[2][Fft1024::E],
                                               double (&si)[2][Fft1024::E], double *dst, bool fast, int t) {
  using F = Fft1024;
  constexpr int E = F::E, n = F::n, T = F::T;
#pragma unroll
  for (int l = 0; l < 2; ++l)
#pragma unroll
    for (int e = 0; e < E; ++e) {
      double pr = 0.0, pi = 0.0;
#pragma unroll
      for (int j = 0; j < 3; ++j) {
        const double2 kv = k[j][l][e];
        pr = __fma_rn(xr[j][e], kv.x, __fma_rn(-xi[j][e], kv.y, pr));
        pi = __fma_rn(xr[j][e], kv.y, __fma_rn(xi[j][e], kv.x, pi));
      }
      sr[l][e] = pr;
      si[l][e] = pi;
      double *d = dst + l * 2 * n + e * T + t;
      if (fast) {  // plain stores: the lines stay in this XCD's L2 for the others' sc1 loads
        d[0] = pr;
        d[n] = pi;
      } else {
        st_sc1(d, pr);
        st_sc1(d + n, pi);
      }
    }
}

// Key prefetcher k of worker w = 2 r + h of message m (br2y_prefetch for the worker's three rows)
__device__ __forceinline__ void br2z_prefetch(const uint32_t *__restrict__ lwe_int, const double2 *__restrict__ bskf,
                                              const uint32_t *flags, int m, int w, int k) {
  constexpr int STEP_LINES = 3 * BR2_ROW * (int)sizeof(double2) / 64;  // 64 B lines of a worker's three rows
  constexpr int PER_THREAD = STEP_LINES / (BR2Z_H * BR2Z_T);
  static_assert(PER_THREAD * BR2Z_H * BR2Z_T == STEP_LINES, "helpers split a step's rows evenly");
  __shared__ int go;
  const int r = w >> 1, h = w & 1;
  const uint32_t *lwe = lwe_int + (size_t)m * (NI + 1);
  uint32_t acc = 0;
  int e = 0;  // executed steps prefetched
#pragma unroll 1
  for (int i = 0; i < NI; ++i) {
    const int a = (int)__builtin_amdgcn_readfirstlane(lwe[i]) & (2 * N2 - 1);
    if (a == 0) continue;
    if (threadIdx.x == 0) {  // the worker has published hand-off e - BR2Z_PF (bounded: a helper may give up)
      int ok = 1, n = 0;
      while ((int)__hip_atomic_load(flags + 4 * m + w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < e - BR2Z_PF) {
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
    const char *rows = reinterpret_cast<const char *>(bskf + ((size_t)i * 2 * D2 + (size_t)r * D2 + 3 * h) * BR2_ROW);
    uint32_t v[PER_THREAD];
#pragma unroll
    for (int u = 0; u < PER_THREAD; ++u)
      v[u] = *reinterpret_cast<const uint32_t *>(rows + (size_t)((u * BR2Z_H + k) * BR2Z_T + (int)threadIdx.x) * 64);
#pragma unroll
    for (int u = 0; u < PER_THREAD; ++u) acc ^= v[u];
    __syncthreads();  // thread 0's next poll after every load of this step returned
    ++e;
  }
  asm volatile("" ::"v"(acc));  // the loads stay live
}

__global__ __launch_bounds__(BR2Z_T, 1) void br2z_kernel(const uint32_t *__restrict__ lwe_int,
                                                         const double2 *__restrict__ bskf,
                                                         const double2 *__restrict__ twg, DeviceTables tb,
                                                         double *xg, uint32_t *flags, int *err,
                                                         uint64_t *__restrict__ out, int nmsg, int w8,
                                                         int allow_fast) {
  using F = Fft1024;
  using M = Mod<2>;
  constexpr int E = F::E, NN = N2, n = F::n, T = F::T;
  __shared__ double2 tws[n];
  __shared__ double2 xf[3][n];  // the forward round's cross-wave buffers
  __shared__ double2 xv[2][n];  // the inverse pair's
  __shared__ double acs[NN];    // this worker's copy of ACC_r (slot_stage positions)
  __shared__ int stop, same_xcd;
  const int m = (int)blockIdx.x % w8, row = (int)blockIdx.x / w8;  // uniform
  if (m >= nmsg) return;
  if (row >= 4) {
    br2z_prefetch(lwe_int, bskf, flags, m, (row - 4) / BR2Z_H, (row - 4) % BR2Z_H);
    return;
  }
  const int w = row, r = w >> 1, h = w & 1, t = (int)threadIdx.x;
  const int pslot = __builtin_amdgcn_readfirstlane(m == 0 ? 8 + 4 * w + (t >> 6) : -1);  // phase trace
  (void)pslot;
  OMR_PHASE_CLOCK(pslot, 0);
  const uint32_t *lwe = lwe_int + (size_t)m * (NI + 1);
  F::load_twiddles(tws, twg, t);
  {  // ACC_r = X^{-b} * LUT2 (body) or 0 (mask)
    const int b = (int)lwe[NI];
    const int rr = (2 * NN - (b % (2 * NN))) % (2 * NN);
    for (int c = t; c < NN; c += T) acs[F::slot_stage(c)] = r == 1 ? canon_small<M>(rot_read<NN>(tb.lut2, c, rr)) : 0.0;
    if (t == 0) {
      stop = 0;
      // XCD ids through global memory (sc1 both ways); a worker that never answers leaves the sc1
      // protocol in place (the step loop's bounded poll then reports it)
      uint32_t *xid = flags + 4 * nmsg + 4 * m;
      const uint32_t mine = (uint32_t)__builtin_amdgcn_s_getreg(6164) + 1u;  // hwreg(HW_REG_XCC_ID, 0, 4)
      __hip_atomic_store(xid + w, mine, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      int same = allow_fast;
      for (int o = 0; o < 4; ++o) {
        if (o == w) continue;
        uint32_t theirs = 0;
        for (int k = 0; k < (1 << 20) && theirs == 0; ++k) {
          theirs = __hip_atomic_load(xid + o, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          if (theirs == 0) __builtin_amdgcn_s_sleep(2);
        }
        same = same && theirs == mine;
      }
      same_xcd = same;
    }
  }
  double2 wc[4][2];  // this thread's forward twiddles of passes 1..4
  F::block_ct<1>(wc[0], twg, t);
  F::block_ct<2>(wc[1], twg, t);
  F::block_ct<3>(wc[2], twg, t);
  F::block_ct<4>(wc[3], twg, t);
  __syncthreads();  // same_xcd, the twiddles and the accumulator visible
  const bool fast = __builtin_amdgcn_readfirstlane(same_xcd) != 0;
  const __amdgpu_buffer_rsrc_t rsrc = bsk2_rsrc(bskf);
  const uint32_t t16 = (uint32_t)t * 16u;
  uint32_t *my_flag = flags + 4 * m + w;
  double2 *const XF[3] = {xf[0], xf[1], xf[2]};
  double2 *const XV[2] = {xv[0], xv[1]};
  RoundGuard<false> rg;
  uint32_t hc = 0;  // hand-offs so far (executed steps)
  double2 ka[3][2][E], kb[3][2][E];
  int pre = -1;  // the step whose rows ka holds
#pragma unroll 1
  for (int i = 0; i < NI; ++i) {
    const int a = (int)__builtin_amdgcn_readfirstlane(lwe[i]) & (2 * NN - 1);
    if (a == 0) continue;  // (X^0 - 1) * ACC = 0 (all four workers of the message skip it)
    OMR_PHASE(pslot, (int)hc, 0);
    const int q0 = i * 2 * D2 + r * D2 + 3 * h;  // the worker's first GGSW row of this step
    // output A's blocks of the three rows (issued before the previous step's inverses when this step
    // runs next; in flight across the digits and the transforms), output B's after the transforms
    if (pre != i) {
#pragma unroll
      for (int j = 0; j < 3; ++j) br2f_load_half(ka[j], rsrc, q0 + j, 0, t16);
    }
    wg_barrier_lds();  // ACC_r (init or the previous update) visible; the previous step's LDS reads done
    uint32_t pw[2][E];  // word h of the digits at the thread's P0 points (coefficients j, j + 1024)
    {
      uint32_t pk[2][E][Digits2S::DW];
      br2f_digits(acs, a, t, pk);
#pragma unroll
      for (int hh = 0; hh < 2; ++hh)
#pragma unroll
        for (int e = 0; e < E; ++e) pw[hh][e] = h ? pk[hh][e][1] : pk[hh][e][0];
    }
    OMR_PHASE(pslot, (int)hc, 1);
    double xr[3][E], xi[3][E];
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      const int wd = h == 1 && j == 2 ? Digits2S::TOP_WIDTH : 7;  // the top digit of word 1
#pragma unroll
      for (int e = 0; e < E; ++e) {
        xr[j][e] = (double)(int)__builtin_amdgcn_sbfe(pw[0][e], 7 * j, wd);
        xi[j][e] = (double)(int)__builtin_amdgcn_sbfe(pw[1][e], 7 * j, wd);
      }
    }
    // output B's blocks issued after the transforms' cross-wave exchange
    br2z_fwd<3>(xr, xi, XF, t, wc, [&]() {
#pragma unroll
      for (int j = 0; j < 3; ++j) br2f_load_half(kb[j], rsrc, q0 + j, 1, t16);
    });
    OMR_PHASE(pslot, (int)hc, 2);
    // hand-off: the four (output, limb) partial spectra of the worker's three rows to its slot hc & 1,
    // output 1 - r first (its stores drain during output r's products); output r's kept
    double sr[2][E], si[2][E], ur[2][E], ui[2][E];
    {
      double *dst = xg + (((size_t)m * 4 + w) * 2 + (hc & 1)) * 8 * n;
      if (r == 0) {
        br2z_mac_store(xr, xi, kb, ur, ui, dst + 4 * n, fast, t);
        br2z_mac_store(xr, xi, ka, sr, si, dst, fast, t);
      } else {
        br2z_mac_store(xr, xi, ka, ur, ui, dst, fast, t);
        br2z_mac_store(xr, xi, kb, sr, si, dst + 4 * n, fast, t);
      }
      OMR_PHASE(pslot, (int)hc, 3);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();
    OMR_PHASE(pslot, (int)hc, 4);
    if (t == 0) {
      if (fast)
        __hip_atomic_store(my_flag, hc + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);  // plain store
      else
        __hip_atomic_store(my_flag, hc + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      for (int o = 0; o < 4 && !stop; ++o) {
        if (o == w) continue;
        int k = 0;
        while (__hip_atomic_load(flags + 4 * m + o, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < hc + 1) {
          if (++k == BR2X_SPIN) {
            stop = 1;
            atomicExch(err, 1);
            break;
          }
          __builtin_amdgcn_s_sleep(2);
        }
      }
    }
    __syncthreads();
    OMR_PHASE(pslot, (int)hc, 5);
    if (stop) break;
    // output r, both limbs: this worker's partial + the other three workers' in increasing order
    // (the other three workers in the order w + 1, w + 2, w + 3 mod 4: every load issued at once)
    double fr[2][E], fi[2][E], vr[3][2][E], vi[3][2][E];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      const int o = (w + 1 + k) & 3;
      const double *src = xg + (((size_t)m * 4 + o) * 2 + (hc & 1)) * 8 * n + (size_t)(r * 2) * 2 * n;
#pragma unroll
      for (int l = 0; l < 2; ++l)
#pragma unroll
        for (int e = 0; e < E; ++e) {
          vr[k][l][e] = ld_sc1(src + l * 2 * n + e * T + t);
          vi[k][l][e] = ld_sc1(src + l * 2 * n + n + e * T + t);
        }
    }
#pragma unroll
    for (int l = 0; l < 2; ++l)
#pragma unroll
      for (int e = 0; e < E; ++e) {
        fr[l][e] = sr[l][e] + vr[0][l][e] + vr[1][l][e] + vr[2][l][e];
        fi[l][e] = si[l][e] + vi[0][l][e] + vi[1][l][e] + vi[2][l][e];
      }
    (void)ur;
    (void)ui;
    asm volatile("" : "+v"(fr[0][0]), "+v"(fr[1][0]), "+v"(fi[0][0]), "+v"(fi[1][0])::"memory");
    OMR_PHASE(pslot, (int)hc, 6);
    if (i + 1 < NI) {  // the next step's output-A blocks (kept when that step runs next)
#pragma unroll
      for (int j = 0; j < 3; ++j) br2f_load_half(ka[j], rsrc, q0 + 2 * D2 + j, 0, t16);
      pre = i + 1;
    }
    br2z_inv<2>(fr, fi, XV, tws, t);
    br2f_update<false>(acs, fr, fi, rg, t);  // rounding, limb recombination mod q2, ACC_r += (in place)
    OMR_PHASE(pslot, (int)hc, 7);
    ++hc;
  }
  OMR_PHASE_CLOCK(pslot, 1);
  __syncthreads();  // the last updates everywhere
  if (h == 0) {     // one copy of ACC_r goes out
    uint64_t *o = out + (size_t)m * 2 * NN + (size_t)r * NN;
    for (int c = t; c < NN; c += T) o[c] = to_u64<M>(acs[F::slot_stage(c)]);
  }
}

}  // namespace omr
