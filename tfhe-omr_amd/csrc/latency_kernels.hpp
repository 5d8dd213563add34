// Latency path of the detect pipeline (small chunks: a single message or a few).
//
// The throughput kernels give one wave to a level-1 rotation and one 4-wave workgroup to a
// level-2 message, so a lone message walks 512 (670) CMUX steps with 10 (14) transforms each on
// one wave (workgroup) while the rest of the chip idles: 9 + 16.6 ms of its 27 ms latency.
// Here every CMUX step's digit transforms are split over more waves, whose partial
// multiply-accumulates are summed through LDS before the inverse transforms:
//   level 1 (br1l_kernel): one 8-wave workgroup per rotation; wave w transforms one of the 8
//     digit polynomials (1 FFT instead of 8) and adds its products into the two output sums in
//     LDS, waves 0 / 1 run the inverse FFT of output A / B and own the mask / body accumulator;
//   level 2 (br2l_kernel): one 8-wave workgroup per message, two groups of four waves; group 0
//     transforms the 6 mask digits, group 1 the 6 body digits, each sums one output and runs one
//     inverse NTT (6 + 1 transforms per group instead of 12 + 2); the trace runs after it
//     (trace_kernel, in place on the output);
//   key switch (ks_mfma_split_kernel + ks_combine_kernel): the 1024 input coefficients split
//     over 32 slices of workgroups (a lone message otherwise gets 21 waves for 88 MB of KSK).
// The arithmetic is the throughput kernels' (same digits, transforms, products and reduction
// points), so the outputs are bit-identical; tests/test_gpu_parity.py checks both paths.
#pragma once

#include "detect_kernels.hpp"

namespace omr {

// Phase timestamps of the latency kernels (tools/phase_trace.py; built only with
// -DOMR_PHASE_TRACE): lane 0 of each traced wave stores clock64() at the phase boundaries of
// executed steps PT_S0 .. PT_S0 + PT_STEPS - 1 (slots 0..7: br1l workgroup 0, waves 0..7; slots
// 8..23: br2x workgroups 0, 1, waves 0..7), plus clock64 / wall_clock64 pairs at kernel entry and
// exit for the clock rate.
#ifdef OMR_PHASE_TRACE
constexpr int PT_S0 = 200, PT_STEPS = 64, PT_K = 8, PT_SLOTS = 32;
__device__ unsigned long long omr_phase_buf[PT_SLOTS * PT_STEPS * PT_K + PT_SLOTS * 4];
__device__ __forceinline__ void phase_mark(int slot, int step, int k) {
  if (slot >= 0 && (threadIdx.x & 63) == 0 && step >= PT_S0 && step < PT_S0 + PT_STEPS)
    omr_phase_buf[(slot * PT_STEPS + (step - PT_S0)) * PT_K + k] = clock64();
}
__device__ __forceinline__ void phase_clock(int slot, int k) {  // k 0: entry, 1: exit
  if (slot >= 0 && (threadIdx.x & 63) == 0) {
    unsigned long long *p = omr_phase_buf + PT_SLOTS * PT_STEPS * PT_K + slot * 4 + 2 * k;
    p[0] = clock64();
    p[1] = wall_clock64();
  }
}
#define OMR_PHASE(slot, step, k) phase_mark(slot, step, k)
#define OMR_PHASE_CLOCK(slot, k) phase_clock(slot, k)
#else
#define OMR_PHASE(slot, step, k) ((void)0)
#define OMR_PHASE_CLOCK(slot, k) ((void)0)
#endif

// ---- level 1 ---------------------------------------------------------------------------------
// Level 1 over eight waves, one workgroup per rotation. Per CMUX step wave w = p * D1 + k extracts
// digit k of polynomial p (p = 0 mask, 1 body: 16 coefficients per lane) and runs its forward FFT
// (GGSW row w's digit spectrum); the eight spectra then cross through LDS (each wave's exchange
// buffer, [e][lane]) and wave v multiplies the 8 spectra's register-slot-v points by the 8 rows'
// keys (its slice of the step, the bsk1l layout: 16 KB contiguous per wave and step), producing
// outputs A and B at those points with plain stores; waves 0 / 1 read output A / B, run its
// inverse and own the mask / body accumulator. Three LDS-only barriers per step (the key loads of
// the next executed step, issued after the multiply-accumulate, stay in flight across them).
// Round 2's form summed the eight waves' products with ds_add_f64 atomics into shared sums: their
// completion tail was ~3,600 cycles of a 17,100-cycle step (tools/phase_trace.py,
// profiles/r03q/phase_br1l_atomics.log); the products now sum in registers in a fixed row order,
// as in br1f_kernel, and the rounded FFT product is exact in either order (device_fft.hpp).
constexpr int BR1L_WAVES = 2 * D1;

// BSK1 rows [512][8 r][2 o][lane * 8 + e] -> the latency layout [512][8 e][8 r][2 o][64 lane]
__global__ __launch_bounds__(256) void bsk1_latency_layout_kernel(const double2 *__restrict__ in,
                                                                  double2 *__restrict__ out, size_t n) {
  const size_t idx = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= n) return;
  const int lane = (int)(idx & 63), o = (int)((idx >> 6) & 1), r = (int)((idx >> 7) & 7), e = (int)((idx >> 10) & 7);
  const size_t i = idx >> 13;
  out[idx] = in[((i * 8 + r) * 2 + o) * 512 + key1_pos(lane, e)];
}

template <bool G>
__device__ __forceinline__ void br1l_body(
    const uint16_t *__restrict__ clue_a, const uint16_t *__restrict__ clue_b,
    const uint16_t *__restrict__ lwe_a, const uint16_t *__restrict__ lwe_b,
    const double2 *__restrict__ bskl, DeviceTables tb, uint32_t *__restrict__ ext_out,
    uint64_t *__restrict__ rlwe_out, int mode, unsigned long long *margin) {
  using F = Fft512;
  constexpr int NF = F::N, W = BR1L_WAVES;
  static_assert(W == 8 && NF == 8 * 64, "one wave per GGSW row and per register slot");
  // [ACC, -ACC] per poly (0 mask, 1 body), Lvl1Off form; 8 KB-aligned for the v_and_or addresses
  __shared__ __attribute__((aligned(8192))) uint32_t ext[2][2 * N1];
  __shared__ double2 xch_all[W][F::BUF];      // per wave: its transform's exchange, then its spectrum [e][lane]
  __shared__ double2 outs[2][8 * 64];         // outputs A, B: [e][lane]
  __shared__ double2 tws[NF];
  __shared__ uint16_t la[N0];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int p = wave / D1, k = wave % D1;
  double2 *xch = xch_all[wave];
  const size_t g = blockIdx.x;  // rotation
  int b;
  if (lwe_a == nullptr) {  // clue g % 7 of message g / 7 (CmLweCiphertext::extract_all, :514)
    const size_t m = g / CLUES;
    const int c = (int)(g % CLUES);
    const uint16_t *A = clue_a + m * N0;
    for (int i = threadIdx.x; i < N0; i += 64 * W)
      la[i] = i <= c ? (uint16_t)(A[c - i] & (Q0 - 1)) : (uint16_t)((Q0 - A[N0 + c - i]) & (Q0 - 1));
    b = clue_b[m * CLUES + c] & (Q0 - 1);
  } else {
    for (int i = threadIdx.x; i < N0; i += 64 * W) la[i] = lwe_a[g * N0 + i] & (Q0 - 1);
    b = lwe_b[g] & (Q0 - 1);
  }
  const int r0 = (2 * N1 - (b % (2 * N1))) % (2 * N1);
  // ACC = (0, X^{-b} * LUT1): wave 0 owns the mask accumulator, wave 1 the body accumulator
  // (the accumulator in br1f's Lvl1Off form: ac'' = ac + H/2 in [0, Q), the stored negacyclic half
  // H - ac'' doubling as the digit operand; br1_fft.hpp, tests/test_lvl1_offset_model.py)
  uint32_t ac[16];
#pragma unroll
  for (int i = 0; i < 16; ++i)
    ac[i] = Lvl1Off::enc(wave == 1 ? (int)canon_small<Mod<1>>(rot_read<N1>(tb.lut1, acc_coef(lane, i), r0)) : 0);
  if (wave < 2) {
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      ext[wave][acc_coef(lane, i)] = ac[i];
      ext[wave][N1 + acc_coef(lane, i)] = Lvl1Off::neg(ac[i]);
    }
  }
  for (int j = threadIdx.x; j < NF; j += 64 * W) tws[j] = tb.fft1[j];
  __syncthreads();
  // Wave v's key slice of an executed step: rows 0..7, outputs A / B at register slot v of every
  // lane (16 KB contiguous per wave), loaded two executed steps ahead (below).
  auto next_step = [&](int i) {  // first i' >= i with a_i' != 0 (uniform)
    while (i < N0 && la[i] == 0) ++i;
    return i;
  };
  double2 kk0[8][2], kk1[8][2];  // [row][output A/B] of two consecutive executed steps
  auto load_slice = [&](double2 (&kk)[8][2], int i) {
    if (i >= N0) return;
    const double2 *kr = bskl + ((size_t)i * 8 + wave) * 16 * 64 + lane;
#pragma unroll
    for (int r = 0; r < 8; ++r)
#pragma unroll
      for (int o = 0; o < 2; ++o) kk[r][o] = kr[(r * 2 + o) * 64];
  };
  const int pslot = __builtin_amdgcn_readfirstlane(blockIdx.x == 0 ? wave : -1);
  int hs = 0;
  RoundGuard<G> rg;  // waves 0 / 1 round the inverses
  (void)pslot;
  (void)hs;
  // one CMUX step at executed step i with its key slice kk (kko: the other slice buffer; inext,
  // inext2: the next two executed steps)
  auto cmux = [&](int i, double2 (&kk)[8][2], double2 (&kko)[8][2], int inext, int inext2) {
    const int a = __builtin_amdgcn_readfirstlane(la[i]);  // != 0: (X^0 - 1) * ACC = 0 is skipped
    OMR_PHASE(pslot, hs, 0);
    double xr[1][8], xi[1][8];
    const uint32_t sbase = (uint32_t)(size_t)(lds_u32 *)ext[p], b4 = (uint32_t)(lane - a) * 4u;
    const uint32_t kWrap = 8u * N1 - 1;  // as br1f_digits: ((b4 + 256 q) & 8191) | sbase
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int j = acc_coef(lane, q);
      uint32_t addr;
      asm("v_and_or_b32 %0, %1, %2, %3" : "=v"(addr) : "v"(b4 + 256u * q), "s"(kWrap), "v"(sbase));
      const uint32_t w = Lvl1Off::digits_u(*(const lds_u32 *)(size_t)addr, ext[p][N1 + j]);
      const double d = Lvl1Off::digit_shifts_u(w, k);
      if (q < 8)
        xr[0][q] = d;
      else
        xi[0][q - 8] = d;
    }
    OMR_PHASE(pslot, hs, 1);
    F::fwd<1, false>(xr, xi, xch, tws, lane);  // pass-0 twiddles from LDS (the lambda loses the
                                               // global table's restrict: vector loads every step)
    wave_lds_fence();  // the spectrum's writes stay below the transform's exchange reads
#pragma unroll
    for (int e = 0; e < 8; ++e) xch[e * 64 + lane] = make_double2(xr[0][e], xi[0][e]);
    OMR_PHASE(pslot, hs, 2);
    // waves 0 / 1 (the inverses' critical path) load the next step's slice here, in the time they
    // wait for waves 4..7, which share their SIMDs and finish their transforms ~2,500 cycles later
    if (wave < 2) load_slice(kko, inext);
    wg_barrier_lds();  // every spectrum is in LDS
    OMR_PHASE(pslot, hs, 3);
    {  // outputs A, B at register slot `wave` of every lane: rows in order, as br1f_step_lds
      double ar = 0.0, ai = 0.0, br = 0.0, bi = 0.0;
#pragma unroll
      for (int r = 0; r < 8; ++r) {
        const double2 x = xch_all[r][wave * 64 + lane];
        const double2 ka = kk[r][0], kB = kk[r][1];
        ar = __fma_rn(x.x, ka.x, __fma_rn(-x.y, ka.y, ar));
        ai = __fma_rn(x.x, ka.y, __fma_rn(x.y, ka.x, ai));
        br = __fma_rn(x.x, kB.x, __fma_rn(-x.y, kB.y, br));
        bi = __fma_rn(x.x, kB.y, __fma_rn(x.y, kB.x, bi));
      }
      outs[0][wave * 64 + lane] = make_double2(ar, ai);
      outs[1][wave * 64 + lane] = make_double2(br, bi);
    }
    wg_barrier_lds();  // outputs complete; every spectrum read (the exchange buffers are free)
    OMR_PHASE(pslot, hs, 4);
    // waves 2..7: the slice two executed steps ahead, into the registers just consumed, issued
    // while waves 0 / 1 run the inverses (issuing 16 KB per wave before the barrier above held
    // every wave there ~2,300 cycles)
    if (wave >= 2) load_slice(kk, inext2);
    if (wave < 2) {  // wave 0: output A (mask accumulator), wave 1: output B (body accumulator)
      double sr[1][8], si[1][8];
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const double2 v = outs[wave][e * 64 + lane];
        sr[0][e] = v.x;
        si[0][e] = v.y;
      }
      OMR_PHASE(pslot, hs, 5);
      F::inv<1, false>(sr, si, xch, tws, lane);
      OMR_PHASE(pslot, hs, 6);
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        ac[q] = Lvl1Off::add(ac[q], Lvl1Off::round<G>(q < 8 ? sr[0][q] : si[0][q - 8], &rg));  // exact (< 2^43)
        ext[wave][acc_coef(lane, q)] = ac[q];
        ext[wave][N1 + acc_coef(lane, q)] = Lvl1Off::neg(ac[q]);
      }
    }
    wg_barrier_lds();  // ACC staged for the next step's digits
    OMR_PHASE(pslot, hs, 7);
    ++hs;
  };
  // key slices alternate between kk0 and kk1: waves 2..7 load each two executed steps ahead,
  // waves 0 / 1 one step ahead (before the first barrier of the step in between)
  int i0 = next_step(0), i1 = next_step(i0 + 1);
  load_slice(kk0, i0);
  if (wave >= 2) load_slice(kk1, i1);
  OMR_PHASE_CLOCK(pslot, 0);
#pragma unroll 1
  while (i0 < N0) {
    const int i2 = __builtin_amdgcn_readfirstlane(next_step(i1 + 1));
    cmux(i0, kk0, kk1, i1, i2);
    if (i1 >= N0) break;
    const int i3 = __builtin_amdgcn_readfirstlane(next_step(i2 + 1));
    cmux(i1, kk1, kk0, i2, i3);
    i0 = i2;
    i1 = i3;
  }
  OMR_PHASE_CLOCK(pslot, 1);
  rg.publish(margin);
  if (mode == 0) {  // extract_lwe_locally (coefficient 0), detector.rs:561
    uint32_t *o = ext_out + g * (N1 + 1);
    for (int j = threadIdx.x; j < N1; j += 64 * W)
      o[j] = Lvl1Int::to_u32(j == 0 ? Lvl1Off::dec(ext[0][0]) : -Lvl1Off::dec(ext[0][N1 - j]));
    if (threadIdx.x == 0) o[N1] = Lvl1Int::to_u32(Lvl1Off::dec(ext[1][0]));
  } else {
    uint64_t *o = rlwe_out + g * 2 * N1;
    for (int j = threadIdx.x; j < N1; j += 64 * W) {
      o[j] = Lvl1Int::to_u32(Lvl1Off::dec(ext[0][j]));
      o[N1 + j] = Lvl1Int::to_u32(Lvl1Off::dec(ext[1][j]));
    }
  }
}

__global__ __launch_bounds__(64 * BR1L_WAVES, 1) void br1l_kernel(
    const uint16_t *__restrict__ clue_a, const uint16_t *__restrict__ clue_b,
    const uint16_t *__restrict__ lwe_a, const uint16_t *__restrict__ lwe_b,
    const double2 *__restrict__ bskl, DeviceTables tb, uint32_t *__restrict__ ext_out,
    uint64_t *__restrict__ rlwe_out, int mode) {
  br1l_body<false>(clue_a, clue_b, lwe_a, lwe_b, bskl, tb, ext_out, rlwe_out, mode, nullptr);
}
__global__ __launch_bounds__(64 * BR1L_WAVES, 1) void br1l_guard_kernel(
    const uint16_t *__restrict__ clue_a, const uint16_t *__restrict__ clue_b,
    const uint16_t *__restrict__ lwe_a, const uint16_t *__restrict__ lwe_b,
    const double2 *__restrict__ bskl, DeviceTables tb, uint32_t *__restrict__ ext_out,
    uint64_t *__restrict__ rlwe_out, int mode, unsigned long long *margin) {
  br1l_body<true>(clue_a, clue_b, lwe_a, lwe_b, bskl, tb, ext_out, rlwe_out, mode, margin);
}

// ---- level 2 ---------------------------------------------------------------------------------
// One workgroup of two 256-thread groups per message: group 0 owns the mask accumulator and its
// 6 digits (GGSW rows 0..5), group 1 the body accumulator and rows 6..11. Per CMUX step each
// group stages its polynomial, transforms its 6 digits and multiply-accumulates both outputs;
// group 0 hands its output-B partial to group 1 and group 1 its output-A partial to group 0
// through `part`; each group then runs one inverse transform. Each group keeps the three-buffer
// discipline of cmux_step3 on its own buffers (staging X1, digits X0 X1 X0 X1 X0 X1, inverse X0:
// consecutive cross-wave uses alternate); the workgroup barriers are a superset of the group's,
// and both groups run the same barrier sequence (a is uniform). Output: the blind rotation in the
// coefficient domain, u64 [2][N2] (mode 1 of br2f_kernel); trace_kernel finishes mode 0.
constexpr int BR2L_T = 2 * BR2_T;

__device__ __forceinline__ void br2l_body(const uint32_t *__restrict__ lwe_int, const double *__restrict__ bsk2,
                                          DeviceTables tb, uint64_t *__restrict__ out) {
  using M = Mod<2>;
  constexpr int T = BR2_T, E = BR2_E, N = N2;
  using NTT = CmuxNtt;
  using DG = Digits2;
  __shared__ double xbuf[2][NTT::LDS_DOUBLES];
  __shared__ double part[2][N];
  __shared__ double tws[N + 136 * 5];  // forward twiddles + the five small-digit stage tables
  const int g = threadIdx.x / T, t = threadIdx.x % T;
  double *X = xbuf[g];
  // pass-0 twiddles read from the LDS copy too (gt = tw): from the global table they were vector
  // loads on every step's critical path (no restrict on DeviceTables' pointers, so no scalar loads)
  const double *tw = tws, *t0 = tws + N;
  const uint32_t *lwe = lwe_int + (size_t)blockIdx.x * (NI + 1);
  double acc[E];
  {
    const int b = (int)lwe[NI];
    const int rr = (2 * N - (b % (2 * N))) % (2 * N);
#pragma unroll
    for (int e = 0; e < E; ++e) acc[e] = g == 1 ? canon_small<M>(rot_read<N>(tb.lut2, t + e * T, rr)) : 0.0;
    for (int j = threadIdx.x; j < N; j += BR2L_T) tws[j] = tb.tw2c[j];
    if (threadIdx.x <= 128) {  // table k: d * c_k, d = tid - 64 (c = tw1, tw2, tw1 tw2, tw3, tw1 tw3)
      const double w1 = tb.tw2[1], w2 = tb.tw2[2], w3 = tb.tw2[3];
      const double c[5] = {w1, w2, canon<M>(mm<M>(w1, w2)), w3, canon<M>(mm<M>(w1, w3))};
#pragma unroll
      for (int k = 0; k < 5; ++k)
        tws[N + 136 * k + threadIdx.x] = canon<M>(mm<M>((double)((int)threadIdx.x - 64), c[k]));
    }
    __syncthreads();
  }
#pragma unroll 1
  for (int i = 0; i < NI; ++i) {
    const int a = (int)__builtin_amdgcn_readfirstlane(lwe[i]) & (2 * N - 1);
    if (a == 0) continue;  // (X^0 - 1) * ACC = 0
    const double *ggsw = bsk2 + ((size_t)i * 2 * D2 + (size_t)g * D2) * 2 * N;
    uint32_t pk[E][DG::DW];
    {  // digits of (X^a - 1) * ACC_g, staged in X1
      double *st = X + N;
#pragma unroll
      for (int e = 0; e < E; ++e) st[t + e * T] = acc[e];
      __syncthreads();
#pragma unroll
      for (int e = 0; e < E; ++e) DG::pack(canon_small<M>(rot_read_lds<N>(st, t + e * T, a) - acc[e]), pk[e]);
      __builtin_amdgcn_wave_barrier();
      __atomic_signal_fence(__ATOMIC_SEQ_CST);
    }
    double accA[E], accB[E];
#pragma unroll
    for (int e = 0; e < E; ++e) accA[e] = accB[e] = 0.0;
    KeyRow<double, E> cur;
    cur.load(ggsw, N, t * E);
    // digits in order (the throughput kernel's (j, j + 3) pairing measured 6 % slower here: its
    // row choice splits the loop body into blocks the scheduler cannot overlap)
#pragma unroll 1
    for (int k2 = 0; k2 < D2; k2 += 2) {
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int k = k2 + h;
        double x[E];
        int f[E];
#pragma unroll
        for (int e = 0; e < E; ++e) f[e] = DG::get_int(pk[e], k) + 64;
        if (h == 0)  // digits on X0, X1, X0, ...
          NTT::template fwd_small<0>(f, t0, x, X, tw, t, tw);
        else
          NTT::template fwd_small<1>(f, t0, x, X, tw, t, tw);
#pragma unroll
        for (int e = 0; e < E; ++e) {
          accA[e] += mm<M>(x[e], cur.a[e]);
          accB[e] += mm<M>(x[e], cur.b[e]);
        }
        if (k == 3) {  // four products on a reduced sum stay below 7.6q (cmux_step3)
#pragma unroll
          for (int e = 0; e < E; ++e) {
            accA[e] = red<M>(accA[e]);
            accB[e] = red<M>(accB[e]);
          }
        }
        if (k + 1 < D2) cur.load(ggsw + (size_t)(k + 1) * 2 * N, N, t * E);
      }
    }
    // exchange the partial the other group owns: group 0 sends B, group 1 sends A
#pragma unroll
    for (int e = 0; e < E; ++e) part[1 - g][e * T + t] = red<M>(g == 0 ? accB[e] : accA[e]);
    __syncthreads();
    double s[E];
#pragma unroll
    for (int e = 0; e < E; ++e) s[e] = red<M>(red<M>(g == 0 ? accA[e] : accB[e]) + part[g][e * T + t]);
    NTT::template inv<0>(s, X, tw, t, tw);
#pragma unroll
    for (int e = 0; e < E; ++e) acc[e] = canon<M>(acc[e] + s[e]);
  }
  uint64_t *o = out + (size_t)blockIdx.x * 2 * N + (size_t)g * N;
#pragma unroll
  for (int e = 0; e < E; ++e) o[t + e * T] = to_u64<M>(acc[e]);
}
__global__ __launch_bounds__(BR2L_T, 1) void br2l_kernel(const uint32_t *__restrict__ lwe_int,
                                                         const double *__restrict__ bsk2, DeviceTables tb,
                                                         uint64_t *__restrict__ out) {
  br2l_body(lwe_int, bsk2, tb, out);
}
// The exact fallback of a guarded throughput level-2 launch (context.hip, launch_br2): the same
// rotation on the modular NTT, run only when that launch's observed rounding margin reached the
// certificate threshold 1 - E2 (every workgroup reads the word and leaves otherwise).
__device__ __forceinline__ bool margin_breached(const unsigned long long *word, double thr) {
  return __longlong_as_double((long long)*word) >= thr;
}
__global__ __launch_bounds__(BR2L_T, 1) void br2l_fallback_kernel(const uint32_t *__restrict__ lwe_int,
                                                                  const double *__restrict__ bsk2, DeviceTables tb,
                                                                  uint64_t *__restrict__ out,
                                                                  const unsigned long long *lmargin, double thr) {
  if (!margin_breached(lmargin, thr)) return;
  br2l_body(lwe_int, bsk2, tb, out);
}

// ---- level 2 over two CUs per message --------------------------------------------------------
// Workgroup 2m + r owns polynomial r (0 mask, 1 body) of message m and its accumulator: its two
// 256-thread groups transform digits 3g .. 3g + 2 of that polynomial (GGSW rows r D2 + 3g + ..)
// and multiply-accumulate both outputs; group 1's partials join group 0's through LDS; the
// output the partner owns (mask CU: B, body CU: A) crosses to it through global memory and the
// partner's arrives the same way; group 0 runs the inverse transform and updates ACC_r. Half the
// transforms of br2l_kernel per CU and step, plus one hand-off.
// The hand-off slots are lane-contiguous (register e of thread t at e * 256 + t): each 8 B sc1 store
// or load instruction covers 512 B of four whole lines (profiles/r03q/handoff_layout_ab.log).
// Hand-off (MI355X_MICROARCH.md, inter-workgroup visibility, the first row of the sc1 table):
// every storing thread stores its payload with sc1 stores (agent-scope relaxed atomics) and waits
// vmcnt(0); a workgroup barrier; one lane stores the sc1 flag (step + 1). The consumer's lane 0
// polls the partner's flag with sc1 loads, a workgroup barrier follows, and every load of the
// payload is an sc1 load. Steps with a_i = 0 are skipped by both workgroups, so the hand-offs are
// numbered by a counter hc of EXECUTED steps: the flag carries hc + 1 and the payload slot is
// hc & 1. Consecutive hand-offs therefore alternate slots, and before a workgroup rewrites slot
// hc & 1 (at hand-off hc + 2) it has seen the partner's flag hc + 2, which the partner publishes
// only after its hand-off-hc read of that slot was consumed. The poll is bounded: after BR2X_SPIN
// polls the workgroup records an error in *err and leaves the loop, so every wave exits. The grid
// (2 workgroups per message, one per CU) must be co-resident: the host launches it with
// hipLaunchCooperativeKernel, which guarantees that or refuses the launch.
constexpr int BR2X_SPIN = 1 << 24;

__device__ __forceinline__ void st_sc1(double *p, double v) {
  __hip_atomic_store(reinterpret_cast<uint64_t *>(p), __builtin_bit_cast(uint64_t, v), __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ double ld_sc1(const double *p) {
  return __builtin_bit_cast(double, __hip_atomic_load(reinterpret_cast<const uint64_t *>(p), __ATOMIC_RELAXED,
                                                       __HIP_MEMORY_SCOPE_AGENT));
}

__global__ __launch_bounds__(BR2L_T, 1) void br2x_kernel(const uint32_t *__restrict__ lwe_int,
                                                         const double *__restrict__ bsk2, DeviceTables tb,
                                                         double *xg, uint32_t *flags, int *err,
                                                         uint64_t *__restrict__ out) {
  using M = Mod<2>;
  constexpr int T = BR2_T, E = BR2_E, N = N2;
  using NTT = CmuxNtt;
  using DG = Digits2;
  constexpr int KD = D2 / 2;  // digits per group
  __shared__ double xbuf[2][NTT::LDS_DOUBLES];
  __shared__ double part[2][N];
  __shared__ double tws[N + 136 * 5];
  __shared__ int stop;
  const int m = blockIdx.x >> 1, r = blockIdx.x & 1;
  const int g = threadIdx.x / T, t = threadIdx.x % T;
  double *X = xbuf[g];
  double *ST = xbuf[0] + N;  // the staged accumulator (group 0's X1), read by both groups
  // pass-0 twiddles read from the LDS copy too (gt = tw): from the global table they were vector
  // loads on every step's critical path (no restrict on DeviceTables' pointers, so no scalar loads)
  const double *tw = tws, *t0 = tws + N;
  const uint32_t *lwe = lwe_int + (size_t)m * (NI + 1);
  double acc[E];  // ACC_r, group 0 only
  {
    const int b = (int)lwe[NI];
    const int rr = (2 * N - (b % (2 * N))) % (2 * N);
#pragma unroll
    for (int e = 0; e < E; ++e) acc[e] = r == 1 ? canon_small<M>(rot_read<N>(tb.lut2, t + e * T, rr)) : 0.0;
    for (int j = threadIdx.x; j < N; j += BR2L_T) tws[j] = tb.tw2c[j];
    if (threadIdx.x <= 128) {  // table k: d * c_k, d = tid - 64 (c = tw1, tw2, tw1 tw2, tw3, tw1 tw3)
      const double w1 = tb.tw2[1], w2 = tb.tw2[2], w3 = tb.tw2[3];
      const double c[5] = {w1, w2, canon<M>(mm<M>(w1, w2)), w3, canon<M>(mm<M>(w1, w3))};
#pragma unroll
      for (int k = 0; k < 5; ++k)
        tws[N + 136 * k + threadIdx.x] = canon<M>(mm<M>((double)((int)threadIdx.x - 64), c[k]));
    }
    if (threadIdx.x == 0) stop = 0;
    __syncthreads();
  }
  uint32_t *my_flag = flags + 2 * m + r, *their_flag = flags + 2 * m + (1 - r);
  uint32_t hc = 0;  // hand-offs so far (executed steps)
  const int pslot = __builtin_amdgcn_readfirstlane(blockIdx.x < 2 ? 8 + 8 * (int)blockIdx.x + (int)(threadIdx.x >> 6) : -1);
  (void)pslot;
  OMR_PHASE_CLOCK(pslot, 0);
#pragma unroll 1
  for (int i = 0; i < NI; ++i) {
    const int a = (int)__builtin_amdgcn_readfirstlane(lwe[i]) & (2 * N - 1);
    if (a == 0) continue;  // (X^0 - 1) * ACC = 0 (both workgroups of the message skip it)
    OMR_PHASE(pslot, (int)hc, 0);
    const size_t slot = hc & 1;
    const double *ggsw = bsk2 + ((size_t)i * 2 * D2 + (size_t)r * D2 + (size_t)g * KD) * 2 * N;
    uint32_t pk[E][DG::DW];
    {  // digits of (X^a - 1) * ACC_r: group 0 stages ACC_r, both groups decompose it
      if (g == 0) {
#pragma unroll
        for (int e = 0; e < E; ++e) ST[t + e * T] = acc[e];
      }
      __syncthreads();
#pragma unroll
      for (int e = 0; e < E; ++e)
        DG::pack(canon_small<M>(rot_read_lds<N>(ST, t + e * T, a) - ST[t + e * T]), pk[e]);
      __builtin_amdgcn_wave_barrier();
      __atomic_signal_fence(__ATOMIC_SEQ_CST);
    }
    OMR_PHASE(pslot, (int)hc, 1);
    double accA[E], accB[E];
#pragma unroll
    for (int e = 0; e < E; ++e) accA[e] = accB[e] = 0.0;
    KeyRow<double, E> cur;
    cur.load(ggsw, N, t * E);
#pragma unroll
    for (int h = 0; h < KD; ++h) {  // three digits: X0, X1, X0 (the staging used group 0's X1)
      const int k = g * KD + h;
      double x[E];
      int f[E];
#pragma unroll
      for (int e = 0; e < E; ++e) f[e] = DG::get_int(pk[e], k) + 64;
      if ((h & 1) == 0)
        NTT::template fwd_small<0>(f, t0, x, X, tw, t, tw);
      else
        NTT::template fwd_small<1>(f, t0, x, X, tw, t, tw);
#pragma unroll
      for (int e = 0; e < E; ++e) {
        accA[e] += mm<M>(x[e], cur.a[e]);
        accB[e] += mm<M>(x[e], cur.b[e]);
      }
      if (h + 1 < KD) cur.load(ggsw + (size_t)(h + 1) * 2 * N, N, t * E);
    }
    // group 1's partials join group 0's (three products on a zero sum: |.| < 5.3q); part[] is
    // lane-contiguous (register e of thread t at e * 256 + t: no LDS bank conflicts)
    if (g == 1) {
#pragma unroll
      for (int e = 0; e < E; ++e) {
        part[0][e * T + t] = red<M>(accA[e]);
        part[1][e * T + t] = red<M>(accB[e]);
      }
    }
    __syncthreads();
    OMR_PHASE(pslot, (int)hc, 3);
    double keep[E];
    if (g == 0) {
#pragma unroll
      for (int e = 0; e < E; ++e) {
        const double sa = red<M>(red<M>(accA[e]) + part[0][e * T + t]);
        const double sb = red<M>(red<M>(accB[e]) + part[1][e * T + t]);
        keep[e] = r == 0 ? sa : sb;
        st_sc1(xg + (((size_t)m * 2 + r) * 2 + slot) * N + e * T + t, r == 0 ? sb : sa);  // the partner's output
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();
    OMR_PHASE(pslot, (int)hc, 4);
    if (threadIdx.x == 0) {
      __hip_atomic_store(my_flag, hc + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      int n = 0;
      while (__hip_atomic_load(their_flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < hc + 1) {
        if (++n == BR2X_SPIN) {
          stop = 1;
          atomicExch(err, 1);
          break;
        }
        __builtin_amdgcn_s_sleep(2);
      }
    }
    __syncthreads();
    OMR_PHASE(pslot, (int)hc, 5);
    if (stop) break;
    if (g == 0) {
      double s[E];
#pragma unroll
      for (int e = 0; e < E; ++e)
        s[e] = red<M>(keep[e] + ld_sc1(xg + (((size_t)m * 2 + (1 - r)) * 2 + slot) * N + e * T + t));
      NTT::template inv<0>(s, X, tw, t, tw);
      OMR_PHASE(pslot, (int)hc, 6);
#pragma unroll
      for (int e = 0; e < E; ++e) acc[e] = canon<M>(acc[e] + s[e]);
    } else {
      __syncthreads();  // the inverse's one workgroup barrier (its cross-wave exchange)
      OMR_PHASE(pslot, (int)hc, 6);
    }
    OMR_PHASE(pslot, (int)hc, 7);
    ++hc;
  }
  OMR_PHASE_CLOCK(pslot, 1);
  if (g == 0) {
    uint64_t *o = out + (size_t)m * 2 * N + (size_t)r * N;
#pragma unroll
    for (int e = 0; e < E; ++e) o[t + e * T] = to_u64<M>(acc[e]);
  }
}

// hom_trace (detector.rs:626-639) in place on blind-rotation outputs (coefficient domain,
// canonical u64 [2][N2] per message) -> NttRlweCiphertext u64 [2][N2].
__device__ __forceinline__ void trace_body(uint64_t *__restrict__ io, const double *__restrict__ tk, DeviceTables tb) {
  using M = Mod<2>;
  constexpr int T = BR2_T, E = BR2_E, N = N2;
  using NTT = WgNtt<M, T, E>;
  __shared__ double xch[NTT::LDS3_DOUBLES];
  __shared__ double tws[N];
  const int tid = threadIdx.x;
  uint64_t *o = io + (size_t)blockIdx.x * 2 * N;
  double acc0[E], acc1[E];
#pragma unroll
  for (int e = 0; e < E; ++e) {
    acc0[e] = from_u64<M>(o[tid + e * T]);
    acc1[e] = from_u64<M>(o[N + tid + e * T]);
    tws[tid + e * T] = tb.tw2[tid + e * T];
    xch[2 * N + tid + e * T] = tb.itw2[tid + e * T];
  }
  __syncthreads();
  hom_trace_store(acc0, acc1, xch, tws, xch + 2 * N, tk, tb, o, tid);
}
__global__ __launch_bounds__(BR2_T, 2) void trace_kernel(uint64_t *__restrict__ io, const double *__restrict__ tk,
                                                         DeviceTables tb) {
  trace_body(io, tk, tb);
}
// trace of br2l_fallback_kernel's output (same condition)
__global__ __launch_bounds__(BR2_T, 2) void trace_fallback_kernel(uint64_t *__restrict__ io, const double *__restrict__ tk,
                                                                  DeviceTables tb, const unsigned long long *lmargin,
                                                                  double thr) {
  if (!margin_breached(lmargin, thr)) return;
  trace_body(io, tk, tb);
}


// hom_trace of the latency path over TRACE_X workgroups (CUs) per message (trace_x_kernel): every
// workgroup keeps the mask and body (redundantly: the per-step updates are cheap), takes the 25
// digits of sigma_g(a) and transforms and multiply-accumulates only digits d = w, w + TRACE_X, ...;
// the partial sums (A, B), reduced, are all-reduced through global memory with br2x's rules (sc1
// stores, vmcnt(0), barrier, one flag per workgroup carrying the step + 1, a bounded poll of every
// partner's flag, sc1 loads; slot = step parity, reusable once every partner has published the
// next step), then every workgroup applies B to the body (NTT domain) and INTT(A) to the mask.
// Workgroup 0 stores NTT(c). The partials are canonicalised before the exchange, so their sum stays
// below TRACE_X q / 2 < 2^53, and the residues are canonicalised as in hom_trace_store: the output
// is bit-identical to it.
// Global slots: xg[m][w][slot][A / B][N2] doubles; flags[m][w].
#ifndef OMR_TRACE_X
#define OMR_TRACE_X 5
#endif
constexpr int TRACE_X = OMR_TRACE_X;  // 25 digits: 5 per workgroup
__global__ __launch_bounds__(BR2_T, 2) void trace_x_kernel(uint64_t *__restrict__ io, const double *__restrict__ tk,
                                                           DeviceTables tb, double *xg, uint32_t *flags, int *err) {
  using M = Mod<2>;
  constexpr int T = BR2_T, E = BR2_E, N = N2;
  using NTT = WgNtt<M, T, E>;
  __shared__ double xch[NTT::LDS_DOUBLES];
  __shared__ double tw[N], itw[N];
  __shared__ int stop;
  const int m = blockIdx.x / TRACE_X, w = blockIdx.x % TRACE_X;
  const int tid = threadIdx.x;
  uint64_t *o = io + (size_t)m * 2 * N;
  constexpr double NINV = -549755813880.0;  // 2048^-1 mod q2, centred (hom_trace_store)
  double ca[E], cb[E];
#pragma unroll
  for (int e = 0; e < E; ++e) {
    ca[e] = canon<M>(mm<M>(from_u64<M>(o[tid + e * T]), NINV));
    cb[e] = canon<M>(mm<M>(from_u64<M>(o[N + tid + e * T]), NINV));
    tw[tid + e * T] = tb.tw2[tid + e * T];
    itw[tid + e * T] = tb.itw2[tid + e * T];
  }
  if (tid == 0) stop = 0;
  __syncthreads();
  NTT::fwd(cb, xch, tw, tid);
#pragma unroll
  for (int e = 0; e < E; ++e) cb[e] = canon<M>(cb[e]);
  uint32_t *fl = flags + (size_t)m * TRACE_X;
#pragma unroll 1
  for (int k = 0; k < TRACE_STEPS; ++k) {
    const uint16_t *src = tb.trace_src + k * N;
    const uint16_t *perm = tb.trace_perm + k * N;
    uint32_t pk[E][DigitsTrace::DW];
#pragma unroll
    for (int e = 0; e < E; ++e) xch[tid + e * T] = ca[e];
    __syncthreads();
#pragma unroll
    for (int e = 0; e < E; ++e) {
      const int sidx = src[tid + e * T];
      DigitsTrace::pack(sidx < N ? xch[sidx] : -xch[sidx - N], pk[e]);  // sigma_g(a)
    }
    __syncthreads();
    double accA[E], accB[E];
#pragma unroll
    for (int e = 0; e < E; ++e) accA[e] = accB[e] = 0.0;
    const double *key = tk + (size_t)k * DT * 2 * N;
    int cnt = 0;
#pragma unroll 1
    for (int d = w; d < DT; d += TRACE_X) {
      const double *ka = key + (size_t)(d * 2) * N + tid * E;
      const double *kb = ka + N;
      double kra[E], krb[E];
#pragma unroll
      for (int e = 0; e < E; ++e) {
        kra[e] = ka[e];
        krb[e] = kb[e];
      }
      double x[E];
#pragma unroll
      for (int e = 0; e < E; ++e) x[e] = DigitsTrace::get(pk[e], d);
      NTT::fwd(x, xch, tw, tid);
#pragma unroll
      for (int e = 0; e < E; ++e) {
        accA[e] += mm<M>(x[e], kra[e]);
        accB[e] += mm<M>(x[e], krb[e]);
      }
      if ((++cnt % 3) == 0) {
#pragma unroll
        for (int e = 0; e < E; ++e) {
          accA[e] = red<M>(accA[e]);
          accB[e] = red<M>(accB[e]);
        }
      }
    }
    // all-reduce of the partials
    const size_t slot = k & 1;
#pragma unroll
    for (int e = 0; e < E; ++e) {
      accA[e] = red<M>(red<M>(accA[e]));  // canonical: TRACE_X of them sum below TRACE_X q / 2
      accB[e] = red<M>(red<M>(accB[e]));
      double *dst = xg + (((size_t)m * TRACE_X + w) * 2 + slot) * 2 * N + e * T + tid;  // lane-contiguous: 512 B per store instruction
      st_sc1(dst, accA[e]);
      st_sc1(dst + N, accB[e]);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) {
      __hip_atomic_store(fl + w, (uint32_t)(k + 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      for (int p = 0; p < TRACE_X && !stop; ++p) {
        if (p == w) continue;
        int n = 0;
        while (__hip_atomic_load(fl + p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < (uint32_t)(k + 1)) {
          if (++n == BR2X_SPIN) {
            stop = 1;
            atomicExch(err, 1);
            break;
          }
          __builtin_amdgcn_s_sleep(2);
        }
      }
    }
    __syncthreads();
    if (stop) break;
#pragma unroll
    for (int p = 0; p < TRACE_X; ++p) {
      if (p == w) continue;
      const double *srcp = xg + (((size_t)m * TRACE_X + p) * 2 + slot) * 2 * N + tid;
#pragma unroll
      for (int e = 0; e < E; ++e) {
        accA[e] += ld_sc1(srcp + e * T);
        accB[e] += ld_sc1(srcp + N + e * T);
      }
    }
    // b_ntt += sigma_g(b)_ntt + B
#pragma unroll
    for (int e = 0; e < E; ++e) xch[tid * E + e] = cb[e];
    __syncthreads();
#pragma unroll
    for (int e = 0; e < E; ++e) cb[e] = canon<M>(cb[e] + xch[perm[tid * E + e]] + red<M>(accB[e]));
    __syncthreads();
    // a += INTT(A) (the sum of partials canonicalised first: a tighter input than the one-group trace's)
#pragma unroll
    for (int e = 0; e < E; ++e) accA[e] = red<M>(red<M>(accA[e]));
    NTT::inv(accA, xch, itw, tid);
#pragma unroll
    for (int e = 0; e < E; ++e) ca[e] = canon<M>(ca[e] + accA[e]);
  }
  if (w != 0 || stop) return;
  NTT::fwd(ca, xch, tw, tid);
#pragma unroll
  for (int e = 0; e < E; ++e) {
    const int t = tid * E + e;
    o[t] = to_u64<M>(canon<M>(ca[e]));
    o[N + t] = to_u64<M>(cb[e]);
  }
}

}  // namespace omr

#include "ks_mfma.hpp"

namespace omr {

// ---- key switch, split over the input coefficients -------------------------------------------
constexpr int KS_SPLIT = 32;  // slices of the 1024 input coefficients

// grid (ceil(B / 64), 21, KS_SPLIT): ks_mfma_kernel's tile over input coefficients
// [z * 1024 / KS_SPLIT, (z + 1) * 1024 / KS_SPLIT); int32 limb sums to part[z][m][col][limb].
__global__ __launch_bounds__(64, 2) void ks_mfma_split_kernel(const uint32_t *__restrict__ lwe1t,
                                                           const uint32_t *__restrict__ kskb,
                                                           int *__restrict__ part, int B, int Bpad) {
  const int lane = threadIdx.x, r = lane & 31, h = lane >> 5;
  const int m0 = blockIdx.x * 64, c0 = blockIdx.y * 32, z = blockIdx.z;
  omr_v16i acc[2][KSM_LIMBS];
#pragma unroll
  for (int tt = 0; tt < 2; ++tt)
#pragma unroll
    for (int l = 0; l < KSM_LIMBS; ++l) acc[tt][l] = omr_v16i{};
  const bool live0 = m0 + r < B, live1 = m0 + 32 + r < B;
  const omr_v4i *bbase = reinterpret_cast<const omr_v4i *>(kskb) + (size_t)(c0 + r) * 2 + h;
  constexpr int SL = N1 / KS_SPLIT;
#pragma unroll 1
  for (int i = z * SL; i < (z + 1) * SL; ++i) {
    const uint32_t x0 = live0 ? lwe1t[(size_t)i * B + m0 + r] : 0u;
    const uint32_t x1 = live1 ? lwe1t[(size_t)i * B + m0 + 32 + r] : 0u;
    const omr_v4i a0 = bit_bytes16(x0, 16 * h), a1 = bit_bytes16(x1, 16 * h);
#pragma unroll
    for (int l = 0; l < KSM_LIMBS; ++l) {
      const omr_v4i bv = bbase[((size_t)i * KSM_LIMBS + l) * KSM_COLS * 2];
      acc[0][l] = __builtin_amdgcn_mfma_i32_32x32x32_i8(a0, bv, acc[0][l], 0, 0, 0);
      acc[1][l] = __builtin_amdgcn_mfma_i32_32x32x32_i8(a1, bv, acc[1][l], 0, 0, 0);
    }
  }
  const int col = c0 + r;
#pragma unroll
  for (int tt = 0; tt < 2; ++tt)
#pragma unroll
    for (int reg = 0; reg < 16; ++reg) {
      const int m = m0 + 32 * tt + (reg & 3) + 8 * (reg >> 2) + 4 * h;
      int *p = part + (((size_t)z * Bpad + m) * KSM_COLS + col) * KSM_LIMBS;
#pragma unroll
      for (int l = 0; l < KSM_LIMBS; ++l) p[l] = acc[tt][l][reg];
    }
}

// Sum of the slices and ks_mfma_kernel's epilogue: one thread per (message, output column).
__global__ void ks_combine_kernel(const int *__restrict__ part, const uint32_t *__restrict__ lwe1t,
                                  uint32_t *__restrict__ lwe_int, int B, int Bpad) {
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= B * (NI + 1)) return;
  const int m = idx / (NI + 1), col = idx % (NI + 1);
  int64_t limb[KSM_LIMBS] = {0, 0, 0, 0};
  for (int z = 0; z < KS_SPLIT; ++z) {
    const int *p = part + (((size_t)z * Bpad + m) * KSM_COLS + col) * KSM_LIMBS;
#pragma unroll
    for (int l = 0; l < KSM_LIMBS; ++l) limb[l] += p[l];
  }
  const uint64_t sum = (uint64_t)limb[0] + ((uint64_t)limb[1] << 7) + ((uint64_t)limb[2] << 14) +
                       ((uint64_t)limb[3] << 21);
  lwe_int[(size_t)m * (NI + 1) + col] = ks_epilogue(sum, lwe1t[(size_t)N1 * B + m], col);
}

}  // namespace omr
