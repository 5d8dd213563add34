// Exactness of the FFT external products ("Worst-case error bound").
//
// Both throughput blind rotations (br1_fft.hpp, br2_fft.hpp) and the latency level 1
// (latency_kernels.hpp) compute sum_r digit_r * key_r with FP64 complex FFTs and round the
// result to the integer it equals. This header holds the three pieces that make that rounding
// provably exact rather than empirically so:
//  - key spectra in double-double: the keys are transformed once, at context creation, by a
//    radix-2 tree FFT in double-double arithmetic with double-double twiddles (accuracy ~2^-100)
//    and rounded once to FP64, so every stored spectral value K^ obeys |K^ - K| <= u |K| (u = 2^-53)
//    instead of carrying an FP64 transform error (key_spectrum_dd_kernel);
//  - kappa_r, the largest |K^| of every stored key row (row_max_abs_kernel): the only key-dependent
//    constants of the a priori bound on |computed - exact| of every rounded product coefficient,
//    E = n D max over steps and outputs of [(2 delta_f + u') sum_r kappa_r + sqrt(2) u sum_k w_k
//    kappa_r(k)] (context.hip: apriori_bound);
//  - the rounding-margin guard (RoundGuard): the guarded kernel variants record the largest
//    |y - rint(y)| over every rounded product coefficient and publish it with one 64-bit atomic
//    max per wave. If E < 0.5 the rounding is exact for every input; otherwise a run whose
//    observed margin m satisfies m < 1 - E is certified exact (an error of 0.5 <= |e| <= E < 1
//    would show as a margin of 1 - |e| >= 1 - E).
#pragma once

#include "common.hpp"

namespace omr {

// ---- double-double arithmetic (Dekker / Knuth; -ffp-contract=off keeps it exact) ----
struct DD {
  double hi, lo;
};
OMR_HD DD dd_two_sum(double a, double b) {
  const double s = a + b, bb = s - a;
  return {s, (a - (s - bb)) + (b - bb)};
}
OMR_HD DD dd_quick(double a, double b) {  // |a| >= |b|
  const double s = a + b;
  return {s, b - (s - a)};
}
OMR_HD DD dd_add(DD a, DD b) {
  DD s = dd_two_sum(a.hi, b.hi);
  const DD t = dd_two_sum(a.lo, b.lo);
  s.lo += t.hi;
  s = dd_quick(s.hi, s.lo);
  s.lo += t.lo;
  return dd_quick(s.hi, s.lo);
}
OMR_HD DD dd_neg(DD a) { return {-a.hi, -a.lo}; }
OMR_HD DD dd_mul(DD a, DD b) {
  const double p = a.hi * b.hi;
  double e = fma(a.hi, b.hi, -p);
  e += a.hi * b.lo + a.lo * b.hi;
  return dd_quick(p, e);
}
struct CDD {
  DD re, im;
};
OMR_HD CDD cdd_add(CDD a, CDD b) { return {dd_add(a.re, b.re), dd_add(a.im, b.im)}; }
OMR_HD CDD cdd_sub(CDD a, CDD b) { return {dd_add(a.re, dd_neg(b.re)), dd_add(a.im, dd_neg(b.im))}; }
OMR_HD CDD cdd_mul(CDD a, CDD b) {
  return {dd_add(dd_mul(a.re, b.re), dd_neg(dd_mul(a.im, b.im))), dd_add(dd_mul(a.re, b.im), dd_mul(a.im, b.re))};
}

// ---- key spectra in double-double -------------------------------------------------------------
// The transforms of device_fft.hpp (Fft512) and br2_fft.hpp (Fft1024) are Cooley-Tukey trees in
// natural index order: stage s (0 .. L-1) splits on index bit L-1-s, node i (the top s bits) has
// twiddle W(s, i) = w^(eps(s, i) / 2) with w = exp(i pi / 2n), and the butterfly on the pair
// (j, j + 2^(L-1-s)) is (x_j + W x_{j'}, x_j - W x_{j'}). Their radix-8/4/2 passes are blocks of
// this tree (fft2_model.py's docstring shows the radix-4 identity), so output index j is the same
// spectral value here. tw: [n - 1] CDD, stage s node i at (1 << s) - 1 + i (built on the host).
// LEVEL 1: u32 canonical keys mod q1, z_j = p_j + i p_{j+512}, out = K / 512 at key1_pos(lane, e)
//          for index jidx(3, lane, e) (br1f_kernel's layout, [npoly][512] double2).
// LEVEL 2: u64 canonical keys mod q2 split into centred 25-bit limbs k = lo + 2^25 hi, each limb
//          transformed, out[poly][limb] = K / 1024 at key_pos(t, e) for index idx(4, t, e)
//          (br2f_kernel's layout, [npoly][2][1024] double2).
constexpr int KDD_T = 256;

template <int L>
__device__ __forceinline__ void dd_tree_fft(double *rh, double *rl, double *ih, double *il, const CDD *__restrict__ tw,
                                            int t) {
  constexpr int n = 1 << L;
#pragma unroll 1
  for (int s = 0; s < L; ++s) {
    const int lh = L - 1 - s, h = 1 << lh;
    for (int p = t; p < n / 2; p += KDD_T) {
      const int blk = p >> lh, j = (blk << (lh + 1)) | (p & (h - 1)), j1 = j + h;
      const CDD w = tw[(1 << s) - 1 + blk];
      const CDD x0 = {{rh[j], rl[j]}, {ih[j], il[j]}}, x1 = {{rh[j1], rl[j1]}, {ih[j1], il[j1]}};
      const CDD v = cdd_mul(w, x1), a = cdd_add(x0, v), b = cdd_sub(x0, v);
      rh[j] = a.re.hi;
      rl[j] = a.re.lo;
      ih[j] = a.im.hi;
      il[j] = a.im.lo;
      rh[j1] = b.re.hi;
      rl[j1] = b.re.lo;
      ih[j1] = b.im.hi;
      il[j1] = b.im.lo;
    }
    __syncthreads();
  }
}

// Largest |z| of n complex values, published as the bits of a non-negative double (which order
// like the value) with one 64-bit atomic max per wave.
__device__ __forceinline__ void wave_max_publish(double v, unsigned long long *word) {
#pragma unroll
  for (int off = 32; off; off >>= 1) v = fmax(v, __shfl_xor(v, off));
  if ((threadIdx.x & 63) == 0) atomicMax(word, (unsigned long long)__double_as_longlong(v));
}
// Largest |K^| of each stored key-spectrum row (len complex values; one workgroup per row):
// kappa_r of the a priori bound, rounded up past sqrt's error.
__global__ __launch_bounds__(256) void row_max_abs_kernel(const double2 *__restrict__ x, int len,
                                                          double *__restrict__ out) {
  __shared__ double wm[4];
  const double2 *row = x + (size_t)blockIdx.x * len;
  double m = 0.0;
  for (int i = threadIdx.x; i < len; i += 256) {
    const double2 v = row[i];
    m = fmax(m, sqrt(v.x * v.x + v.y * v.y) * (1.0 + 0x1p-50));
  }
#pragma unroll
  for (int off = 32; off; off >>= 1) m = fmax(m, __shfl_xor(m, off));
  if ((threadIdx.x & 63) == 0) wm[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0) out[blockIdx.x] = fmax(fmax(wm[0], wm[1]), fmax(wm[2], wm[3]));
}

// ---- rounding-margin guard ----------------------------------------------------------------------
// RoundGuard<true>::note(y, r) keeps max |y - r| (r = the integer y was rounded to); publish()
// leaves it in *word (one atomic per wave). RoundGuard<false> compiles to nothing: the production
// kernels are the G = false instantiations, the guarded ones separate kernels (context.hip).
template <bool G>
struct RoundGuard {
  double m = 0.0;
  __device__ __forceinline__ void note(double y, double r) {
    if constexpr (G) m = fmax(m, fabs(y - r));
  }
  __device__ __forceinline__ void publish(unsigned long long *word) {
    if constexpr (G) wave_max_publish(m, word);
  }
};

// ---- the exactness contract of a context (context.hip) -----------------------------------------
// Guard words per context: [0, 1] the largest margin of levels 1, 2 since the last reset (what
// omr_ctx_rounding_margin reports), [2, 3] the margin of the launch in flight (zeroed before each
// guarded launch, written by its kernels), [4, 5] the number of launches whose margin reached the
// threshold 1 - E (that launch was then re-run on the exact NTT: br1n_fallback_kernel,
// br2l_fallback_kernel + trace_fallback_kernel).
constexpr int GUARD_WORDS = 6;
constexpr int GUARD_ERR_HANDOFF = 1;  // bit of the context's error word: a two-CU hand-off timed out
__global__ void guard_fold_kernel(unsigned long long *words, int level, double thr) {
  if (threadIdx.x != 0) return;
  const unsigned long long m = words[2 + level];
  atomicMax(&words[level], m);
  if (__longlong_as_double((long long)m) >= thr) atomicAdd(&words[4 + level], 1ull);
}

}  // namespace omr
