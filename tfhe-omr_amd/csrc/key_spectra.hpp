// Key spectra of the FFT blind rotations in double-double (context creation; exactness.hpp).
// Replaces the FP64 key transforms of rounds 1-3 (key_to_fft1_kernel / key_to_fft2_kernel, still
// used by the test entry omr_fft1_mul): the stored spectrum of every key polynomial is the exact
// transform rounded once to FP64, which the a priori error bound of DESIGN.md §3 relies on.
#pragma once

#include "br2_fft.hpp"
#include "exactness.hpp"

namespace omr {

// One workgroup per key polynomial (level 1) or per (polynomial, limb) (level 2).
template <int LEVEL>
__global__ __launch_bounds__(KDD_T) void key_spectrum_dd_kernel(const void *__restrict__ in_v, double2 *__restrict__ out,
                                                                size_t npoly, const CDD *__restrict__ tw) {
  constexpr int L = LEVEL == 1 ? 9 : 10, n = 1 << L;
  __shared__ double rh[n], rl[n], ih[n], il[n];
  const int t = threadIdx.x;
  const size_t poly = LEVEL == 1 ? blockIdx.x : blockIdx.x >> 1;
  const int limb = LEVEL == 1 ? 0 : (int)(blockIdx.x & 1);
  if (poly >= npoly) return;
  for (int j = t; j < n; j += KDD_T) {
    double re, im;
    if constexpr (LEVEL == 1) {
      const uint32_t *src = static_cast<const uint32_t *>(in_v) + poly * N1;
      re = from_u64<Mod<1>>(src[j]);
      im = from_u64<Mod<1>>(src[j + n]);
    } else {  // the limb split of br2_fft.hpp (k = lo + 2^25 hi, |lo|, |hi| <= 2^24)
      const uint64_t *src = static_cast<const uint64_t *>(in_v) + poly * N2;
      double v[2];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const double k = from_u64<Mod<2>>(src[j + h * n]);
        const double hi = rint(k * (1.0 / LIMB));
        v[h] = limb ? hi : __fma_rn(-hi, LIMB, k);
      }
      re = v[0];
      im = v[1];
    }
    rh[j] = re;
    rl[j] = 0.0;
    ih[j] = im;
    il[j] = 0.0;
  }
  __syncthreads();
  dd_tree_fft<L>(rh, rl, ih, il, tw, t);
  // slot -> spectral index: level 1 key1_pos(lane, e) = e * 64 + lane holds jidx(3, lane, e);
  // level 2 key_pos(t', e) = e * 256 + t' holds idx(4, t', e)
  double2 *dst = out + (poly * (LEVEL == 1 ? 1 : 2) + limb) * n;
  for (int slot = t; slot < n; slot += KDD_T) {
    int j;
    if constexpr (LEVEL == 1)
      j = Fft512::jidx(3, slot & 63, slot >> 6);
    else
      j = Fft1024::idx(4, slot & 255, slot >> 8);
    // a normalised double-double's hi is its value rounded to the nearest double; 1/n is exact
    dst[slot] = make_double2(rh[j] * (1.0 / n), ih[j] * (1.0 / n));
  }
}

}  // namespace omr
