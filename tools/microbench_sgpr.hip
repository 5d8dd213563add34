// Issue cost of an FP64 FMA whose multiplier is an SGPR pair vs a VGPR pair, and the FP64 rate one,
// two and four waves per SIMD reach with CH independent FMA chains per lane (round 6: the level-1
// twiddle experiments). The multiplier is either wave-uniform in SGPRs ("s"
// constraint) or held in a VGPR pair ("v" constraint); UNR rounds of the CH chains per loop
// iteration keep the branch out of the measurement. 256 x 4 x W waves (W waves per SIMD).
//   hipcc -O3 --offload-arch=gfx950 tools/microbench_sgpr.hip -o tools/microbench_sgpr
#include <hip/hip_runtime.h>

#include <cstdio>

constexpr int ITER = 512, UNR = 16;

template <bool SGPR, int CH>
__global__ void k_fma(double *out, double w0) {
  double v[CH];
  for (int c = 0; c < CH; ++c) v[c] = threadIdx.x + c;
  const double w = w0;  // kernel argument: uniform, in SGPRs unless copied
  double wv;
  asm volatile("v_mov_b64 %0, %1" : "=v"(wv) : "s"(w));  // a VGPR copy
#pragma unroll 1
  for (int i = 0; i < ITER; ++i) {
#pragma unroll
    for (int c = 0; c < CH * UNR; ++c) {
      if constexpr (SGPR)
        asm volatile("v_fma_f64 %0, %0, %1, 0.5" : "+v"(v[c % CH]) : "s"(w));
      else
        asm volatile("v_fma_f64 %0, %0, %1, 0.5" : "+v"(v[c % CH]) : "v"(wv));
    }
  }
  double r = 0;
  for (int c = 0; c < CH; ++c) r += v[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

int main() {
  int cus = 0;
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  double *buf;
  (void)hipMalloc(&buf, (size_t)cus * 4 * 1024 * sizeof(double));
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  auto run = [&](auto kern, int wps, const char *what, int ch) {
    float best = 1e30f;
    for (int rep = 0; rep < 3; ++rep) {
      (void)hipEventRecord(a);
      kern<<<cus * wps, 256>>>(buf, 1.0000001);
      (void)hipEventRecord(b);
      (void)hipEventSynchronize(b);
      float ms;
      (void)hipEventElapsedTime(&ms, a, b);
      best = ms < best ? ms : best;
    }
    const double fmas = (double)cus * wps * 256 * ITER * UNR * ch;
    printf("waves/SIMD %d  chains %2d  multiplier in %s: %.3f ms  %.1f G lane-FMA/s  (%.2f cycles per wave-FMA per SIMD at 2.4 GHz; 4 = FP64 peak)\n",
           wps, ch, what, best, fmas / (best * 1e6), (best * 1e-3 * 2.4e9) / (fmas / 64 / (cus * 4)));
  };
  for (int wps = 1; wps <= 4; wps *= 2) {
    run(k_fma<false, 8>, wps, "VGPR", 8);
    run(k_fma<true, 8>, wps, "SGPR", 8);
    run(k_fma<false, 16>, wps, "VGPR", 16);
    run(k_fma<true, 16>, wps, "SGPR", 16);
  }
  (void)hipFree(buf);
  return 0;
}
