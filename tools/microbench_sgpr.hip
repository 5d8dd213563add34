// Issue cost of an FP64 FMA whose multiplier is an SGPR pair vs a VGPR pair (round 6: the level-1
// twiddle experiments). Each lane runs 8 independent FMA chains (enough ILP to keep
// the FP64 pipe busy); the multiplier is either wave-uniform in SGPRs ("s" constraint) or held in a
// VGPR pair ("v" constraint). 256 x 4 x W waves (W waves per SIMD).
//   hipcc -O3 --offload-arch=gfx950 tools/microbench_sgpr.hip -o tools/microbench_sgpr
#include <hip/hip_runtime.h>

#include <cstdio>

constexpr int ITER = 4096, CH = 8;

template <bool SGPR>
__global__ void k_fma(double *out, double w0) {
  double v[CH];
  for (int c = 0; c < CH; ++c) v[c] = threadIdx.x + c;
  const double w = w0;  // kernel argument: uniform, in SGPRs unless copied
  double wv;
  asm volatile("v_mov_b64 %0, %1" : "=v"(wv) : "s"(w));  // a VGPR copy
#pragma unroll 1
  for (int i = 0; i < ITER; ++i) {
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      if constexpr (SGPR)
        asm volatile("v_fma_f64 %0, %0, %1, 0.5" : "+v"(v[c]) : "s"(w));
      else
        asm volatile("v_fma_f64 %0, %0, %1, 0.5" : "+v"(v[c]) : "v"(wv));
    }
  }
  double r = 0;
  for (int c = 0; c < CH; ++c) r += v[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

int main() {
  int cus = 0;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  double *buf;
  hipMalloc(&buf, (size_t)cus * 4 * 1024 * sizeof(double));
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  for (int wps = 1; wps <= 4; wps *= 2) {  // waves per SIMD: blocks of 256 threads, wps per CU
    for (int s = 0; s < 2; ++s) {
      float best = 1e30f;
      for (int rep = 0; rep < 3; ++rep) {
        hipEventRecord(a);
        if (s)
          k_fma<true><<<cus * wps, 256>>>(buf, 1.0000001);
        else
          k_fma<false><<<cus * wps, 256>>>(buf, 1.0000001);
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms;
        hipEventElapsedTime(&ms, a, b);
        best = ms < best ? ms : best;
      }
      const double fmas = (double)cus * wps * 256 * ITER * CH;
      printf("waves/SIMD %d  multiplier in %s: %.3f ms  %.1f G lane-FMA/s  (%.2f cycles per wave-FMA per SIMD at 2.4 GHz)\n",
             wps, s ? "SGPR" : "VGPR", best, fmas / (best * 1e6), (best * 1e-3 * 2.4e9) / (fmas / 64 / (cus * 4)));
    }
  }
  hipFree(buf);
  return 0;
}
