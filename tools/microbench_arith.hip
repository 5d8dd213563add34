// Instruction-throughput microbenchmark for the modular-arithmetic choices of the
// detect path on gfx950: 32-bit Shoup, 64-bit Shoup (integer), FP64 exact modmul.
// Reports Gop/s (modmuls per second over the whole chip).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cmath>

#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

constexpr int ITER = 1024;
constexpr int CH = 8;

__global__ void k_mul_lo_u32(uint32_t* out, uint32_t s) {
  uint32_t v[CH];
  for (int c = 0; c < CH; ++c) v[c] = threadIdx.x + c * 77 + s;
  for (int i = 0; i < ITER; ++i)
#pragma unroll
    for (int c = 0; c < CH; ++c) v[c] = v[c] * (v[c] | 1u);
  uint32_t r = 0; for (int c = 0; c < CH; ++c) r ^= v[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}
__global__ void k_mul_hi_u32(uint32_t* out, uint32_t s) {
  uint32_t v[CH];
  for (int c = 0; c < CH; ++c) v[c] = threadIdx.x + c * 77 + s;
  for (int i = 0; i < ITER; ++i)
#pragma unroll
    for (int c = 0; c < CH; ++c) v[c] = __umulhi(v[c], s) + v[c];
  uint32_t r = 0; for (int c = 0; c < CH; ++c) r ^= v[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}
__global__ void k_mul_u24(uint32_t* out, uint32_t s) {
  uint32_t v[CH];
  for (int c = 0; c < CH; ++c) v[c] = threadIdx.x + c * 77 + s;
  for (int i = 0; i < ITER; ++i)
#pragma unroll
    for (int c = 0; c < CH; ++c) v[c] = (uint32_t)__mul24((int)v[c], (int)s) + 1u;
  uint32_t r = 0; for (int c = 0; c < CH; ++c) r ^= v[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}
__global__ void k_add_u32(uint32_t* out, uint32_t s) {
  uint32_t v[CH];
  for (int c = 0; c < CH; ++c) v[c] = threadIdx.x + c * 77 + s;
  for (int i = 0; i < ITER; ++i)
#pragma unroll
    for (int c = 0; c < CH; ++c) v[c] = (v[c] + s) ^ c;
  uint32_t r = 0; for (int c = 0; c < CH; ++c) r ^= v[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}
// 32-bit Shoup modmul: r = a*w - umulhi(a, w')*q, lazy in [0,2q)
__global__ void k_shoup32(uint32_t* out, uint32_t w, uint32_t wp, uint32_t q) {
  uint32_t v[CH];
  for (int c = 0; c < CH; ++c) v[c] = (threadIdx.x + c * 77) % q;
  for (int i = 0; i < ITER; ++i)
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      uint32_t a = v[c];
      uint32_t qe = __umulhi(a, wp);
      uint32_t r = a * w - qe * q;
      v[c] = r >= q ? r - q : r;
    }
  uint32_t r = 0; for (int c = 0; c < CH; ++c) r ^= v[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}
// 64-bit Shoup modmul (q < 2^62)
__global__ void k_shoup64(uint64_t* out, uint64_t w, uint64_t wp, uint64_t q) {
  uint64_t v[CH];
  for (int c = 0; c < CH; ++c) v[c] = (threadIdx.x + c * 7777ull) % q;
  for (int i = 0; i < ITER; ++i)
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      uint64_t a = v[c];
      uint64_t qe = __umul64hi(a, wp);
      uint64_t r = a * w - qe * q;
      v[c] = r >= q ? r - q : r;
    }
  uint64_t r = 0; for (int c = 0; c < CH; ++c) r ^= v[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}
// FP64 exact modmul (q < 2^50): h=a*w, l=fma(a,w,-h), qe=rint(h*qi), r=fma(-qe,q,h)+l
__global__ void k_fp64mm(double* out, double w, double q, double qi) {
  double v[CH];
  for (int c = 0; c < CH; ++c) v[c] = (double)((threadIdx.x + c * 7777ull) % (1ull << 40));
  for (int i = 0; i < ITER; ++i)
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      double a = v[c];
      double h = a * w;
      double l = __fma_rn(a, w, -h);
      double qe = rint(h * qi);
      double r = __fma_rn(-qe, q, h) + l;
      v[c] = r;
    }
  double r = 0; for (int c = 0; c < CH; ++c) r += v[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}
// FP64 modmul with magic-number rounding instead of rint
__global__ void k_fp64mm_magic(double* out, double w, double q, double qi) {
  const double M = 6755399441055744.0;  // 1.5*2^52
  double v[CH];
  for (int c = 0; c < CH; ++c) v[c] = (double)((threadIdx.x + c * 7777ull) % (1ull << 40));
  for (int i = 0; i < ITER; ++i)
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      double a = v[c];
      double h = a * w;
      double l = __fma_rn(a, w, -h);
      double qe = __fma_rn(h, qi, M) - M;
      double r = __fma_rn(-qe, q, h) + l;
      v[c] = r;
    }
  double r = 0; for (int c = 0; c < CH; ++c) r += v[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}
__global__ void k_fma64(double* out, double w) {
  double v[CH];
  for (int c = 0; c < CH; ++c) v[c] = threadIdx.x + c;
  for (int i = 0; i < ITER; ++i)
#pragma unroll
    for (int c = 0; c < CH; ++c) v[c] = __fma_rn(v[c], w, 0.5);
  double r = 0; for (int c = 0; c < CH; ++c) r += v[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}
__global__ void k_fma32(float* out, float w) {
  float v[CH];
  for (int c = 0; c < CH; ++c) v[c] = threadIdx.x + c;
  for (int i = 0; i < ITER; ++i)
#pragma unroll
    for (int c = 0; c < CH; ++c) v[c] = __fmaf_rn(v[c], w, 0.5f);
  float r = 0; for (int c = 0; c < CH; ++c) r += v[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

template <typename F>
double timeit(F f, int reps) {
  hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
  f(); hipDeviceSynchronize();
  hipEventRecord(a);
  for (int i = 0; i < reps; ++i) f();
  hipEventRecord(b); hipEventSynchronize(b);
  float ms; hipEventElapsedTime(&ms, a, b);
  return ms / reps;
}

int main() {
  const int blocks = 256 * 16, threads = 256;
  const double nops = (double)blocks * threads * ITER * CH;
  void* buf; CHK(hipMalloc(&buf, (size_t)blocks * threads * 8));
  const uint32_t q1 = 134215681u; const uint64_t q2 = 1125899906826241ull;
  uint32_t w1 = 12345677u; uint32_t w1p = (uint32_t)(((uint64_t)w1 << 32) / q1);
  uint64_t w2 = 987654321987ull; uint64_t w2p = (uint64_t)(((unsigned __int128)w2 << 64) / q2);
  struct { const char* name; double ms; } r[16]; int n = 0;
#define RUN(NAME, ...) r[n].name = NAME; r[n].ms = timeit([&]{ hipLaunchKernelGGL(__VA_ARGS__); }, 5); ++n;
  RUN("mul_lo_u32", k_mul_lo_u32, dim3(blocks), dim3(threads), 0, 0, (uint32_t*)buf, 3u)
  RUN("mul_hi_u32(+add)", k_mul_hi_u32, dim3(blocks), dim3(threads), 0, 0, (uint32_t*)buf, 3u)
  RUN("mul_u24", k_mul_u24, dim3(blocks), dim3(threads), 0, 0, (uint32_t*)buf, 3u)
  RUN("add+xor_u32", k_add_u32, dim3(blocks), dim3(threads), 0, 0, (uint32_t*)buf, 3u)
  RUN("shoup32 modmul", k_shoup32, dim3(blocks), dim3(threads), 0, 0, (uint32_t*)buf, w1, w1p, q1)
  RUN("shoup64 modmul", k_shoup64, dim3(blocks), dim3(threads), 0, 0, (uint64_t*)buf, w2, w2p, q2)
  RUN("fp64 modmul rint", k_fp64mm, dim3(blocks), dim3(threads), 0, 0, (double*)buf, (double)w2, (double)q2, 1.0 / (double)q2)
  RUN("fp64 modmul magic", k_fp64mm_magic, dim3(blocks), dim3(threads), 0, 0, (double*)buf, (double)w2, (double)q2, 1.0 / (double)q2)
  RUN("fma_f64", k_fma64, dim3(blocks), dim3(threads), 0, 0, (double*)buf, 1.0000001)
  RUN("fma_f32", k_fma32, dim3(blocks), dim3(threads), 0, 0, (float*)buf, 1.0000001f)
  hipDeviceProp_t p; hipGetDeviceProperties(&p, 0);
  printf("device %s CUs %d clock %d kHz\n", p.gcnArchName, p.multiProcessorCount, p.clockRate);
  for (int i = 0; i < n; ++i)
    printf("%-22s %8.3f ms  %9.1f Gop/s (per lane-op)\n", r[i].name, r[i].ms, nops / (r[i].ms * 1e6));
  return 0;
}
