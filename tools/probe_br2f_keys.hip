// Feasibility probe for a level-2 blind rotation on the complex FFT (two 25-bit key limbs):
// can a 256-thread workgroup per message stream 768 KB of FFT-domain key per CMUX step (twice
// the NTT key's bytes) at the FFT's compute rate? Each step reads 12 rows x 4 (output, limb)
// blocks of 1,024 double2, thread t reading points 4t..4t+3 of each block (16 dwordx4 loads per
// row), and spends `work` FP64 FMAs per row on them plus two workgroup barriers (the exchanges).
// Modes: 0 no key loads (compute only), 1 one message per 256-thread workgroup (2 per CU),
// 2 two messages per 512-thread workgroup whose halves read the same rows in lockstep (L1
// sharing). Prints ms per launch of `msgs` messages and the key bytes per message-step.
//   hipcc -O3 --offload-arch=gfx950 tools/probe_br2f_keys.hip -o tools/probe_br2f_keys
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CHK(x)                                                                      \
  do {                                                                              \
    hipError_t e = (x);                                                             \
    if (e != hipSuccess) {                                                          \
      printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__);               \
      return 1;                                                                     \
    }                                                                               \
  } while (0)

constexpr int ROWS = 12, BLK = 4, PTS = 1024, STEP_D2 = ROWS * BLK * PTS;  // double2 per step

// MODE 3: the NTT design's key bytes (2 blocks per row, 384 KB per step) for calibration
template <int MODE>
__global__ __launch_bounds__(MODE == 2 ? 512 : 256, MODE == 2 ? 1 : 2) void probe(const double2 *__restrict__ key,
                                                                                  double *out, int steps, int work) {
  constexpr int NB = MODE == 3 ? 2 : BLK;
  const int t = threadIdx.x & 255;
  __shared__ double sink[512];
  double acc[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) acc[i] = 1.0 + 1e-9 * (threadIdx.x + i);
  double2 k[BLK][4];
#pragma unroll 1
  for (int s = 0; s < steps; ++s) {
#pragma unroll 1
    for (int r = 0; r < ROWS; ++r) {
      if (MODE != 0) {
        const double2 *row = key + (size_t)s * STEP_D2 + (size_t)r * NB * PTS + t * 4;
#pragma unroll
        for (int b = 0; b < BLK; ++b)
#pragma unroll
          for (int e = 0; e < 4; ++e) k[b][e] = row[(b % NB) * PTS + e];
      } else {
#pragma unroll
        for (int b = 0; b < BLK; ++b)
#pragma unroll
          for (int e = 0; e < 4; ++e) k[b][e] = make_double2(1e-9 * (b + e + r), 1e-9 * (s + e));
      }
      // the FFT's FP64 work per row, 8 independent chains, consuming the key
#pragma unroll 1
      for (int w = 0; w < work; w += 32) {
#pragma unroll
        for (int i = 0; i < 8; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j) acc[i] = __fma_rn(acc[i], 0.999999, 1e-12);
      }
#pragma unroll
      for (int b = 0; b < BLK; ++b)
#pragma unroll
        for (int e = 0; e < 4; ++e) acc[(b * 4 + e) & 7] = __fma_rn(k[b][e].x, k[b][e].y, acc[(b * 4 + e) & 7]);
      __syncthreads();  // the transform's cross-wave exchange
      sink[threadIdx.x & 511] = acc[0];
      __syncthreads();
    }
  }
  double s = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) s += acc[i];
  out[(size_t)blockIdx.x * blockDim.x + threadIdx.x] = s + sink[(threadIdx.x + 1) & 511];
}

int main(int argc, char **argv) {
  const int steps = argc > 1 ? atoi(argv[1]) : 670;
  const int msgs = argc > 2 ? atoi(argv[2]) : 8192;
  const int work = argc > 3 ? atoi(argv[3]) : 256;
  double2 *key;
  double *out;
  CHK(hipMalloc(&key, (size_t)steps * STEP_D2 * sizeof(double2)));
  CHK(hipMemset(key, 0, (size_t)steps * STEP_D2 * sizeof(double2)));
  CHK(hipMalloc(&out, (size_t)msgs * 256 * sizeof(double)));
  hipEvent_t a, b;
  CHK(hipEventCreate(&a));
  CHK(hipEventCreate(&b));
  for (int mode = 0; mode < 4; ++mode) {
    for (int rep = 0; rep < 2; ++rep) {
      CHK(hipEventRecord(a));
      if (mode == 0) probe<0><<<msgs, 256>>>(key, out, steps, work);
      if (mode == 1) probe<1><<<msgs, 256>>>(key, out, steps, work);
      if (mode == 2) probe<2><<<msgs / 2, 512>>>(key, out, steps, work);
      if (mode == 3) probe<3><<<msgs, 256>>>(key, out, steps, work);
      CHK(hipGetLastError());
      CHK(hipEventRecord(b));
      CHK(hipEventSynchronize(b));
      float ms = 0;
      CHK(hipEventElapsedTime(&ms, a, b));
      printf("mode %d rep %d: %d msgs x %d steps, work %d FMA/row: %.1f ms, %.2f us/msg-step, key %.0f KB/msg-step\n",
             mode, rep, msgs, steps, work, ms, ms * 1e3 / ((double)msgs * steps) * 512.0 / 512.0,
             mode ? STEP_D2 * 16.0 / 1024 / (mode == 3 ? 2 : 1) : 0.0);
    }
  }
  return 0;
}
