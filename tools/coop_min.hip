// Minimal reproducer for the exit-time fault of profiled processes that made cooperative launches
// (DESIGN.md §5a): does `rocprofv3 --kernel-trace --stats -- ./coop_min coop`
// also end in SIGSEGV? If it does, the fault is the runtime's (HIP exit handler -> HSA teardown
// after the profiler tool finalised) with no state of libomr_gpu.so involved.
//   coop   one hipLaunchCooperativeKernel of a trivial kernel on the null stream, sync, free, exit
//   plain  the same with a plain launch (control)
//   lib    the library's pattern: a non-blocking stream, the cooperative launch, the error word
//          copied to pinned host memory on that stream, then hipHostFree / hipStreamDestroy
// build: hipcc --offload-arch=gfx950 -O2 tools/coop_min.hip -o tools/coop_min
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstring>

__global__ void fill(int *p) { p[blockIdx.x * blockDim.x + threadIdx.x] = (int)threadIdx.x; }

#define CHECK(x)                                                                 \
  do {                                                                           \
    hipError_t e_ = (x);                                                         \
    if (e_ != hipSuccess) {                                                      \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));               \
      return 1;                                                                  \
    }                                                                            \
  } while (0)

int main(int argc, char **argv) {
  const char *mode = argc > 1 ? argv[1] : "coop";
  int *d = nullptr;
  CHECK(hipMalloc(&d, 4 * 256 * sizeof(int)));
  void *args[] = {(void *)&d};
  if (!std::strcmp(mode, "plain")) {
    fill<<<4, 256>>>(d);
    CHECK(hipGetLastError());
  } else if (!std::strcmp(mode, "lib")) {
    hipStream_t st;
    int *herr = nullptr;
    CHECK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    CHECK(hipHostMalloc((void **)&herr, sizeof(int), hipHostMallocDefault));
    CHECK(hipLaunchCooperativeKernel((const void *)fill, dim3(4), dim3(256), args, 0, st));
    CHECK(hipMemcpyAsync(herr, d, sizeof(int), hipMemcpyDeviceToHost, st));
    CHECK(hipStreamSynchronize(st));
    CHECK(hipHostFree(herr));
    CHECK(hipStreamDestroy(st));
  } else {
    CHECK(hipLaunchCooperativeKernel((const void *)fill, dim3(4), dim3(256), args, 0, nullptr));
  }
  CHECK(hipDeviceSynchronize());
  int h[4];
  CHECK(hipMemcpy(h, d + 255, sizeof(h), hipMemcpyDeviceToHost));
  CHECK(hipFree(d));
  std::printf("coop_min %s: ok (%d %d)\n", mode, h[0], h[1]);
  return 0;
}
