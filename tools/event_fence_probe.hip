// Cost of a hipEventRecord between back-to-back streaming kernels on MI355X, by event flags.
// The robust engine records one "op done" event per device op; the N=1 kernel trace showed a
// 6 us gap after every 37 us copy where kernels without a record in between run back to back.
//   hipcc --offload-arch=gfx950 -O3 -o build/bin/event_fence_probe tools/event_fence_probe.hip
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>

#define CHECK(x)                                                                  \
  do {                                                                            \
    hipError_t e_ = (x);                                                          \
    if (e_ != hipSuccess) {                                                       \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(1);                                                                    \
    }                                                                             \
  } while (0)

__global__ __launch_bounds__(256) void CopyKernel(uint4 *__restrict__ d, const uint4 *__restrict__ s,
                                                  size_t n) {
  const size_t i = blockIdx.x * static_cast<size_t>(blockDim.x) + threadIdx.x;
  if (i < n) d[i] = s[i];
}

int main(int argc, char **argv) {
  const size_t bytes = (argc > 1 ? atol(argv[1]) : 128) << 20;
  const int iters = argc > 2 ? atoi(argv[2]) : 50;
  const size_t n = bytes / 16;
  uint4 *a, *b;
  CHECK(hipMalloc(&a, bytes));
  CHECK(hipMalloc(&b, bytes));
  CHECK(hipMemset(a, 1, bytes));
  hipStream_t st;
  CHECK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  struct Variant {
    const char *name;
    int record;
    unsigned flags;
  } vs[] = {{"no_event", 0, 0},
            {"DisableTiming", 1, hipEventDisableTiming},
            {"DisableTiming|DisableSystemFence", 1, hipEventDisableTiming | hipEventDisableSystemFence},
            {"DisableTiming|ReleaseToDevice", 1, hipEventDisableTiming | hipEventReleaseToDevice},
            {"DisableTiming|ReleaseToSystem", 1, hipEventDisableTiming | hipEventReleaseToSystem}};
  const int grid = static_cast<int>((n + 255) / 256);
  for (int round = 0; round < 3; ++round) {
    for (const Variant &v : vs) {
      hipEvent_t ev;
      CHECK(hipEventCreateWithFlags(&ev, v.flags ? v.flags : hipEventDisableTiming));
      for (int w = 0; w < 5; ++w) hipLaunchKernelGGL(CopyKernel, grid, 256, 0, st, b, a, n);
      CHECK(hipStreamSynchronize(st));
      const auto t0 = std::chrono::steady_clock::now();
      for (int i = 0; i < iters; ++i) {
        hipLaunchKernelGGL(CopyKernel, grid, 256, 0, st, b, a, n);
        if (v.record) CHECK(hipEventRecord(ev, st));
      }
      CHECK(hipStreamSynchronize(st));
      const double us =
          std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count() /
          iters;
      printf("{\"round\": %d, \"variant\": \"%s\", \"bytes\": %zu, \"us_per_iter\": %.2f}\n", round,
             v.name, bytes, us);
      CHECK(hipEventDestroy(ev));
    }
  }
  return 0;
}
