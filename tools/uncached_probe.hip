// Streaming bandwidth of uncached HBM (hipDeviceMallocUncached: the direct transport's stage
// buffers, flags and symmetric heap) against ordinary hipMalloc memory, on one MI355X.
//   hipcc --offload-arch=gfx950 -O3 -o build/bin/uncached_probe tools/uncached_probe.hip
// Prints one JSON line per (source, destination) pair: us per 128 MiB copy, median of 20.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHECK(x)                                                                        \
  do {                                                                                  \
    hipError_t e_ = (x);                                                                \
    if (e_ != hipSuccess) {                                                             \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(1);                                                                          \
    }                                                                                   \
  } while (0)

__global__ __launch_bounds__(256) void CopyKernel(uint4 *__restrict__ d, const uint4 *__restrict__ s,
                                                  size_t n) {
  const size_t i = blockIdx.x * static_cast<size_t>(blockDim.x) + threadIdx.x;
  if (i < n) d[i] = s[i];
}

int main(int argc, char **argv) {
  const size_t bytes = static_cast<size_t>(argc > 1 ? atol(argv[1]) : 128) << 20;
  const size_t n = bytes / 16;
  uint4 *buf[2][2];  // [uncached][which]
  for (int u = 0; u < 2; ++u) {
    for (int w = 0; w < 2; ++w) {
      void *p = nullptr;
      if (u) {
        CHECK(hipExtMallocWithFlags(&p, bytes, hipDeviceMallocUncached));
      } else {
        CHECK(hipMalloc(&p, bytes));
      }
      CHECK(hipMemset(p, w + 1, bytes));
      buf[u][w] = static_cast<uint4 *>(p);
    }
  }
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  const int grid = static_cast<int>((n + 255) / 256);
  const char *name[2] = {"cached", "uncached"};
  for (int su = 0; su < 2; ++su) {
    for (int du = 0; du < 2; ++du) {
      uint4 *src = buf[su][0], *dst = buf[du][1];
      for (int w = 0; w < 3; ++w) hipLaunchKernelGGL(CopyKernel, grid, 256, 0, 0, dst, src, n);
      std::vector<float> t;
      for (int r = 0; r < 20; ++r) {
        CHECK(hipEventRecord(a, 0));
        hipLaunchKernelGGL(CopyKernel, grid, 256, 0, 0, dst, src, n);
        CHECK(hipEventRecord(b, 0));
        CHECK(hipEventSynchronize(b));
        float ms = 0;
        CHECK(hipEventElapsedTime(&ms, a, b));
        t.push_back(ms * 1000.f);
      }
      std::sort(t.begin(), t.end());
      printf("{\"src\": \"%s\", \"dst\": \"%s\", \"bytes\": %zu, \"us\": %.1f, \"TBps\": %.2f}\n",
             name[su], name[du], bytes, t[10], 2.0 * bytes / (t[10] * 1e-6) / 1e12);
    }
  }
  return 0;
}
