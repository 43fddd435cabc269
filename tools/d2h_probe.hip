// D2H / H2D bandwidth of a 256 MiB hipMemcpyAsync per pinned-host allocation flag (the memory
// kind behind the checkpoint mirror).  Build: hipcc --offload-arch=gfx950 -O2 tools/d2h_probe.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));              \
      std::exit(1);                                                             \
    }                                                                           \
  } while (0)

int main() {
  const size_t bytes = size_t(256) << 20;
  void *dev = nullptr;
  CK(hipMalloc(&dev, bytes));
  CK(hipMemset(dev, 1, bytes));
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  struct Kind {
    const char *name;
    unsigned flags;
  } kinds[] = {{"default", hipHostMallocDefault},
               {"coherent", hipHostMallocCoherent},
               {"noncoherent", hipHostMallocNonCoherent},
               {"writecombined", hipHostMallocWriteCombined},
               {"numa_user", hipHostMallocNumaUser}};
  for (const Kind &k : kinds) {
    void *host = nullptr;
    if (hipHostMalloc(&host, bytes, k.flags) != hipSuccess) {
      (void)hipGetLastError();
      std::printf("{\"kind\":\"%s\",\"error\":\"hipHostMalloc failed\"}\n", k.name);
      continue;
    }
    float best_d2h = 1e30f, best_h2d = 1e30f;
    for (int rep = 0; rep < 6; ++rep) {
      float ms = 0;
      CK(hipEventRecord(a, s));
      CK(hipMemcpyAsync(host, dev, bytes, hipMemcpyDeviceToHost, s));
      CK(hipEventRecord(b, s));
      CK(hipEventSynchronize(b));
      CK(hipEventElapsedTime(&ms, a, b));
      if (rep > 0 && ms < best_d2h) best_d2h = ms;
      CK(hipEventRecord(a, s));
      CK(hipMemcpyAsync(dev, host, bytes, hipMemcpyHostToDevice, s));
      CK(hipEventRecord(b, s));
      CK(hipEventSynchronize(b));
      CK(hipEventElapsedTime(&ms, a, b));
      if (rep > 0 && ms < best_h2d) best_h2d = ms;
    }
    std::printf("{\"kind\":\"%s\",\"d2h_ms\":%.3f,\"d2h_GBps\":%.1f,\"h2d_ms\":%.3f,\"h2d_GBps\":%.1f}\n",
                k.name, best_d2h, bytes / best_d2h / 1e6, best_h2d, bytes / best_h2d / 1e6);
    CK(hipHostFree(host));
  }
  return 0;
}
