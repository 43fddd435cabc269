// Variant sweep for the read-only streaming reduction behind rabit's checksum (kernels.hip):
// grid size, vectors in flight per lane, plain vs nontemporal loads, 64-bit vs 32-bit-pair
// position weights.  One JSON line per variant: median us over 20 launches of 128 MiB.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/checksum_variants.hip -o build/bin/checksum_variants
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHECK(x)                                                                             \
  do {                                                                                       \
    hipError_t e = (x);                                                                      \
    if (e != hipSuccess) {                                                                   \
      fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); \
      exit(1);                                                                               \
    }                                                                                        \
  } while (0)

constexpr int kBlock = 256;
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

template <bool NT>
__device__ __forceinline__ uint4 Ld(const uint4 *p) {
  if (NT) {
    u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(p));
    return make_uint4(v.x, v.y, v.z, v.w);
  }
  return *p;
}

// MODE 0: s2 += (v + 1) * q in 64 bits (current).  MODE 1: the same sum computed from two
// 32-bit products per vector (idx split into hi / lo words) — fewer quarter-rate multiplies.
template <int U, bool NT, int MODE>
__global__ __launch_bounds__(kBlock) void K(const uint4 *__restrict__ w, size_t nvec,
                                            unsigned long long *out) {
  unsigned long long s1 = 0, s2 = 0;
  const size_t ntile = (nvec + static_cast<size_t>(kBlock) * U - 1) / (kBlock * U);
  for (size_t t = blockIdx.x; t < ntile; t += gridDim.x) {
    const size_t base = t * kBlock * U + threadIdx.x;
    uint4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const size_t i = base + u * kBlock;
      v[u] = i < nvec ? Ld<NT>(w + i) : make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const unsigned long long idx = base + u * kBlock + 1ull;
      const unsigned long long q = static_cast<unsigned long long>(v[u].x) + 2ull * v[u].y +
                                   3ull * v[u].z + 4ull * v[u].w;
      s1 += static_cast<unsigned long long>(v[u].x) + v[u].y + v[u].z + v[u].w;
      if (MODE == 0) {
        s2 += idx * q;
      } else {
        // idx < 2^32 for any buffer below 64 GiB: one 32x64 product
        const unsigned int id32 = static_cast<unsigned int>(idx);
        s2 += static_cast<unsigned long long>(id32) * static_cast<unsigned int>(q) +
              ((static_cast<unsigned long long>(id32) * static_cast<unsigned int>(q >> 32)) << 32);
      }
    }
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    s1 += __shfl_down(s1, off, 64);
    s2 += __shfl_down(s2, off, 64);
  }
  if ((threadIdx.x & 63) == 0) {  // one partial pair per wave (no contended atomics)
    const size_t slot = static_cast<size_t>(blockIdx.x) * (kBlock / 64) + threadIdx.x / 64;
    out[2 * slot] = s1;
    out[2 * slot + 1] = s2;
  }
}

template <int U, bool NT, int MODE>
void Run(const uint4 *w, size_t nvec, unsigned long long *out, int grid, hipEvent_t a,
         hipEvent_t b) {
  std::vector<float> ts;
  for (int r = 0; r < 22; ++r) {
    CHECK(hipEventRecord(a, 0));
    for (int k = 0; k < 5; ++k) hipLaunchKernelGGL((K<U, NT, MODE>), dim3(grid), dim3(kBlock), 0, 0, w, nvec, out);
    CHECK(hipEventRecord(b, 0));
    CHECK(hipEventSynchronize(b));
    float ms = 0;
    CHECK(hipEventElapsedTime(&ms, a, b));
    if (r >= 2) ts.push_back(ms * 1000.f / 5);
  }
  std::sort(ts.begin(), ts.end());
  const float med = ts[ts.size() / 2];
  printf("{\"U\": %d, \"nt\": %d, \"mode\": %d, \"grid\": %d, \"median_us\": %.1f, \"TBps\": %.2f}\n",
         U, NT ? 1 : 0, MODE, grid, med, nvec * 16.0 / med / 1e6);
  fflush(stdout);
}

int main() {
  const size_t bytes = 128u << 20;
  const size_t nvec = bytes / 16;
  uint4 *w;
  unsigned long long *out;
  CHECK(hipMalloc(&w, bytes));
  CHECK(hipMalloc(&out, 16u * 32768 * 4));
  CHECK(hipMemset(w, 1, bytes));
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  for (int grid : {1024, 2048, 4096, 8192}) {
    Run<4, false, 0>(w, nvec, out, grid, a, b);
    Run<4, false, 1>(w, nvec, out, grid, a, b);
    Run<8, false, 1>(w, nvec, out, grid, a, b);
    Run<4, true, 1>(w, nvec, out, grid, a, b);
    Run<2, false, 1>(w, nvec, out, grid, a, b);
  }
  // one-tile-per-workgroup grids (no grid-stride loop)
  Run<4, false, 1>(w, nvec, out, static_cast<int>(nvec / (kBlock * 4)), a, b);
  Run<1, false, 1>(w, nvec, out, static_cast<int>(nvec / kBlock), a, b);
  return 0;
}
