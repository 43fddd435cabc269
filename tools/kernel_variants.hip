// Variant sweep for the streaming kernels of the device data plane (copy and dst += src).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/kernel_variants.hip -o build/bin/kernel_variants
// Prints one JSON line per variant: median time and GB/s over interleaved rounds, 128 MiB f32.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <string>
#include <vector>

#define CHECK(x)                                                               \
  do {                                                                         \
    hipError_t e = (x);                                                        \
    if (e != hipSuccess) {                                                     \
      fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); \
      exit(1);                                                                 \
    }                                                                          \
  } while (0)

__device__ __forceinline__ uint4 add4(uint4 a, uint4 b) {
  float x[4], y[4];
  __builtin_memcpy(x, &a, 16);
  __builtin_memcpy(y, &b, 16);
#pragma unroll
  for (int j = 0; j < 4; ++j) x[j] += y[j];
  uint4 r;
  __builtin_memcpy(&r, x, 16);
  return r;
}

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
template <bool NT>
__device__ __forceinline__ uint4 ld(const uint4 *p) {
  if (NT) {
    u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(p));
    return make_uint4(v.x, v.y, v.z, v.w);
  }
  return *p;
}
template <bool NT>
__device__ __forceinline__ void st(uint4 *p, uint4 v) {
  if (NT) {
    u32x4 w = {v.x, v.y, v.z, v.w};
    __builtin_nontemporal_store(w, reinterpret_cast<u32x4 *>(p));
  } else {
    *p = v;
  }
}

// grid-stride, U vectors per lane per iteration
template <int U, bool NT, bool ADD>
__global__ __launch_bounds__(256) void KStride(uint4 *__restrict__ d, const uint4 *__restrict__ s,
                                               size_t nvec) {
  const size_t stride = (size_t)gridDim.x * 256;
  size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  for (; i + (U - 1) * stride < nvec; i += U * stride) {
    uint4 a[U], b[U];
#pragma unroll
    for (int u = 0; u < U; ++u) a[u] = ld<NT>(s + i + u * stride);
    if (ADD) {
#pragma unroll
      for (int u = 0; u < U; ++u) b[u] = ld<NT>(d + i + u * stride);
#pragma unroll
      for (int u = 0; u < U; ++u) a[u] = add4(a[u], b[u]);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) st<NT>(d + i + u * stride, a[u]);
  }
  for (; i < nvec; i += stride) st<NT>(d + i, ADD ? add4(ld<NT>(s + i), ld<NT>(d + i)) : ld<NT>(s + i));
}

// one-shot: block b owns the contiguous tile [b*256*U, (b+1)*256*U) vectors
template <int U, bool NT, bool ADD>
__global__ __launch_bounds__(256) void KTile(uint4 *__restrict__ d, const uint4 *__restrict__ s,
                                             size_t nvec) {
  const size_t base = (size_t)blockIdx.x * 256 * U + threadIdx.x;
  uint4 a[U], b[U];
  if (base + (U - 1) * 256 < nvec) {
#pragma unroll
    for (int u = 0; u < U; ++u) a[u] = ld<NT>(s + base + u * 256);
    if (ADD) {
#pragma unroll
      for (int u = 0; u < U; ++u) b[u] = ld<NT>(d + base + u * 256);
#pragma unroll
      for (int u = 0; u < U; ++u) a[u] = add4(a[u], b[u]);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) st<NT>(d + base + u * 256, a[u]);
  } else {
    for (int u = 0; u < U; ++u) {
      size_t i = base + u * 256;
      if (i < nvec) st<NT>(d + i, ADD ? add4(ld<NT>(s + i), ld<NT>(d + i)) : ld<NT>(s + i));
    }
  }
}

// generalized tile: B lanes per block, U vectors per lane; XCD: tiles of one XCD contiguous
// (workgroups are dispatched round-robin over the 8 XCDs); MODE 0 copy, 1 d += s, 2 o = d + s
template <int B, int U, bool XCD, int MODE, bool NTS = false>
__global__ __launch_bounds__(B) void KTileG(uint4 *__restrict__ d, const uint4 *__restrict__ s,
                                            uint4 *__restrict__ o, size_t nvec) {
  size_t tile = blockIdx.x;
  if (XCD) {
    const size_t g = gridDim.x, per = g / 8;
    if (per * 8 == g) tile = (blockIdx.x % 8) * per + blockIdx.x / 8;
  }
  const size_t base = tile * B * U + threadIdx.x;
  uint4 *out = MODE == 2 ? o : d;
  if (base + (U - 1) * B < nvec) {
    uint4 a[U], b[U];
#pragma unroll
    for (int u = 0; u < U; ++u) a[u] = s[base + u * B];
    if (MODE != 0) {
#pragma unroll
      for (int u = 0; u < U; ++u) b[u] = d[base + u * B];
#pragma unroll
      for (int u = 0; u < U; ++u) a[u] = add4(a[u], b[u]);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) st<NTS>(out + base + u * B, a[u]);
  } else {
    for (int u = 0; u < U; ++u) {
      size_t i = base + u * B;
      if (i < nvec) st<NTS>(out + i, MODE != 0 ? add4(s[i], d[i]) : s[i]);
    }
  }
}

struct Variant {
  std::string name;
  std::function<void(uint4 *, const uint4 *, size_t, hipStream_t)> run;
  bool add;
};

static uint4 *g_out = nullptr;  // third buffer for out-of-place variants
static uint4 *g_out_base = nullptr;

template <int B, int U, bool XCD, int MODE, bool NTS = false, int OFF = 0>
Variant TileG() {
  char nm[96];
  const char *m = MODE == 0 ? "copy" : (MODE == 1 ? "add" : "add3");
  snprintf(nm, sizeof(nm), "%s_tileg_b%d_u%d%s%s_off%d", m, B, U, XCD ? "_xcd" : "",
           NTS ? "_nts" : "", OFF);
  return {nm,
          [](uint4 *d, const uint4 *s, size_t n, hipStream_t st) {
            size_t g = (n + (size_t)B * U - 1) / ((size_t)B * U);
            uint4 *o = g_out_base + OFF / 16;
            hipLaunchKernelGGL((KTileG<B, U, XCD, MODE, NTS>), dim3(g), dim3(B), 0, st, d, s, o, n);
          },
          MODE != 0};
}

template <int U, bool NT, bool ADD>
Variant Stride(int grid) {
  char nm[96];
  snprintf(nm, sizeof(nm), "%s_stride_g%d_u%d%s", ADD ? "add" : "copy", grid, U, NT ? "_nt" : "");
  return {nm,
          [grid](uint4 *d, const uint4 *s, size_t n, hipStream_t st) {
            hipLaunchKernelGGL((KStride<U, NT, ADD>), dim3(grid), dim3(256), 0, st, d, s, n);
          },
          ADD};
}
template <int U, bool NT, bool ADD>
Variant Tile() {
  char nm[96];
  snprintf(nm, sizeof(nm), "%s_tile_u%d%s", ADD ? "add" : "copy", U, NT ? "_nt" : "");
  return {nm,
          [](uint4 *d, const uint4 *s, size_t n, hipStream_t st) {
            size_t g = (n + 256 * U - 1) / (256 * U);
            hipLaunchKernelGGL((KTile<U, NT, ADD>), dim3(g), dim3(256), 0, st, d, s, n);
          },
          ADD};
}

int main(int argc, char **argv) {
  const size_t mb = argc > 1 ? atoi(argv[1]) : 128;
  const size_t bytes = mb << 20, nvec = bytes / 16;
  uint4 *a, *b, *c;
  CHECK(hipMalloc(&a, bytes));
  CHECK(hipMalloc(&b, bytes));
  CHECK(hipMalloc(&c, bytes));
  CHECK(hipMalloc(&g_out_base, bytes + (1 << 20)));
  g_out = g_out_base;
  std::vector<float> h(bytes / 4);
  for (size_t i = 0; i < h.size(); ++i) h[i] = (float)((i * 2654435761u) % 1000) * 1e-3f;
  CHECK(hipMemcpy(a, h.data(), bytes, hipMemcpyHostToDevice));
  CHECK(hipMemcpy(b, h.data(), bytes, hipMemcpyHostToDevice));
  hipStream_t st;
  CHECK(hipStreamCreate(&st));
  std::vector<Variant> vs = {
      Stride<4, false, false>(2048), Stride<8, false, false>(2048), Stride<4, false, false>(1024),
      Stride<4, true, false>(2048),  Tile<4, false, false>(),       Tile<8, false, false>(),
      Tile<16, false, false>(),      Tile<8, true, false>(),        Stride<4, false, true>(2048),
      Stride<8, false, true>(2048),  Stride<2, false, true>(4096),  Tile<4, false, true>(),
      Tile<8, false, true>(),        Tile<8, true, true>(),         Tile<2, false, true>(),
  };
  {
    std::vector<Variant> more = {
        TileG<256, 4, false, 0>(),  TileG<256, 4, true, 0>(),   TileG<512, 4, false, 0>(),
        TileG<1024, 2, false, 0>(), TileG<128, 1, false, 0>(),  TileG<256, 1, false, 0>(),
        TileG<256, 2, true, 0>(),   TileG<256, 4, false, 1>(),  TileG<256, 4, true, 1>(),
        TileG<512, 2, false, 1>(),  TileG<128, 1, false, 1>(),  TileG<256, 1, false, 1>(),
        TileG<256, 4, false, 2>(),  TileG<256, 1, false, 2>(),  TileG<128, 1, false, 2>(),
        TileG<256, 2, true, 2>(),
        TileG<256, 1, false, 2, true>(),  TileG<256, 1, false, 0, true>(),
        TileG<256, 1, false, 2, false, 4096>(), TileG<256, 1, false, 2, false, 65536>(),
        TileG<256, 1, false, 2, false, 256>(),  TileG<256, 1, false, 1, true>(),
    };
    vs.insert(vs.end(), more.begin(), more.end());
  }
  vs.push_back({"copy_hipMemcpyAsync",
                [bytes](uint4 *d, const uint4 *s, size_t, hipStream_t st) {
                  (void)hipMemcpyAsync(d, s, bytes, hipMemcpyDeviceToDevice, st);
                },
                false});
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  const int rounds = 5, reps = 20;
  std::vector<std::vector<float>> times(vs.size());
  for (int r = 0; r < rounds; ++r) {
    for (size_t k = 0; k < vs.size(); ++k) {
      uint4 *dst = vs[k].add ? b : c;
      vs[k].run(dst, a, nvec, st);  // warm
      for (int i = 0; i < reps; ++i) {
        CHECK(hipEventRecord(e0, st));
        vs[k].run(dst, a, nvec, st);
        CHECK(hipEventRecord(e1, st));
        CHECK(hipEventSynchronize(e1));
        float ms;
        CHECK(hipEventElapsedTime(&ms, e0, e1));
        times[k].push_back(ms);
      }
    }
  }
  for (size_t k = 0; k < vs.size(); ++k) {
    auto &t = times[k];
    std::sort(t.begin(), t.end());
    const float med = t[t.size() / 2];
    const double moved = vs[k].add ? 3.0 * bytes : 2.0 * bytes;
    printf("{\"variant\": \"%s\", \"median_us\": %.1f, \"best_us\": %.1f, \"GBps\": %.0f}\n",
           vs[k].name.c_str(), med * 1e3, t[0] * 1e3, moved / (med * 1e-3) / 1e9);
  }
  return 0;
}
