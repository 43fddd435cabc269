// Does the 8-source reduce of the direct allreduce gain anything from the matrix cores or from
// LDS staging?  (BASELINE.json's north star asks for "MFMA packed-vector accumulate and LDS
// staging"; SURVEY §7.2 step 5: "benchmark both and keep the faster".)
//
// Shape: the local step of an 8-rank two-shot allreduce of 128 MiB fp32 — each rank sums the
// 16 MiB segment it owns over 8 sources (128 MiB read, 16 MiB written).
//
//  valu : each lane loads one float4 per source and adds them with packed fp32 adds, one
//         16-B store (the production ReduceMultiTileKernel's structure)
//  mfma : the sum is a ones-vector GEMM on the matrix cores: v_mfma_f32_32x32x2_f32 with A = 1
//         (32x2) and B = 2 sources x 32 columns; lane l feeds B[l/32][l%32], so one wave
//         accumulates 2 sources x 32 columns per instruction; 4 accumulators (one per float4
//         component) x 4 source pairs = 16 MFMAs per 128 elements.  Row 0 of D is the sum.
//  lds  : a workgroup stages its 8 source tiles in LDS (16 KiB x 8 = 128 KiB), barrier, then
//         sums from LDS
//
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/mfma_reduce_probe.hip -o build/bin/mfma_reduce_probe
// Prints one JSON line per variant (median of interleaved rounds) after checking every output
// against a host fp32 sum.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHECK(x)                                                                            \
  do {                                                                                      \
    hipError_t e = (x);                                                                     \
    if (e != hipSuccess) {                                                                  \
      fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); \
      exit(1);                                                                              \
    }                                                                                       \
  } while (0)

constexpr int kSrc = 8;
struct Srcs {
  const float *p[kSrc];
};

// ------------------------------------------------------------------------------------- valu
__global__ __launch_bounds__(256) void ValuReduce(float *__restrict__ dst, Srcs s, size_t nvec) {
  const size_t i = static_cast<size_t>(blockIdx.x) * 256 + threadIdx.x;
  if (i >= nvec) return;
  float4 a = reinterpret_cast<const float4 *>(s.p[0])[i];
#pragma unroll
  for (int k = 1; k < kSrc; ++k) {
    const float4 b = reinterpret_cast<const float4 *>(s.p[k])[i];
    a.x += b.x;
    a.y += b.y;
    a.z += b.z;
    a.w += b.w;
  }
  reinterpret_cast<float4 *>(dst)[i] = a;
}

// ------------------------------------------------------------------------------------- mfma
typedef float f32x16 __attribute__((ext_vector_type(16)));

// one wave: 128 consecutive elements (32 lanes x float4) per chunk
__global__ __launch_bounds__(256) void MfmaReduce(float *__restrict__ dst, Srcs s, size_t nchunk) {
  const int lane = threadIdx.x & 63;
  const int half = lane >> 5, j = lane & 31;
  const size_t c = static_cast<size_t>(blockIdx.x) * 4 + (threadIdx.x >> 6);
  if (c >= nchunk) return;
  const size_t at = c * 128 + 4 * static_cast<size_t>(j);
  float4 v[kSrc / 2];
#pragma unroll
  for (int m = 0; m < kSrc / 2; ++m) v[m] = *reinterpret_cast<const float4 *>(s.p[2 * m + half] + at);
  f32x16 acc0 = {}, acc1 = {}, acc2 = {}, acc3 = {};
#pragma unroll
  for (int m = 0; m < kSrc / 2; ++m) {
    // D[i][j] += sum_k A[i][k] * B[k][j], A = 1: column j collects sources 2m and 2m+1
    acc0 = __builtin_amdgcn_mfma_f32_32x32x2f32(1.0f, v[m].x, acc0, 0, 0, 0);
    acc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(1.0f, v[m].y, acc1, 0, 0, 0);
    acc2 = __builtin_amdgcn_mfma_f32_32x32x2f32(1.0f, v[m].z, acc2, 0, 0, 0);
    acc3 = __builtin_amdgcn_mfma_f32_32x32x2f32(1.0f, v[m].w, acc3, 0, 0, 0);
  }
  // every row of D holds the column sums; lanes 0-31 own columns 0-31 in register 0
  if (half == 0) {
    *reinterpret_cast<float4 *>(dst + at) = make_float4(acc0[0], acc1[0], acc2[0], acc3[0]);
  }
}

// -------------------------------------------------------------------------------------- lds
constexpr int kLdsVec = 1024;  // float4 per source per workgroup (16 KiB), x8 sources = 128 KiB
__global__ __launch_bounds__(256) void LdsReduce(float *__restrict__ dst, Srcs s, size_t nvec) {
  extern __shared__ float4 tile[];  // [kSrc][kLdsVec]
  const size_t base = static_cast<size_t>(blockIdx.x) * kLdsVec;
#pragma unroll
  for (int k = 0; k < kSrc; ++k) {
    for (int v = threadIdx.x; v < kLdsVec; v += 256) {
      if (base + v < nvec) tile[k * kLdsVec + v] = reinterpret_cast<const float4 *>(s.p[k])[base + v];
    }
  }
  __syncthreads();
  for (int v = threadIdx.x; v < kLdsVec; v += 256) {
    if (base + v >= nvec) break;
    float4 a = tile[v];
#pragma unroll
    for (int k = 1; k < kSrc; ++k) {
      const float4 b = tile[k * kLdsVec + v];
      a.x += b.x;
      a.y += b.y;
      a.z += b.z;
      a.w += b.w;
    }
    reinterpret_cast<float4 *>(dst)[base + v] = a;
  }
}

int main(int argc, char **argv) {
  const size_t n = argc > 1 ? strtoull(argv[1], nullptr, 10) : (size_t(16) << 20) / 4;  // floats
  const int rounds = argc > 2 ? atoi(argv[2]) : 20;
  if (n % 4096 != 0) {
    fprintf(stderr, "n must be a multiple of 4096\n");
    return 1;
  }
  std::vector<float> h(n * kSrc);
  for (size_t i = 0; i < h.size(); ++i) h[i] = static_cast<float>((i * 2654435761u) % 1000) * 1e-3f;
  std::vector<float> want(n, 0.f);
  for (size_t i = 0; i < n; ++i) {
    float a = h[i];
    for (int k = 1; k < kSrc; ++k) a += h[k * n + i];
    want[i] = a;
  }
  float *src = nullptr, *dst = nullptr;
  CHECK(hipMalloc(&src, n * kSrc * sizeof(float)));
  CHECK(hipMalloc(&dst, n * sizeof(float)));
  CHECK(hipMemcpy(src, h.data(), h.size() * sizeof(float), hipMemcpyHostToDevice));
  Srcs s;
  for (int k = 0; k < kSrc; ++k) s.p[k] = src + k * n;
  const size_t nvec = n / 4, nchunk = n / 128;
  CHECK(hipFuncSetAttribute(reinterpret_cast<const void *>(LdsReduce),
                            hipFuncAttributeMaxDynamicSharedMemorySize,
                            kSrc * kLdsVec * sizeof(float4)));
  struct V {
    const char *name;
    void (*launch)(float *, Srcs, size_t, size_t);
  };
  V vs[] = {
      {"valu", [](float *d, Srcs s, size_t nv, size_t) {
         hipLaunchKernelGGL(ValuReduce, dim3((nv + 255) / 256), dim3(256), 0, 0, d, s, nv);
       }},
      {"mfma", [](float *d, Srcs s, size_t, size_t nc) {
         hipLaunchKernelGGL(MfmaReduce, dim3((nc + 3) / 4), dim3(256), 0, 0, d, s, nc);
       }},
      {"lds", [](float *d, Srcs s, size_t nv, size_t) {
         hipLaunchKernelGGL(LdsReduce, dim3((nv + kLdsVec - 1) / kLdsVec), dim3(256),
                            kSrc * kLdsVec * sizeof(float4), 0, d, s, nv);
       }},
  };
  const int nv = sizeof(vs) / sizeof(vs[0]);
  std::vector<float> got(n);
  for (auto &v : vs) {  // correctness first
    CHECK(hipMemset(dst, 0, n * sizeof(float)));
    v.launch(dst, s, nvec, nchunk);
    CHECK(hipGetLastError());
    CHECK(hipDeviceSynchronize());
    CHECK(hipMemcpy(got.data(), dst, n * sizeof(float), hipMemcpyDeviceToHost));
    double maxrel = 0;
    for (size_t i = 0; i < n; ++i) {
      maxrel = std::max(maxrel, std::fabs(double(got[i]) - want[i]) / std::max(1e-6, std::fabs(double(want[i]))));
    }
    printf("{\"variant\": \"%s\", \"check_max_rel_err\": %.3g}\n", v.name, maxrel);
    if (maxrel > 1e-5) return 2;
  }
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  std::vector<std::vector<float>> t(nv);
  for (int r = 0; r < rounds; ++r) {
    for (int k = 0; k < nv; ++k) {  // interleaved so clocks/thermals hit all variants alike
      CHECK(hipEventRecord(a));
      vs[k].launch(dst, s, nvec, nchunk);
      CHECK(hipEventRecord(b));
      CHECK(hipEventSynchronize(b));
      float ms = 0;
      CHECK(hipEventElapsedTime(&ms, a, b));
      t[k].push_back(ms * 1e3f);
    }
  }
  const double bytes = double(n) * sizeof(float) * (kSrc + 1);
  for (int k = 0; k < nv; ++k) {
    std::sort(t[k].begin(), t[k].end());
    const double us = t[k][t[k].size() / 2];
    printf("{\"variant\": \"%s\", \"sources\": %d, \"elems\": %zu, \"median_us\": %.2f, "
           "\"min_us\": %.2f, \"TBps\": %.2f}\n",
           vs[k].name, kSrc, n, us, t[k][0], bytes / us / 1e6);
  }
  return 0;
}
