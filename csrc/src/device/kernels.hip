/*!
 * \file kernels.hip
 * \brief gfx950 (MI355X, CDNA4) kernels of the device data plane.
 *
 * All kernels here are HBM-bandwidth bound (element-wise: 2-9 bytes moved per FLOP), so
 * the design goal is to stream at the HBM roof (~6.3 TB/s measured on MI355X):
 *  - 64-lane waves, 256-thread workgroups, grid capped at 2048 workgroups
 *    (256 CUs x 8) and grid-stride beyond that;
 *  - 16 bytes per lane per access (global_load_dwordx4 / global_store_dwordx4);
 *  - kUnroll independent 16-byte loads per lane issued before any use, so every wave keeps
 *    several KB in flight (latency hiding by ILP as well as by occupancy);
 *  - the multi-source reduce is templated on the source count so all loads of one
 *    element-vector are issued back to back.
 * MFMA is deliberately not used: an element-wise reduce has no reuse, a ones-vector GEMM
 * over stacked peer buffers moves the same bytes and adds matrix-pipe work.
 */
#include <hip/hip_runtime.h>

#include <cstdint>
#include <type_traits>

#include "device/kernels.h"

namespace rabit {
namespace device {
namespace {

constexpr int kBlock = 256;
constexpr int kMaxGrid = 2048;
constexpr int kUnroll = 4;

enum OpCode : int { kOpMax = 0, kOpMin = 1, kOpSum = 2, kOpOr = 3 };

template <typename T, int OP>
struct Apply;
template <typename T>
struct Apply<T, kOpMax> {
  __device__ __forceinline__ static T f(T a, T b) { return b > a ? b : a; }
};
template <typename T>
struct Apply<T, kOpMin> {
  __device__ __forceinline__ static T f(T a, T b) { return b < a ? b : a; }
};
template <typename T>
struct Apply<T, kOpSum> {
  __device__ __forceinline__ static T f(T a, T b) { return a + b; }
};
template <typename T>
struct Apply<T, kOpOr> {
  __device__ __forceinline__ static T f(T a, T b) { return a | b; }
};

/*! \brief 16-byte pack of T */
template <typename T>
struct alignas(16) Pack {
  static constexpr int kLanes = 16 / sizeof(T);
  T v[kLanes];
};

inline int GridFor(size_t items) {
  size_t blocks = (items + kBlock - 1) / kBlock;
  if (blocks < 1) blocks = 1;
  if (blocks > static_cast<size_t>(kMaxGrid)) blocks = kMaxGrid;
  return static_cast<int>(blocks);
}

inline bool Aligned16(const void *p) { return (reinterpret_cast<uintptr_t>(p) & 15u) == 0; }

// ---------------------------------------------------------------- two-operand reduce
template <typename T, int OP>
__global__ __launch_bounds__(kBlock) void ReduceVecKernel(T *__restrict__ dst,
                                                          const T *__restrict__ src, size_t n) {
  using P = Pack<T>;
  constexpr int L = P::kLanes;
  const size_t nvec = n / L;
  P *d = reinterpret_cast<P *>(dst);
  const P *s = reinterpret_cast<const P *>(src);
  const size_t stride = static_cast<size_t>(gridDim.x) * kBlock;
  size_t i = static_cast<size_t>(blockIdx.x) * kBlock + threadIdx.x;
  for (; i + (kUnroll - 1) * stride < nvec; i += kUnroll * stride) {
    P a[kUnroll], b[kUnroll];
#pragma unroll
    for (int u = 0; u < kUnroll; ++u) {
      a[u] = d[i + u * stride];
      b[u] = s[i + u * stride];
    }
#pragma unroll
    for (int u = 0; u < kUnroll; ++u) {
#pragma unroll
      for (int j = 0; j < L; ++j) a[u].v[j] = Apply<T, OP>::f(a[u].v[j], b[u].v[j]);
      d[i + u * stride] = a[u];
    }
  }
  for (; i < nvec; i += stride) {
    P a = d[i], b = s[i];
#pragma unroll
    for (int j = 0; j < L; ++j) a.v[j] = Apply<T, OP>::f(a.v[j], b.v[j]);
    d[i] = a;
  }
  // tail (< L elements), first threads of the grid
  const size_t tail = nvec * L;
  const size_t t = static_cast<size_t>(blockIdx.x) * kBlock + threadIdx.x;
  if (tail + t < n) dst[tail + t] = Apply<T, OP>::f(dst[tail + t], src[tail + t]);
}

template <typename T, int OP>
__global__ __launch_bounds__(kBlock) void ReduceScalarKernel(T *__restrict__ dst,
                                                             const T *__restrict__ src,
                                                             size_t n) {
  const size_t stride = static_cast<size_t>(gridDim.x) * kBlock;
  for (size_t i = static_cast<size_t>(blockIdx.x) * kBlock + threadIdx.x; i < n; i += stride) {
    dst[i] = Apply<T, OP>::f(dst[i], src[i]);
  }
}

template <typename T, int OP>
hipError_t Reduce2(void *dst, const void *src, size_t n, hipStream_t st) {
  T *d = static_cast<T *>(dst);
  const T *s = static_cast<const T *>(src);
  if (Aligned16(dst) && Aligned16(src)) {
    const size_t nvec = n / Pack<T>::kLanes;
    hipLaunchKernelGGL((ReduceVecKernel<T, OP>), dim3(GridFor((nvec + kUnroll - 1) / kUnroll)),
                       dim3(kBlock), 0, st, d, s, n);
  } else {
    hipLaunchKernelGGL((ReduceScalarKernel<T, OP>), dim3(GridFor(n)), dim3(kBlock), 0, st, d, s,
                       n);
  }
  return hipGetLastError();
}

// ---------------------------------------------------------------- multi-source reduce
struct SrcList {
  const void *p[kMaxReduceSources];
};

template <typename T, int OP, int NSRC>
__global__ __launch_bounds__(kBlock) void ReduceMultiVecKernel(T *dst, SrcList srcs,
                                                               size_t n) {
  using P = Pack<T>;
  constexpr int L = P::kLanes;
  const size_t nvec = n / L;
  const size_t stride = static_cast<size_t>(gridDim.x) * kBlock;
  for (size_t i = static_cast<size_t>(blockIdx.x) * kBlock + threadIdx.x; i < nvec;
       i += stride) {
    P x[NSRC];
#pragma unroll
    for (int k = 0; k < NSRC; ++k) x[k] = reinterpret_cast<const P *>(srcs.p[k])[i];
    P acc = x[0];
#pragma unroll
    for (int k = 1; k < NSRC; ++k) {
#pragma unroll
      for (int j = 0; j < L; ++j) acc.v[j] = Apply<T, OP>::f(acc.v[j], x[k].v[j]);
    }
    reinterpret_cast<P *>(dst)[i] = acc;
  }
  const size_t tail = nvec * L;
  const size_t t = static_cast<size_t>(blockIdx.x) * kBlock + threadIdx.x;
  if (tail + t < n) {
    T acc = static_cast<const T *>(srcs.p[0])[tail + t];
#pragma unroll
    for (int k = 1; k < NSRC; ++k) {
      acc = Apply<T, OP>::f(acc, static_cast<const T *>(srcs.p[k])[tail + t]);
    }
    dst[tail + t] = acc;
  }
}

template <typename T, int OP>
__global__ __launch_bounds__(kBlock) void ReduceMultiScalarKernel(T *dst,
                                                                  SrcList srcs, int nsrc,
                                                                  size_t n) {
  const size_t stride = static_cast<size_t>(gridDim.x) * kBlock;
  for (size_t i = static_cast<size_t>(blockIdx.x) * kBlock + threadIdx.x; i < n; i += stride) {
    T acc = static_cast<const T *>(srcs.p[0])[i];
    for (int k = 1; k < nsrc; ++k) acc = Apply<T, OP>::f(acc, static_cast<const T *>(srcs.p[k])[i]);
    dst[i] = acc;
  }
}

template <typename T, int OP, int NSRC>
void LaunchMultiVec(T *dst, const SrcList &sl, size_t n, hipStream_t st) {
  const size_t nvec = n / Pack<T>::kLanes;
  hipLaunchKernelGGL((ReduceMultiVecKernel<T, OP, NSRC>), dim3(GridFor(nvec)), dim3(kBlock), 0,
                     st, dst, sl, n);
}

template <typename T, int OP>
hipError_t ReduceMulti(void *dst, const void *const *srcs, int nsrc, size_t n, hipStream_t st) {
  SrcList sl;
  bool aligned = Aligned16(dst);
  for (int k = 0; k < kMaxReduceSources; ++k) {
    sl.p[k] = k < nsrc ? srcs[k] : nullptr;
    if (k < nsrc) aligned = aligned && Aligned16(srcs[k]);
  }
  T *d = static_cast<T *>(dst);
  if (!aligned) {
    hipLaunchKernelGGL((ReduceMultiScalarKernel<T, OP>), dim3(GridFor(n)), dim3(kBlock), 0, st, d,
                       sl, nsrc, n);
    return hipGetLastError();
  }
  switch (nsrc) {
    case 1: LaunchMultiVec<T, OP, 1>(d, sl, n, st); break;
    case 2: LaunchMultiVec<T, OP, 2>(d, sl, n, st); break;
    case 3: LaunchMultiVec<T, OP, 3>(d, sl, n, st); break;
    case 4: LaunchMultiVec<T, OP, 4>(d, sl, n, st); break;
    case 5: LaunchMultiVec<T, OP, 5>(d, sl, n, st); break;
    case 6: LaunchMultiVec<T, OP, 6>(d, sl, n, st); break;
    case 7: LaunchMultiVec<T, OP, 7>(d, sl, n, st); break;
    case 8: LaunchMultiVec<T, OP, 8>(d, sl, n, st); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

// ---------------------------------------------------------------- lazy prepare
template <typename T>
__device__ __forceinline__ T PrepApply(T x, int prep, T alpha) {
  switch (prep) {
    case kPrepSquare: return x * x;
    case kPrepScale: return x * alpha;
    case kPrepAbs: return x < T(0) ? T(0) - x : x;
    default: return x;
  }
}

template <typename T>
__global__ __launch_bounds__(kBlock) void PrepareVecKernel(T *__restrict__ dst,
                                                           T *__restrict__ dst2,
                                                           const T *__restrict__ src, size_t n,
                                                           int prep, T alpha) {
  using P = Pack<T>;
  constexpr int L = P::kLanes;
  const size_t nvec = n / L;
  const size_t stride = static_cast<size_t>(gridDim.x) * kBlock;
  size_t i = static_cast<size_t>(blockIdx.x) * kBlock + threadIdx.x;
  for (; i + (kUnroll - 1) * stride < nvec; i += kUnroll * stride) {
    P a[kUnroll];
#pragma unroll
    for (int u = 0; u < kUnroll; ++u) a[u] = reinterpret_cast<const P *>(src)[i + u * stride];
#pragma unroll
    for (int u = 0; u < kUnroll; ++u) {
#pragma unroll
      for (int j = 0; j < L; ++j) a[u].v[j] = PrepApply<T>(a[u].v[j], prep, alpha);
      reinterpret_cast<P *>(dst)[i + u * stride] = a[u];
      if (dst2 != nullptr) reinterpret_cast<P *>(dst2)[i + u * stride] = a[u];
    }
  }
  for (; i < nvec; i += stride) {
    P a = reinterpret_cast<const P *>(src)[i];
#pragma unroll
    for (int j = 0; j < L; ++j) a.v[j] = PrepApply<T>(a.v[j], prep, alpha);
    reinterpret_cast<P *>(dst)[i] = a;
    if (dst2 != nullptr) reinterpret_cast<P *>(dst2)[i] = a;
  }
  const size_t tail = nvec * L;
  const size_t t = static_cast<size_t>(blockIdx.x) * kBlock + threadIdx.x;
  if (tail + t < n) {
    T y = PrepApply<T>(src[tail + t], prep, alpha);
    dst[tail + t] = y;
    if (dst2 != nullptr) dst2[tail + t] = y;
  }
}

template <typename T>
__global__ __launch_bounds__(kBlock) void PrepareScalarKernel(T *dst, T *dst2, const T *src,
                                                              size_t n, int prep, T alpha) {
  const size_t stride = static_cast<size_t>(gridDim.x) * kBlock;
  for (size_t i = static_cast<size_t>(blockIdx.x) * kBlock + threadIdx.x; i < n; i += stride) {
    T y = PrepApply<T>(src[i], prep, alpha);
    dst[i] = y;
    if (dst2 != nullptr) dst2[i] = y;
  }
}

template <typename T>
hipError_t Prepare(void *dst, void *dst2, const void *src, size_t n, int prep, double alpha,
                   hipStream_t st) {
  T *d = static_cast<T *>(dst);
  T *d2 = static_cast<T *>(dst2);
  const T *s = static_cast<const T *>(src);
  const T a = static_cast<T>(alpha);
  if (Aligned16(dst) && Aligned16(src) && (dst2 == nullptr || Aligned16(dst2))) {
    const size_t nvec = n / Pack<T>::kLanes;
    hipLaunchKernelGGL(PrepareVecKernel<T>, dim3(GridFor((nvec + kUnroll - 1) / kUnroll)),
                       dim3(kBlock), 0, st, d, d2, s, n, prep, a);
  } else {
    hipLaunchKernelGGL(PrepareScalarKernel<T>, dim3(GridFor(n)), dim3(kBlock), 0, st, d, d2, s, n,
                       prep, a);
  }
  return hipGetLastError();
}

// ---------------------------------------------------------------- checksum
__global__ __launch_bounds__(kBlock) void ChecksumKernel(const uint32_t *__restrict__ w,
                                                         size_t nwords,
                                                         unsigned long long *__restrict__ out) {
  const size_t stride = static_cast<size_t>(gridDim.x) * kBlock;
  unsigned long long s1 = 0, s2 = 0;
  const size_t nvec = nwords / 4;
  const uint4 *w4 = reinterpret_cast<const uint4 *>(w);
  for (size_t i = static_cast<size_t>(blockIdx.x) * kBlock + threadIdx.x; i < nvec; i += stride) {
    uint4 v = w4[i];
    const unsigned long long base = 4ull * i + 1ull;
    s1 += static_cast<unsigned long long>(v.x) + v.y + v.z + v.w;
    s2 += base * v.x + (base + 1) * v.y + (base + 2) * v.z + (base + 3) * v.w;
  }
  const size_t t = static_cast<size_t>(blockIdx.x) * kBlock + threadIdx.x;
  if (4 * nvec + t < nwords) {
    s1 += w[4 * nvec + t];
    s2 += (4ull * nvec + t + 1ull) * w[4 * nvec + t];
  }
  // wave64 reduction, then across the 4 waves of the workgroup through LDS
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    s1 += __shfl_down(s1, off, 64);
    s2 += __shfl_down(s2, off, 64);
  }
  __shared__ unsigned long long part[2][kBlock / 64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if (lane == 0) {
    part[0][wave] = s1;
    part[1][wave] = s2;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned long long a = 0, b = 0;
#pragma unroll
    for (int k = 0; k < kBlock / 64; ++k) {
      a += part[0][k];
      b += part[1][k];
    }
    atomicAdd(&out[0], a);
    atomicAdd(&out[1], b);
  }
}

// ---------------------------------------------------------------- copy
/*! \brief 16-byte-per-lane streaming copy, kUnroll loads in flight per lane */
__global__ __launch_bounds__(kBlock) void CopyVecKernel(uint4 *__restrict__ dst,
                                                       const uint4 *__restrict__ src,
                                                       size_t nvec) {
  const size_t stride = static_cast<size_t>(gridDim.x) * kBlock;
  size_t i = static_cast<size_t>(blockIdx.x) * kBlock + threadIdx.x;
  for (; i + (kUnroll - 1) * stride < nvec; i += kUnroll * stride) {
    uint4 v[kUnroll];
#pragma unroll
    for (int u = 0; u < kUnroll; ++u) v[u] = src[i + u * stride];
#pragma unroll
    for (int u = 0; u < kUnroll; ++u) dst[i + u * stride] = v[u];
  }
  for (; i < nvec; i += stride) dst[i] = src[i];
}

// ---------------------------------------------------------------- fill
template <typename T>
__global__ __launch_bounds__(kBlock) void FillKernel(T *dst, size_t n, T value) {
  const size_t stride = static_cast<size_t>(gridDim.x) * kBlock;
  for (size_t i = static_cast<size_t>(blockIdx.x) * kBlock + threadIdx.x; i < n; i += stride) {
    dst[i] = value;
  }
}

// dtype code -> C++ type; integer-only ops reject float types
template <typename Fn>
hipError_t DispatchType(int dtype, bool int_only, Fn &&fn) {
  switch (dtype) {
    case 0: return fn(static_cast<int8_t *>(nullptr));
    case 1: return fn(static_cast<uint8_t *>(nullptr));
    case 2: return fn(static_cast<int32_t *>(nullptr));
    case 3: return fn(static_cast<uint32_t *>(nullptr));
    case 4: return fn(static_cast<int64_t *>(nullptr));
    case 5: return fn(static_cast<uint64_t *>(nullptr));
    case 6: return int_only ? hipErrorInvalidValue : fn(static_cast<float *>(nullptr));
    case 7: return int_only ? hipErrorInvalidValue : fn(static_cast<double *>(nullptr));
    case 8: return fn(static_cast<int64_t *>(nullptr));
    case 9: return fn(static_cast<uint64_t *>(nullptr));
    default: return hipErrorInvalidValue;
  }
}

template <typename T>
struct OrTag {
  // BitOR is only instantiated for integral types
  template <typename U = T>
  static typename std::enable_if<std::is_integral<U>::value, hipError_t>::type Reduce2Or(
      void *d, const void *s, size_t n, hipStream_t st) {
    return Reduce2<U, kOpOr>(d, s, n, st);
  }
  template <typename U = T>
  static typename std::enable_if<!std::is_integral<U>::value, hipError_t>::type Reduce2Or(
      void *, const void *, size_t, hipStream_t) {
    return hipErrorInvalidValue;
  }
  template <typename U = T>
  static typename std::enable_if<std::is_integral<U>::value, hipError_t>::type MultiOr(
      void *d, const void *const *s, int k, size_t n, hipStream_t st) {
    return ReduceMulti<U, kOpOr>(d, s, k, n, st);
  }
  template <typename U = T>
  static typename std::enable_if<!std::is_integral<U>::value, hipError_t>::type MultiOr(
      void *, const void *const *, int, size_t, hipStream_t) {
    return hipErrorInvalidValue;
  }
};
}  // namespace

hipError_t LaunchReduce(void *dst, const void *src, size_t count, int dtype, int op,
                        hipStream_t stream) {
  if (count == 0) return hipSuccess;
  return DispatchType(dtype, op == kOpOr, [&](auto *tag) -> hipError_t {
    using T = typename std::remove_pointer<decltype(tag)>::type;
    switch (op) {
      case kOpMax: return Reduce2<T, kOpMax>(dst, src, count, stream);
      case kOpMin: return Reduce2<T, kOpMin>(dst, src, count, stream);
      case kOpSum: return Reduce2<T, kOpSum>(dst, src, count, stream);
      case kOpOr: return OrTag<T>::Reduce2Or(dst, src, count, stream);
      default: return hipErrorInvalidValue;
    }
  });
}

hipError_t LaunchReduceMulti(void *dst, const void *const *srcs, int nsrc, size_t count,
                             int dtype, int op, hipStream_t stream) {
  if (count == 0) return hipSuccess;
  if (nsrc < 1 || nsrc > kMaxReduceSources) return hipErrorInvalidValue;
  return DispatchType(dtype, op == kOpOr, [&](auto *tag) -> hipError_t {
    using T = typename std::remove_pointer<decltype(tag)>::type;
    switch (op) {
      case kOpMax: return ReduceMulti<T, kOpMax>(dst, srcs, nsrc, count, stream);
      case kOpMin: return ReduceMulti<T, kOpMin>(dst, srcs, nsrc, count, stream);
      case kOpSum: return ReduceMulti<T, kOpSum>(dst, srcs, nsrc, count, stream);
      case kOpOr: return OrTag<T>::MultiOr(dst, srcs, nsrc, count, stream);
      default: return hipErrorInvalidValue;
    }
  });
}

hipError_t LaunchPrepare(void *dst, void *dst2, const void *src, size_t count, int dtype,
                         int prep, double alpha, hipStream_t stream) {
  if (count == 0) return hipSuccess;
  return DispatchType(dtype, false, [&](auto *tag) -> hipError_t {
    using T = typename std::remove_pointer<decltype(tag)>::type;
    return Prepare<T>(dst, dst2, src, count, prep, alpha, stream);
  });
}

hipError_t LaunchChecksum(const void *buf, size_t nbytes, unsigned long long *out,
                          hipStream_t stream) {
  if (nbytes % 4 != 0 || !Aligned16(buf)) return hipErrorInvalidValue;
  const size_t nwords = nbytes / 4;
  if (nwords == 0) return hipSuccess;
  hipLaunchKernelGGL(ChecksumKernel, dim3(GridFor(nwords / 4 + 1)), dim3(kBlock), 0, stream,
                     static_cast<const uint32_t *>(buf), nwords, out);
  return hipGetLastError();
}

hipError_t LaunchCopy(void *dst, const void *src, size_t bytes, hipStream_t stream) {
  if (bytes == 0 || dst == src) return hipSuccess;
  const size_t nvec = Aligned16(dst) && Aligned16(src) ? bytes / 16 : 0;
  if (nvec != 0) {
    hipLaunchKernelGGL(CopyVecKernel, dim3(GridFor((nvec + kUnroll - 1) / kUnroll)),
                       dim3(kBlock), 0, stream, static_cast<uint4 *>(dst),
                       static_cast<const uint4 *>(src), nvec);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  const size_t done = nvec * 16;
  if (done < bytes) {
    return hipMemcpyAsync(static_cast<char *>(dst) + done, static_cast<const char *>(src) + done,
                          bytes - done, hipMemcpyDeviceToDevice, stream);
  }
  return hipSuccess;
}

hipError_t LaunchFill(void *dst, size_t count, int dtype, double value, hipStream_t stream) {
  if (count == 0) return hipSuccess;
  return DispatchType(dtype, false, [&](auto *tag) -> hipError_t {
    using T = typename std::remove_pointer<decltype(tag)>::type;
    hipLaunchKernelGGL(FillKernel<T>, dim3(GridFor(count)), dim3(kBlock), 0, stream,
                       static_cast<T *>(dst), count, static_cast<T>(value));
    return hipGetLastError();
  });
}
}  // namespace device
}  // namespace rabit
