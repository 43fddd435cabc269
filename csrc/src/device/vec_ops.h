/*!
 * \file vec_ops.h
 * \brief Device-side building blocks shared by the gfx950 streaming kernels (kernels.hip) and
 *        the direct transport's fused allreduce (fused_allreduce.hip): the reduction ops of
 *        rabit (reference `include/rabit/internal/rabit-inl.h:67-102`) applied lane-wise to
 *        16-byte vectors, the lazy-prepare transforms and the nontemporal 16-byte store.
 *        Include from .hip translation units only.
 */
#ifndef XRABIT_DEVICE_VEC_OPS_H_
#define XRABIT_DEVICE_VEC_OPS_H_

#include <hip/hip_runtime.h>

#include <cstdint>
#include <type_traits>

#include "device/kernels.h"
#include "rabit/internal/half.h"

namespace rabit {
namespace device {
namespace vec {

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

/*! \brief lane-wise op on the T lanes of two 16-byte vectors */
template <typename T, int OP>
__device__ __forceinline__ uint4 Combine(uint4 a, uint4 b) {
  constexpr int L = 16 / sizeof(T);
  T x[L], y[L];
  __builtin_memcpy(x, &a, 16);
  __builtin_memcpy(y, &b, 16);
#pragma unroll
  for (int j = 0; j < L; ++j) x[j] = Apply<T, OP>::f(x[j], y[j]);
  uint4 r;
  __builtin_memcpy(&r, x, 16);
  return r;
}

typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));
/*! \brief streaming (nontemporal) 16-byte store: for outputs that are not the buffer just read
 *  (two inputs -> third buffer measured 71 -> 57 us per 128 MiB; neutral for in-place / copy) */
__device__ __forceinline__ void StoreNT(uint4 *p, uint4 v) {
  u32x4_t w = {v.x, v.y, v.z, v.w};
  // compiler-only barrier: without it a later pass rebuilds this store as <4 x float> and drops
  // the !nontemporal tag in the multi-source kernel (seen in the LLVM IR of hipcc, ROCm 7.2)
  asm volatile("" ::: "memory");
  __builtin_nontemporal_store(w, reinterpret_cast<u32x4_t *>(p));
}

template <typename T>
__device__ __forceinline__ T PrepApply(T x, int prep, T alpha) {
  switch (prep) {
    case kPrepSquare: return x * x;
    case kPrepScale: return x * alpha;
    case kPrepAbs:
      if constexpr (std::is_signed<T>::value || IsHalfType<T>::value) {
        return x < T(0) ? T(0) - x : x;
      }
      return x;
    default: return x;
  }
}

template <typename T>
__device__ __forceinline__ uint4 PrepVec(uint4 v, int prep, T alpha) {
  constexpr int L = 16 / sizeof(T);
  T x[L];
  __builtin_memcpy(x, &v, 16);
#pragma unroll
  for (int j = 0; j < L; ++j) x[j] = PrepApply<T>(x[j], prep, alpha);
  uint4 r;
  __builtin_memcpy(&r, x, 16);
  return r;
}

/*! \brief op over NSRC 16-byte vectors, then the optional post scale.  16-bit floats are
 *  widened: every element is accumulated over all sources in fp32 and rounded once */
template <typename T, int OP, int NSRC>
__device__ __forceinline__ uint4 ReduceVecs(const uint4 *v, double post) {
  if constexpr (IsHalfType<T>::value) {
    constexpr int L = 8;
    T t[L];
    float acc[L];
    __builtin_memcpy(t, &v[0], 16);
#pragma unroll
    for (int j = 0; j < L; ++j) acc[j] = t[j].f();
#pragma unroll
    for (int k = 1; k < NSRC; ++k) {
      __builtin_memcpy(t, &v[k], 16);
#pragma unroll
      for (int j = 0; j < L; ++j) acc[j] = Apply<float, OP>::f(acc[j], t[j].f());
    }
    const float ps = static_cast<float>(post);
#pragma unroll
    for (int j = 0; j < L; ++j) t[j] = T(post != 0.0 ? acc[j] * ps : acc[j]);
    uint4 r;
    __builtin_memcpy(&r, t, 16);
    return r;
  } else {
    uint4 acc = v[0];
#pragma unroll
    for (int k = 1; k < NSRC; ++k) acc = Combine<T, OP>(acc, v[k]);
    if (post != 0.0) acc = PrepVec<T>(acc, kPrepScale, static_cast<T>(post));
    return acc;
  }
}

/*! \brief ReduceVecs over a run-time number of sources n <= MAXN (v[k] for k >= n unused);
 *  sources are combined in index order, so every rank computes the same bits */
template <typename T, int OP, int MAXN>
__device__ __forceinline__ uint4 ReduceVecsN(const uint4 *v, int n, double post) {
  if constexpr (IsHalfType<T>::value) {
    constexpr int L = 8;
    T t[L];
    float acc[L];
    __builtin_memcpy(t, &v[0], 16);
#pragma unroll
    for (int j = 0; j < L; ++j) acc[j] = t[j].f();
#pragma unroll
    for (int k = 1; k < MAXN; ++k) {
      if (k < n) {
        __builtin_memcpy(t, &v[k], 16);
#pragma unroll
        for (int j = 0; j < L; ++j) acc[j] = Apply<float, OP>::f(acc[j], t[j].f());
      }
    }
    const float ps = static_cast<float>(post);
#pragma unroll
    for (int j = 0; j < L; ++j) t[j] = T(post != 0.0 ? acc[j] * ps : acc[j]);
    uint4 r;
    __builtin_memcpy(&r, t, 16);
    return r;
  } else {
    uint4 acc = v[0];
#pragma unroll
    for (int k = 1; k < MAXN; ++k) {
      if (k < n) acc = Combine<T, OP>(acc, v[k]);
    }
    if (post != 0.0) acc = PrepVec<T>(acc, kPrepScale, static_cast<T>(post));
    return acc;
  }
}

/*! \brief scalar reduce of element i over n sources (tails) */
template <typename T, int OP>
__device__ __forceinline__ T ReduceScalarN(const T *const *src, int n, size_t i, double post) {
  if constexpr (IsHalfType<T>::value) {
    float acc = src[0][i].f();
    for (int k = 1; k < n; ++k) acc = Apply<float, OP>::f(acc, src[k][i].f());
    if (post != 0.0) acc *= static_cast<float>(post);
    return T(acc);
  } else {
    T acc = src[0][i];
    for (int k = 1; k < n; ++k) acc = Apply<T, OP>::f(acc, src[k][i]);
    if (post != 0.0) acc = acc * static_cast<T>(post);
    return acc;
  }
}

}  // namespace vec
}  // namespace device
}  // namespace rabit
#endif  // XRABIT_DEVICE_VEC_OPS_H_
