/*!
 * \file kernels.hip
 * \brief gfx950 (MI355X, CDNA4) kernels of the device data plane.
 *
 * All kernels here are HBM-bandwidth bound (element-wise: no reuse), so the goal is the HBM
 * roof (~6.3-7 TB/s achievable on MI355X).  Structure, chosen by measurement
 * (tools/kernel_variants.hip; profiles/r1_s5_kernels, profiles/r1_s12_variants): a one-shot
 * grid in which workgroup b owns the contiguous tile of 256 x U 16-byte vectors at b*256*U:
 *  - every wave instruction moves 1 KiB contiguous (64 lanes x 16 B: global_load_dwordx4);
 *  - U = 1 (32768 workgroups per 128 MiB): copy 39.7 us / dst += src 56.8 us, vs 41.2 / 58.6
 *    at U = 4 and 44.4 / 66.8 for the best grid-stride loops (2048-4096 workgroups);
 *  - all loads of a lane (x sources) are issued before any arithmetic or store;
 *  - the data is loaded as uint4 and re-interpreted in registers, so the compiler cannot split
 *    a 16-byte access into halves (it did with struct-of-T packs: 4.8 TB/s, half-width stores);
 *  - stores to a buffer other than the one just read (multi-source reduce, prepare, dual
 *    store) are nontemporal: two inputs -> third buffer 71 -> 57 us per 128 MiB; nontemporal
 *    loads, and nontemporal stores for in-place / copy, measured neutral to 9 % slower.
 * MFMA is deliberately not used: an element-wise reduce has no data reuse; a ones-vector GEMM
 * over stacked peer buffers moves the same bytes and only adds matrix-pipe work.  Measured
 * (tools/mfma_reduce_probe.hip, profiles/r1_mfma_probe/): 8-source fp32 sum of 16 MiB segments,
 * VALU 28.2 us vs v_mfma_f32_32x32x2_f32 33.1 us vs LDS-staged 48.2 us.
 */
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <map>
#include <mutex>
#include <type_traits>

#include "device/kernels.h"
#include "device/vec_ops.h"
#include "rabit/internal/half.h"

namespace rabit {
namespace device {
namespace {
using namespace vec;  // NOLINT

constexpr int kBlock = 256;

inline bool Aligned16(const void *p) { return (reinterpret_cast<uintptr_t>(p) & 15u) == 0; }

/*! \brief workgroups for a one-shot tile grid over nvec vectors (>= 1) */
inline unsigned TileGrid(size_t nvec, int unroll) {
  size_t per = static_cast<size_t>(kBlock) * unroll;
  size_t g = (nvec + per - 1) / per;
  return static_cast<unsigned>(g == 0 ? 1 : g);
}

/*! \brief elements past the last full 16-byte vector, handled by workgroup 0 */
template <typename T, typename F>
__device__ __forceinline__ void Tail(size_t nvec, size_t n, F &&f) {
  constexpr size_t L = 16 / sizeof(T);
  if (blockIdx.x == 0) {
    for (size_t i = nvec * L + threadIdx.x; i < n; i += kBlock) f(i);
  }
}

// ---------------------------------------------------------------- two-operand reduce
template <typename T, int OP, int U>
__global__ __launch_bounds__(kBlock) void ReduceTileKernel(T *__restrict__ dst,
                                                           const T *__restrict__ src, size_t n) {
  const size_t nvec = n * sizeof(T) / 16;
  uint4 *d = reinterpret_cast<uint4 *>(dst);
  const uint4 *s = reinterpret_cast<const uint4 *>(src);
  const size_t base = static_cast<size_t>(blockIdx.x) * kBlock * U + threadIdx.x;
  if (base + (U - 1) * kBlock < nvec) {
    uint4 a[U], b[U];
#pragma unroll
    for (int u = 0; u < U; ++u) a[u] = d[base + u * kBlock];
#pragma unroll
    for (int u = 0; u < U; ++u) b[u] = s[base + u * kBlock];
#pragma unroll
    for (int u = 0; u < U; ++u) d[base + u * kBlock] = Combine<T, OP>(a[u], b[u]);
  } else {
    for (int u = 0; u < U; ++u) {
      const size_t i = base + u * kBlock;
      if (i < nvec) d[i] = Combine<T, OP>(d[i], s[i]);
    }
  }
  Tail<T>(nvec, n, [&](size_t i) { dst[i] = Apply<T, OP>::f(dst[i], src[i]); });
}

template <typename T, int OP>
__global__ __launch_bounds__(kBlock) void ReduceScalarKernel(T *__restrict__ dst,
                                                             const T *__restrict__ src,
                                                             size_t n) {
  const size_t i = static_cast<size_t>(blockIdx.x) * kBlock + threadIdx.x;
  if (i < n) dst[i] = Apply<T, OP>::f(dst[i], src[i]);
}

template <typename T, int OP>
hipError_t Reduce2(void *dst, const void *src, size_t n, hipStream_t st) {
  T *d = static_cast<T *>(dst);
  const T *s = static_cast<const T *>(src);
  if (Aligned16(dst) && Aligned16(src)) {
    constexpr int U = 1;  // one 16-B vector per lane, 32768 workgroups per 128 MiB (fastest)
    hipLaunchKernelGGL((ReduceTileKernel<T, OP, U>), dim3(TileGrid(n * sizeof(T) / 16, U)),
                       dim3(kBlock), 0, st, d, s, n);
  } else {
    hipLaunchKernelGGL((ReduceScalarKernel<T, OP>), dim3(TileGrid(n, 1)), dim3(kBlock), 0, st, d,
                       s, n);
  }
  return hipGetLastError();
}

// ---------------------------------------------------------------- multi-source reduce
struct SrcList {
  const void *p[kMaxReduceSources];
  const int *guard;  // optional: skip the whole launch when *guard != 0 (failed peer barrier)
  const void *const *table;  // optional: device table of source pointers (overrides p)
  double post_scale;         // != 0: multiply the reduced value by it (floating types)
  void *dst2;                // optional second destination (same values as dst)
  int prep;                  // PrepOp applied to sources prep_from.. as they are loaded (the
  int prep_from;             // lazy prepare fused into the reduce: no separate pass)
  double prep_alpha;
  int coherent;  // 1: sources are read with system-scope loads (see LoadSys16)
};

/*!
 * \brief system-scope 16-byte load (buffer_load_dwordx4 sc0 sc1): never served from a cache line
 *        another agent may have left stale.  The direct transport's pull reduce reads its peers'
 *        inputs in place (zero copy, peer_registry.h) from ordinary cacheable HBM of another
 *        process or GPU, written there by that rank's kernels; this GPU's L2 may still hold the
 *        same addresses from the previous op.  (Stage buffers and the symmetric heap are uncached
 *        anyway, where the scope changes nothing.)  Offsets are 32-bit: callers keep the source
 *        below 2 GiB (one chunk of the stage at most).
 */
__device__ __forceinline__ uint4 LoadSys16(const void *base, size_t vec_index) {
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<void *>(base), 0, 0x7fffffff, 0x00020000);
  const u32x4_t v =
      __builtin_amdgcn_raw_buffer_load_b128(rs, static_cast<int>(vec_index * 16), 0, 1 | 16);
  return make_uint4(v.x, v.y, v.z, v.w);
}

/*! \brief element i of a source with a system-scope load (tails of LoadSys16 reads) */
template <typename T>
__device__ __forceinline__ T LoadSysElem(const void *base, size_t i) {
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<void *>(base), 0, 0x7fffffff, 0x00020000);
  const int off = static_cast<int>(i * sizeof(T));
  T x;
  if constexpr (sizeof(T) == 1) {
    const unsigned char v = __builtin_amdgcn_raw_buffer_load_b8(rs, off, 0, 1 | 16);
    __builtin_memcpy(&x, &v, 1);
  } else if constexpr (sizeof(T) == 2) {
    const unsigned short v = __builtin_amdgcn_raw_buffer_load_b16(rs, off, 0, 1 | 16);
    __builtin_memcpy(&x, &v, 2);
  } else if constexpr (sizeof(T) == 4) {
    const unsigned int v = __builtin_amdgcn_raw_buffer_load_b32(rs, off, 0, 1 | 16);
    __builtin_memcpy(&x, &v, 4);
  } else {
    typedef unsigned int u32x2_t __attribute__((ext_vector_type(2)));
    const u32x2_t v = __builtin_amdgcn_raw_buffer_load_b64(rs, off, 0, 1 | 16);
    __builtin_memcpy(&x, &v, 8);
  }
  return x;
}

/*! \brief source k: from the device table when given (written by an earlier kernel, e.g. a
 *  peer barrier that resolved where each peer's input lives), else the launch argument */
__device__ __forceinline__ const void *Src(const SrcList &s, int k) {
  return s.table != nullptr ? s.table[k] : s.p[k];
}

__device__ __forceinline__ bool Guarded(const int *guard) {
  return guard != nullptr &&
         __hip_atomic_load(guard, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0;
}

/*! \brief scalar form of ReduceVecs over nsrc sources (tails, unaligned buffers) */
template <typename T>
__device__ __forceinline__ T LoadSrc(const SrcList &srcs, int k, size_t i) {
  const T x = srcs.coherent ? LoadSysElem<T>(Src(srcs, k), i)
                            : static_cast<const T *>(Src(srcs, k))[i];
  return srcs.prep != 0 && k >= srcs.prep_from
             ? PrepApply<T>(x, srcs.prep, static_cast<T>(srcs.prep_alpha))
             : x;
}

template <typename T, int OP>
__device__ __forceinline__ T ReduceScalar(const SrcList &srcs, int nsrc, size_t i) {
  if constexpr (IsHalfType<T>::value) {
    float acc = LoadSrc<T>(srcs, 0, i).f();
    for (int k = 1; k < nsrc; ++k) acc = Apply<float, OP>::f(acc, LoadSrc<T>(srcs, k, i).f());
    if (srcs.post_scale != 0.0) acc *= static_cast<float>(srcs.post_scale);
    return T(acc);
  } else {
    T acc = LoadSrc<T>(srcs, 0, i);
    for (int k = 1; k < nsrc; ++k) acc = Apply<T, OP>::f(acc, LoadSrc<T>(srcs, k, i));
    if (srcs.post_scale != 0.0) acc = acc * static_cast<T>(srcs.post_scale);
    return acc;
  }
}

template <typename T, int OP, int NSRC, int U>
__global__ __launch_bounds__(kBlock) void ReduceMultiTileKernel(T *dst, SrcList srcs, size_t n) {
  if (Guarded(srcs.guard)) return;
  const size_t nvec = n * sizeof(T) / 16;
  const size_t base = static_cast<size_t>(blockIdx.x) * kBlock * U + threadIdx.x;
  uint4 *d = reinterpret_cast<uint4 *>(dst);
  uint4 *d2 = reinterpret_cast<uint4 *>(srcs.dst2);
  if (base + (U - 1) * kBlock < nvec) {
    uint4 x[NSRC][U];
#pragma unroll
    for (int k = 0; k < NSRC; ++k) {
      const uint4 *sk = reinterpret_cast<const uint4 *>(Src(srcs, k));
      if (srcs.coherent) {  // uniform branch
#pragma unroll
        for (int u = 0; u < U; ++u) x[k][u] = LoadSys16(sk, base + u * kBlock);
      } else {
#pragma unroll
        for (int u = 0; u < U; ++u) x[k][u] = sk[base + u * kBlock];
      }
    }
    if (srcs.prep != 0) {  // uniform branch: the fused lazy prepare, applied on load
#pragma unroll
      for (int k = 0; k < NSRC; ++k) {
        if (k < srcs.prep_from) continue;
#pragma unroll
        for (int u = 0; u < U; ++u) {
          x[k][u] = PrepVec<T>(x[k][u], srcs.prep, static_cast<T>(srcs.prep_alpha));
        }
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      uint4 v[NSRC];
#pragma unroll
      for (int k = 0; k < NSRC; ++k) v[k] = x[k][u];
      const uint4 acc = ReduceVecs<T, OP, NSRC>(v, srcs.post_scale);
      StoreNT(d + base + u * kBlock, acc);
      if (d2 != nullptr) StoreNT(d2 + base + u * kBlock, acc);
    }
  } else {
    for (int u = 0; u < U; ++u) {
      const size_t i = base + u * kBlock;
      if (i >= nvec) break;
      uint4 v[NSRC];
#pragma unroll
      for (int k = 0; k < NSRC; ++k) {
        v[k] = srcs.coherent ? LoadSys16(Src(srcs, k), i)
                             : reinterpret_cast<const uint4 *>(Src(srcs, k))[i];
        if (srcs.prep != 0 && k >= srcs.prep_from) {
          v[k] = PrepVec<T>(v[k], srcs.prep, static_cast<T>(srcs.prep_alpha));
        }
      }
      const uint4 acc = ReduceVecs<T, OP, NSRC>(v, srcs.post_scale);
      StoreNT(d + i, acc);  // same store kind as the main path (merged stores keep nt)
      if (d2 != nullptr) StoreNT(d2 + i, acc);
    }
  }
  Tail<T>(nvec, n, [&](size_t i) {
    const T acc = ReduceScalar<T, OP>(srcs, NSRC, i);
    dst[i] = acc;
    if (srcs.dst2 != nullptr) static_cast<T *>(srcs.dst2)[i] = acc;
  });
}

template <typename T, int OP>
__global__ __launch_bounds__(kBlock) void ReduceMultiScalarKernel(T *dst, SrcList srcs, int nsrc,
                                                                  size_t n) {
  const size_t i = static_cast<size_t>(blockIdx.x) * kBlock + threadIdx.x;
  if (i >= n || Guarded(srcs.guard)) return;
  const T acc = ReduceScalar<T, OP>(srcs, nsrc, i);
  dst[i] = acc;
  if (srcs.dst2 != nullptr) static_cast<T *>(srcs.dst2)[i] = acc;
}

template <typename T, int OP, int NSRC>
void LaunchMultiTile(T *dst, const SrcList &sl, size_t n, hipStream_t st) {
  // keep ~8 16-byte loads in flight per lane
  constexpr int U = 1;
  hipLaunchKernelGGL((ReduceMultiTileKernel<T, OP, NSRC, U>),
                     dim3(TileGrid(n * sizeof(T) / 16, U)), dim3(kBlock), 0, st, dst, sl, n);
}

template <typename T, int OP>
hipError_t ReduceMulti(void *dst, const void *const *srcs, int nsrc, size_t n, hipStream_t st,
                       const int *guard, const void *const *table, double post_scale,
                       void *dst2, int prep = 0, double prep_alpha = 1.0, int prep_from = 0) {
  SrcList sl;
  sl.guard = guard;
  sl.table = table;
  sl.post_scale = post_scale;
  sl.dst2 = dst2;
  sl.prep = prep;
  sl.prep_from = prep_from;
  sl.prep_alpha = prep_alpha;
  // sources resolved on the device (a barrier's table) may be peers' inputs read in place
  sl.coherent = table != nullptr && n * sizeof(T) < (size_t(1) << 31) ? 1 : 0;
  bool aligned = Aligned16(dst) && (dst2 == nullptr || Aligned16(dst2));
  for (int k = 0; k < kMaxReduceSources; ++k) {
    sl.p[k] = k < nsrc ? srcs[k] : nullptr;
    if (k < nsrc) aligned = aligned && Aligned16(srcs[k]);
  }
  T *d = static_cast<T *>(dst);
  if (!aligned) {
    hipLaunchKernelGGL((ReduceMultiScalarKernel<T, OP>), dim3(TileGrid(n, 1)), dim3(kBlock), 0, st,
                       d, sl, nsrc, n);
    return hipGetLastError();
  }
  switch (nsrc) {
    case 1: LaunchMultiTile<T, OP, 1>(d, sl, n, st); break;
    case 2: LaunchMultiTile<T, OP, 2>(d, sl, n, st); break;
    case 3: LaunchMultiTile<T, OP, 3>(d, sl, n, st); break;
    case 4: LaunchMultiTile<T, OP, 4>(d, sl, n, st); break;
    case 5: LaunchMultiTile<T, OP, 5>(d, sl, n, st); break;
    case 6: LaunchMultiTile<T, OP, 6>(d, sl, n, st); break;
    case 7: LaunchMultiTile<T, OP, 7>(d, sl, n, st); break;
    case 8: LaunchMultiTile<T, OP, 8>(d, sl, n, st); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

// ---------------------------------------------------------------- lazy prepare
template <typename T, int U>
__global__ __launch_bounds__(kBlock) void PrepareTileKernel(T *dst, T *dst2, const T *src,
                                                            size_t n, int prep, T alpha) {
  const size_t nvec = n * sizeof(T) / 16;
  const size_t base = static_cast<size_t>(blockIdx.x) * kBlock * U + threadIdx.x;
  const uint4 *s = reinterpret_cast<const uint4 *>(src);
  uint4 *d = reinterpret_cast<uint4 *>(dst);
  uint4 *d2 = reinterpret_cast<uint4 *>(dst2);
  if (base + (U - 1) * kBlock < nvec) {
    uint4 a[U];
#pragma unroll
    for (int u = 0; u < U; ++u) a[u] = s[base + u * kBlock];
#pragma unroll
    for (int u = 0; u < U; ++u) a[u] = PrepVec<T>(a[u], prep, alpha);
#pragma unroll
    for (int u = 0; u < U; ++u) StoreNT(d + base + u * kBlock, a[u]);
    if (d2 != nullptr) {
#pragma unroll
      for (int u = 0; u < U; ++u) StoreNT(d2 + base + u * kBlock, a[u]);
    }
  } else {
    for (int u = 0; u < U; ++u) {
      const size_t i = base + u * kBlock;
      if (i >= nvec) break;
      const uint4 y = PrepVec<T>(s[i], prep, alpha);
      StoreNT(d + i, y);
      if (d2 != nullptr) StoreNT(d2 + i, y);
    }
  }
  Tail<T>(nvec, n, [&](size_t i) {
    const T y = PrepApply<T>(src[i], prep, alpha);
    dst[i] = y;
    if (dst2 != nullptr) dst2[i] = y;
  });
}

template <typename T>
__global__ __launch_bounds__(kBlock) void PrepareScalarKernel(T *dst, T *dst2, const T *src,
                                                              size_t n, int prep, T alpha) {
  const size_t i = static_cast<size_t>(blockIdx.x) * kBlock + threadIdx.x;
  if (i >= n) return;
  const T y = PrepApply<T>(src[i], prep, alpha);
  dst[i] = y;
  if (dst2 != nullptr) dst2[i] = y;
}

template <typename T>
hipError_t Prepare(void *dst, void *dst2, const void *src, size_t n, int prep, double alpha,
                   hipStream_t st) {
  T *d = static_cast<T *>(dst);
  T *d2 = static_cast<T *>(dst2);
  const T *s = static_cast<const T *>(src);
  const T a = static_cast<T>(alpha);
  if (Aligned16(dst) && Aligned16(src) && (dst2 == nullptr || Aligned16(dst2))) {
    constexpr int U = 1;
    hipLaunchKernelGGL((PrepareTileKernel<T, U>), dim3(TileGrid(n * sizeof(T) / 16, U)),
                       dim3(kBlock), 0, st, d, d2, s, n, prep, a);
  } else {
    hipLaunchKernelGGL(PrepareScalarKernel<T>, dim3(TileGrid(n, 1)), dim3(kBlock), 0, st, d, d2, s,
                       n, prep, a);
  }
  return hipGetLastError();
}

// ---------------------------------------------------------------- copy
template <int U>
__global__ __launch_bounds__(kBlock) void CopyTileKernel(uint4 *__restrict__ dst,
                                                        const uint4 *__restrict__ src,
                                                        size_t nvec) {
  const size_t base = static_cast<size_t>(blockIdx.x) * kBlock * U + threadIdx.x;
  if (base + (U - 1) * kBlock < nvec) {
    uint4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = src[base + u * kBlock];
#pragma unroll
    for (int u = 0; u < U; ++u) dst[base + u * kBlock] = v[u];
  } else {
    for (int u = 0; u < U; ++u) {
      const size_t i = base + u * kBlock;
      if (i < nvec) dst[i] = src[i];
    }
  }
}

/*!
 * Narrow copy for device -> pinned host memory (rabit_device_mirror_engine=kernel for
 * checkpoint mirrors): `ctas` workgroups walk the buffer grid-stride, 4 x 16 B per lane in
 * flight, with nontemporal stores.  PCIe (~55 GB/s) bounds the copy, so a few workgroups reach
 * it.  It is NOT the default: measured against 20 bf16 8192^3 GEMMs on the caller's stream
 * (tools/mirror_probe.py, profiles/r2_s15_mirror), a 256 MiB mirror by hipMemcpyAsync (a blit
 * kernel in PyTorch processes) costs the step +0.4 %, by this kernel at 4-1024 workgroups
 * 2.7-4 ms: a few CUs slowed for the whole copy stretch the GEMM's last wave of tiles.
 */
__global__ __launch_bounds__(kBlock) void CopyNarrowKernel(uint4 *__restrict__ dst,
                                                          const uint4 *__restrict__ src,
                                                          size_t nvec) {
  constexpr int U = 4;
  const size_t stride = static_cast<size_t>(gridDim.x) * kBlock;
  size_t i = static_cast<size_t>(blockIdx.x) * kBlock + threadIdx.x;
  for (; i + (U - 1) * stride < nvec; i += U * stride) {
    uint4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = src[i + u * stride];
#pragma unroll
    for (int u = 0; u < U; ++u) StoreNT(&dst[i + u * stride], v[u]);
  }
  for (; i < nvec; i += stride) StoreNT(&dst[i], src[i]);
}

// ---------------------------------------------------------------- checksum
/*!
 * Position-weighted checksum over 16-byte vectors v (words w0..w3):
 *   s1 = sum of all 32-bit words,  s2 = sum_v (v+1) * (w0 + 2 w1 + 3 w2 + 4 w3)   (mod 2^64)
 * One 64-bit multiply per 16 bytes keeps it bandwidth-bound; order changes across vectors
 * and within a vector both change s2.
 */
constexpr int kChecksumGrid = 1024;  // 4 workgroups per CU, tiles walked grid-stride (measured
                                     // best with 4 vectors per lane: tools/checksum_variants.hip)
constexpr int kChecksumShards = 8;   // arrival counters, one 128-byte line each

__device__ __forceinline__ void BlockSum2(unsigned long long &s1, unsigned long long &s2) {
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
    s1 = s2 = 0;
#pragma unroll
    for (int k = 0; k < kBlock / 64; ++k) {
      s1 += part[0][k];
      s2 += part[1][k];
    }
  }
}

/*!
 * \brief one launch: each workgroup folds its tiles into one (s1, s2) partial, and the workgroup
 *        that arrives last (agent-scope counter) adds all partials into out and re-arms the
 *        counter.  No atomics on the sums themselves (8192 workgroups adding into one word
 *        serialise, measured 3.3x slower than partials) and no second launch (a dependent
 *        one-workgroup kernel costs ~4 us, 15 % of a 128 MiB checksum).
 */
template <int U>
__global__ __launch_bounds__(kBlock) void ChecksumKernel(const uint4 *__restrict__ w, size_t nvec,
                                                         unsigned long long *partial,
                                                         unsigned int *arrived,
                                                         unsigned long long *out) {
  unsigned long long s1 = 0, s2 = 0;
  const size_t ntile = (nvec + static_cast<size_t>(kBlock) * U - 1) / (kBlock * U);
  for (size_t t = blockIdx.x; t < ntile; t += gridDim.x) {
    const size_t base = t * kBlock * U + threadIdx.x;
    uint4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const size_t i = base + u * kBlock;
      v[u] = i < nvec ? w[i] : make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const unsigned long long idx = base + u * kBlock + 1ull;
      const unsigned long long q = static_cast<unsigned long long>(v[u].x) + 2ull * v[u].y +
                                   3ull * v[u].z + 4ull * v[u].w;
      s1 += static_cast<unsigned long long>(v[u].x) + v[u].y + v[u].z + v[u].w;
      s2 += idx * q;
    }
  }
  BlockSum2(s1, s2);
  // Hand-off (MI355X_MICROARCH.md, inter-workgroup visibility): every partial is stored sc1
  // (written through, agent scope) and drained (vmcnt(0)) before the same lane's agent-scope
  // add to the counter of its shard (blockIdx % 8: one 128-byte line each, so 8 chains of
  // ~grid/8 adds instead of one chain of grid adds: a single counter took 20 us at 2048
  // workgroups).  The workgroup whose add completes its shard releases (agent fence) and adds
  // to the top counter; the one that completes the top counter acquires and sums all partials.
  __shared__ bool last;
  if (threadIdx.x == 0) {
    __hip_atomic_store(&partial[2 * blockIdx.x], s1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(&partial[2 * blockIdx.x + 1], s2, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const unsigned shard = blockIdx.x % kChecksumShards;
    const unsigned members = (gridDim.x - shard + kChecksumShards - 1) / kChecksumShards;
    const unsigned shards = gridDim.x < kChecksumShards ? gridDim.x : kChecksumShards;
    bool top = false;
    if (__hip_atomic_fetch_add(arrived + shard * 32, 1u, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT) == members - 1) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      top = __hip_atomic_fetch_add(arrived + kChecksumShards * 32, 1u, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT) == shards - 1;
      if (top) {
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
    }
    last = top;
  }
  __syncthreads();
  if (!last) return;
  s1 = s2 = 0;
  for (unsigned i = threadIdx.x; i < gridDim.x; i += kBlock) {
    s1 += __hip_atomic_load(&partial[2 * i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s2 += __hip_atomic_load(&partial[2 * i + 1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  BlockSum2(s1, s2);
  if (threadIdx.x == 0) {
    out[0] += s1;
    out[1] += s2;
    // re-armed for the next launch on this device (stream order)
    for (int k = 0; k <= kChecksumShards; ++k) {
      __hip_atomic_store(arrived + k * 32, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

// ---------------------------------------------------------------- fill
template <typename T>
__global__ __launch_bounds__(kBlock) void FillKernel(T *dst, size_t n, T value) {
  const size_t i = static_cast<size_t>(blockIdx.x) * kBlock + threadIdx.x;
  if (i < n) dst[i] = value;
}

// ---------------------------------------------------------------- fault injection
__global__ __launch_bounds__(64) void HangKernel(const volatile int *release, long long max_ticks) {
  if (threadIdx.x != 0) return;
  const long long t0 = wall_clock64();
  while (*release == 0 && wall_clock64() - t0 < max_ticks) __builtin_amdgcn_s_sleep(127);
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
    case 10: return int_only ? hipErrorInvalidValue : fn(static_cast<half_t *>(nullptr));
    case 11: return int_only ? hipErrorInvalidValue : fn(static_cast<bf16_t *>(nullptr));
    default: return hipErrorInvalidValue;
  }
}

template <typename T>
struct OrTag {
  // BitOR is only instantiated for integral types
  static hipError_t Reduce2Or(void *d, const void *s, size_t n, hipStream_t st) {
    if constexpr (std::is_integral<T>::value) return Reduce2<T, kOpOr>(d, s, n, st);
    return hipErrorInvalidValue;
  }
  static hipError_t MultiOr(void *d, const void *const *s, int k, size_t n, hipStream_t st,
                            const int *guard, const void *const *table, void *d2, int prep,
                            double alpha, int prep_from) {
    if constexpr (std::is_integral<T>::value) {
      return ReduceMulti<T, kOpOr>(d, s, k, n, st, guard, table, 0.0, d2, prep, alpha, prep_from);
    }
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
                             int dtype, int op, hipStream_t stream, const int *guard,
                             const void *const *table, double post_scale, void *dst2, int prep,
                             double prep_alpha, int prep_from) {
  if (count == 0) return hipSuccess;
  if (post_scale != 0.0 && dtype != 6 && dtype != 7 && dtype != 10 && dtype != 11) {
    return hipErrorInvalidValue;  // floating types only
  }
  if (nsrc < 1 || nsrc > kMaxReduceSources) return hipErrorInvalidValue;
  return DispatchType(dtype, op == kOpOr, [&](auto *tag) -> hipError_t {
    using T = typename std::remove_pointer<decltype(tag)>::type;
    switch (op) {
      case kOpMax:
        return ReduceMulti<T, kOpMax>(dst, srcs, nsrc, count, stream, guard, table, post_scale,
                                      dst2, prep, prep_alpha, prep_from);
      case kOpMin:
        return ReduceMulti<T, kOpMin>(dst, srcs, nsrc, count, stream, guard, table, post_scale,
                                      dst2, prep, prep_alpha, prep_from);
      case kOpSum:
        return ReduceMulti<T, kOpSum>(dst, srcs, nsrc, count, stream, guard, table, post_scale,
                                      dst2, prep, prep_alpha, prep_from);
      case kOpOr:
        return OrTag<T>::MultiOr(dst, srcs, nsrc, count, stream, guard, table, dst2, prep,
                                 prep_alpha, prep_from);
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

hipError_t LaunchCopy(void *dst, const void *src, size_t bytes, hipStream_t stream) {
  if (bytes == 0 || dst == src) return hipSuccess;
  const size_t nvec = Aligned16(dst) && Aligned16(src) ? bytes / 16 : 0;
  if (nvec != 0) {
    constexpr int U = 1;
    hipLaunchKernelGGL(CopyTileKernel<U>, dim3(TileGrid(nvec, U)), dim3(kBlock), 0, stream,
                       static_cast<uint4 *>(dst), static_cast<const uint4 *>(src), nvec);
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

hipError_t LaunchCopyNarrow(void *dst, const void *src, size_t bytes, int ctas,
                            hipStream_t stream) {
  if (bytes == 0 || dst == src) return hipSuccess;
  const size_t nvec = Aligned16(dst) && Aligned16(src) ? bytes / 16 : 0;
  if (nvec != 0) {
    const size_t per = static_cast<size_t>(kBlock) * 4;
    const unsigned grid = static_cast<unsigned>(
        std::max<size_t>(1, std::min<size_t>(std::max(ctas, 1), (nvec + per - 1) / per)));
    hipLaunchKernelGGL(CopyNarrowKernel, dim3(grid), dim3(kBlock), 0, stream,
                       static_cast<uint4 *>(dst), static_cast<const uint4 *>(src), nvec);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  const size_t done = nvec * 16;
  if (done < bytes) {
    return hipMemcpyAsync(static_cast<char *>(dst) + done, static_cast<const char *>(src) + done,
                          bytes - done, hipMemcpyDefault, stream);
  }
  return hipSuccess;
}

hipError_t LaunchChecksum(const void *buf, size_t nbytes, unsigned long long *out,
                          hipStream_t stream) {
  if (nbytes % 16 != 0 || !Aligned16(buf)) return hipErrorInvalidValue;
  const size_t nvec = nbytes / 16;
  if (nvec == 0) return hipSuccess;
  // per-device scratch: 2 x kChecksumGrid u64 partials + the arrival counter (zeroed once;
  // the last workgroup of every launch re-arms it).  Launches of one device must not overlap
  // (they are stream-ordered in the engine).
  static std::mutex mu;
  static std::map<int, unsigned long long *> scratch;
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return e;
  unsigned long long *partial;
  {
    std::lock_guard<std::mutex> lk(mu);
    auto it = scratch.find(dev);
    if (it == scratch.end()) {
      void *p = nullptr;
      const size_t bytes =
          sizeof(unsigned long long) * 2 * kChecksumGrid + 128 * (kChecksumShards + 1);
      e = hipMalloc(&p, bytes);
      if (e != hipSuccess) return e;
      e = hipMemset(p, 0, bytes);
      if (e == hipSuccess) e = hipDeviceSynchronize();
      if (e != hipSuccess) return e;
      it = scratch.emplace(dev, static_cast<unsigned long long *>(p)).first;
    }
    partial = it->second;
  }
  constexpr int U = 4;
  const unsigned grid = std::min<unsigned>(TileGrid(nvec, U), kChecksumGrid);
  hipLaunchKernelGGL(ChecksumKernel<U>, dim3(grid), dim3(kBlock), 0, stream,
                     static_cast<const uint4 *>(buf), nvec, partial,
                     reinterpret_cast<unsigned int *>(partial + 2 * kChecksumGrid), out);
  return hipGetLastError();
}

hipError_t LaunchHang(const volatile int *release, long long max_ticks, hipStream_t stream) {
  hipLaunchKernelGGL(HangKernel, dim3(1), dim3(64), 0, stream, release, max_ticks);
  return hipGetLastError();
}

hipError_t LaunchFill(void *dst, size_t count, int dtype, double value, hipStream_t stream) {
  if (count == 0) return hipSuccess;
  return DispatchType(dtype, false, [&](auto *tag) -> hipError_t {
    using T = typename std::remove_pointer<decltype(tag)>::type;
    hipLaunchKernelGGL(FillKernel<T>, dim3(TileGrid(count, 1)), dim3(kBlock), 0, stream,
                       static_cast<T *>(dst), count, static_cast<T>(value));
    return hipGetLastError();
  });
}
}  // namespace device
}  // namespace rabit
