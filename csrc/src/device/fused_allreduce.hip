/*!
 * \file fused_allreduce.hip
 * \brief gfx950 kernel of the direct transport's fused two-shot allreduce (one launch per chunk;
 *        see FusedAllreduceArgs in peer_coll.h for the protocol).
 *
 * It replaces the reference's ring reduce-scatter + allgather (`src/allreduce_base.cc:958-977`)
 * for GPUs that read each other's HBM: every rank reduces 1/n of the chunk from all n inputs and
 * everyone gathers the n reduced segments, so 2(n-1)/n of the payload crosses xGMI per rank,
 * over all 7 links at once.  The classic form (peer_coll.cc) launches 5 kernels per chunk and
 * meets the peers at two whole-GPU barriers; here each tile is handed over on its own:
 *
 *  - hand-off (MI355X_MICROARCH.md, "inter-workgroup visibility"): every handed-off byte is in
 *    the uncached stage allocations, so the producer only waits for its stores to complete
 *    (s_waitcnt vmcnt(0) in every wave, workgroup barrier) before wave 0 stores the epoch into
 *    the flags (relaxed, system scope).  Bytes it pushes into a peer's stage go through this
 *    GPU's mapping of that memory, which may be cacheable here: they leave as system-scope
 *    write-through stores (sc0 sc1), and a tile with element-wise tails releases at system scope
 *    (L2 write-back) before its flag.
 *    Consumer: wave 0 polls (relaxed, s_sleep back-off), one system-scope acquire fence (a peer's
 *    mapping may be cacheable on this GPU), vmcnt(0), workgroup barrier, then loads;
 *  - every poll gives up on the host abort word (peer failure seen on the TCP control plane), the
 *    wall-clock deadline, or a failure another workgroup already recorded; the failure goes to
 *    the group's device status word (guard of every later kernel) and to a pinned host word;
 *  - streaming: each lane keeps one 16-byte load per source in flight (n remote loads at once;
 *    4 for the staging copy), 4 workgroups per CU (128 VGPRs), results leave with nontemporal
 *    stores;
 *  - tiles shrink (down to 8 KiB) for small chunks so the grid still covers the GPU; a rank whose
 *    own buffers are unaligned touches them element-wise, the protocol is the same everywhere.
 */
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <type_traits>

#include "device/peer_coll.h"
#include "device/vec_ops.h"
#include "rabit/internal/half.h"

namespace rabit {
namespace device {
namespace {
using namespace vec;  // NOLINT

constexpr int kBlock = 256;
constexpr int kFlagBase = 64;  // u64 words before the ready array (word 0: mailbox)
constexpr int kCpolSystem = 1 | 16;      // cache policy sc0 | sc1: system scope, write-through
constexpr int kRsrcWord3 = 0x00020000;   // buffer descriptor word 3 for raw 32-bit offsets (gfx950)

__device__ __forceinline__ unsigned long long *ReadyFlag(const FusedAllreduceArgs &a, int owner,
                                                         int i) {
  return a.flags[owner] + kFlagBase + i;
}
__device__ __forceinline__ unsigned long long *DoneFlag(const FusedAllreduceArgs &a, int owner,
                                                        int i) {
  return a.flags[owner] + kFlagBase + a.tiles_cap + i;
}
/*! \brief inbox flag at `owner` for the tile `sender` pushed */
__device__ __forceinline__ unsigned long long *InboxFlag(const FusedAllreduceArgs &a, int owner,
                                                         int sender, int i) {
  return a.flags[owner] + kFlagBase + static_cast<size_t>(2 + sender) * a.tiles_cap + i;
}

__device__ __forceinline__ bool GroupFailed(const FusedAllreduceArgs &a) {
  return __hip_atomic_load(a.dev_status, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0;
}

/*! \brief element range [lo, hi) of tile i of segment q */
__device__ __forceinline__ void TileRange(const FusedAllreduceArgs &a, int q, int i, size_t *lo,
                                          size_t *hi) {
  const size_t s0 = static_cast<size_t>(q) * a.seg;
  const size_t l = s0 + static_cast<size_t>(i) * a.tile;
  *lo = l < a.count ? l : a.count;
  size_t h = l + a.tile;
  if (h > s0 + a.seg) h = s0 + a.seg;
  if (h > a.count) h = a.count;
  *hi = h > *lo ? h : *lo;
}

/*!
 * \brief producer side of a hand-off: wait until this workgroup's stores have completed, then
 *        wave 0 stores the epoch into the flags its lanes name (lane k: flag(k), unless null).
 *        Every handed-off byte lives in uncached memory (stage buffers: hipDeviceMallocUncached,
 *        also for peers' pushes), so a completed store is visible to any reader and no L2
 *        write-back is needed (the out / out2 results are only read after the launch).
 */
template <typename FlagOf>
__device__ __forceinline__ void Publish(const FusedAllreduceArgs &a, int nflags, FlagOf flag,
                                        bool remote_stores = false) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x < 64) {
    if (remote_stores) {
      // some handed-off bytes went into a PEER's memory with plain stores (element-wise tails):
      // this GPU's mapping of it may be cacheable, so write this XCD's L2 back (system-scope
      // release) before the flag; the wait keeps the flag behind the write-back
      // (MI355X_MICROARCH.md, compiler hazard)
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    const int k = static_cast<int>(threadIdx.x);
    if (k < nflags) {
      unsigned long long *f = flag(k);
      if (f != nullptr) {
        __hip_atomic_store(f, a.epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      }
    }
  }
}

/*!
 * \brief consumer side: wave 0 lane k polls flag(k) (k < nflags, non-null) until it reaches the
 *        epoch; false (failure recorded) if any gives up.  Every thread returns the same value.
 */
template <typename FlagOf>
__device__ __forceinline__ bool Await(const FusedAllreduceArgs &a, int *s_bad, int nflags,
                                      FlagOf flag) {
  if (threadIdx.x < 64) {
    const int k = static_cast<int>(threadIdx.x);
    bool ok = true;
    if (k < nflags) {
      unsigned long long *f = flag(k);
      if (f != nullptr) {
        const long long t0 = wall_clock64();
        while (__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) < a.epoch) {
          if (*a.abort_word != 0 || *a.peer_abort != 0 || wall_clock64() - t0 > a.deadline_ticks ||
              GroupFailed(a)) {
            ok = false;
            break;
          }
          __builtin_amdgcn_s_sleep(2);
        }
      }
    }
    if (!ok) {
      __hip_atomic_store(a.dev_status, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      __hip_atomic_store(a.host_status, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      *s_bad = 1;
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
  return *s_bad == 0;
}

/*! \brief 16-byte store of v at byte offset `off` of the buffer `rs` describes.  REMOTE: a peer's
 *  memory through this GPU's mapping of it, which may be cacheable here, so the store is
 *  system-scope write-through (cache policy sc0 sc1): once it completes (vmcnt) it is visible to
 *  the peer with no L2 write-back of this XCD (MI355X_MICROARCH.md, inter-workgroup visibility;
 *  cdna_hip_programming.md Guideline 16 R1, at system instead of agent scope) */
template <bool REMOTE>
__device__ __forceinline__ void StoreStage(uint4 *dv, __amdgpu_buffer_rsrc_t rs, size_t v,
                                           uint4 x) {
  if (REMOTE) {
    u32x4_t w = {x.x, x.y, x.z, x.w};
    __builtin_amdgcn_raw_buffer_store_b128(w, rs, static_cast<int>(v * 16), 0, kCpolSystem);
  } else {
    dv[v] = x;
  }
}

/*! \brief d[0, n) = prep(s[0, n)) by the workgroup: 4 x 16-byte loads in flight per lane when
 *  both are 16-byte aligned (d always is: stage memory), element-wise otherwise.  Returns true
 *  if any element went out element-wise (plain stores: a REMOTE hand-off of those needs a
 *  system-scope release before its flag). */
template <typename T, bool REMOTE>
__device__ __forceinline__ bool CopyPrep(T *d, const T *s, size_t n, int prep, T alpha,
                                         bool vec_src) {
  constexpr size_t L = 16 / sizeof(T);
  size_t nvec = 0;
  if (vec_src) {
    nvec = n / L;
    const uint4 *sv = reinterpret_cast<const uint4 *>(s);
    uint4 *dv = reinterpret_cast<uint4 *>(d);
    // one descriptor per call (d and n are uniform over the workgroup; n * sizeof(T) is at most
    // one tile, far below the 4 GiB of a descriptor's 32-bit offsets)
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc(d, 0, static_cast<int>(nvec * 16), kRsrcWord3);
    size_t v = threadIdx.x;
    for (; v + 3 * kBlock < nvec; v += 4 * kBlock) {
      uint4 t[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) t[u] = sv[v + u * kBlock];
      if (prep != kPrepCopy) {
#pragma unroll
        for (int u = 0; u < 4; ++u) t[u] = PrepVec<T>(t[u], prep, alpha);
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) StoreStage<REMOTE>(dv, rs, v + u * kBlock, t[u]);
    }
    for (; v < nvec; v += kBlock) {
      StoreStage<REMOTE>(dv, rs, v, prep == kPrepCopy ? sv[v] : PrepVec<T>(sv[v], prep, alpha));
    }
  }
  for (size_t e = nvec * L + threadIdx.x; e < n; e += kBlock) {
    d[e] = PrepApply<T>(s[e], prep, alpha);
  }
  return nvec * L < n;
}

/*! \brief store the 16-byte vector v as elements [e, e + 16 / sizeof(T)) of dst */
template <typename T>
__device__ __forceinline__ void PutVec(T *dst, size_t e, uint4 v, bool vec) {
  if (vec) {
    StoreNT(reinterpret_cast<uint4 *>(dst + e), v);
  } else {
    constexpr int L = 16 / sizeof(T);
    T x[L];
    __builtin_memcpy(x, &v, 16);
#pragma unroll
    for (int j = 0; j < L; ++j) dst[e + j] = x[j];
  }
}

/*!
 * \brief reduce phase of one tile: res / out / out2 [v] = op over the n sources s_in[k][v] for
 *        the nvec 16-byte vectors of the tile.  Each lane loads U vectors of every source before
 *        it combines or stores any (MAXN x U x 16 B in flight per lane; MAXN x U <= 16 keeps the
 *        4-workgroups-per-CU register budget), sources in rank order.
 */
template <typename T, int OP, int MAXN, int U>
__device__ __forceinline__ void ReduceTileVec(const char *const *s_in, int n, size_t nvec, T *out,
                                              T *out2, uint4 *res, size_t lo, bool vout,
                                              double post) {
  constexpr size_t L = 16 / sizeof(T);
  size_t v = threadIdx.x;
  for (; v + (U - 1) * kBlock < nvec; v += U * kBlock) {
    uint4 x[U][MAXN];
#pragma unroll
    for (int k = 0; k < MAXN; ++k) {
      if (k < n) {
        const uint4 *sk = reinterpret_cast<const uint4 *>(s_in[k]);
#pragma unroll
        for (int u = 0; u < U; ++u) x[u][k] = sk[v + u * kBlock];
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint4 y = ReduceVecsN<T, OP, MAXN>(x[u], n, post);
      const size_t e = lo + (v + u * kBlock) * L;
      PutVec<T>(out, e, y, vout);
      if (out2 != nullptr) PutVec<T>(out2, e, y, vout);
      res[v + u * kBlock] = y;
    }
  }
  for (; v < nvec; v += kBlock) {
    uint4 x[MAXN];
#pragma unroll
    for (int k = 0; k < MAXN; ++k) {
      if (k < n) x[k] = reinterpret_cast<const uint4 *>(s_in[k])[v];
    }
    const uint4 y = ReduceVecsN<T, OP, MAXN>(x, n, post);
    PutVec<T>(out, lo + v * L, y, vout);
    if (out2 != nullptr) PutVec<T>(out2, lo + v * L, y, vout);
    res[v] = y;
  }
}

/*!
 * \brief gather phase of one tile index: copy the reduced tile of every other rank p (s_nv[p]
 *        elements at s_lo[p] of its stage; 0 for this rank) into out / out2, U vectors per peer
 *        per lane loaded before any store (whole 16-byte vectors; the element tails follow in
 *        the caller)
 */
template <typename T, int MAXN, int U>
__device__ __forceinline__ void GatherTileVec(const FusedAllreduceArgs &a, const size_t *s_lo,
                                              const size_t *s_nv, int n, T *out, T *out2,
                                              bool vout) {
  constexpr size_t L = 16 / sizeof(T);
  const size_t most = (a.tile + L - 1) / L;
  for (size_t v = threadIdx.x; v < most; v += U * kBlock) {
    uint4 x[U][MAXN];
#pragma unroll
    for (int p = 0; p < MAXN; ++p) {
      if (p < n) {
        const size_t nv = s_nv[p] / L;
        const uint4 *sp =
            reinterpret_cast<const uint4 *>(reinterpret_cast<const T *>(a.stage[p]) + s_lo[p]);
#pragma unroll
        for (int u = 0; u < U; ++u) {
          if (v + u * kBlock < nv) x[u][p] = sp[v + u * kBlock];
        }
      }
    }
#pragma unroll
    for (int p = 0; p < MAXN; ++p) {
      if (p < n) {
        const size_t nv = s_nv[p] / L;
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const size_t w = v + u * kBlock;
          if (w < nv) {
            PutVec<T>(out, s_lo[p] + w * L, x[u][p], vout);
            if (out2 != nullptr) PutVec<T>(out2, s_lo[p] + w * L, x[u][p], vout);
          }
        }
      }
    }
  }
}

template <typename T, int OP>
__global__ __launch_bounds__(kBlock, 4) void FusedAllreduceKernel(FusedAllreduceArgs a) {
  __shared__ int s_bad;
  __shared__ const char *s_in[kMaxPeers];
  if (GroupFailed(a)) return;  // an earlier op of this group failed: touch nothing
  if (threadIdx.x == 0) s_bad = 0;
  __syncthreads();
  const int n = a.n, r = a.rank;
  constexpr size_t L = 16 / sizeof(T);
  const T alpha = static_cast<T>(a.alpha);
  const T *src = reinterpret_cast<const T *>(a.src);
  T *out = reinterpret_cast<T *>(a.out);
  T *out2 = reinterpret_cast<T *>(a.out2);
  T *mine = reinterpret_cast<T *>(a.stage[r]);
  // the caller's buffers may be unaligned on this rank only (views): that changes how this rank
  // touches its own memory, never the protocol, which every rank runs identically
  const bool vsrc = (reinterpret_cast<uintptr_t>(src) & 15u) == 0;
  const bool vout = (reinterpret_cast<uintptr_t>(out) & 15u) == 0 &&
                    (reinterpret_cast<uintptr_t>(out2) & 15u) == 0;

  // ---- 1. stage (pull) or push this workgroup's tiles of every segment, then publish them
  for (int i = blockIdx.x; i < a.tiles; i += gridDim.x) {
    bool scalar_remote = false;  // some pushed element left with a plain (cacheable) store
    if (a.push || !a.zero_copy) {
      for (int q = 0; q < n; ++q) {
        size_t lo, hi;
        TileRange(a, q, i, &lo, &hi);
        if (hi <= lo) continue;
        if (a.push && q != r) {
          T *d = reinterpret_cast<T *>(a.stage[q]) + static_cast<size_t>(r) * a.seg +
                 (lo - static_cast<size_t>(q) * a.seg);
          scalar_remote |= CopyPrep<T, true>(d, src + lo, hi - lo, a.prep, alpha, vsrc);
        } else {
          T *d = a.push ? reinterpret_cast<T *>(a.stage[q]) + static_cast<size_t>(r) * a.seg +
                              (lo - static_cast<size_t>(q) * a.seg)
                        : mine + lo;
          CopyPrep<T, false>(d, src + lo, hi - lo, a.prep, alpha, vsrc);
        }
      }
    }
    if (a.push) {
      // scalar_remote is the same in every thread of the workgroup (sizes and alignment only)
      Publish(a, n, [&](int q) { return InboxFlag(a, q, r, i); }, scalar_remote);
    } else {
      // pull: where this rank's input is (its stage, or its input in place in the symmetric
      // heap) goes out with the flag; every rank chooses for itself
      if (threadIdx.x == 0) {
        __hip_atomic_store(a.flags[r], a.mailbox, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      }
      Publish(a, 1, [&](int) { return ReadyFlag(a, r, i); });
    }
  }

  // ---- 2. reduce this rank's segment: n sources in rank order -> out, out2, own stage
  for (int i = blockIdx.x; i < a.tiles; i += gridDim.x) {
    bool ok;
    if (a.push) {
      ok = Await(a, &s_bad, n, [&](int p) { return InboxFlag(a, r, p, i); });
    } else {
      ok = Await(a, &s_bad, n, [&](int p) { return ReadyFlag(a, p, i); });
    }
    if (!ok) return;
    size_t lo, hi;
    TileRange(a, r, i, &lo, &hi);
    if (threadIdx.x < static_cast<unsigned>(n)) {
      const int p = static_cast<int>(threadIdx.x);
      const char *base;
      if (a.push) {
        // inbox slot p of this rank's stage holds sender p's copy of this segment
        base = a.stage[r] + static_cast<ptrdiff_t>(p - r) *
                                static_cast<ptrdiff_t>(a.seg * sizeof(T));
      } else {
        const unsigned long long m =
            __hip_atomic_load(a.flags[p], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        base = ((m & kMailboxHeap) != 0 ? a.heap[p] : a.alloc[p]) + (m & ~kMailboxHeap);
      }
      s_in[p] = base + lo * sizeof(T);  // this tile of source p
    }
    __syncthreads();
    if (hi > lo) {
      const size_t nvec = (hi - lo) / L;
      uint4 *res = reinterpret_cast<uint4 *>(mine + lo);
      // U vectors per lane per step, every load of the step issued before any store: with one
      // load per source in flight a lane waited a full (remote) latency per 16 bytes
      if (n <= 4) {
        ReduceTileVec<T, OP, 4, 4>(s_in, n, nvec, out, out2, res, lo, vout, a.post);
      } else {
        ReduceTileVec<T, OP, kMaxPeers, 2>(s_in, n, nvec, out, out2, res, lo, vout, a.post);
      }
      for (size_t e = nvec * L + threadIdx.x; e < hi - lo; e += kBlock) {
        const T *srcs[kMaxPeers];
        for (int k = 0; k < n; ++k) srcs[k] = reinterpret_cast<const T *>(s_in[k]);
        const T y = ReduceScalarN<T, OP>(srcs, n, e, a.post);
        out[lo + e] = y;
        if (out2 != nullptr) out2[lo + e] = y;
        mine[lo + e] = y;
      }
    }
    Publish(a, 1, [&](int) { return DoneFlag(a, r, i); });
  }

  // ---- 3. gather every other rank's reduced segment from its stage
  __shared__ size_t s_lo[kMaxPeers], s_nv[kMaxPeers];
  for (int i = blockIdx.x; i < a.tiles; i += gridDim.x) {
    if (!Await(a, &s_bad, n, [&](int p) { return p == r ? nullptr : DoneFlag(a, p, i); })) {
      return;
    }
    if (threadIdx.x < kMaxPeers) {
      const int p = static_cast<int>(threadIdx.x);
      size_t lo = 0, hi = 0;
      if (p < n && p != r) TileRange(a, p, i, &lo, &hi);
      s_lo[p] = lo;
      s_nv[p] = hi - lo;  // elements
    }
    __syncthreads();
    if (n <= 4) {
      GatherTileVec<T, 4, 4>(a, s_lo, s_nv, n, out, out2, vout);
    } else {
      GatherTileVec<T, kMaxPeers, 2>(a, s_lo, s_nv, n, out, out2, vout);
    }
    for (int p = 0; p < n; ++p) {
      const size_t nel = s_nv[p];
      const T *sp = reinterpret_cast<const T *>(a.stage[p]) + s_lo[p];
      for (size_t e = nel / L * L + threadIdx.x; e < nel; e += kBlock) {
        out[s_lo[p] + e] = sp[e];
        if (out2 != nullptr) out2[s_lo[p] + e] = sp[e];
      }
    }
    __syncthreads();  // s_lo / s_nv are rewritten by the next tile
  }
}

/*!
 * \brief one-shot allreduce of a small chunk in ONE launch (instead of stage copy + barrier
 *        kernel + reduce kernel): workgroup i stages tile i of this rank's input into its stage,
 *        raises the tile's ready flag, waits for every rank's ready flag of that tile, then
 *        reduces the tile from all n stages in rank order (identical bits everywhere) into out
 *        and out2.  Stage buffers alternate by parity and a rank's next launch on the same
 *        parity starts only after every peer raised its flags of the launch in between, which a
 *        peer does after its reads of this one: no second hand-off is needed.  The grid is at
 *        most a few dozen workgroups, so every one is resident.
 */
/*! \brief completion signal of a launch (FusedAllreduceArgs::done_word): the workgroup that
 *  counts itself in last re-arms the counter and stores the epoch into pinned host memory */
__device__ __forceinline__ void SignalDone(const FusedAllreduceArgs &a) {
  if (a.done_word == nullptr || threadIdx.x != 0) return;
  // this workgroup's stores (the result, possibly a peer's stage) are complete before it counts
  // in; the host then sees the word only after every workgroup did
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  const unsigned old =
      __hip_atomic_fetch_add(a.done_count, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (old == gridDim.x - 1) {
    __hip_atomic_store(a.done_count, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(a.done_word, a.epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

template <typename T, int OP>
__global__ __launch_bounds__(kBlock) void FusedOneshotKernel(FusedAllreduceArgs a) {
  __shared__ int s_bad;
  __shared__ const char *s_in[kMaxPeers];
  if (GroupFailed(a)) {
    SignalDone(a);
    return;
  }
  if (threadIdx.x == 0) s_bad = 0;
  __syncthreads();
  const int n = a.n, r = a.rank;
  constexpr size_t L = 16 / sizeof(T);
  const T alpha = static_cast<T>(a.alpha);
  const T *src = reinterpret_cast<const T *>(a.src);
  T *out = reinterpret_cast<T *>(a.out);
  T *out2 = reinterpret_cast<T *>(a.out2);
  T *mine = reinterpret_cast<T *>(a.stage[r]);
  const bool vsrc = (reinterpret_cast<uintptr_t>(src) & 15u) == 0;
  const bool vout = (reinterpret_cast<uintptr_t>(out) & 15u) == 0 &&
                    (reinterpret_cast<uintptr_t>(out2) & 15u) == 0;
  for (int i = blockIdx.x; i < a.tiles; i += gridDim.x) {
    const size_t lo = static_cast<size_t>(i) * a.tile;
    const size_t hi = lo + a.tile < a.count ? lo + a.tile : a.count;
    CopyPrep<T, false>(mine + lo, src + lo, hi - lo, a.prep, alpha, vsrc);
    Publish(a, 1, [&](int) { return ReadyFlag(a, r, i); });
    if (!Await(a, &s_bad, n, [&](int p) { return p == r ? nullptr : ReadyFlag(a, p, i); })) {
      break;  // failure recorded; still count in below
    }
    if (threadIdx.x < static_cast<unsigned>(n)) {
      s_in[threadIdx.x] = a.stage[threadIdx.x] + lo * sizeof(T);
    }
    __syncthreads();
    const size_t nvec = (hi - lo) / L;
    for (size_t v = threadIdx.x; v < nvec; v += kBlock) {
      uint4 x[kMaxPeers];
#pragma unroll
      for (int k = 0; k < kMaxPeers; ++k) {
        if (k < n) x[k] = reinterpret_cast<const uint4 *>(s_in[k])[v];
      }
      const uint4 y = ReduceVecsN<T, OP, kMaxPeers>(x, n, a.post);
      PutVec<T>(out, lo + v * L, y, vout);
      if (out2 != nullptr) PutVec<T>(out2, lo + v * L, y, vout);
    }
    for (size_t e = nvec * L + threadIdx.x; e < hi - lo; e += kBlock) {
      const T *srcs[kMaxPeers];
      for (int k = 0; k < n; ++k) srcs[k] = reinterpret_cast<const T *>(s_in[k]);
      const T y = ReduceScalarN<T, OP>(srcs, n, e, a.post);
      out[lo + e] = y;
      if (out2 != nullptr) out2[lo + e] = y;
    }
    __syncthreads();  // s_in is rewritten by the next tile
  }
  SignalDone(a);
}

template <typename T>
hipError_t LaunchOneshotT(const FusedAllreduceArgs &args, int grid, hipStream_t st) {
  switch (args.op) {
    case kOpMax:
      hipLaunchKernelGGL((FusedOneshotKernel<T, kOpMax>), dim3(grid), dim3(kBlock), 0, st, args);
      break;
    case kOpMin:
      hipLaunchKernelGGL((FusedOneshotKernel<T, kOpMin>), dim3(grid), dim3(kBlock), 0, st, args);
      break;
    case kOpSum:
      hipLaunchKernelGGL((FusedOneshotKernel<T, kOpSum>), dim3(grid), dim3(kBlock), 0, st, args);
      break;
    case kOpOr:
      if constexpr (std::is_integral<T>::value) {
        hipLaunchKernelGGL((FusedOneshotKernel<T, kOpOr>), dim3(grid), dim3(kBlock), 0, st,
                           args);
        break;
      }
      return hipErrorInvalidValue;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

template <typename T>
hipError_t LaunchT(const FusedAllreduceArgs &args, int grid, hipStream_t st) {
  switch (args.op) {
    case kOpMax:
      hipLaunchKernelGGL((FusedAllreduceKernel<T, kOpMax>), dim3(grid), dim3(kBlock), 0, st, args);
      break;
    case kOpMin:
      hipLaunchKernelGGL((FusedAllreduceKernel<T, kOpMin>), dim3(grid), dim3(kBlock), 0, st, args);
      break;
    case kOpSum:
      hipLaunchKernelGGL((FusedAllreduceKernel<T, kOpSum>), dim3(grid), dim3(kBlock), 0, st, args);
      break;
    case kOpOr:
      if constexpr (std::is_integral<T>::value) {
        hipLaunchKernelGGL((FusedAllreduceKernel<T, kOpOr>), dim3(grid), dim3(kBlock), 0, st,
                           args);
        break;
      }
      return hipErrorInvalidValue;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}
}  // namespace

int FusedResidentBlocks(int device) {
  int cus = 0;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess) {
    (void)hipGetLastError();
    return 0;
  }
  // the least resident instantiation bounds them all
  int per_cu = 1 << 30;
  auto take = [&](const void *fn) {
    int b = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&b, fn, kBlock, 0) != hipSuccess) {
      (void)hipGetLastError();
      b = 1;
    }
    per_cu = std::min(per_cu, std::max(b, 1));
  };
  take(reinterpret_cast<const void *>(&FusedAllreduceKernel<float, kOpSum>));
  take(reinterpret_cast<const void *>(&FusedAllreduceKernel<double, kOpMax>));
  take(reinterpret_cast<const void *>(&FusedAllreduceKernel<bf16_t, kOpSum>));
  take(reinterpret_cast<const void *>(&FusedAllreduceKernel<int8_t, kOpOr>));
  return cus * per_cu;
}

hipError_t LaunchFusedOneshot(const FusedAllreduceArgs &args, int grid, hipStream_t stream) {
  if (args.n < 1 || args.n > kMaxPeers || args.rank < 0 || args.rank >= args.n || grid < 1 ||
      args.tiles < 1 || args.tiles > args.tiles_cap || args.tile % 256 != 0 ||
      args.count > args.tile * static_cast<size_t>(args.tiles) || args.push || args.zero_copy) {
    return hipErrorInvalidValue;
  }
  if (args.post != 0.0 && args.dtype != 6 && args.dtype != 7 && args.dtype != 10 &&
      args.dtype != 11) {
    return hipErrorInvalidValue;
  }
  switch (args.dtype) {
    case 0: return LaunchOneshotT<int8_t>(args, grid, stream);
    case 1: return LaunchOneshotT<uint8_t>(args, grid, stream);
    case 2: return LaunchOneshotT<int32_t>(args, grid, stream);
    case 3: return LaunchOneshotT<uint32_t>(args, grid, stream);
    case 4:
    case 8: return LaunchOneshotT<int64_t>(args, grid, stream);
    case 5:
    case 9: return LaunchOneshotT<uint64_t>(args, grid, stream);
    case 6: return LaunchOneshotT<float>(args, grid, stream);
    case 7: return LaunchOneshotT<double>(args, grid, stream);
    case 10: return LaunchOneshotT<half_t>(args, grid, stream);
    case 11: return LaunchOneshotT<bf16_t>(args, grid, stream);
    default: return hipErrorInvalidValue;
  }
}

hipError_t LaunchFusedAllreduce(const FusedAllreduceArgs &args, int grid, hipStream_t stream) {
  if (args.n < 1 || args.n > kMaxPeers || args.rank < 0 || args.rank >= args.n || grid < 1 ||
      args.tiles < 1 || args.tiles > args.tiles_cap || args.seg % 256 != 0 ||
      args.tile % 256 != 0 || args.count > args.seg * static_cast<size_t>(args.n)) {
    return hipErrorInvalidValue;
  }
  if (args.post != 0.0 && args.dtype != 6 && args.dtype != 7 && args.dtype != 10 &&
      args.dtype != 11) {
    return hipErrorInvalidValue;
  }
  switch (args.dtype) {
    case 0: return LaunchT<int8_t>(args, grid, stream);
    case 1: return LaunchT<uint8_t>(args, grid, stream);
    case 2: return LaunchT<int32_t>(args, grid, stream);
    case 3: return LaunchT<uint32_t>(args, grid, stream);
    case 4:
    case 8: return LaunchT<int64_t>(args, grid, stream);
    case 5:
    case 9: return LaunchT<uint64_t>(args, grid, stream);
    case 6: return LaunchT<float>(args, grid, stream);
    case 7: return LaunchT<double>(args, grid, stream);
    case 10: return LaunchT<half_t>(args, grid, stream);
    case 11: return LaunchT<bf16_t>(args, grid, stream);
    default: return hipErrorInvalidValue;
  }
}
}  // namespace device
}  // namespace rabit
