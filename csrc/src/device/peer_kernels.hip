/*!
 * \file peer_kernels.hip
 * \brief gfx950 kernels of the direct (IPC / xGMI peer-memory) transport: a cross-process
 *        flag barrier and a batched multi-segment copy that pulls peer segments over xGMI.
 *
 * Barrier: every rank owns an array of one 64-bit flag per peer inside its IPC-exported,
 * uncached staging allocation.  Arriving at barrier number e, rank r stores e into slot r of
 * every peer's array (system-scope release) and then spins until all n slots of its own array
 * are >= e (system-scope acquire).  Epochs only grow, so flags never need resetting.  The
 * number e is kept on the device (a counter word the barrier kernel advances), so barriers
 * recorded in a hipGraph are numbered afresh on every replay.  Each lane
 * polls with s_sleep back-off and gives up when the host raises the abort word (peer failure
 * seen on the TCP control plane) or the wall-clock deadline passes — every wave reaches an exit.
 * A failure is recorded in a device word (the guard every later kernel of the group checks
 * first, so nothing is written after a failed barrier) and in a pinned host word.
 *
 * Copy batch: up to kMaxCopySegs (dst, src[, dst2]) segments in one launch; workgroup b takes
 * tile b / nseg of segment b % nseg, so the workgroups in flight read from every peer at once
 * and all xGMI links carry traffic together.  Remote segments (pushes into a peer's memory) may
 * share a launch with pulls: the pipelined allreduce sends one chunk out while it gathers an
 * older one in, over both directions of every link at once.  Tiles are 256 lanes x 16 B
 * (kUnroll = 1: 4 KiB per workgroup), like the other streaming kernels (kernels.hip).
 */
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>

#include "device/peer_coll.h"

namespace rabit {
namespace device {
namespace {

constexpr int kBlock = 256;
constexpr int kUnroll = 1;  // 4 KiB tiles: as for the streaming kernels of kernels.hip
constexpr size_t kTileBytes = static_cast<size_t>(kBlock) * kUnroll * 16;

template <bool RESOLVE>
__global__ __launch_bounds__(64) void PeerBarrierKernel(PeerFlagTable flags, int rank, int n,
                                                        unsigned long long *counter,
                                                        const volatile int *abort_word,
                                                        int *dev_status, int *host_status,
                                                        long long deadline_ticks,
                                                        int peer_abort_on, ResolveArgs resolve) {
  const int t = threadIdx.x;
  // an earlier barrier of this group failed: stay failed, signal nothing
  if (__hip_atomic_load(dev_status, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0) return;
  // this barrier's number: one more than the last barrier of this rank's group (kernels of the
  // group run one after the other on one stream, so a plain read-modify-write by one lane holds)
  __shared__ unsigned long long s_epoch;
  if (t == 0) {
    s_epoch = __hip_atomic_load(counter, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1;
    __hip_atomic_store(counter, s_epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  const unsigned long long epoch = s_epoch;
  auto mailbox = [&](int p) {
    return reinterpret_cast<unsigned long long *>(reinterpret_cast<char *>(flags.p[p]) +
                                                  kPeerMailboxOffset) +
           resolve.parity;
  };
  // the allgather slice layout (begin, size) of this window, by parity like the mailbox
  auto meta = [&](int p) {
    return reinterpret_cast<unsigned long long *>(reinterpret_cast<char *>(flags.p[p]) +
                                                  kPeerMetaOffset) +
           2 * resolve.parity;
  };
  if (RESOLVE) {
    if (t == 0) {
      if (resolve.table != nullptr) {
        __hip_atomic_store(mailbox(rank), resolve.my_mailbox, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_SYSTEM);
      }
      if (resolve.meta_table != nullptr) {
        __hip_atomic_store(meta(rank), resolve.my_meta[0], __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_SYSTEM);
        __hip_atomic_store(meta(rank) + 1, resolve.my_meta[1], __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_SYSTEM);
      }
    }
    __syncthreads();  // the mailbox / meta stores precede every lane's flag store below
  }
  // make the bytes written by earlier kernels of this stream visible before signalling
  __threadfence_system();
  // raised by a peer that aborted the group (kPeerAbortOffset of this rank's own flag area)
  const volatile int *peer_abort = reinterpret_cast<const volatile int *>(
      reinterpret_cast<const char *>(flags.p[rank]) + kPeerAbortOffset);
  if (t < n) {
    __hip_atomic_store(flags.p[t] + rank, epoch, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    unsigned long long *mine = flags.p[rank] + t;
    const long long t0 = wall_clock64();
    while (__hip_atomic_load(mine, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) < epoch) {
      if (*abort_word != 0 || (peer_abort_on && *peer_abort != 0) ||
          wall_clock64() - t0 > deadline_ticks) {
        // the reason, for the host's log: 1 the host raised the abort word, 4 a peer aborted
        // the group, 3 the deadline
        const int why = *abort_word != 0 ? 1 : (peer_abort_on && *peer_abort != 0 ? 4 : 3);
        if (peer_abort_on && why != 4) {
          // this rank gives up on its own account: every peer's waits give up too
          for (int p = 0; p < n; ++p) {
            if (p == rank) continue;
            __hip_atomic_store(reinterpret_cast<int *>(reinterpret_cast<char *>(flags.p[p]) +
                                                       kPeerAbortOffset),
                               1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
          }
        }
        __hip_atomic_store(dev_status, why, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __hip_atomic_store(host_status, why, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        break;
      }
      __builtin_amdgcn_s_sleep(4);
    }
  }
  __threadfence_system();
  if (RESOLVE) {
    __syncthreads();
    if (t < n && resolve.meta_table != nullptr &&
        __hip_atomic_load(dev_status, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) == 0) {
      resolve.meta_table[2 * t] =
          __hip_atomic_load(meta(t), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      resolve.meta_table[2 * t + 1] =
          __hip_atomic_load(meta(t) + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    if (t < n && resolve.table != nullptr &&
        __hip_atomic_load(dev_status, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) == 0) {
      const unsigned long long m =
          __hip_atomic_load(mailbox(t), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      const char *src;
      if ((m & kMailboxHeap) != 0) {
        src = resolve.heap_base[t] + (m & ~kMailboxHeap);
      } else if ((m & kMailboxReg) != 0) {
        // a registered allocation of peer t: its mapping from the registry's device table (the
        // peer only publishes one this rank acknowledged, see peer_registry.h)
        const int slot = static_cast<int>((m >> kMailboxRegShift) & (kMaxRegs - 1));
        const char *base = resolve.reg_table != nullptr
                               ? resolve.reg_table[t * kMaxRegs + slot] : nullptr;
        if (t == rank) {
          // this rank's own input, in place (its mailbox offset is into its own allocation)
          base = resolve.own_src - (m & kMailboxOffsetMask);
        }
        if (base == nullptr) {
          // cannot happen by the protocol; fail the op (the group is rebuilt) instead of
          // reading through a null mapping
          __hip_atomic_store(dev_status, 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
          __hip_atomic_store(host_status, 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
          return;
        }
        src = base + (m & kMailboxOffsetMask);
      } else {
        src = resolve.stage_base[t] + m;
      }
      resolve.table[t] = src + resolve.seg_off;
    }
  }
}

typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void StoreNT(uint4 *p, uint4 v) {
  u32x4_t w = {v.x, v.y, v.z, v.w};
  // compiler-only barrier: without it a later pass rebuilds this store as <4 x float> and drops
  // the !nontemporal tag in the multi-source kernel (seen in the LLVM IR of hipcc, ROCm 7.2)
  asm volatile("" ::: "memory");
  __builtin_nontemporal_store(w, reinterpret_cast<u32x4_t *>(p));
}

__host__ __device__ __forceinline__ bool Al16(const void *p) {
  return (reinterpret_cast<uintptr_t>(p) & 15u) == 0;
}

/*!
 * \brief one tile of a push segment into a peer's memory.  The destination is reached through
 *        this GPU's mapping of the peer's allocation, which may be cacheable here, so every byte
 *        leaves with a 16-byte system-scope write-through store (sc0 sc1): once the kernel has
 *        ended the peer sees it, whatever its cache type (the barrier kernel that follows signals
 *        from one workgroup, whose release cannot write back the other XCDs' L2s).  The inbox
 *        slot is 16-byte aligned and padded to whole 256-element blocks, so a tail word may carry
 *        zero padding past `bytes`; the source is read only within `bytes`.
 */
__device__ __forceinline__ void PushTile(const CopySeg &g, size_t lo, size_t hi) {
  typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
  const size_t nw = (hi - lo + 15) / 16;
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
      g.dst + lo, 0, static_cast<int>(nw * 16), 0x00020000);
  const bool vsrc = Al16(g.src + lo);
  for (size_t w = threadIdx.x; w < nw; w += kBlock) {
    uint4 v;
    if (vsrc && lo + (w + 1) * 16 <= hi) {
      v = reinterpret_cast<const uint4 *>(g.src + lo)[w];
    } else {
      unsigned char b[16];
#pragma unroll
      for (int k = 0; k < 16; ++k) {
        const size_t at = lo + w * 16 + k;
        b[k] = at < hi ? static_cast<unsigned char>(g.src[at]) : 0;
      }
      __builtin_memcpy(&v, b, 16);
    }
    const u32x4 x = {v.x, v.y, v.z, v.w};
    __builtin_amdgcn_raw_buffer_store_b128(x, rs, static_cast<int>(w * 16), 0, 1 | 16);
  }
}

__device__ __forceinline__ void CopyBatchBody(const CopyBatch &batch);

__global__ __launch_bounds__(kBlock) void CopyBatchKernel(CopyBatch batch) {
  CopyBatchBody(batch);
  if (batch.done_word != nullptr && threadIdx.x == 0) {
    // this workgroup's stores are complete before it counts in; the last one to count in
    // re-arms the counter and tells the host (pinned word)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const unsigned old =
        __hip_atomic_fetch_add(batch.done_count, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (old == gridDim.x - 1) {
      __hip_atomic_store(batch.done_count, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(batch.done_word, batch.epoch, __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
}

__device__ __forceinline__ void CopyBatchBody(const CopyBatch &batch) {
  if (batch.guard != nullptr &&
      __hip_atomic_load(batch.guard, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0) {
    return;
  }
  const int s = static_cast<int>(blockIdx.x % static_cast<unsigned>(batch.n));
  const size_t tile = blockIdx.x / static_cast<unsigned>(batch.n);
  const CopySeg &g = batch.seg[s];
  const size_t lo = tile * kTileBytes;
  if (lo >= g.bytes) return;
  const size_t hi = std::min(g.bytes, lo + kTileBytes);
  if (batch.remote || g.remote) {
    PushTile(g, lo, hi);
    return;
  }
  const bool vec = Al16(g.dst) && Al16(g.src) && (g.dst2 == nullptr || Al16(g.dst2));
  if (vec) {
    const size_t nv = (hi - lo) / 16;  // lo is a multiple of 16
    const uint4 *src = reinterpret_cast<const uint4 *>(g.src + lo);
    uint4 *dst = reinterpret_cast<uint4 *>(g.dst + lo);
    uint4 *dst2 = g.dst2 != nullptr ? reinterpret_cast<uint4 *>(g.dst2 + lo) : nullptr;
    if (nv == static_cast<size_t>(kBlock) * kUnroll) {
      uint4 v[kUnroll];
#pragma unroll
      for (int u = 0; u < kUnroll; ++u) v[u] = src[threadIdx.x + u * kBlock];
#pragma unroll
      for (int u = 0; u < kUnroll; ++u) StoreNT(dst + threadIdx.x + u * kBlock, v[u]);
      if (dst2 != nullptr) {
#pragma unroll
        for (int u = 0; u < kUnroll; ++u) StoreNT(dst2 + threadIdx.x + u * kBlock, v[u]);
      }
    } else {
      for (size_t i = threadIdx.x; i < nv; i += kBlock) {
        const uint4 v = src[i];
        dst[i] = v;
        if (dst2 != nullptr) dst2[i] = v;
      }
      // trailing bytes of the segment (< 16)
      for (size_t i = lo + nv * 16 + threadIdx.x; i < hi; i += kBlock) {
        const char c = g.src[i];
        g.dst[i] = c;
        if (g.dst2 != nullptr) g.dst2[i] = c;
      }
    }
  } else {
    for (size_t i = lo + threadIdx.x; i < hi; i += kBlock) {
      const char c = g.src[i];
      g.dst[i] = c;
      if (g.dst2 != nullptr) g.dst2[i] = c;
    }
  }
}
/*! \brief a workgroup copies [0, bytes) of src to dst (and dst2): 16-byte vectors when the three
 *  share their alignment modulo 16 (head and tail bytes apart), bytes otherwise */
__device__ __forceinline__ void BlockCopy(char *dst, const char *src, char *dst2, size_t bytes) {
  const uintptr_t md = reinterpret_cast<uintptr_t>(dst) & 15u;
  const uintptr_t ms = reinterpret_cast<uintptr_t>(src) & 15u;
  const uintptr_t m2 = dst2 != nullptr ? reinterpret_cast<uintptr_t>(dst2) & 15u : md;
  size_t head = bytes, nv = 0;
  if (md == ms && m2 == md) {
    head = md != 0 ? std::min<size_t>(bytes, 16 - md) : 0;
    nv = (bytes - head) / 16;
  }
  for (size_t i = threadIdx.x; i < head; i += kBlock) {
    dst[i] = src[i];
    if (dst2 != nullptr) dst2[i] = src[i];
  }
  const uint4 *s4 = reinterpret_cast<const uint4 *>(src + head);
  uint4 *d4 = reinterpret_cast<uint4 *>(dst + head);
  uint4 *e4 = dst2 != nullptr ? reinterpret_cast<uint4 *>(dst2 + head) : nullptr;
  for (size_t i = threadIdx.x; i < nv; i += kBlock) {
    const uint4 v = s4[i];
    d4[i] = v;
    if (e4 != nullptr) e4[i] = v;
  }
  for (size_t i = head + nv * 16 + threadIdx.x; i < bytes; i += kBlock) {
    dst[i] = src[i];
    if (dst2 != nullptr) dst2[i] = src[i];
  }
}

__global__ __launch_bounds__(kBlock) void AllgatherWindowKernel(AllgatherWindowArgs a) {
  if (a.guard != nullptr &&
      __hip_atomic_load(a.guard, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0) {
    return;
  }
  __shared__ unsigned long long s_meta[2 * kMaxPeers];
  if (threadIdx.x < 2 * a.n) s_meta[threadIdx.x] = a.meta_table[threadIdx.x];
  __syncthreads();
  const size_t tlo = a.wlo + static_cast<size_t>(blockIdx.x) * kTileBytes;
  if (tlo >= a.whi) return;
  const size_t thi = std::min(a.whi, tlo + kTileBytes);
  for (int p = 0; p < a.n; ++p) {
    if (p == a.rank) continue;
    const size_t size = static_cast<size_t>(s_meta[2 * p + 1]);
    if (size == 0 || a.total == 0) continue;
    const size_t begin = static_cast<size_t>(s_meta[2 * p]) % a.total;
    // the slice [begin, begin + size) mod total: at most two ranges
    size_t lo[2] = {begin, 0}, hi[2] = {std::min(a.total, begin + size), 0};
    const int k = begin + size > a.total ? 2 : 1;
    if (k == 2) hi[1] = begin + size - a.total;
    for (int j = 0; j < k; ++j) {
      const size_t x0 = std::max(lo[j], tlo), x1 = std::min(hi[j], thi);
      if (x1 <= x0) continue;
      BlockCopy(a.buf + x0, a.stage[p] + (x0 - a.wlo), a.log != nullptr ? a.log + x0 : nullptr,
                x1 - x0);
    }
  }
}
}  // namespace

hipError_t LaunchAllgatherWindow(const AllgatherWindowArgs &args, hipStream_t stream) {
  if (args.n < 1 || args.n > kMaxPeers || args.rank < 0 || args.rank >= args.n ||
      args.whi < args.wlo || args.meta_table == nullptr) {
    return hipErrorInvalidValue;
  }
  const size_t tiles = (args.whi - args.wlo + kTileBytes - 1) / kTileBytes;
  if (tiles == 0) return hipSuccess;
  if (tiles > 0x7fffffffu) return hipErrorInvalidValue;
  hipLaunchKernelGGL(AllgatherWindowKernel, dim3(static_cast<unsigned>(tiles)), dim3(kBlock), 0,
                     stream, args);
  return hipGetLastError();
}

hipError_t LaunchPeerBarrier(const PeerFlagTable &flags, int rank, int n,
                             unsigned long long *counter, const volatile int *abort_word,
                             int *dev_status, int *host_status, long long deadline_ticks,
                             int peer_abort_on,
                             const ResolveArgs *resolve, hipStream_t stream) {
  if (n < 1 || n > kMaxPeers || rank < 0 || rank >= n || counter == nullptr) {
    return hipErrorInvalidValue;
  }
  if (resolve != nullptr) {
    hipLaunchKernelGGL(PeerBarrierKernel<true>, dim3(1), dim3(64), 0, stream, flags, rank, n,
                       counter, abort_word, dev_status, host_status, deadline_ticks, peer_abort_on,
                       *resolve);
  } else {
    ResolveArgs none{};
    hipLaunchKernelGGL(PeerBarrierKernel<false>, dim3(1), dim3(64), 0, stream, flags, rank, n,
                       counter, abort_word, dev_status, host_status, deadline_ticks, peer_abort_on,
                       none);
  }
  return hipGetLastError();
}

hipError_t LaunchCopyBatch(const CopyBatch &batch, hipStream_t stream) {
  if (batch.n < 0 || batch.n > kMaxCopySegs) return hipErrorInvalidValue;
  for (int i = 0; i < batch.n; ++i) {
    // push destinations are whole-16-byte inbox slots (PushTile pads the last word)
    if ((batch.remote || batch.seg[i].remote) &&
        (!Al16(batch.seg[i].dst) || batch.seg[i].dst2 != nullptr)) {
      return hipErrorInvalidValue;
    }
  }
  size_t tiles = 0;
  for (int i = 0; i < batch.n; ++i) {
    tiles = std::max(tiles, (batch.seg[i].bytes + kTileBytes - 1) / kTileBytes);
  }
  if (tiles == 0) return hipSuccess;
  const size_t grid = tiles * static_cast<size_t>(batch.n);
  if (grid > 0x7fffffffu) return hipErrorInvalidValue;
  hipLaunchKernelGGL(CopyBatchKernel, dim3(static_cast<unsigned>(grid)), dim3(kBlock), 0, stream,
                     batch);
  return hipGetLastError();
}
}  // namespace device
}  // namespace rabit
