/*!
 * \file peer_coll.cc
 * \brief Host side of the direct (IPC peer-memory) transport; see peer_coll.h.
 */
#include "device/peer_coll.h"

#include <unistd.h>

#include <algorithm>
#include <cstdio>
#include <cstring>

#include "core/exit.h"
#include "device/ar_plan.h"
#include "device/bcast_plan.h"
#include "device/device_plane.h"
#include "device/kernels.h"
#include "rabit/internal/utils.h"

namespace rabit {
namespace device {
namespace {
size_t ElemBytes(int dtype) {
  switch (dtype) {
    case 0:
    case 1: return 1;
    case 10:
    case 11: return 2;
    case 2:
    case 3:
    case 6: return 4;
    default: return 8;
  }
}

inline size_t RoundUp(size_t x, size_t m) { return (x + m - 1) / m * m; }

/*! \brief [lo, hi) of segment p when c items are cut into n segments of `seg` */
inline void SegRange(size_t c, size_t seg, int p, size_t *lo, size_t *hi) {
  *lo = std::min(c, seg * static_cast<size_t>(p));
  *hi = std::min(c, *lo + seg);
}

void AddSeg(CopyBatch *b, char *dst, const char *src, char *dst2, size_t bytes,
            bool remote = false) {
  if (bytes == 0) return;
  utils::Assert(b->n < kMaxCopySegs, "copy batch overflow");
  b->seg[b->n++] = CopySeg{dst, src, dst2, bytes, remote ? 1 : 0};
}

/*! \brief dst[0, bytes) = src[0, bytes) as equal 4 KiB-aligned segments in the batch's free
 *  slots: a large local copy then shares a launch with a gather, and the two run at once (one
 *  HBM-bound, the other xGMI-bound on separate GPUs) */
void AddSplit(CopyBatch *b, char *dst, const char *src, size_t bytes) {
  if (bytes == 0) return;
  const size_t slots = static_cast<size_t>(std::max(1, kMaxCopySegs - b->n));
  const size_t piece = RoundUp((bytes + slots - 1) / slots, 4096);
  for (size_t o = 0; o < bytes; o += piece) {
    AddSeg(b, dst + o, src + o, nullptr, std::min(piece, bytes - o));
  }
}

/*! \brief the (at most two) byte ranges of a wrapping slice [begin, begin+size) mod total */
int SliceRanges(size_t begin, size_t size, size_t total, size_t lo[2], size_t hi[2]) {
  if (size == 0) return 0;
  begin %= total;
  lo[0] = begin;
  hi[0] = std::min(total, begin + size);
  if (begin + size <= total) return 1;
  lo[1] = 0;
  hi[1] = begin + size - total;
  return 2;
}
}  // namespace

PeerGroup::PeerGroup(int device, size_t stage_bytes, double deadline_sec, hipStream_t stream,
                     const SymHeapInfo &heap)
    : device_(device), stage_bytes_(RoundUp(std::max<size_t>(stage_bytes, 1 << 20), 1 << 16)),
      stream_(stream), heap_(heap) {
  CheckHip(hipSetDevice(device_), "hipSetDevice");
  // fused allreduce: a segment is at most a stage, a tile kFusedTileBytes
  tiles_cap_ = static_cast<int>((stage_bytes_ + kFusedTileMinBytes - 1) / kFusedTileMinBytes);
  fused_block_bytes_ = RoundUp(FusedFlagWords(tiles_cap_) * sizeof(unsigned long long), 1 << 16);
  const size_t flag_bytes = kPeerFlagBytes + 2 * fused_block_bytes_;
  void *p = nullptr;
  // uncached: peers poll the flags and stream the stage buffers over xGMI; nothing of it may
  // linger in a (non-coherent) L2 between ops
  CheckHip(hipExtMallocWithFlags(&p, flag_bytes + 2 * stage_bytes_, hipDeviceMallocUncached),
           "hipExtMallocWithFlags(peer stage)");
  base_ = static_cast<char *>(p);
  CheckHip(hipMemset(base_, 0, flag_bytes), "hipMemset(flags)");
  CheckHip(hipDeviceSynchronize(), "hipDeviceSynchronize");
  hipIpcMemHandle_t h;
  CheckHip(hipIpcGetMemHandle(&h, base_), "hipIpcGetMemHandle");
  static_assert(sizeof(h) <= sizeof(local_.ipc), "ipc handle size");
  std::memcpy(local_.ipc, &h, sizeof(h));
  CheckHip(hipDeviceGetPCIBusId(local_.pci, sizeof(local_.pci), device_), "hipDeviceGetPCIBusId");
  gethostname(local_.host, sizeof(local_.host) - 1);
  local_.stage_bytes = stage_bytes_;
  local_.pid = static_cast<int32_t>(getpid());
  local_.device = device_;
  local_.heap_bytes = heap_.base != nullptr ? heap_.bytes : 0;
  local_.fused_cap = FusedResidentBlocks(device_);
  std::memcpy(local_.heap_ipc, heap_.ipc, sizeof(local_.heap_ipc));
  // zero-copy registry page (a failure only leaves ordinary inputs staged)
  std::string rwhy;
  if (registry_.Create(&rwhy)) {
    std::strncpy(local_.reg_name, registry_.name(), sizeof(local_.reg_name) - 1);
  }
  void *tbl = nullptr;
  CheckHip(hipMalloc(&tbl, kMaxPeers * sizeof(void *)), "hipMalloc(source table)");
  table_ = static_cast<const void **>(tbl);
  void *mt = nullptr;
  CheckHip(hipMalloc(&mt, 2 * kMaxPeers * sizeof(unsigned long long)), "hipMalloc(meta table)");
  meta_table_ = static_cast<unsigned long long *>(mt);
  void *hw = nullptr;
  CheckHip(hipHostMalloc(&hw, 64, hipHostMallocCoherent | hipHostMallocMapped),
           "hipHostMalloc(peer words)");
  host_words_ = static_cast<int *>(hw);
  std::memset(host_words_, 0, 64);
  CheckHip(hipDeviceGetAttribute(&clock_khz_, hipDeviceAttributeWallClockRate, device_),
           "wall clock");
  set_deadline_sec(deadline_sec);
}

PeerGroup::~PeerGroup() {
  (void)hipSetDevice(device_);
  if (timing_) {
    for (auto &e : ev_) (void)hipEventDestroy(e);
  }
  for (size_t r = 0; r < peer_base_.size(); ++r) {
    if (peer_base_[r] != nullptr && peer_base_[r] != base_) {
      (void)hipIpcCloseMemHandle(peer_base_[r]);
    }
  }
  for (size_t r = 0; r < peer_heap_.size(); ++r) {
    if (peer_heap_[r] != nullptr && peer_heap_[r] != heap_.base) {
      (void)hipIpcCloseMemHandle(peer_heap_[r]);
    }
  }
  if (table_ != nullptr) (void)hipFree(const_cast<void **>(table_));
  if (meta_table_ != nullptr) (void)hipFree(meta_table_);
  if (base_ != nullptr) (void)hipFree(base_);
  if (host_words_ != nullptr) (void)hipHostFree(host_words_);
}

bool PeerGroup::Open(const std::vector<PeerRecord> &all, int rank, std::string *why) {
  const int n = static_cast<int>(all.size());
  if (n < 1 || n > kMaxPeers) {
    *why = "group size " + std::to_string(n) + " not in [1, 8]";
    return false;
  }
  for (int r = 0; r < n; ++r) {
    if (std::strncmp(all[r].host, local_.host, sizeof(local_.host)) != 0) {
      *why = std::string("rank ") + std::to_string(r) + " is on another host";
      return false;
    }
    if (all[r].stage_bytes != stage_bytes_) {
      *why = "stage sizes differ";
      return false;
    }
  }
  peer_base_.assign(n, nullptr);
  for (int r = 0; r < n; ++r) {
    if (r == rank) {
      peer_base_[r] = base_;
      continue;
    }
    hipIpcMemHandle_t h;
    std::memcpy(&h, all[r].ipc, sizeof(h));
    void *p = nullptr;
    hipError_t e = hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess);
    if (e != hipSuccess) {
      (void)hipGetLastError();
      *why = std::string("hipIpcOpenMemHandle(rank ") + std::to_string(r) +
             "): " + hipGetErrorString(e);
      return false;
    }
    peer_base_[r] = static_cast<char *>(p);
  }
  peer_heap_.assign(n, nullptr);
  for (int r = 0; r < n; ++r) {
    if (all[r].heap_bytes == 0) continue;
    if (r == rank) {
      peer_heap_[r] = heap_.base;
      continue;
    }
    hipIpcMemHandle_t h;
    std::memcpy(&h, all[r].heap_ipc, sizeof(h));
    void *p = nullptr;
    hipError_t e = hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess);
    if (e != hipSuccess) {
      (void)hipGetLastError();
      *why = std::string("hipIpcOpenMemHandle(heap of rank ") + std::to_string(r) +
             "): " + hipGetErrorString(e);
      return false;
    }
    peer_heap_[r] = static_cast<char *>(p);
  }
  n_ = n;
  rank_ = rank;
  {
    std::vector<std::string> names(n);
    bool all_named = true;
    for (int r = 0; r < n; ++r) {
      names[r] = std::string(all[r].reg_name, strnlen(all[r].reg_name, sizeof(all[r].reg_name)));
      all_named = all_named && !names[r].empty();
    }
    std::string rwhy;
    registry_ok_ = all_named && n >= 2 && registry_.Open(names, rank, &rwhy);
  }
  // a fused launch waits on the other ranks' launches: when ranks share a GPU, no rank's grid
  // may take every slot of it, or the others' workgroups could never start; each gets at most
  // its share of the resident capacity.  Every rank derives the same grid from the same records
  // (the launch's no-deadlock argument needs equal grids).
  int share = 1;
  for (int a = 0; a < n; ++a) {
    int c = 0;
    for (int b = 0; b < n; ++b) c += std::strncmp(all[a].pci, all[b].pci, sizeof(all[a].pci)) == 0;
    share = std::max(share, c);
  }
  // capacity of an MI355X (256 CUs x 4 resident workgroups), lowered by what any rank's GPU
  // reports, so that all ranks use the same value
  int cap = 1024;
  for (int a = 0; a < n; ++a) {
    if (all[a].fused_cap > 0) cap = std::min(cap, static_cast<int>(all[a].fused_cap));
  }
  gpu_share_ = share;
  fused_grid_ = fused_grid_req_ > 0 ? fused_grid_req_ : std::max(16, cap / share);
  opened_ = true;
  return true;
}

char *PeerGroup::stage(int rank, int which) const {
  return peer_base_[rank] + kPeerFlagBytes + 2 * fused_block_bytes_ +
         static_cast<size_t>(which) * stage_bytes_;
}

void PeerGroup::SignalAbort() {
  if (host_words_ != nullptr) {
    __atomic_store_n(&host_words_[0], 1, __ATOMIC_SEQ_CST);
  }
  // (a barrier kernel that sees this word passes the abort on to every peer: kPeerAbortOffset)
}

bool PeerGroup::failed() const {
  return host_words_ != nullptr && __atomic_load_n(&host_words_[1], __ATOMIC_SEQ_CST) != 0;
}

hipError_t PeerGroup::Barrier(const ResolveArgs *resolve) {
  PeerFlagTable t;
  for (int p = 0; p < kMaxPeers; ++p) {
    t.p[p] = p < n_ ? reinterpret_cast<unsigned long long *>(peer_base_[p]) : nullptr;
  }
  ++epoch_;  // (statistics: the barrier's number itself lives in barrier_counter())
  return LaunchPeerBarrier(t, rank_, n_, barrier_counter(), &host_words_[0], dev_status(),
                           &host_words_[1], deadline_ticks_, peer_abort_ ? 1 : 0, resolve, stream_);
}

#define XRABIT_TRY_HIP(expr)              \
  do {                                    \
    hipError_t e_ = (expr);               \
    if (e_ != hipSuccess) return e_;      \
  } while (0)

hipError_t PeerGroup::Allreduce(const void *send, void *recv, void *recv2, size_t count,
                                int dtype, int op, int prep, double alpha) {
  ReduceStep step = [dtype, op](void *dst, const void *const *srcs, int n, size_t c,
                                const int *guard, const void *const *table, double post,
                                hipStream_t st) {
    return LaunchReduceMulti(dst, srcs, n, c, dtype, op, st, guard, table, post);
  };
  return AllreduceImpl(send, recv, recv2, count, ElemBytes(dtype), dtype, prep, alpha, step,
                       true, op == 2, op);
}

hipError_t PeerGroup::AllreduceCustom(const void *send, void *recv, void *recv2, size_t count,
                                      size_t type_nbytes, const ReduceStep &step) {
  // user reductions take host-computed source pointers: every rank stages its input
  return AllreduceImpl(send, recv, recv2, count, type_nbytes, -1, kPrepCopy, 1.0, step, false);
}

hipError_t PeerGroup::AllreduceImpl(const void *send, void *recv, void *recv2, size_t count,
                                    size_t tn, int dtype, int prep, double alpha,
                                    const ReduceStep &step, bool indirect, bool op_is_sum,
                                    int builtin_op) {
  utils::Assert(opened_, "peer group not opened");
  // segments are multiples of 256 elements: 256-byte aligned for any element size
  const size_t quantum = 256 * static_cast<size_t>(n_);
  const size_t chunk = std::max(quantum, (stage_bytes_ / tn) / quantum * quantum);
  utils::Check(chunk * tn <= stage_bytes_, "peer stage buffer too small for %zu-byte elements",
               tn);
  const char *in = static_cast<const char *>(send);
  char *out = static_cast<char *>(recv);
  char *out2 = static_cast<char *>(recv2);
  // sum(a x_p) = a sum(x_p): exact reordering only for the linear op
  const bool post_scale =
      indirect && op_is_sum && prep == kPrepScale &&
      (dtype == 6 || dtype == 7 || dtype == 10 || dtype == 11);
  const int stage_prep = post_scale ? kPrepCopy : prep;
  // per-phase timing of single-chunk ops (rabit_device_phase_timing=1)
  const bool timed = timing_ && count <= chunk;
  auto mark = [&](int k) { return timed ? hipEventRecord(ev_[k], stream_) : hipSuccess; };
  bool did_fused = false;
  done_pending_ = false;
  // Registered zero copy (peer_registry.h): every rank counts this op alike, maps the peers'
  // newly exported allocations ahead of its kernels, and reads in place from the peers that
  // published one.  Only the pull two-shot stages its input (push and pipelined forms read it
  // where it is), so only that form asks for its own input to be exported.
  ++op_seq_;
  const bool registry = registry_ok_ && !no_registry_ && indirect;
  // (a replaced mapping waits for the stream to drain: at most twice the barrier deadline)
  if (registry) {
    const double drain_sec = 2.0 * static_cast<double>(deadline_ticks_) / (clock_khz_ * 1e3);
    XRABIT_TRY_HIP(registry_.Refresh(op_seq_, stream_, drain_sec));
  }
  unsigned long long reg_mailbox = 0;
  const bool reg_input = registry && zero_copy_min_ != 0 && count * tn >= zero_copy_min_ &&
                         count * tn > oneshot_max_ && !push_ && !fused_ &&
                         stage_prep == kPrepCopy && !InHeap(in, count * tn) &&
                         registry_.Resolve(in, count * tn, op_seq_, &reg_mailbox);
  // pipelined push form (ar_plan.h): ops above the one-shot size, raw inputs
  if (pipeline_ && push_ && n_ >= 2 && stage_prep == kPrepCopy &&
      !(indirect && count * tn <= oneshot_max_)) {
    timing_pending_ = false;  // no phase events in this form
    return AllreducePipelined(in, out, out2, count, tn, post_scale ? alpha : 0.0, step);
  }
  // A second destination (the robust engine's user buffer) may only change once the op has
  // succeeded on this rank, so that a retry after a failure still finds the input there.  The
  // gather of the LAST chunk follows the op's last barrier and stores it in the same pass; the
  // chunks before it are gathered into `out` alone and copied over by extra segments of that same
  // launch, which the group's failure word guards (it does nothing if any barrier of the op gave
  // up), so the local copy runs while the last gather reads over the links.  The fused
  // kernels hand tiles over one by one, with no last barrier: a peer dying inside one leaves some
  // tiles delivered and others not, so they never store the second destination themselves.
  const size_t last_off = count == 0 || !defer_second_ ? 0 : (count - 1) / chunk * chunk;
  bool tail_signal = false;  // the second destination's tail copy carries the done signal
  size_t tail_end = last_off;  // [0, tail_end) reaches out2 through the guarded copy
  for (size_t off = 0; off < count; off += chunk) {
    const size_t c = std::min(chunk, count - off);
    const int which = parity_;
    parity_ ^= 1;
    char *mine = stage(rank_, which);
    const char *chunk_src = in + off * tn;
    char *out2_now = off >= last_off ? out2 : nullptr;  // second destination in this chunk
    // zero copy: an input in the symmetric heap is read in place by the peers (its location
    // goes out in this rank's mailbox; each rank decides for itself).  A floating-point scale
    // (gradient averaging) is applied once after the sum on every rank, so inputs stay raw.
    // One-shot ops never read in place: with a single barrier nothing would stop this rank
    // from overwriting its input (second destination, the caller's next kernels) while a slower
    // peer is still reading it.  Two-shot reads all inputs before the second barrier.
    const bool oneshot = indirect && c * tn <= oneshot_max_ && count <= chunk;
    const size_t seg = RoundUp((c + n_ - 1) / n_, 256);
    // push: the owners' inboxes receive the input segments directly (n * seg <= chunk always
    // holds: chunk is a multiple of 256 n)
    const bool use_push = push_ && !oneshot && stage_prep == kPrepCopy &&
                          n_ * seg * tn <= stage_bytes_;
    const bool aligned_src = (reinterpret_cast<uintptr_t>(chunk_src) & 15u) == 0;
    const bool heap_zero_copy = indirect && !oneshot && !use_push && stage_prep == kPrepCopy &&
                                InHeap(chunk_src, c * tn) && aligned_src;
    const bool reg_zero_copy = reg_input && !oneshot && !use_push && aligned_src;
    const bool zero_copy = heap_zero_copy || reg_zero_copy;
    // where this rank's input of the chunk is: its stage, the heap, or a registered allocation
    const unsigned long long my_mailbox =
        heap_zero_copy ? (kMailboxHeap | static_cast<unsigned long long>(chunk_src - heap_.base))
        : reg_zero_copy ? reg_mailbox + static_cast<unsigned long long>(off * tn)
                        : static_cast<unsigned long long>(mine - base_);
    char *chunk_out = out + off * tn;
    char *chunk_out2 = out2_now != nullptr ? out2_now + off * tn : nullptr;
    // every input of this decision is the same on all ranks (the kernel copes with this rank's
    // unaligned buffers itself), so all ranks run the same form of the chunk
    if (fused_ && !oneshot && builtin_op >= 0 && c * tn >= fused_min_bytes_) {
      // one launch for the whole chunk (per-tile hand-offs instead of two GPU-wide barriers)
      FusedAllreduceArgs fa{};
      for (int p = 0; p < n_; ++p) {
        fa.stage[p] = stage(p, which);
        fa.alloc[p] = peer_base_[p];
        fa.heap[p] = peer_heap_.empty() ? nullptr : peer_heap_[p];
        fa.flags[p] = fused_flags(p, which);
      }
      fa.src = chunk_src;
      fa.out = chunk_out;
      fa.out2 = defer_second_ ? nullptr : chunk_out2;
      if (defer_second_ && chunk_out2 != nullptr) tail_end = off + c;
      fa.count = c;
      fa.seg = seg;
      // about one tile per workgroup of the grid, 8-64 KiB, a multiple of 256 elements
      const size_t per_wg = RoundUp(seg * tn / static_cast<size_t>(fused_grid_), 256 * tn);
      fa.tile = std::min(kFusedTileBytes, std::max(kFusedTileMinBytes, per_wg)) / tn;
      fa.tiles = static_cast<int>((seg + fa.tile - 1) / fa.tile);
      fa.tiles_cap = tiles_cap_;
      fa.n = n_;
      fa.rank = rank_;
      fa.push = use_push ? 1 : 0;
      fa.zero_copy = heap_zero_copy ? 1 : 0;  // (reg_input is off with the fused form)
      fa.mailbox = my_mailbox;
      fa.epoch = ++fused_epoch_;
      fa.dtype = dtype;
      fa.op = builtin_op;
      fa.prep = stage_prep;
      fa.alpha = alpha;
      fa.post = post_scale ? alpha : 0.0;
      fa.abort_word = &host_words_[0];
      fa.peer_abort = peer_abort_ ? peer_abort() : &host_words_[0];
      fa.dev_status = dev_status();
      fa.host_status = &host_words_[1];
      fa.deadline_ticks = deadline_ticks_;
      const int grid = std::min(fused_grid_, fa.tiles);
      XRABIT_TRY_HIP(LaunchFusedAllreduce(fa, grid, stream_));
      ++fused_chunks_;
      did_fused = true;
      if (use_push) ++push_chunks_;
      if (zero_copy) ++zero_copy_chunks_;
      continue;
    }
    if (oneshot && c * tn <= fused_oneshot_max_ && builtin_op >= 0) {
      // small op in one launch: stage, per-tile ready flags, reduce of all stages (the classic
      // form below takes 3 launches: stage copy, barrier, reduce).  Up to 64 KiB it is faster
      // with 2-8 ranks (4 KiB: 28 vs 32 us with 2 ranks sharing a GPU, 64 vs 101 us with 8);
      // at 256 KiB its 64 workgroups lose to the classic reduce kernel's full grid.
      FusedAllreduceArgs fa{};
      for (int p = 0; p < n_; ++p) {
        fa.stage[p] = stage(p, which);
        fa.alloc[p] = peer_base_[p];
        fa.flags[p] = fused_flags(p, which);
      }
      fa.src = chunk_src;
      fa.out = chunk_out;
      fa.out2 = defer_second_ ? nullptr : chunk_out2;
      if (defer_second_ && chunk_out2 != nullptr) tail_end = off + c;
      fa.count = c;
      // 4 KiB tiles (at least 256 elements; larger when the op needs more than the flag
      // slots): up to 64 workgroups for the default largest one-shot op (256 KiB)
      fa.tile = RoundUp(std::max<size_t>(4096 / tn, (c + tiles_cap_ - 1) / tiles_cap_), 256);
      fa.tiles = static_cast<int>((c + fa.tile - 1) / fa.tile);
      fa.seg = fa.tile;
      fa.tiles_cap = tiles_cap_;
      fa.n = n_;
      fa.rank = rank_;
      fa.epoch = ++fused_epoch_;
      fa.dtype = dtype;
      fa.op = builtin_op;
      fa.prep = stage_prep;
      fa.alpha = alpha;
      fa.post = post_scale ? alpha : 0.0;
      fa.abort_word = &host_words_[0];
      fa.peer_abort = peer_abort_ ? peer_abort() : &host_words_[0];
      fa.dev_status = dev_status();
      fa.host_status = &host_words_[1];
      fa.deadline_ticks = deadline_ticks_;
      // single-launch op; with a deferred second destination the tail copy after it signals
      // instead (the host must not see the op done before that copy is)
      const bool signal = done_signal_ && count <= chunk && (out2 == nullptr || !defer_second_);
      if (done_signal_ && count <= chunk && !signal) tail_signal = true;
      if (signal) {
        fa.done_count = done_count();
        fa.done_word = done_word();
      }
      XRABIT_TRY_HIP(LaunchFusedOneshot(fa, std::min(fa.tiles, fused_grid_), stream_));
      if (signal) {
        done_pending_ = true;
        done_epoch_ = fa.epoch;
      }
      ++oneshot_ops_;
      ++fused_oneshots_;
      did_fused = true;
      continue;
    }
    XRABIT_TRY_HIP(mark(0));
    if (use_push) {
      // no staging: this rank's own stage is its inbox, written by the peers
    } else if (zero_copy) {
      ++zero_copy_chunks_;
      if (reg_zero_copy) ++reg_zero_copy_chunks_;
    } else if (stage_prep == kPrepCopy) {
      XRABIT_TRY_HIP(LaunchCopy(mine, chunk_src, c * tn, stream_));
    } else {
      XRABIT_TRY_HIP(
          LaunchPrepare(mine, nullptr, chunk_src, c, dtype, stage_prep, alpha, stream_));
    }
    XRABIT_TRY_HIP(mark(1));
    if (oneshot) {
      // one-shot (small ops): one barrier, then every rank reduces the whole chunk from all
      // peers' inputs itself, in rank order (identical results everywhere), straight into the
      // destination — no second barrier, no gather
      ResolveArgs ra{};
      ra.my_mailbox = my_mailbox;
      ra.reg_table = registry_ok_ ? registry_.device_table() : nullptr;
      ra.own_src = chunk_src;
      ra.parity = which;
      for (int p = 0; p < n_; ++p) {
        ra.stage_base[p] = peer_base_[p];
        ra.heap_base[p] = peer_heap_.empty() ? nullptr : peer_heap_[p];
      }
      ra.seg_off = 0;
      ra.table = table_;
      XRABIT_TRY_HIP(Barrier(&ra));
      XRABIT_TRY_HIP(mark(2));
      const void *srcs[kMaxPeers];
      for (int p = 0; p < n_; ++p) srcs[p] = stage(p, which);
      if (builtin_op >= 0) {
        // built-in op: the same kernel also stores the result into the second destination
        XRABIT_TRY_HIP(LaunchReduceMulti(out + off * tn, srcs, n_, c, dtype, builtin_op, stream_,
                                         dev_status(), table_, post_scale ? alpha : 0.0,
                                         out2 != nullptr ? out2 + off * tn : nullptr));
      } else {
        XRABIT_TRY_HIP(step(out + off * tn, srcs, n_, c, dev_status(), table_,
                            post_scale ? alpha : 0.0, stream_));
      }
      XRABIT_TRY_HIP(mark(3));
      XRABIT_TRY_HIP(mark(4));  // (no second barrier)
      if (out2 != nullptr && builtin_op < 0) {
        CopyBatch b;
        NewBatch(&b);
        AddSeg(&b, out2 + off * tn, out + off * tn, nullptr, c * tn);
        XRABIT_TRY_HIP(LaunchCopyBatch(b, stream_));
      }
      XRABIT_TRY_HIP(mark(5));
      ++oneshot_ops_;
      continue;
    }
    size_t lo, hi;
    SegRange(c, seg, rank_, &lo, &hi);
    if (use_push) {
      // segment q of this rank's input goes to inbox slot `rank_` of rank q's stage (posted
      // remote writes, read from the input where it is), then every inbox is local memory
      CopyBatch b;
      NewBatch(&b);
      b.remote = 1;  // (this rank's own inbox slot too: the same store kind everywhere)
      for (int q = 0; q < n_; ++q) {
        size_t qlo, qhi;
        SegRange(c, seg, q, &qlo, &qhi);
        AddSeg(&b, stage(q, which) + (static_cast<size_t>(rank_) * seg) * tn,
               chunk_src + qlo * tn, nullptr, (qhi - qlo) * tn);
      }
      if (b.n > 0) XRABIT_TRY_HIP(LaunchCopyBatch(b, stream_));
      XRABIT_TRY_HIP(Barrier());
      if (die_mid_ && off > 0) DieMidOp();  // as below, for the pull form
      XRABIT_TRY_HIP(mark(2));
      if (hi > lo) {
        const void *srcs[kMaxPeers];
        for (int p = 0; p < n_; ++p) srcs[p] = mine + (static_cast<size_t>(p) * seg) * tn;
        // the result lands in this rank's own slot, where the gather of every peer reads it
        XRABIT_TRY_HIP(step(mine + (static_cast<size_t>(rank_) * seg) * tn, srcs, n_, hi - lo,
                            dev_status(), nullptr, post_scale ? alpha : 0.0, stream_));
      }
      XRABIT_TRY_HIP(mark(3));
      XRABIT_TRY_HIP(Barrier());
      XRABIT_TRY_HIP(mark(4));
      NewBatch(&b);
      for (int p = 0; p < n_; ++p) {
        size_t plo, phi;
        SegRange(c, seg, p, &plo, &phi);
        const size_t at = (off + plo) * tn;
        AddSeg(&b, out + at, stage(p, which) + (static_cast<size_t>(p) * seg) * tn,
               out2_now != nullptr ? out2_now + at : nullptr, (phi - plo) * tn);
      }
      if (out2_now != nullptr && tail_end > 0) {
        // the earlier chunks into the second destination in the same launch (after the op's
        // last barrier, guarded like the gather)
        AddSplit(&b, out2, out, tail_end * tn);
        tail_end = 0;
      }
      XRABIT_TRY_HIP(LaunchCopyBatch(b, stream_));
      XRABIT_TRY_HIP(mark(5));
      ++push_chunks_;
      continue;
    }
    if (indirect) {
      ResolveArgs ra{};
      ra.my_mailbox = my_mailbox;
      ra.reg_table = registry_ok_ ? registry_.device_table() : nullptr;
      ra.own_src = chunk_src;
      ra.parity = which;
      for (int p = 0; p < n_; ++p) {
        ra.stage_base[p] = peer_base_[p];
        ra.heap_base[p] = peer_heap_.empty() ? nullptr : peer_heap_[p];
      }
      ra.seg_off = lo * tn;
      ra.table = table_;
      XRABIT_TRY_HIP(Barrier(&ra));
    } else {
      XRABIT_TRY_HIP(Barrier());
    }
    // every peer passed this barrier with the previous chunk gathered into its output
    if (die_mid_ && off > 0) DieMidOp();
    XRABIT_TRY_HIP(mark(2));
    if (hi > lo) {
      const void *srcs[kMaxPeers];
      // host pointers: the staged locations (the table, when used, holds the real ones; both
      // are 256-byte aligned)
      for (int p = 0; p < n_; ++p) srcs[p] = stage(p, which) + lo * tn;  // rank order: identical
      XRABIT_TRY_HIP(step(mine + lo * tn, srcs, n_, hi - lo, dev_status(),
                          indirect ? table_ : nullptr, post_scale ? alpha : 0.0, stream_));
    }
    XRABIT_TRY_HIP(mark(3));
    XRABIT_TRY_HIP(Barrier());
    XRABIT_TRY_HIP(mark(4));
    CopyBatch b;
    NewBatch(&b);
    for (int p = 0; p < n_; ++p) {
      SegRange(c, seg, p, &lo, &hi);
      const size_t at = (off + lo) * tn;
      AddSeg(&b, out + at, stage(p, which) + lo * tn, out2_now != nullptr ? out2_now + at : nullptr,
             (hi - lo) * tn);
    }
    if (out2_now != nullptr && tail_end > 0) {
      AddSplit(&b, out2, out, tail_end * tn);  // as in the push form above
      tail_end = 0;
    }
    XRABIT_TRY_HIP(LaunchCopyBatch(b, stream_));
    XRABIT_TRY_HIP(mark(5));
  }
  if (out2 != nullptr && tail_end > 0) {
    // fused chunks (and chunks before a fused last one) into the second destination, only if
    // every barrier and hand-off of the op held
    CopyBatch b;
    NewBatch(&b);
    AddSeg(&b, out2, out, nullptr, tail_end * tn);
    if (tail_signal) {
      b.done_count = done_count();
      b.done_word = done_word();
      b.epoch = ++fused_epoch_;
    }
    XRABIT_TRY_HIP(LaunchCopyBatch(b, stream_));
    if (tail_signal) {
      done_pending_ = true;
      done_epoch_ = b.epoch;
    }
  }
  timing_pending_ = timed && !did_fused;  // phases exist only in the classic form
  return hipSuccess;
}

hipError_t PeerGroup::LinkProbe(size_t bytes, double out[kLinkProbeValues]) {
  utils::Assert(opened_, "peer group not opened");
  for (int i = 0; i < kLinkProbeValues; ++i) out[i] = 0;
  if (n_ < 2) return hipSuccess;
  const size_t total = std::max<size_t>(4096, std::min(bytes, stage_bytes_) / 4096 * 4096);
  const size_t per = std::max<size_t>(4096, total / static_cast<size_t>(n_ - 1) / 4096 * 4096);
  hipEvent_t e0, e1;
  XRABIT_TRY_HIP(hipEventCreate(&e0));
  XRABIT_TRY_HIP(hipEventCreate(&e1));
  // sources in parity 0 of the stages, destinations in parity 1
  auto timed = [&](const CopyBatch &b, double *ms) -> hipError_t {
    XRABIT_TRY_HIP(Barrier());
    XRABIT_TRY_HIP(hipEventRecord(e0, stream_));
    XRABIT_TRY_HIP(LaunchCopyBatch(b, stream_));
    XRABIT_TRY_HIP(hipEventRecord(e1, stream_));
    XRABIT_TRY_HIP(hipEventSynchronize(e1));
    float m = 0;
    XRABIT_TRY_HIP(hipEventElapsedTime(&m, e0, e1));
    *ms = m;
    return hipSuccess;
  };
  hipError_t err = hipSuccess;
  double ms = 0, sum_pull = 0, sum_push = 0;
  for (int k = 1; k < n_ && err == hipSuccess; ++k) {
    const int to = (rank_ + k) % n_;
    CopyBatch b;
    NewBatch(&b);
    AddSeg(&b, stage(rank_, 1), stage(to, 0), nullptr, total);
    err = timed(b, &ms);
    sum_pull += total / (ms * 1e-3) / 1e9;
    if (err != hipSuccess) break;
    NewBatch(&b);
    AddSeg(&b, stage(to, 1), stage(rank_, 0), nullptr, total, true);
    err = timed(b, &ms);
    sum_push += total / (ms * 1e-3) / 1e9;
  }
  if (err == hipSuccess) {
    out[0] = sum_pull / (n_ - 1);
    out[1] = sum_push / (n_ - 1);
    CopyBatch pull, push, both;
    NewBatch(&pull);
    NewBatch(&push);
    NewBatch(&both);
    for (int k = 1; k < n_; ++k) {
      const int q = (rank_ + k) % n_;
      // pulls land in slices [0, n) of the puller's parity-1 stage and pushes in slices
      // [n, 2n) of the receiver's, one slice per writer: no two writers overlap
      char *remote_dst = stage(q, 1) + static_cast<size_t>(n_ + rank_) * per;
      char *local_dst = stage(rank_, 1) + static_cast<size_t>(q) * per;
      AddSeg(&pull, local_dst, stage(q, 0), nullptr, per);
      AddSeg(&push, remote_dst, stage(rank_, 0), nullptr, per, true);
      AddSeg(&both, local_dst, stage(q, 0), nullptr, per);
      AddSeg(&both, remote_dst, stage(rank_, 0), nullptr, per, true);
    }
    const double moved = static_cast<double>(per) * (n_ - 1);
    if (per * static_cast<size_t>(2 * n_) <= stage_bytes_) {
      err = timed(pull, &ms);
      if (err == hipSuccess) out[2] = moved / (ms * 1e-3) / 1e9;
      if (err == hipSuccess) err = timed(push, &ms);
      if (err == hipSuccess) out[3] = moved / (ms * 1e-3) / 1e9;
      if (err == hipSuccess) err = timed(both, &ms);
      if (err == hipSuccess) out[4] = moved / (ms * 1e-3) / 1e9;
    }
  }
  // nobody's next op may write a stage a peer's probe copy still touches
  if (err == hipSuccess) err = Barrier();
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  return err;
}

hipError_t PeerGroup::AllreduceGraphable(void *buf, size_t count, int dtype, int op,
                                         hipStream_t stream) {
  // the classic forms only: the fused kernels and the pipelined form number their hand-offs
  // on the host, which a replayed graph would repeat
  const hipStream_t saved_stream = stream_;
  const bool saved_timing = timing_, saved_fused = fused_, saved_pipe = pipeline_,
             saved_done = done_signal_;
  const size_t saved_fused_oneshot = fused_oneshot_max_;
  stream_ = stream;
  timing_ = false;
  fused_ = false;
  pipeline_ = false;
  done_signal_ = false;
  fused_oneshot_max_ = 0;
  no_registry_ = true;  // no host drain or table copy may be captured
  // A replay runs its stage parities as captured, whatever the op before it left behind: a
  // barrier on each side keeps every peer's reads of the neighbouring ops out of this op's
  // stage writes (the previous op has completed on every rank once all arrive here; nobody
  // starts the next op before all finished this one).
  hipError_t e = Barrier();
  if (e == hipSuccess) e = Allreduce(buf, buf, nullptr, count, dtype, op, kPrepCopy, 1.0);
  if (e == hipSuccess) e = Barrier();
  stream_ = saved_stream;
  timing_ = saved_timing;
  fused_ = saved_fused;
  pipeline_ = saved_pipe;
  done_signal_ = saved_done;
  fused_oneshot_max_ = saved_fused_oneshot;
  no_registry_ = false;
  done_pending_ = false;
  timing_pending_ = false;
  ++graphable_ops_;
  return e;
}

void PeerGroup::DieMidOp() {
  die_mid_ = false;
  (void)hipStreamSynchronize(stream_);
  fprintf(stderr, "[%d]@@@Hit Mock Die Mid Op: exiting inside a multi-chunk device allreduce\n",
          rank_);
  fflush(stderr);
  utils::ExitProcess(kMockDieMidExitCode);
}

hipError_t PeerGroup::AllreducePipelined(const char *in, char *out, char *out2, size_t count,
                                         size_t tn, double post, const ReduceStep &step) {
  // a configured chunk is rounded to whole 256 n-element blocks and held to what n + 1 slots
  // of a stage can take (the automatic choice already is)
  const size_t q = 256 * static_cast<size_t>(n_);
  const size_t cap = stage_bytes_ / tn / static_cast<size_t>(n_ + 1) / 256 * q;
  const size_t chunk = pipeline_chunk_ != 0
                           ? std::max(q, std::min(cap, pipeline_chunk_ / tn / q * q))
                           : ArPipeline::AutoChunk(count, tn, n_, stage_bytes_);
  const ArPipeline plan(count, chunk, n_);
  utils::Check(plan.stage_bytes(tn) <= stage_bytes_,
               "pipelined allreduce: a chunk of %zu elements needs %zu stage bytes, %zu available",
               chunk, plan.stage_bytes(tn), stage_bytes_);
  const int base = parity_;
  for (size_t t = 0; t < plan.rounds(); ++t) {
    // pushes of chunk t (remote writes) and gathers of chunk t-2 (remote reads) in one launch:
    // opposite directions of every link
    CopyBatch b;
    NewBatch(&b);
    for (const ArCopy &c : plan.Copies(rank_, t)) {
      const int p = ArPipeline::parity(base, c.chunk);
      const size_t at = (c.chunk * plan.chunk + c.lo) * tn;
      const size_t bytes = (c.hi - c.lo) * tn;
      if (c.push) {
        AddSeg(&b, stage(c.peer, p) + plan.inbox(rank_) * tn, in + at, nullptr, bytes, true);
      } else {
        char *second = out2 != nullptr && (plan.second_in_gather(c.chunk) || !defer_second_)
                           ? out2 + at
                           : nullptr;
        AddSeg(&b, out + at, stage(c.peer, p) + plan.result() * tn, second, bytes);
      }
    }
    const bool final_round = t + 1 == plan.rounds();
    if (final_round && out2 != nullptr && defer_second_) {
      // after the last barrier: the earlier chunks into the second destination, in the launch
      // of the last gather (local HBM copy and xGMI reads at once)
      AddSplit(&b, out2, out, plan.second_tail() * tn);
    }
    if (b.n > 0) XRABIT_TRY_HIP(LaunchCopyBatch(b, stream_));
    // the reduce of chunk t-1: this rank's n inbox slots into its result slot
    const ArReduce red = plan.Reduce(rank_, t);
    if (red.any) {
      char *mine = stage(rank_, ArPipeline::parity(base, red.chunk));
      const void *srcs[kMaxPeers];
      for (int s = 0; s < n_; ++s) srcs[s] = mine + plan.inbox(s) * tn;
      XRABIT_TRY_HIP(step(mine + plan.result() * tn, srcs, n_, red.hi - red.lo, dev_status(),
                          nullptr, post, stream_));
    }
    if (plan.barrier_after(t)) {
      XRABIT_TRY_HIP(Barrier());
      // after round 2's barrier every peer has gathered chunk 0 into its output
      if (die_mid_ && t >= 2 && plan.nchunks >= 2) DieMidOp();
    }
    ++pipelined_rounds_;
  }
  parity_ = plan.next_parity(base);
  ++pipelined_ops_;
  push_chunks_ += plan.nchunks;
  return hipSuccess;
}

void PeerGroup::EnableTiming() {
  if (timing_) return;
  for (auto &e : ev_) CheckHip(hipEventCreate(&e), "hipEventCreate(phase)");
  timing_ = true;
}

void PeerGroup::CollectTiming() {
  if (!timing_pending_) return;
  timing_pending_ = false;
  for (int k = 0; k < kPhases; ++k) {
    float ms = 0;
    if (hipEventElapsedTime(&ms, ev_[k], ev_[k + 1]) != hipSuccess) {
      (void)hipGetLastError();
      return;
    }
    phase_ms_[k] += ms;
  }
  ++timed_ops_;
}

hipError_t PeerGroup::Broadcast(void *buf, size_t bytes, int root, void *log) {
  utils::Assert(opened_, "peer group not opened");
  done_pending_ = false;
  char *user = static_cast<char *>(buf);
  char *lg = static_cast<char *>(log);
  if (bytes == 0) return hipSuccess;
  CopyBatch b;
  if (n_ == 1) {
    // a one-rank group: the data is already in place, only the log slot needs it
    if (lg != nullptr) XRABIT_TRY_HIP(LaunchCopy(lg, user, bytes, stream_));
    return hipSuccess;
  }
  // scatter of chunk k+1 and allgather of chunk k in the same round (bcast_plan.h)
  const size_t chunk = bcast_chunk_ != 0 ? std::min(bcast_chunk_, stage_bytes_)
                                         : BcastPipeline::AutoChunk(bytes, stage_bytes_);
  const BcastPipeline plan(bytes, chunk, n_, root);
  const int base = parity_;
  for (size_t t = 0; t < plan.rounds(); ++t) {
    if (plan.barrier_before(t)) XRABIT_TRY_HIP(Barrier());
    NewBatch(&b);
    for (const BcastCopy &c : plan.Round(rank_, t)) {
      const int which = BcastPipeline::parity(base, c.chunk);
      const size_t at = c.chunk * plan.chunk + c.off;  // byte offset in the user buffer
      const char *src = c.from < 0 ? user + at : stage(c.from, which) + c.off;
      char *dsts[3];
      int nd = 0;
      if (c.to_stage) dsts[nd++] = stage(rank_, which) + c.off;
      if (c.to_user) dsts[nd++] = user + at;
      if (c.to_log && lg != nullptr) dsts[nd++] = lg + at;
      utils::Assert(nd <= 2, "broadcast plan: more than two destinations");
      if (nd == 0) continue;
      AddSeg(&b, dsts[0], src, nd > 1 ? dsts[1] : nullptr, c.bytes);
    }
    if (b.n > 0) XRABIT_TRY_HIP(LaunchCopyBatch(b, stream_));
  }
  parity_ = plan.next_parity(base);
  ++bcast_ops_;
  bcast_chunks_ += plan.nchunks;
  return hipSuccess;
}

hipError_t PeerGroup::AllgatherV(void *buf, size_t total, const std::vector<size_t> &begin,
                                 const std::vector<size_t> &size, void *log) {
  utils::Assert(opened_, "peer group not opened");
  done_pending_ = false;
  char *user = static_cast<char *>(buf);
  char *lg = static_cast<char *>(log);
  for (size_t wlo = 0; wlo < total; wlo += stage_bytes_) {
    const size_t whi = std::min(total, wlo + stage_bytes_);
    const int which = parity_;
    parity_ ^= 1;
    CopyBatch b;
    NewBatch(&b);
    for (int p = 0; p < n_; ++p) {
      size_t lo[2], hi[2];
      const int k = SliceRanges(begin[p], size[p], total, lo, hi);
      for (int j = 0; j < k; ++j) {
        const size_t a = std::max(lo[j], wlo), z = std::min(hi[j], whi);
        if (z <= a) continue;
        if (p == rank_) {
          // own slice into the stage (and the log slot, dual store)
          AddSeg(&b, stage(rank_, which) + (a - wlo), user + a, lg != nullptr ? lg + a : nullptr,
                 z - a);
        }
      }
    }
    if (b.n > 0) XRABIT_TRY_HIP(LaunchCopyBatch(b, stream_));
    XRABIT_TRY_HIP(Barrier());
    NewBatch(&b);
    for (int p = 0; p < n_; ++p) {
      if (p == rank_) continue;
      size_t lo[2], hi[2];
      const int k = SliceRanges(begin[p], size[p], total, lo, hi);
      for (int j = 0; j < k; ++j) {
        const size_t a = std::max(lo[j], wlo), z = std::min(hi[j], whi);
        if (z > a) {
          AddSeg(&b, user + a, stage(p, which) + (a - wlo), lg != nullptr ? lg + a : nullptr,
                 z - a);
        }
      }
    }
    if (b.n > 0) XRABIT_TRY_HIP(LaunchCopyBatch(b, stream_));
  }
  return hipSuccess;
}
hipError_t PeerGroup::AllgatherResolved(void *buf, size_t total, size_t begin, size_t size,
                                        void *log) {
  utils::Assert(opened_, "peer group not opened");
  done_pending_ = false;
  if (total == 0) return hipSuccess;
  char *user = static_cast<char *>(buf);
  char *lg = static_cast<char *>(log);
  begin %= total;
  size_t lo[2], hi[2];
  const int k = SliceRanges(begin, size, total, lo, hi);
  for (size_t wlo = 0; wlo < total; wlo += stage_bytes_) {
    const size_t whi = std::min(total, wlo + stage_bytes_);
    const int which = parity_;
    parity_ ^= 1;
    // own slice's part of the window into the stage (and the log slot, dual store)
    CopyBatch b;
    NewBatch(&b);
    for (int j = 0; j < k; ++j) {
      const size_t a = std::max(lo[j], wlo), z = std::min(hi[j], whi);
      if (z > a) {
        AddSeg(&b, stage(rank_, which) + (a - wlo), user + a, lg != nullptr ? lg + a : nullptr,
               z - a);
      }
    }
    if (b.n > 0) XRABIT_TRY_HIP(LaunchCopyBatch(b, stream_));
    // the barrier publishes this rank's slice and resolves everybody's into the meta table
    ResolveArgs ra{};
    ra.parity = which;
    ra.table = nullptr;
    ra.my_meta[0] = static_cast<unsigned long long>(begin);
    ra.my_meta[1] = static_cast<unsigned long long>(size);
    ra.meta_table = meta_table_;
    XRABIT_TRY_HIP(Barrier(&ra));
    AllgatherWindowArgs ga{};
    for (int p = 0; p < n_; ++p) ga.stage[p] = stage(p, which);
    ga.meta_table = meta_table_;
    ga.buf = user;
    ga.log = lg;
    ga.total = total;
    ga.wlo = wlo;
    ga.whi = whi;
    ga.n = n_;
    ga.rank = rank_;
    ga.guard = dev_status();
    XRABIT_TRY_HIP(LaunchAllgatherWindow(ga, stream_));
  }
  ++resolved_allgathers_;
  return hipSuccess;
}

hipError_t PeerGroup::Exchange(const std::vector<ExchangeItem> &plan, size_t *bytes_in) {
  utils::Assert(opened_, "peer group not opened");
  done_pending_ = false;
  *bytes_in = 0;
  // every sender's distinct payloads, back to back (256-B aligned) in plan order: the byte
  // stream it pushes through its stage buffer.  All ranks derive the same layout.
  std::vector<size_t> stream_len(n_, 0), at(plan.size(), 0);
  std::vector<std::vector<std::pair<int, size_t>>> first(n_);  // (key, offset) per sender
  for (size_t i = 0; i < plan.size(); ++i) {
    const ExchangeItem &x = plan[i];
    utils::Check(x.src >= 0 && x.src < n_ && x.dst >= 0 && x.dst < n_,
                 "device exchange: rank out of range");
    if (x.src == x.dst || x.bytes == 0) continue;
    auto &seen = first[x.src];
    auto it = std::find_if(seen.begin(), seen.end(),
                           [&](const std::pair<int, size_t> &p) { return p.first == x.key; });
    if (it != seen.end()) {
      at[i] = it->second;
      continue;
    }
    at[i] = stream_len[x.src];
    seen.emplace_back(x.key, at[i]);
    stream_len[x.src] += RoundUp(x.bytes, 256);
  }
  CopyBatch b;
  NewBatch(&b);
  auto add = [&](char *dst, const char *src, size_t bytes) -> hipError_t {
    if (bytes == 0) return hipSuccess;
    if (b.n == kMaxCopySegs) {
      XRABIT_TRY_HIP(LaunchCopyBatch(b, stream_));
      NewBatch(&b);
    }
    AddSeg(&b, dst, src, nullptr, bytes);
    return hipSuccess;
  };
  auto flush = [&]() -> hipError_t {
    if (b.n > 0) XRABIT_TRY_HIP(LaunchCopyBatch(b, stream_));
    NewBatch(&b);
    return hipSuccess;
  };
  // copies a rank makes to itself never touch the stage
  for (const ExchangeItem &x : plan) {
    if (x.src == rank_ && x.dst == rank_) {
      XRABIT_TRY_HIP(add(static_cast<char *>(x.dst_ptr), static_cast<const char *>(x.src_ptr),
                         x.bytes));
    }
  }
  XRABIT_TRY_HIP(flush());
  size_t rounds = 0;
  for (int s = 0; s < n_; ++s) {
    rounds = std::max(rounds, (stream_len[s] + stage_bytes_ - 1) / stage_bytes_);
  }
  for (size_t r = 0; r < rounds; ++r) {
    const size_t lo = r * stage_bytes_, hi = lo + stage_bytes_;
    const int which = parity_;
    parity_ ^= 1;
    // 1. my window of my stream into my stage (each distinct payload once)
    std::vector<int> staged;
    for (size_t i = 0; i < plan.size(); ++i) {
      const ExchangeItem &x = plan[i];
      if (x.src != rank_ || x.dst == rank_ || x.bytes == 0) continue;
      if (std::find(staged.begin(), staged.end(), x.key) != staged.end()) continue;
      staged.push_back(x.key);
      const size_t a = std::max(lo, at[i]), z = std::min(hi, at[i] + x.bytes);
      if (z > a) {
        XRABIT_TRY_HIP(add(stage(rank_, which) + (a - lo),
                           static_cast<const char *>(x.src_ptr) + (a - at[i]), z - a));
      }
    }
    XRABIT_TRY_HIP(flush());
    XRABIT_TRY_HIP(Barrier());
    // 2. pull the parts of this window addressed to me
    for (size_t i = 0; i < plan.size(); ++i) {
      const ExchangeItem &x = plan[i];
      if (x.dst != rank_ || x.src == rank_ || x.bytes == 0) continue;
      const size_t a = std::max(lo, at[i]), z = std::min(hi, at[i] + x.bytes);
      if (z > a) {
        XRABIT_TRY_HIP(add(static_cast<char *>(x.dst_ptr) + (a - at[i]),
                           stage(x.src, which) + (a - lo), z - a));
        *bytes_in += z - a;
      }
    }
    XRABIT_TRY_HIP(flush());
  }
  return hipSuccess;
}
#undef XRABIT_TRY_HIP
}  // namespace device
}  // namespace rabit
