/*!
 * \file peer_coll.h
 * \brief Direct transport of the device plane: collectives that read peer HBM through IPC
 *        mappings (xGMI between the GPUs of one MI355X node).
 *
 * Every rank exports one uncached allocation [flags | stage 0 | stage 1] and maps its peers'.
 * An op stages its input in the local stage buffer, meets the peers at a flag barrier, and then
 * pulls what it needs from the peers' stage buffers with streaming kernels, so each of the 7
 * xGMI links of a GPU carries 1/7 of the traffic at the same time (a ring uses one link per
 * direction).  Stage buffers alternate between ops, which lets two barriers per allreduce
 * suffice (SURVEY §5.8 "direct peer access with our own multi-source reduce kernel").
 *
 *  - Allreduce (two-shot): stage; barrier; rank r reduces segment r of all n stage buffers
 *    in place with the multi-source kernel; barrier; everyone gathers the n reduced segments
 *    (optionally storing them twice: result log + user buffer).  Per rank, 2(n-1)/n of the
 *    payload crosses xGMI — the bandwidth-optimal amount — spread over all links.
 *    Push variant (set_push): every rank writes segment q of its input straight into rank q's
 *    stage (an inbox slot per sender); barrier; rank r reduces its n local inbox slots;
 *    barrier; everyone gathers as above.  The calibration picks pull or push per machine.
 *  - Broadcast: root stages; barrier; rank p pulls segment p from the root; barrier; everyone
 *    pulls the other segments from their owners (scatter + allgather: the root's links carry
 *    2/n of the payload each instead of all of it).
 *  - AllgatherV (rabit's variable, wrapping slices): stage own slice; barrier; pull the rest.
 *
 * Ranks that share one GPU also work (IPC within a device), which is how the multi-rank device
 * path is tested on a one-GPU machine.  Failure handling: the barrier gives up when the host
 * raises the abort word or a deadline passes, and reports it in a status word; the owner then
 * drops the whole group (epochs are not resynchronised, a new group is built).
 */
#ifndef XRABIT_DEVICE_PEER_COLL_H_
#define XRABIT_DEVICE_PEER_COLL_H_

#include <hip/hip_runtime_api.h>

#include <cstddef>
#include <functional>
#include <algorithm>
#include <cstdint>
#include <string>
#include <atomic>
#include <vector>

#include "device/peer_registry.h"

namespace rabit {
namespace device {

constexpr int kMaxPeers = 8;
constexpr int kMaxCopySegs = 16;
/*! \brief bytes of the flag area at the start of each exported allocation: kMaxPeers arrival
 *  flags at offset 0, the local failure word at kPeerStatusOffset */
constexpr size_t kPeerFlagBytes = 64 * 1024;
/*! \brief exit status of a rank leaving through the mock_die_mid hook (the launcher restarts it) */
constexpr int kMockDieMidExitCode = 250;
constexpr size_t kPeerStatusOffset = 4096;
/*! \brief an int that peers raise when they give up on the group: a barrier kernel that gives up
 *  on its own account (the host raised the abort word: it saw a failure, e.g. a dead peer's
 *  sockets closing; or the deadline passed) stores it into every peer's flag area over the IPC
 *  mappings, and every barrier and fused wait polls its own copy next to the host abort word.
 *  The rank that sees a failure first so ends every rank's spinning kernels at once, instead of
 *  each rank waiting to learn of it on its own TCP links.  No stream and no host call is involved
 *  (a HIP stream per group cost tens of ms of bring-up with 8 ranks on one GPU,
 *  profiles/r4_recovery/).  A group stays failed after an abort and the next epoch builds a new,
 *  zeroed one, so the word needs no reset */
constexpr size_t kPeerAbortOffset = kPeerStatusOffset + 1024;
/*! \brief two mailbox words (by stage parity): where this rank's input of the current chunk
 *  lives, published before the first barrier of the chunk (see ResolveArgs) */
constexpr size_t kPeerMailboxOffset = 8192;
/*! \brief per parity, this rank's (begin, size) slice of the current allgather window, published
 *  by the window's barrier (ResolveArgs::meta_table): peers resolve the whole slice layout on the
 *  device, so no host round exchanges it (PeerGroup::AllgatherResolved) */
constexpr size_t kPeerMetaOffset = kPeerMailboxOffset + 64;
/*! \brief mailbox flag: the offset is into the symmetric heap, not the stage allocation */
constexpr unsigned long long kMailboxHeap = 1ull << 63;

struct PeerFlagTable {
  unsigned long long *p[kMaxPeers];
};

struct CopySeg {
  char *dst;
  const char *src;
  char *dst2;  // optional second destination (nullptr: none)
  size_t bytes;
  int remote;  // 1: dst is a peer's memory (push): system-scope write-through stores, dst
               // 16-byte aligned, no dst2
};

struct CopyBatch {
  CopySeg seg[kMaxCopySegs];
  int n;
  const int *guard;  // optional device word: the launch does nothing when it is non-zero
  int remote;        // 1: every segment is remote (as CopySeg::remote)
  // optional completion signal (as FusedAllreduceArgs::done_word): the last workgroup stores
  // epoch into done_word once every workgroup is through, guarded launches included
  unsigned int *done_count;
  unsigned long long *done_word;
  unsigned long long epoch;
};

/*!
 * \brief optional work of a chunk's first barrier: publish where this rank's input is (its
 *        mailbox word) before signalling, and after the wait turn every peer's mailbox into a
 *        source pointer for this rank's segment (table[p] = base_p + offset_p + seg_off) in
 *        cached device memory, so the reduce kernel reads n scalars instead of n remote words
 *        per workgroup.
 */
struct ResolveArgs {
  unsigned long long my_mailbox;    // value to publish
  int parity;                       // mailbox slot
  const char *stage_base[kMaxPeers];
  const char *heap_base[kMaxPeers];  // nullptr: that peer has no symmetric heap
  size_t seg_off;                   // byte offset of this rank's segment in the chunk
  const void **table;               // out: n source pointers
  // registered allocations (peer_registry.h): [peer][slot] mapped bases, for kMailboxReg words
  // of the peers; this rank's own registered input is own_src (the table maps peers only)
  const char *const *reg_table;
  const char *own_src;
  // optional allgather slice layout: publish my_meta (begin, size) before signalling, and after
  // the wait copy every rank's pair into meta_table[2 p .. 2 p + 1] (device memory)
  unsigned long long my_meta[2];
  unsigned long long *meta_table;
};

/*!
 * \brief the gather of one allgather window whose slice layout lives on the device (meta_table,
 *        filled by the window's barrier): every byte of [wlo, whi) that belongs to another rank's
 *        slice (slices partition [0, total) and may wrap) is copied from that rank's stage (at
 *        offset - wlo) into buf, and into log when given
 */
struct AllgatherWindowArgs {
  const char *stage[kMaxPeers];            // stage of this window's parity, per rank (mapped)
  const unsigned long long *meta_table;    // 2 n words: (begin, size) per rank
  char *buf, *log;
  size_t total, wlo, whi;
  int n, rank;
  const int *guard;                        // the group's failure word
};
hipError_t LaunchAllgatherWindow(const AllgatherWindowArgs &args, hipStream_t stream);

/*!
 * \brief the fused two-shot allreduce of one chunk (fused_allreduce.hip): ONE launch replaces
 *        stage copy + barrier + reduce + barrier + gather.  The chunk is cut into n segments
 *        (segment q reduced by rank q) of `tiles` tiles each; workgroup w owns tiles
 *        w, w + G, ... of every segment, on every rank, and hands them over with per-tile flags
 *        instead of whole-GPU barriers:
 *          1. stage (pull: own stage; push: inbox slot `rank` of each owner's stage) its tiles of
 *             every segment, then raise ready[tile] (push: inbox[rank][tile] at each owner);
 *          2. for its tiles of segment `rank`: wait for every rank's ready flag, reduce the n
 *             sources in rank order into out/out2 and into the own stage (where peers gather
 *             it), raise done[tile];
 *          3. for its tiles of every other segment p: wait for done[tile] of rank p, copy.
 *        A workgroup only ever waits for the workgroup with the SAME index on another rank, which
 *        produces before it waits, so the launch cannot deadlock whatever subset of either grid
 *        is resident (grids are equal on every rank).  Every wait gives up on the host abort
 *        word, the wall-clock deadline, or a failure seen by another workgroup.
 */
constexpr size_t kFusedTileBytes = 64 * 1024;     // largest tile
constexpr size_t kFusedTileMinBytes = 8 * 1024;   // smallest tile (small chunks, big grids)
struct FusedAllreduceArgs {
  char *stage[kMaxPeers];                 // stage buffer of this parity, per rank (mapped)
  const char *alloc[kMaxPeers];           // exported allocation base per rank (zero copy)
  const char *heap[kMaxPeers];            // symmetric heap base per rank (zero copy)
  unsigned long long *flags[kMaxPeers];   // fused flag block of this parity, per rank
  const char *src;                        // this rank's input chunk
  char *out, *out2;                       // result chunk (out2: optional second copy)
  size_t count;                           // elements in the chunk
  size_t seg;                             // elements per segment (multiple of 256)
  size_t tile;                            // elements per tile (multiple of 256)
  int tiles;                              // tiles per segment
  int tiles_cap;                          // flag slots per array in a flag block
  int n, rank, push, zero_copy;
  unsigned long long mailbox;             // zero copy: where this rank's input is
  unsigned long long epoch;
  int dtype, op, prep;
  double alpha, post;
  const volatile int *abort_word;
  const volatile int *peer_abort;  // this rank's copy of the peers' abort word (kPeerAbortOffset)
  int *dev_status, *host_status;
  long long deadline_ticks;
  // optional completion signal (fused one-shot): every workgroup counts itself in on done_count
  // (device memory, re-armed by the last one), and the last one stores `epoch` into done_word
  // (pinned host memory) — the host polls that word instead of an event (no hipEventRecord /
  // hipEventQuery round trips on the small-op path)
  unsigned int *done_count;
  unsigned long long *done_word;
};
/*! \brief u64 words of one fused flag block (one parity) for tiles_cap tiles per segment */
inline size_t FusedFlagWords(int tiles_cap) {
  return 64 + static_cast<size_t>(2 + kMaxPeers) * static_cast<size_t>(tiles_cap);
}
/*! \brief workgroups of the fused kernel that fit on `device` at once (0: unknown) */
int FusedResidentBlocks(int device);
/*! \brief enqueue the fused allreduce of one chunk on `grid` workgroups */
hipError_t LaunchFusedAllreduce(const FusedAllreduceArgs &args, int grid, hipStream_t stream);
/*! \brief enqueue a small chunk's one-shot allreduce as one launch (tiles of args.tile elements
 *  over args.count; stage copy, per-tile ready flags, reduce of all n stages into out / out2) */
hipError_t LaunchFusedOneshot(const FusedAllreduceArgs &args, int grid, hipStream_t stream);

/*!
 * \brief the group's flag barrier.  Its number comes from `counter`, a word in this rank's own
 *        flag area that the barrier kernel itself advances: every rank runs the same sequence
 *        of barriers, so the counters agree, and a captured hipGraph that replays barriers gets
 *        fresh numbers on every replay (a host-side number would be baked into the graph)
 */
hipError_t LaunchPeerBarrier(const PeerFlagTable &flags, int rank, int n,
                             unsigned long long *counter, const volatile int *abort_word,
                             int *dev_status, int *host_status, long long deadline_ticks,
                             int peer_abort_on, const ResolveArgs *resolve, hipStream_t stream);
hipError_t LaunchCopyBatch(const CopyBatch &batch, hipStream_t stream);

/*! \brief fixed-size record every rank contributes when a group is built */
struct PeerRecord {
  char ipc[64];      // hipIpcMemHandle_t of the exported allocation
  char pci[32];      // PCI bus id of the GPU
  char host[64];     // host name
  uint64_t stage_bytes;
  int32_t pid;
  int32_t device;
  char heap_ipc[64];   // hipIpcMemHandle_t of the symmetric heap (heap_bytes != 0)
  uint64_t heap_bytes;
  int32_t fused_cap;   // fused-kernel workgroups resident at once on this GPU
  int32_t pad;
  char reg_name[48];   // shm name of the zero-copy registry page ("" : none, peer_registry.h)
};

/*!
 * \brief one point-to-point copy of a device exchange (every rank passes the same global plan;
 *        src_ptr is only meaningful on rank src, dst_ptr only on rank dst).  Items of one
 *        sender with the same key carry the same bytes (sent once, read by several receivers).
 */
struct ExchangeItem {
  int src, dst;
  int key;
  size_t bytes;
  const void *src_ptr;
  void *dst_ptr;
};

/*! \brief this rank's symmetric heap (owned by the DevicePlane, outlives peer groups) */
struct SymHeapInfo {
  char *base{nullptr};
  size_t bytes{0};
  char ipc[64]{};
};

class PeerGroup {
 public:
  /*! \brief allocate and export the local buffers; stage_bytes per stage buffer */
  PeerGroup(int device, size_t stage_bytes, double deadline_sec, hipStream_t stream,
            const SymHeapInfo &heap = SymHeapInfo());
  ~PeerGroup();
  PeerGroup(const PeerGroup &) = delete;
  PeerGroup &operator=(const PeerGroup &) = delete;

  const PeerRecord &local() const { return local_; }
  /*!
   * \brief map every peer's allocation; all must be on this host with equal stage sizes.
   * \return false (and an explanation in why) when the group cannot be built
   */
  bool Open(const std::vector<PeerRecord> &all, int rank, std::string *why);
  int size() const { return n_; }
  void set_stream(hipStream_t s) { stream_ = s; }
  size_t stage_bytes() const { return stage_bytes_; }

  // enqueue on the stream given at construction (the caller waits / checks status)
  hipError_t Allreduce(const void *send, void *recv, void *recv2, size_t count, int dtype, int op,
                       int prep, double alpha);
  /*! \brief reduction step of a custom allreduce: dst = reduce(srcs[0..n)) over count
   *  elements on `stream`, doing nothing when *guard != 0 */
  typedef std::function<hipError_t(void *dst, const void *const *srcs, int n, size_t count,
                                   const int *guard, const void *const *table,
                                   double post_scale, hipStream_t stream)>
      ReduceStep;
  /*! \brief allreduce of count elements of type_nbytes bytes with a caller-provided reduction */
  hipError_t AllreduceCustom(const void *send, void *recv, void *recv2, size_t count,
                             size_t type_nbytes, const ReduceStep &step);
  /*!
   * \brief broadcast from root, pipelined over chunks: the scatter of chunk k+1 (root -> its
   *        non-roots) and the allgather of chunk k (among the non-roots) share a round, because
   *        they use disjoint xGMI link directions (bcast_plan.h).  log != nullptr: every byte of
   *        the result is also stored there by the same kernels (the robust engine's result-log
   *        slot: no copy after the collective)
   */
  hipError_t Broadcast(void *buf, size_t bytes, int root, void *log = nullptr);
  /*! \brief pipeline chunk of a broadcast (0: automatic, BcastPipeline::AutoChunk) */
  void set_bcast_chunk(size_t b) { bcast_chunk_ = b; }
  uint64_t bcast_ops() const { return bcast_ops_; }
  uint64_t bcast_chunks() const { return bcast_chunks_; }
  hipError_t AllgatherV(void *buf, size_t total, const std::vector<size_t> &begin,
                        const std::vector<size_t> &size, void *log = nullptr);
  /*!
   * \brief rabit's allgather knowing only this rank's slice [begin, begin + size) mod total:
   *        every window's barrier publishes the slice and resolves everybody's on the device,
   *        and the gather kernel finds each byte's owner there (no host metadata round)
   */
  hipError_t AllgatherResolved(void *buf, size_t total, size_t begin, size_t size,
                               void *log = nullptr);
  uint64_t resolved_allgathers() const { return resolved_allgathers_; }
  /*!
   * \brief point-to-point copies between ranks (a collective: every rank passes the same plan).
   *        Each sender streams the distinct payloads it owns through its stage buffer, one
   *        stage-sized window per round; after the round's barrier every receiver pulls the
   *        parts addressed to it from the senders' stages.  Ranks that neither send nor receive
   *        only join the barriers (no payload bytes move through them).
   *        *bytes_in receives the payload bytes this rank pulled from peers.
   */
  hipError_t Exchange(const std::vector<ExchangeItem> &plan, size_t *bytes_in);

  /*!
   * \brief xGMI link probe (a collective: every rank of the group calls it between the same
   *        ops).  Copies of `bytes` (at most a stage) through the IPC mappings, each started
   *        right after a barrier and timed with hipEvents on this rank:
   *          [0] one link, reads: every rank pulls from rank + k at once, mean over k = 1..n-1
   *          [1] one link, writes: every rank pushes to rank + k at once, mean over k
   *          [2] all links, reads: every rank pulls bytes / (n-1) from each peer at once
   *          [3] all links, writes: every rank pushes bytes / (n-1) to each peer at once
   *          [4] all links, both directions: [2] and [3] in one launch (bytes each way)
   *        out[i] = GB/s of this rank (bytes moved per direction / its time).  The stages'
   *        contents are garbage afterwards; a barrier at the end keeps the next op's stage
   *        writes behind every probe copy.
   */
  hipError_t LinkProbe(size_t bytes, double out[5]);
  static constexpr int kLinkProbeValues = 5;
  /*!
   * \brief in-place allreduce that may be captured into a hipGraph and replayed (non-fault-
   *        tolerant engines): the classic pull / push form on `stream`, with no host wait, no
   *        event and no completion word, between two extra barriers, so no stage access of the
   *        op overlaps one of the ops around it and a replay may run on any stage parity (its
   *        parities are the captured ones, whatever the previous op used).  Barrier numbers come
   *        from the device counter.  Graph replays and other ops of the group must be ordered
   *        (one stream, or joined streams).
   */
  hipError_t AllreduceGraphable(void *buf, size_t count, int dtype, int op, hipStream_t stream);
  /*! \brief make spinning barriers give up (host side; safe at any time) */
  void SignalAbort();
  /*! \brief true when a barrier gave up (read after the stream drained) */
  bool failed() const;
  /*! \brief why the group failed: 1 abort word, 2 unmapped zero-copy source, 3 deadline,
   *         4 a peer aborted the group */
  int fail_reason() const {
    return host_words_ != nullptr ? __atomic_load_n(&host_words_[1], __ATOMIC_SEQ_CST) : 0;
  }
  uint64_t barriers() const { return epoch_; }
  /*! \brief chunks whose input was read in place (symmetric heap or a registered allocation:
   *  no stage copy) */
  uint64_t zero_copy_chunks() const { return zero_copy_chunks_; }
  /*! \brief of those, chunks of registered ordinary allocations (peer_registry.h) */
  uint64_t reg_zero_copy_chunks() const { return reg_zero_copy_chunks_; }
  const PeerRegistry &registry() const { return registry_; }
  /*! \brief ordinary allocations are registered for zero copy (rabit_device_zero_copy) from
   *  this many bytes per op (0: never) */
  void set_zero_copy_min(size_t b) { zero_copy_min_ = b; }
  /*! \brief every peer mapped this rank's registry page: drop its name */
  void SealRegistry() { registry_.Seal(); }
  /*! \brief ops of at most this many bytes use the one-shot allreduce (one barrier) */
  void set_oneshot_max(size_t b) { oneshot_max_ = b; }
  /*!
   * \brief reduce-scatter by remote WRITES (push) instead of remote reads: every rank writes
   *        segment q of its input into an inbox slot of rank q's stage buffer, then reduces
   *        its inbox locally; the gather still pulls.  Posted writes need no round trip per
   *        request over xGMI; which variant is faster is measured by the calibration.
   */
  void set_push(bool v) { push_ = v; }
  bool push() const { return push_; }
  uint64_t push_chunks() const { return push_chunks_; }
  uint64_t oneshot_ops() const { return oneshot_ops_; }
  /*!
   * \brief two-shot allreduces as the PIPELINED push form (ar_plan.h): the push reduce-scatter
   *        of chunk k (outgoing links) and the gather of chunk k-2 (incoming links) share a
   *        round, one barrier per round.  Applies with set_push(true) to ops above the one-shot
   *        size; the calibration times it as a form of its own.
   */
  void set_pipeline(bool v) { pipeline_ = v; }
  bool pipeline() const { return pipeline_; }
  /*! \brief bytes per pipeline chunk (0: ArPipeline::AutoChunk) */
  void set_pipeline_chunk(size_t bytes) { pipeline_chunk_ = bytes; }
  uint64_t pipelined_ops() const { return pipelined_ops_; }
  uint64_t graphable_ops() const { return graphable_ops_; }
  uint64_t pipelined_rounds() const { return pipelined_rounds_; }
  /*!
   * \brief test hook (mock_die_mid): the next multi-chunk allreduce exits the process in the
   *        middle, right after a barrier that every peer passed only with the op's first chunk
   *        already gathered into its output, so survivors fail the op with part of it delivered
   */
  void ArmDieMidOp() { die_mid_ = true; }
  /*! \brief test knob (rabit_device_defer_second=0): store the second destination in every
   *  chunk's gather, as before the deferral, to show what the deferral protects */
  void set_defer_second(bool v) { defer_second_ = v; }
  /*!
   * \brief two-shot chunks of built-in ops run as ONE fused kernel (per-tile flags, see
   *        FusedAllreduceArgs) instead of stage + barrier + reduce + barrier + gather launches
   */
  void set_fused(bool v) { fused_ = v; }
  /*! \brief one-shot ops of at most this many bytes as one fused launch, larger ones (and all
   *  with 0) as stage copy + barrier + reduce */
  void set_fused_oneshot_max(size_t b) { fused_oneshot_max_ = b; }
  uint64_t fused_oneshots() const { return fused_oneshots_; }
  bool fused() const { return fused_; }
  /*! \brief workgroups of a fused launch (0: automatic, from the ranks sharing a GPU) */
  void set_fused_grid(int g) { fused_grid_req_ = g; }
  /*! \brief chunks below this many bytes keep the classic form */
  void set_fused_min_bytes(size_t b) { fused_min_bytes_ = b; }
  int fused_grid() const { return fused_grid_; }
  /*! \brief the most ranks of this group on one GPU (1: every rank has its own) */
  int gpu_share() const { return gpu_share_; }
  uint64_t fused_chunks() const { return fused_chunks_; }
  /*!
   * \brief the op just enqueued ends with a kernel that signals its completion in pinned host
   *        memory: *word reaches `epoch` once every workgroup is done (failed ones included;
   *        failed() tells).  False (and nothing to poll) otherwise.  Consumes the signal.
   */
  bool TakeDoneSignal(const volatile unsigned long long **word, unsigned long long *epoch) {
    if (!done_pending_) return false;
    done_pending_ = false;
    *word = done_word();
    *epoch = done_epoch_;
    return true;
  }
  /*! \brief an abort also raises every peer's abort word (rabit_device_peer_abort) */
  void set_peer_abort(bool on) { peer_abort_ = on; }
  /*! \brief polling the done word instead of an event (rabit_device_done_word) */
  void set_done_signal(bool v) { done_signal_ = v; }
  /*! \brief record hipEvents between the phases of single-chunk allreduces */
  void EnableTiming();
  /*! \brief stop timing phases (the events stay for a later EnableTiming) */
  void DisableTiming() { timing_ = false; }
  /*! \brief forget the phase times accumulated so far */
  void ResetTiming() {
    for (double &m : phase_ms_) m = 0;
    timed_ops_ = 0;
  }
  /*! \brief fold the last timed op into the phase totals (call after the stream drained) */
  void CollectTiming();
  static constexpr int kPhases = 5;  // stage copy, barrier, reduce, barrier, gather
  const double *phase_ms() const { return phase_ms_; }
  uint64_t timed_ops() const { return timed_ops_; }
  void set_deadline_sec(double sec) {
    deadline_ticks_ = static_cast<long long>(std::max(sec, 0.1) * clock_khz_ * 1000.0);
  }

 private:
  hipError_t Barrier(const ResolveArgs *resolve = nullptr);
  hipError_t AllreduceImpl(const void *send, void *recv, void *recv2, size_t count, size_t tn,
                           int dtype, int prep, double alpha, const ReduceStep &step,
                           bool indirect, bool op_is_sum = false, int builtin_op = -1);
  /*! \brief the pipelined push form of AllreduceImpl (ar_plan.h) */
  hipError_t AllreducePipelined(const char *in, char *out, char *out2, size_t count, size_t tn,
                                double post, const ReduceStep &step);
  /*! \brief mock_die_mid: wait for the stream, then leave the process (see ArmDieMidOp) */
  void DieMidOp();
  /*! \brief true if [p, p + bytes) lies in this rank's symmetric heap */
  bool InHeap(const void *p, size_t bytes) const {
    const char *c = static_cast<const char *>(p);
    return heap_.base != nullptr && c >= heap_.base && c + bytes <= heap_.base + heap_.bytes;
  }
  char *stage(int rank, int which) const;
  /*! \brief fused flag block of `rank` for stage parity `which` */
  unsigned long long *fused_flags(int rank, int which) const {
    return reinterpret_cast<unsigned long long *>(peer_base_[rank] + kPeerFlagBytes +
                                                  static_cast<size_t>(which) * fused_block_bytes_);
  }
  int *dev_status() const { return reinterpret_cast<int *>(base_ + kPeerStatusOffset); }
  int *peer_abort() const { return reinterpret_cast<int *>(base_ + kPeerAbortOffset); }
  unsigned int *done_count() const {
    return reinterpret_cast<unsigned int *>(base_ + kPeerStatusOffset + 256);
  }
  unsigned long long *barrier_counter() const {
    return reinterpret_cast<unsigned long long *>(base_ + kPeerStatusOffset + 512);
  }
  unsigned long long *done_word() const {
    return reinterpret_cast<unsigned long long *>(host_words_ + 8);  // bytes 32..39
  }
  void NewBatch(CopyBatch *b) const {
    b->n = 0;
    b->guard = dev_status();
    b->remote = 0;
    b->done_count = nullptr;
    b->done_word = nullptr;
    b->epoch = 0;
  }

  int device_;
  size_t stage_bytes_;
  hipStream_t stream_;
  long long deadline_ticks_{0};
  int clock_khz_{100000};
  char *base_{nullptr};                 // local allocation
  std::vector<char *> peer_base_;       // mapped allocations (own = base_)
  SymHeapInfo heap_;                    // own symmetric heap (not owned)
  std::vector<char *> peer_heap_;       // mapped heaps (own = heap_.base), nullptr if none
  const void **table_{nullptr};         // device table of resolved reduce sources
  int *host_words_{nullptr};            // pinned: [0] abort, [1] status
  bool peer_abort_{false};              // rabit_device_peer_abort
  int n_{0}, rank_{0};
  unsigned long long epoch_{0};
  int parity_{0};
  PeerRecord local_{};
  bool opened_{false};
  bool timing_{false}, timing_pending_{false};
  hipEvent_t ev_[kPhases + 1]{};
  double phase_ms_[kPhases]{};
  uint64_t timed_ops_{0};
  uint64_t zero_copy_chunks_{0};
  uint64_t reg_zero_copy_chunks_{0};
  PeerRegistry registry_;
  bool registry_ok_{false};
  size_t zero_copy_min_{1u << 20};
  bool no_registry_{false};  // set while an op is captured into a hipGraph
  uint64_t op_seq_{0};       // AllreduceImpl calls (every rank of the group counts alike)
  size_t oneshot_max_{256u << 10};
  uint64_t oneshot_ops_{0};
  bool push_{false};
  uint64_t push_chunks_{0};
  bool pipeline_{false};
  size_t pipeline_chunk_{0};
  uint64_t pipelined_ops_{0}, pipelined_rounds_{0};
  uint64_t graphable_ops_{0};
  bool die_mid_{false};
  bool defer_second_{true};
  bool fused_{true};
  size_t fused_oneshot_max_{64u << 10};
  uint64_t fused_oneshots_{0};
  int fused_grid_req_{0}, fused_grid_{256}, gpu_share_{1};
  size_t fused_min_bytes_{0};
  int tiles_cap_{0};                // flag slots per array of a fused flag block
  size_t fused_block_bytes_{0};     // bytes of one fused flag block (2 per allocation)
  unsigned long long fused_epoch_{0};
  uint64_t fused_chunks_{0};
  bool done_signal_{true};
  size_t bcast_chunk_{0};
  uint64_t bcast_ops_{0}, bcast_chunks_{0};
  uint64_t resolved_allgathers_{0};
  unsigned long long *meta_table_{nullptr};  // device: 2 kMaxPeers words
  bool done_pending_{false};
  unsigned long long done_epoch_{0};
};

}  // namespace device
}  // namespace rabit
#endif  // XRABIT_DEVICE_PEER_COLL_H_
