/*!
 * \file device_plane.h
 * \brief Device data plane: RCCL over xGMI + gfx950 kernels for HBM buffers.
 *
 * MI355X design:
 *  - one process per GPU, one RCCL communicator per engine; the ncclUniqueId travels over the
 *    host control plane (the engine broadcasts it on the TCP tree), and a new communicator
 *    (new epoch) is built after every recovery;
 *  - built-in Sum/Max/Min go to ncclAllReduce; ops RCCL lacks (BitOR) use
 *    all-to-all + our multi-source reduce kernel + allgather (bandwidth-optimal, all 7 links);
 *  - rabit's variable, wrapping Allgather slices become a group of ncclBroadcast calls;
 *  - collectives run on a private non-blocking stream ordered after the caller's stream by
 *    events; the host waits on completion while probing for peer failure (TCP hang-up) and
 *    RCCL async errors, and aborts the communicator (ncclCommAbort) so a dead peer can never
 *    wedge the process.
 */
#ifndef XRABIT_DEVICE_DEVICE_PLANE_H_
#define XRABIT_DEVICE_DEVICE_PLANE_H_

#include <hip/hip_runtime_api.h>
#include <rccl/rccl.h>

#include <functional>
#include <memory>
#include <string>
#include <vector>

#include "device/p2p_plan.h"
#include "device/host_stager.h"
#include "device/peer_coll.h"
#include "net/socket.h"

namespace rabit {
namespace device {

using net::Status;

/*! \brief returns true when a peer failure was detected (checked while waiting) */
typedef std::function<bool()> FailureProbe;

struct DeviceConfig {
  int device{-1};                      // -1: LOCAL_RANK env, else rank % device count
  bool sync{true};                     // host waits for each collective to complete
  double op_timeout_sec{-1};           // deadline of a device op: < 0 auto (size-scaled), 0 none
  double drain_timeout_sec{30};        // after an abort, the stream must drain within this
  size_t arena_chunk{256u << 20};      // result-log arena growth step
  size_t arena_reserve{0};             // first result-log chunk (0: arena_chunk)
  size_t arena_cap{size_t(64) << 30};  // HBM result-log cap; beyond it (or when hipMalloc fails)
                                       // results spill to pinned host memory
  size_t spill_cap{size_t(1) << 40};   // pinned host bytes the result log may spill (0: no spill,
                                       // a full HBM log is then an error)
  int spin_us{5000};                   // busy-poll window before sleeping while waiting
  int algo{0};                         // 0 auto, 1 RCCL only, 2 direct (IPC peer memory) only
  size_t peer_stage{256u << 20};       // direct transport: bytes per stage buffer (x2 per rank)
  double peer_deadline_sec{120};       // direct transport: barrier gives up after this long
  size_t direct_min_bytes{1u << 20};   // auto: ops of at least this size use the direct path
  bool phase_timing{false};            // direct transport: hipEvent timing of each phase
  bool ops_on_user_stream{true};       // enqueue collectives on the caller's stream
  size_t sym_heap{0};                  // bytes of the symmetric (IPC-exported) heap, 0: none
  size_t oneshot_max{256u << 10};      // direct allreduce: one-shot up to this many bytes
  int direct_mode{0};                  // direct reduce-scatter: 0 calibrated, 1 pull, 2 push
  int fused_mode{0};                   // direct two-shot chunks as one fused kernel: 0 never
                                       // (default: the 5-launch form measured faster from
                                       // 1 MiB up, profiles/r3_fused_vs_classic), 1 always,
                                       // 2 as the calibration finds faster
  int fused_grid{0};                   // workgroups of a fused launch (0: automatic)
  size_t fused_oneshot_max{64u << 10}; // one-shot direct ops up to this size as one fused
                                       // launch (0: never; above it the 3-launch form)
  size_t fused_min_bytes{0};           // chunks below this keep the classic 5-launch form
  size_t calib_big{128u << 20};        // large calibration point (bytes, at most a stage)
  size_t bcast_chunk{0};               // direct broadcast pipeline chunk (0: sqrt(S x 4 MiB))
  int pipeline_mode{2};                // direct two-shot as the pipelined push form (ar_plan.h):
                                       // 0 never, 1 always (with push), 2 as the calibration
                                       // finds faster
  size_t pipeline_chunk{0};            // its chunk in bytes (0: ArPipeline::AutoChunk)
  size_t zero_copy_min{1u << 20};      // direct pull two-shot: ordinary HBM inputs of at least
                                       // this size are IPC-registered and read in place by the
                                       // peers (peer_registry.h); 0: never
  bool defer_second{true};             // multi-chunk ops: the second destination only after
                                       // the last barrier (0: test knob, the old behaviour)
  // host-buffer allreduce staged through HBM (rabit_host_via_device): pipelined in chunks of
  // this size through pinned slots (host_stager.h), or one whole copy each way (0)
  size_t host_stage_chunk{16u << 20};
  int host_stage_threads{0};           // memcpy threads of the staging (0: host share /
                                       // local ranks)
  int host_stage_streams{3};           // 3: H2D / collective / D2H on separate streams; 1: all on
                                       // the plane stream
  int rccl_min_ctas{0};                // ncclConfig_t minCTAs / maxCTAs (0: RCCL's choice)
  int rccl_max_ctas{0};
  // RCCL communicator lifecycle: the bring-up (init and the connection
  // of every channel) runs on a helper thread watched by the failure probe and a deadline, so
  // a peer that dies mid-init costs kAborted / kTimeout instead of a hang (see InitComm)
  double comm_init_timeout_sec{120};   // deadline of communicator bring-up (0: none)
  bool peer_abort{true};               // an abort raises the peers' abort words too
                                       // (rabit_device_peer_abort, PeerGroup::SignalAbort)
  bool done_word{true};                // small direct ops: poll a kernel-written host word for
                                       // completion instead of an event
  int rccl_max_failures{8};            // consecutive aborted RCCL ops before the error is fatal
  size_t rccl_warm_bytes{128u << 20};  // largest allreduce of the bring-up's warm-up (64 KiB,
                                       // 4 MiB and this size connect RCCL's algorithm paths)
  int mock_rccl_error{0};              // test hook: the n-th RCCL enqueue (1-based) fails with
                                       // ncclRemoteError instead of running
};

/*! \brief exit status of a rank whose own device stream stayed wedged after an abort (the
 *  launcher restarts it; its peers recover as from a crash) */
constexpr int kDeviceHangExitCode = 251;
/*! \brief auto deadline of a device op of this many bytes: 60 s plus 1 s per GB */
inline double AutoOpDeadline(size_t bytes) { return 60.0 + static_cast<double>(bytes) * 1e-9; }

/*! \brief HBM arena for the robust engine's result log and checkpoints (bump allocator over
 *  chunks; Reset() keeps the chunks so steady-state iterations never call hipMalloc).  A pinned
 *  arena holds page-locked host memory instead (the result log's spill space past its HBM cap) */
class DeviceArena {
 public:
  ~DeviceArena();
  /*! \brief chunk: smallest growth step; reserve: size of the first chunk (one allocation up
   *  front instead of many during the first iterations); HBM arenas then grow geometrically
   *  (each new chunk as large as everything reserved so far, at most kMaxStep), so a long
   *  stretch between checkpoints costs O(log) hipMallocs, not one per chunk */
  void Configure(size_t chunk, size_t cap, bool pinned = false, size_t reserve = 0) {
    chunk_ = chunk;
    cap_ = cap;
    pinned_ = pinned;
    reserve_ = reserve;
  }
  static constexpr size_t kMaxStep = size_t(8) << 30;
  bool pinned() const { return pinned_; }
  /*! \brief 256-byte aligned slot, nullptr when over the cap or out of memory */
  void *Alloc(size_t bytes);
  /*! \brief give back the most recent allocation (ResultLog::DropLast) */
  void PopTo(void *ptr);
  void Reset();
  size_t used() const;
  size_t reserved() const;

 private:
  struct Chunk {
    char *base;
    size_t size, used;
  };
  std::vector<Chunk> chunks_;
  size_t cur_{0};
  size_t chunk_{256u << 20}, cap_{size_t(64) << 30}, reserve_{0};
  bool pinned_{false};
};

/*!
 * \brief makes `device` current for a scope (allocations and launches of the plane go to its
 *        GPU even if the calling thread switched devices in between), then restores it
 */
class DeviceGuard {
 public:
  explicit DeviceGuard(int device) {
    if (device < 0) return;
    int cur = -1;
    if (hipGetDevice(&cur) == hipSuccess && cur != device && hipSetDevice(device) == hipSuccess) {
      prev_ = cur;
    }
  }
  ~DeviceGuard() {
    if (prev_ >= 0) (void)hipSetDevice(prev_);
  }
  DeviceGuard(const DeviceGuard &) = delete;
  DeviceGuard &operator=(const DeviceGuard &) = delete;

 private:
  int prev_{-1};
};

class DevicePlane {
 public:
  /*!
   * \brief process-wide RCCL settings the plane relies on, applied before any thread starts
   *        (setenv is not safe against concurrent getenv): NCCL_RUNTIME_CONNECT=0 makes RCCL
   *        connect its collective channels inside communicator init (InitComm's helper thread,
   *        watched by the failure probe) instead of lazily inside the first collective that needs
   *        them, where a dead peer would block the enqueueing thread with no deadline.  This is a
   *        side effect on every RCCL user of the process (torch.distributed included): their
   *        communicators connect eagerly too.  A value the user set wins.
   */
  static void ConfigureRcclEnv();
  /*! \brief number of visible GPUs (0 when HIP has no device) */
  static int DeviceCount();
  DevicePlane(const DeviceConfig &cfg, int rank_hint);
  ~DevicePlane();

  int device() const { return device_; }
  bool IsDevicePtr(const void *p) const;
  /*!
   * \brief the caller's stream.  With ops_on_user_stream (default) collectives are enqueued on
   *        it directly — no cross-stream events per op; a change of stream is ordered after the
   *        previous one, so collectives stay in issue order on the GPU.
   */
  void SetUserStream(hipStream_t s);
  hipStream_t stream() const { return stream_; }
  DeviceArena *arena() { return &arena_; }
  /*! \brief pinned host arena the result log spills to (nullptr: spilling disabled) */
  DeviceArena *spill_arena() { return cfg_.spill_cap != 0 ? &spill_ : nullptr; }
  /*! \brief scratch slot staging spilled results (HBM side of the D2H / H2D copies) */
  static constexpr int kSpillScratch = 3;
  /*! \brief scratch slot of the calibration's second destination */
  static constexpr int kCalibScratch = 4;
  const DeviceConfig &config() const { return cfg_; }

  // ---- communicator lifecycle
  /*! \brief serialized ncclUniqueId (NCCL_UNIQUE_ID_BYTES bytes) */
  static std::string NewUniqueId();
  /*!
   * \brief collective over all ranks: build the communicator of a new epoch and connect all
   *        its channels, on a helper thread, while this thread watches `probe` and
   *        comm_init_timeout_sec: a rank that never joins (or dies during the bring-up) costs the
   *        others kAborted / kTimeout, not a hang.
   */
  Status InitComm(const std::string &id, int nranks, int rank, const FailureProbe &probe);
  /*! \brief abort the communicator and the peer group (unblocks in-flight kernels), drop them */
  void AbortComm();
  /*! \brief drop the RCCL communicator alone (no op in flight on it), keep the peer group */
  void DropComm();
  bool has_comm() const { return comm_ != nullptr; }
  bool has_peers() const { return peers_ != nullptr; }
  /*! \brief a transport for world > 1 is up */
  bool ready() const { return comm_ != nullptr || peers_ != nullptr; }
  int epoch() const { return epoch_; }
  /*! \brief count a new communicator epoch (after InitComm and/or OpenPeers) */
  void BeginEpoch(int nranks, int rank) {
    nranks_ = nranks;
    rank_ = rank;
    ++epoch_;
  }

  // ---- peer preflight (before the direct transport maps anything)
  /*! \brief what this rank found out about the link to one peer */
  struct PeerLinkInfo {
    int rank{-1};
    int ordinal{-1};      // the peer's GPU as this process numbers it (-1: not visible)
    int can_access{-1};   // hipDeviceCanAccessPeer (-1: not checked)
    int link_type{-1};    // hipExtGetLinkTypeAndHopCount: 4 = xGMI, 2 = PCIe (-1: unknown)
    int hops{-1};
    bool same_gpu{false};
  };
  /*!
   * \brief map every peer's GPU (by PCI bus id) to a local ordinal, check peer access and the
   *        link type; false (with why) if a visible peer GPU cannot be accessed, in which case
   *        the direct transport must stay off (RCCL only)
   */
  bool Preflight(const std::vector<PeerRecord> &all, int rank, std::string *why);
  const std::vector<PeerLinkInfo> &peer_links() const { return links_; }
  /*! \brief links_ as a JSON array */
  std::string PeerLinksJson() const;

  // ---- direct transport (IPC peer memory over xGMI)
  /*! \brief allocate and export the local stage buffers; false (with why) if impossible */
  bool PreparePeers(PeerRecord *rec, std::string *why);
  /*! \brief map every rank's buffers (records in rank order) */
  bool OpenPeers(const std::vector<PeerRecord> &all, int rank, std::string *why);
  void DropPeers();
  /*! \brief route an op of this many bytes over the direct transport */
  bool UseDirect(size_t bytes) const {
    if (peers_ == nullptr) return false;
    if (force_ >= 0) return force_ == 1;
    if (comm_ == nullptr || cfg_.algo == 2) return true;
    if (!transport_bands_.empty()) return BandAt(transport_bands_, bytes).direct != 0;
    return bytes >= cfg_.direct_min_bytes || bytes < direct_below_bytes_;
  }
  /*! \brief what the calibration chose for one band of op sizes: the transport, and the form of
   *  the direct two-shot path */
  struct RouteChoice {
    size_t lo;  // ops of at least lo bytes (up to the next band)
    int8_t direct, push, pipeline, fused;
  };
  /*!
   * \brief the calibrated piecewise routing (engine/routing.h): transport bands (direct or
   *        RCCL per size) and form bands (the fastest direct form per size, used whenever an op
   *        goes direct).  Empty vectors: the two-threshold routing and one fixed form.  Clears
   *        a forced form.
   */
  void SetRoutes(const std::vector<RouteChoice> &transport, const std::vector<RouteChoice> &form) {
    transport_bands_ = transport;
    form_bands_ = form;
    form_forced_ = false;
  }
  const std::vector<RouteChoice> &transport_bands() const { return transport_bands_; }
  const std::vector<RouteChoice> &form_bands() const { return form_bands_; }
  /*! \brief back to the calibrated transport and form (undo ForceTransport / forced forms) */
  void RestoreCalibrated() {
    force_ = -1;
    form_forced_ = false;
    if (peers_ != nullptr && form_bands_.empty()) {
      peers_->set_push(default_form_.push != 0);
      peers_->set_pipeline(default_form_.pipeline != 0);
      peers_->set_fused(default_form_.fused != 0);
    }
  }
  const RouteChoice &default_form() const { return default_form_; }
  /*! \brief the form used when no form bands exist (the configured or calibrated one) */
  void SetDefaultForm(bool push, bool pipeline, bool fused) {
    default_form_ = RouteChoice{0, 1, static_cast<int8_t>(push), static_cast<int8_t>(pipeline),
                                static_cast<int8_t>(fused)};
  }
  /*! \brief route a broadcast of this many bytes over the direct transport: by its own
   *  calibration once that ran (a broadcast moves each byte once per link, an allreduce twice,
   *  so the crossover differs), by the allreduce routing before */
  bool UseDirectBcast(size_t bytes) const {
    if (peers_ == nullptr) return false;
    if (force_ >= 0 || !bcast_routed_ || comm_ == nullptr || cfg_.algo == 2) {
      return UseDirect(bytes);
    }
    return bytes >= bcast_min_bytes_ || bytes < bcast_below_bytes_;
  }
  void set_bcast_routing(size_t min_bytes, size_t below_bytes) {
    bcast_routed_ = true;
    bcast_min_bytes_ = min_bytes;
    bcast_below_bytes_ = below_bytes;
  }
  bool bcast_routed() const { return bcast_routed_; }
  size_t bcast_min_bytes() const { return bcast_min_bytes_; }
  size_t bcast_below_bytes() const { return bcast_below_bytes_; }
  uint64_t bcast_ops() const { return peers_ ? peers_->bcast_ops() : 0; }
  uint64_t bcast_chunks() const { return peers_ ? peers_->bcast_chunks() : 0; }
  void set_direct_min_bytes(size_t b) { cfg_.direct_min_bytes = b; }
  /*! \brief ops below this size go direct too (the calibration found the direct transport
   *  faster for small ops and RCCL for large ones) */
  void set_direct_below_bytes(size_t b) { direct_below_bytes_ = b; }
  size_t direct_below_bytes() const { return direct_below_bytes_; }
  size_t direct_min_bytes() const { return cfg_.direct_min_bytes; }
  /*! \brief calibration: -1 normal routing, 0 force RCCL, 1 force direct */
  void ForceTransport(int which) { force_ = which; }
  /*! \brief channel (CTA) bounds of the next communicator (0: RCCL's choice) */
  void set_rccl_ctas(int min_ctas, int max_ctas) {
    cfg_.rccl_min_ctas = min_ctas;
    cfg_.rccl_max_ctas = max_ctas;
  }
  int rccl_min_ctas() const { return cfg_.rccl_min_ctas; }
  /*! \brief direct reduce-scatter by remote writes (push) instead of remote reads */
  void SetDirectPush(bool v) {
    form_forced_ = true;
    if (peers_ != nullptr) peers_->set_push(v);
  }
  bool direct_push() const { return peers_ != nullptr && peers_->push(); }
  uint64_t push_chunks() const { return peers_ ? peers_->push_chunks() : 0; }
  /*! \brief direct two-shot allreduces as the pipelined push form (with SetDirectPush(true)) */
  void SetPipeline(bool v) {
    form_forced_ = true;
    if (peers_ != nullptr) peers_->set_pipeline(v);
  }
  bool pipeline() const { return peers_ != nullptr && peers_->pipeline(); }
  uint64_t pipelined_ops() const { return peers_ ? peers_->pipelined_ops() : 0; }
  uint64_t pipelined_rounds() const { return peers_ ? peers_->pipelined_rounds() : 0; }
  /*!
   * \brief xGMI link probe over the direct transport (PeerGroup::LinkProbe; a collective
   *        outside the fault-tolerance log, every rank calls it between the same ops).  GB/s of
   *        this rank: one link read / write, all links read / write, all links both ways.  A
   *        failed barrier aborts the group (the next op rebuilds it) and returns kAborted.
   */
  Status LinkProbe(size_t bytes, double out[PeerGroup::kLinkProbeValues]);
  /*! \brief test hook (mock_die_mid): the next multi-chunk direct allreduce exits mid-op */
  void ArmDieMidOp() {
    if (peers_ != nullptr) peers_->ArmDieMidOp();
  }
  /*! \brief barrier deadline of the direct transport (calibration runs with a short one) */
  void SetPeerDeadline(double sec) {
    if (peers_ != nullptr) peers_->set_deadline_sec(sec);
  }
  /*! \brief average per-phase time (us) of timed direct allreduces; false if none */
  bool DirectPhaseUs(double out[PeerGroup::kPhases], uint64_t *nops) const;
  /*!
   * \brief allocate from the symmetric heap: HBM that peers map through IPC, so the direct
   *        transport reads an allreduce input there in place (no stage copy).  nullptr when
   *        the heap is disabled (rabit_device_symmetric_heap=0) or full.  Bump allocation,
   *        freed with the engine.
   */
  void *SymAlloc(size_t bytes);
  const SymHeapInfo &sym_heap() const { return heap_; }
  size_t sym_heap_used() const { return heap_used_; }
  uint64_t zero_copy_chunks() const { return peers_ ? peers_->zero_copy_chunks() : 0; }
  uint64_t reg_zero_copy_chunks() const { return peers_ ? peers_->reg_zero_copy_chunks() : 0; }
  /*! \brief ordinary inputs of at least this size are registered for zero copy (0: never) */
  void SetZeroCopyMin(size_t b) {
    cfg_.zero_copy_min = b;
    if (peers_ != nullptr) peers_->set_zero_copy_min(b);
  }
  /*! \brief zero-copy registry counters as JSON ({} without a peer group) */
  std::string RegistryJson() const;
  /*! \brief every rank opened the group: drop the names of the shared registry pages */
  void SealPeers() {
    if (peers_ != nullptr) peers_->SealRegistry();
  }
  uint64_t oneshot_ops() const { return peers_ ? peers_->oneshot_ops() : 0; }
  uint64_t fused_chunks() const { return peers_ ? peers_->fused_chunks() : 0; }
  uint64_t fused_oneshots() const { return peers_ ? peers_->fused_oneshots() : 0; }
  void SetFused(bool v) {
    form_forced_ = true;
    if (peers_ != nullptr) peers_->set_fused(v);
  }
  bool fused() const { return peers_ != nullptr && peers_->fused(); }
  /*! \brief hipEvent timing of the classic direct form's phases from now on (fresh totals),
   *  or off; false without a peer group */
  bool SetPhaseTiming(bool on) {
    if (peers_ == nullptr) return false;
    if (on) {
      peers_->EnableTiming();
      peers_->ResetTiming();
    } else {
      peers_->DisableTiming();
    }
    return true;
  }
  int fused_grid() const { return peers_ ? peers_->fused_grid() : 0; }
  /*! \brief ranks of the direct group share a GPU (a rehearsal or test setup) */
  bool peers_share_gpu() const { return peers_ && peers_->gpu_share() > 1; }
  /*! \brief fill PeerRecord host/pci fields only (ranks without a peer group) */
  void DescribeDevice(PeerRecord *rec) const;

  // ---- collectives (enqueue then wait)
  /*!
   * \brief recv = reduce(prep(send)) over ranks, also stored to recv2 when given; send may equal
   *        recv.  prep is a PrepOp (kPrepCopy: none).  recv2 is written only when the op
   *        succeeds on this rank, so a retry still finds the input.
   */
  /*!
   * \brief in-place allreduce enqueued on `stream` and nothing else: no host wait, no event,
   *        no result log, so it may be captured into a hipGraph.  RCCL, or the direct
   *        transport's classic form with device-numbered barriers (PeerGroup::
   *        AllreduceGraphable) when the routing sends ops of this size there or RCCL is not up.
   *        Outside fault tolerance (non-robust engines only).  0 on success, -2 without a
   *        transport, -3 for a dtype/op the path lacks (BitOR), -5 when the enqueue fails.
   */
  int GraphAllreduce(void *buf, size_t count, int dtype, int op, hipStream_t stream);
  /*! \brief graphable allreduces that went over the direct transport */
  uint64_t graph_direct_ops() const { return graph_direct_ops_; }
  Status Allreduce(const void *send, void *recv, void *recv2, size_t count, int dtype, int op,
                   int prep, double alpha, const FailureProbe &probe);
  /*! \brief launcher of a user device reduction (IEngine::DeviceReduceLauncher) */
  typedef int(DeviceReduceLauncher)(void *dst, const void *const *srcs, int nsrc, size_t count,
                                    const int *guard, void *stream);
  /*! \brief allreduce of count elements of type_nbytes with a user device reduction */
  Status AllreduceCustom(const void *send, void *recv, void *recv2, size_t count,
                         size_t type_nbytes, DeviceReduceLauncher *launcher,
                         const FailureProbe &probe);
  /*! \brief in-place broadcast; log != nullptr: the result is also stored there once the op
   *  succeeded (the direct transport's kernels store it in the same pass, RCCL by a copy that
   *  Finish enqueues) */
  Status Broadcast(void *buf, size_t bytes, int root, const FailureProbe &probe,
                   void *log = nullptr);
  /*! \brief rabit Allgather: slice r = [begin[r], begin[r]+size[r]) mod total, in place
   *  (log: as for Broadcast) */
  Status AllgatherV(void *buf, size_t total, const std::vector<size_t> &begin,
                    const std::vector<size_t> &size, const FailureProbe &probe,
                    void *log = nullptr);
  /*! \brief true when an allgather of this size needs every rank's slice on the host first
   *  (RCCL's grouped broadcasts); the direct transport resolves the layout on the device */
  bool AllgatherNeedsLayout(size_t total) const { return !UseDirect(total); }
  /*! \brief rabit Allgather knowing only this rank's slice (direct transport only: see
   *  AllgatherNeedsLayout) */
  Status AllgatherResolved(void *buf, size_t total, size_t begin, size_t size,
                           void *log = nullptr);
  uint64_t resolved_allgathers() const { return peers_ ? peers_->resolved_allgathers() : 0; }
  /*!
   * \brief point-to-point copies over xGMI (see ExchangeItem; every rank passes the same plan).
   *        With RCCL: one grouped ncclSend/ncclRecv call on the ranks that take part (the others
   *        do nothing); otherwise the direct transport's stage exchange.  Enqueue only: the
   *        caller waits with Finish().  *bytes_in: payload bytes this rank received from peers.
   */
  Status Exchange(const std::vector<ExchangeItem> &plan, size_t *bytes_in,
                  const FailureProbe &probe = FailureProbe());
  /*! \brief reusable page-locked host buffer of at least bytes (grows, never shrinks): the
   *  staging area of device ops whose reduction runs on the host (user reducers) */
  void *PinnedScratch(size_t bytes);
  /*! \brief stage a host-reducer allreduce through pinned host memory */
  void StageToHost(void *host, const void *dev, size_t bytes);
  void StageToDevice(void *dev, const void *host, size_t bytes);
  /*!
   * \brief collective: host_out = allreduce(host_in) of host memory through HBM, pipelined
   *        (H2D of chunk k+1, the device allreduce of chunk k and the D2H of chunk k-1 overlap;
   *        multi-threaded copies between pageable and pinned memory).  Returns like a device
   *        allreduce followed by Finish.
   */
  Status AllreduceHostStaged(void *host_out, const void *host_in, size_t count, int dtype, int op,
                             const FailureProbe &probe);
  uint64_t host_staged_ops() const { return host_staged_ops_; }
  /*! \brief create the staging pipeline (pinned slots, copy threads, streams) ahead of use */
  void PrepareHostStager();
  int host_stage_threads() const { return stager_ ? stager_->threads() : 0; }
  /*! \brief the staging's time split as JSON (ms over all staged ops; {} before the first) */
  std::string HostStageJson() const;
  /*! \brief ranks of the job on this host (sizes the staging's thread pool) */
  void set_local_ranks(int n) { local_ranks_ = n; }

  // ---- device failure handling
  /*!
   * \brief fault injection (mock_dev_hang): enqueue a kernel that wedges this stream (it ignores
   *        aborts) for at most max_sec; the collective queued behind it never starts
   */
  void InjectHang(double max_sec);
  /*! \brief end an injected hang (also called from the watchdog thread) */
  static void ReleaseHang();
  /*! \brief poll until the plane stream is idle; false after sec seconds */
  bool DrainStream(double sec);
  /*!
   * \brief this rank's own device work does not finish even after the communicators were
   *        aborted: end the process with kDeviceHangExitCode for a restart (the peers see the
   *        links drop and recover as from a crash).  Injected hangs are released first so that
   *        no wave outlives the process.
   */
  [[noreturn]] static void WedgedExit(const char *why);
  /*! \brief bytes of the op being waited for (auto deadline) */
  void set_op_bytes(size_t b) { op_bytes_ = b; }

  // ---- memory / ordering
  /*! \brief async copy on the plane stream (any memory kinds) */
  void CopyAsync(void *dst, const void *src, size_t bytes);
  /*! \brief async HBM-to-HBM copy with the gfx950 copy kernel */
  void CopyDeviceAsync(void *dst, const void *src, size_t bytes);
  /*! \brief order the plane stream after the user stream */
  void EnterFromUser();
  /*! \brief record completion, order the user stream after it, host-wait if sync */
  Status Finish(const FailureProbe &probe, bool host_wait = true);
  /*! \brief block until the plane stream is idle */
  void Synchronize();
  /*! \brief reusable scratch buffer of at least bytes */
  void *Scratch(size_t bytes, int slot = 0);

  /*! \brief RCCL enqueue calls made so far, and the ones that returned ncclInProgress and were
   *  settled by polling (non-blocking communicator) */
  uint64_t rccl_calls() const { return rccl_calls_; }
  uint64_t rccl_settled() const { return rccl_settled_; }
  /*! \brief RCCL results turned into kAborted / kTimeout (the engine recovered) */
  uint64_t rccl_aborts() const { return rccl_aborts_; }
  /*! \brief communicator bring-ups given up while RCCL's bootstrap still waited on a peer */
  uint64_t init_abandoned() const { return init_abandoned_; }
  /*! \brief multi-rank bring-ups refused because kMaxAbandonedInits helpers were still live */
  uint64_t init_refused() const { return init_refused_; }
  /*! \brief abandoned bring-up helpers of this process still blocked in RCCL */
  static int LiveAbandonedInits();
  /*! \brief at most this many abandoned bring-up helpers may be live at once */
  static constexpr int kMaxAbandonedInits = 2;
  /*! \brief ops whose completion was read from a kernel-written host word */
  uint64_t done_words() const { return done_words_; }

 private:
  Status WaitEvent(hipEvent_t ev, const FailureProbe &probe);
  /*! \brief wait (bounded by drain_timeout_sec) for a bring-up's warm-up stream to go idle */
  void DrainBringUp(hipStream_t s);
  /*! \brief wait until a kernel stored `epoch` (or more) into the pinned host word */
  Status WaitWord(const volatile unsigned long long *word, unsigned long long epoch,
                  const FailureProbe &probe);
  /*! \brief the completion wait: poll() returns hipSuccess / hipErrorNotReady / an error;
   *  meanwhile RCCL async errors, the failure probe and the op deadline are watched */
  template <typename Poll>
  Status WaitUntil(const Poll &poll, const FailureProbe &probe);
  /*!
   * \brief map an RCCL return code to a Status: success; ncclInProgress (non-blocking
   *        communicator) is polled to completion under the probe and the op deadline; a result a
   *        dead peer can cause aborts the communicator and returns kAborted (the engine
   *        recovers); a usage error is fatal
   */
  Status Rccl(int result, const char *what, const FailureProbe &probe);
  /*! \brief poll ncclCommGetAsyncError until the communicator leaves ncclInProgress; abort it on
   *  an error, a peer failure or after limit_sec (> 0) */
  Status Settle(const char *what, const FailureProbe &probe, double limit_sec);
  /*! \brief abort the communicator after a failed RCCL call (kAborted), or throw if the call
   *  cannot have failed because of a peer */
  Status FailRccl(const char *what, int result);
  /*! \brief count one RCCL enqueue; true when the mock_rccl_error hook makes it fail */
  bool MockRcclFault();
  /*! \brief one grouped ncclSend / ncclRecv call over ops (pointers from at(i, op)) */
  Status RunP2P(const std::vector<P2POp> &ops,
                const std::function<char *(size_t, const P2POp &)> &at,
                const char *what, const FailureProbe &probe);
  /*! \brief one reduce pass of the kernel-reduced allreduce: dst = reduce(srcs) over count
   *  elements; acc_first: srcs[0] is the running result of an earlier pass (not prepared) */
  typedef std::function<hipError_t(void *dst, const void *const *srcs, int nsrc, size_t count,
                                   bool acc_first, hipStream_t stream)>
      PassFn;
  /*! \brief RCCL allreduce for what ncclAllReduce cannot do (BitOR, custom and prepared
   *  reductions): grouped p2p reduce-scatter (SegmentPlan), `pass`, grouped p2p allgather */
  Status AllreduceByKernel(const void *send, void *recv, size_t count, size_t type_nbytes,
                           const PassFn &pass, const FailureProbe &probe);

  static const RouteChoice &BandAt(const std::vector<RouteChoice> &bands, size_t bytes) {
    size_t i = 0;
    while (i + 1 < bands.size() && bytes >= bands[i + 1].lo) ++i;
    return bands[i];
  }
  /*! \brief a direct op of this size is about to run: its calibrated form, unless forced */
  void ApplyForm(size_t bytes) {
    if (form_forced_ || form_bands_.empty() || peers_ == nullptr) return;
    const RouteChoice &c = BandAt(form_bands_, bytes);
    peers_->set_push(c.push != 0);
    peers_->set_pipeline(c.pipeline != 0);
    peers_->set_fused(c.fused != 0);
  }

  DeviceConfig cfg_;
  int device_{-1};
  std::vector<RouteChoice> transport_bands_, form_bands_;
  RouteChoice default_form_{0, 1, 0, 0, 0};
  bool form_forced_{false};
  hipStream_t stream_{nullptr};       // stream collectives are enqueued on
  hipStream_t own_stream_{nullptr};   // private non-blocking stream (ops_on_user_stream=false)
  hipStream_t user_stream_{nullptr};
  hipEvent_t ev_switch_{nullptr};
  hipEvent_t ev_in_{nullptr}, ev_done_{nullptr};
  ncclComm_t comm_{nullptr};
  int nranks_{0}, rank_{0}, epoch_{0};
  DeviceArena arena_;
  DeviceArena spill_;
  std::unique_ptr<PeerGroup> peers_;
  std::unique_ptr<HostStager> stager_;  // created by the first staged host allreduce
  uint64_t host_staged_ops_{0};
  int local_ranks_{0};
  int spin_us_override_{-1};  // >= 0: the busy-poll window of the current wait (host staging)
  SymHeapInfo heap_;
  size_t heap_used_{0};
  int force_{-1};
  size_t direct_below_bytes_{0};
  bool bcast_routed_{false};
  size_t bcast_min_bytes_{static_cast<size_t>(-1)}, bcast_below_bytes_{0};
  void *pending_dst_{nullptr};  // second destination of the last RCCL allreduce (see Finish)
  const void *pending_src_{nullptr};
  size_t pending_bytes_{0};
  // 0/1: all-to-all path (and calibration), 2: host-buffer staging, 3: spilled results,
  // 4: calibration second destination
  static constexpr int kScratchSlots = 5;
  void *scratch_[kScratchSlots]{};
  size_t scratch_bytes_[kScratchSlots]{};
  void *pinned_{nullptr};
  size_t pinned_bytes_{0};
  size_t op_bytes_{0};
  std::vector<PeerLinkInfo> links_;
  uint64_t rccl_calls_{0}, rccl_settled_{0}, rccl_aborts_{0}, init_abandoned_{0};
  uint64_t done_words_{0};
  uint64_t graph_direct_ops_{0};
  uint64_t init_refused_{0};
  int rccl_fail_streak_{0};  // aborted RCCL ops since the last op that completed
};

/*! \brief throw rabit::Error on a HIP failure */
void CheckHip(hipError_t e, const char *what);
}  // namespace device
}  // namespace rabit
#endif  // XRABIT_DEVICE_DEVICE_PLANE_H_
