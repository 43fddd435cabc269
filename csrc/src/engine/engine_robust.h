/*!
 * \file engine_robust.h
 * \brief Fault-tolerant engine: consensus, result log, checkpoints and replay recovery.
 *
 * Parity: reference AllreduceRobust (`src/allreduce_robust.{h,cc}`, `allreduce_robust-inl.h`).
 * Semantics kept: every collective is identified by (version, seqno); a restarted worker
 * reloads the last checkpoint from peers and replays the results of every collective since
 * then from the peers' result logs, without re-running its lazy prepare functions; survivors
 * block and serve it.  MI355X-specific design:
 *  - results of HBM collectives are logged in an HBM arena (no host round trip on the hot
 *    path); RCCL writes the result straight into its log slot (out-of-place), then one D2D
 *    copy lands it in the user buffer;
 *  - the per-op consensus round is elided in steady state (all ranks agreed on "execute" at
 *    the previous op and nobody has seen a failure since); any failure or special action
 *    (checkpoint, load, bootstrap cache) re-enables it, so the replay protocol is unchanged;
 *  - a real watchdog: on timeout it aborts the device communicator and the process instead
 *    of throwing into a discarded future (reference quirk).
 */
#ifndef XRABIT_ENGINE_ENGINE_ROBUST_H_
#define XRABIT_ENGINE_ENGINE_ROBUST_H_

#include <atomic>
#include <condition_variable>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "engine/engine_base.h"
#include "engine/local_replicas.h"

namespace rabit {
namespace engine {

class EngineRobust : public EngineBase {
 public:
  EngineRobust();
  ~EngineRobust() override;
  bool Init(int argc, char *argv[]) override;
  bool Shutdown() override;
  void SetParam(const char *name, const char *val) override;

  void Allgather(void *sendrecvbuf, size_t total_size, size_t slice_begin, size_t slice_end,
                 size_t size_prev_slice, const char *_file, const int _line,
                 const char *_caller) override;
  void Allreduce(void *sendrecvbuf_, size_t type_nbytes, size_t count, ReduceFunction reducer,
                 PreprocFunction prepare_fun, void *prepare_arg, const char *_file,
                 const int _line, const char *_caller) override;
  void AllreduceDevice(void *sendrecvbuf_, size_t type_nbytes, size_t count,
                       DeviceReduceLauncher *dev_reducer, ReduceFunction host_reducer,
                       PreprocFunction prepare_fun, void *prepare_arg, const char *_file,
                       const int _line, const char *_caller) override;
  void AllreduceTyped(void *sendrecvbuf_, size_t count, mpi::DataType dtype, mpi::OpType op,
                      ReduceFunction reducer, PreprocFunction prepare_fun, void *prepare_arg,
                      const char *_file, const int _line, const char *_caller) override;
  void Broadcast(void *sendrecvbuf_, size_t total_size, int root, const char *_file,
                 const int _line, const char *_caller) override;
  void InitAfterException() override;
  int LoadCheckPoint(Serializable *global_model, Serializable *local_model) override;
  void CheckPointDevice(const Serializable *global_model,
                        const Serializable *local_model) override {
    CheckPointImpl(global_model, local_model, true);
  }
  void CheckPoint(const Serializable *global_model, const Serializable *local_model) override {
    CheckPointImpl(global_model, local_model, false);
  }
  void LazyCheckPoint(const Serializable *global_model) override {
    CheckPointImpl(global_model, nullptr, true);
  }
  const char *EngineName() const override { return "robust"; }
  void DevAllreducePrepared(void *dst, const void *src, size_t count, int dtype, int op,
                            int prep, double alpha, const char *_file, const int _line,
                            const char *_caller) override;

  // ---- hooks used by unit tests (white-box)
  /*! \brief called when the watchdog expires (default: log and terminate the process) */
  typedef void (*TimeoutHandler)(int rank, int timeout_sec);
  void SetTimeoutHandler(TimeoutHandler h) { timeout_handler_ = h; }
  /*! \brief exit status of a rank that rabit_hang_timeout_sec found stuck inside an op */
  static constexpr int kHangExitCode = 252;
  /*! \brief feed CheckAndRecover directly (tests); returns its result */
  bool TestCheckAndRecover(Status s) { return CheckAndRecover(s); }
  bool watchdog_fired() const { return watchdog_fired_.load(); }
  bool consensus_elided() const { return fast_mode_; }

 protected:
  /*! \brief role of a node in a recovery transfer */
  enum RecoverType { kHaveData = 0, kRequestData = 1, kPassData = 2 };
  enum SeqType { kSeq = 0, kCache = 1 };

  /*!
   * \brief 8-byte consensus message (reference allreduce_robust.h:224-322):
   *   seqcode    = (min seqno << 5) | action flags
   *   maxseqcode = (max bootstrap-cache seqno << 5) | cache-role flag
   */
  struct ActionSummary {
    static constexpr uint32_t kSpecialOp = 1u << 26;
    static constexpr uint32_t kLocalCheckPoint = (1u << 26) - 2;
    static constexpr uint32_t kLocalCheckAck = (1u << 26) - 1;
    static constexpr int kLoadCheck = 1;
    static constexpr int kCheckPoint = 2;
    static constexpr int kCheckAck = 4;
    static constexpr int kDiffSeq = 8;
    static constexpr int kLoadBootstrapCache = 16;
    uint32_t seqcode{0}, maxseqcode{0};
    ActionSummary() = default;
    ActionSummary(int flag, int cache_flag, uint32_t minseqno = kSpecialOp,
                  uint32_t maxseqno = kSpecialOp)
        : seqcode((minseqno << 5) | static_cast<uint32_t>(flag)),
          maxseqcode((maxseqno << 5) | static_cast<uint32_t>(cache_flag)) {}
    uint32_t code(SeqType t) const { return t == kSeq ? seqcode : maxseqcode; }
    uint32_t seqno(SeqType t = kSeq) const { return code(t) >> 5; }
    int flag(SeqType t = kSeq) const { return static_cast<int>(code(t) & 31); }
    bool load_check(SeqType t = kSeq) const { return (code(t) & kLoadCheck) != 0; }
    bool load_cache(SeqType t = kSeq) const { return (code(t) & kLoadBootstrapCache) != 0; }
    bool check_point(SeqType t = kSeq) const { return (code(t) & kCheckPoint) != 0; }
    bool check_ack(SeqType t = kSeq) const { return (code(t) & kCheckAck) != 0; }
    bool diff_seq() const { return (seqcode & kDiffSeq) != 0; }
    static void Reducer(const void *src, void *dst, int len, const MPI::Datatype &);
  };

  /*!
   * \brief append-only log of collective results since the last checkpoint; each entry lives
   *        in host memory or in the HBM arena of the device plane
   */
  class ResultLog {
   public:
    struct Entry {
      int seqno;
      size_t size;
      bool on_device;  // ptr is HBM
      void *ptr;       // host arena, HBM arena or pinned spill slot
      bool spilled;    // result of an HBM op kept in pinned host memory (HBM log was full)
    };
    /*! \brief HBM arena for device results, and the pinned arena they spill to past its cap */
    void SetArena(device::DeviceArena *a, device::DeviceArena *spill) {
      arena_ = a;
      spill_ = spill;
    }
    /*! \brief growth step of the host arena (small for logs of short keys) */
    void SetHostChunk(size_t bytes) { host_.set_min_chunk(bytes); }
    void Clear();
    /*!
     * \brief scratch slot for the next result (not visible until PushTemp).  A device result
     *        that does not fit the HBM arena spills to pinned host memory (temp_spilled()).
     */
    void *AllocTemp(size_t size, bool device);
    bool temp_spilled() const { return temp_.spilled; }
    size_t n_spilled() const { return n_spilled_; }
    void PushTemp(int seqno, size_t size);
    /*! \brief stored entry for seqno or nullptr */
    const Entry *Query(int seqno) const;
    void *Data(const Entry &e) { return e.ptr; }
    void DropLast();
    int LastSeqNo() const { return entries_.empty() ? -1 : entries_.back().seqno; }
    size_t size() const { return entries_.size(); }

   private:
    /*! \brief host counterpart of device::DeviceArena: 64-byte aligned bump allocation over
     *  chunks that are kept across checkpoints (no reallocation copies, no zero-fill, and
     *  steady-state iterations touch no fresh pages) */
    class HostArena {
     public:
      ~HostArena();
      void *Alloc(size_t bytes);
      void PopTo(void *ptr);
      void Reset();
      void set_min_chunk(size_t b) { min_chunk_ = b; }

     private:
      struct Chunk {
        char *base;
        size_t size, used;
      };
      std::vector<Chunk> chunks_;
      size_t cur_{0};
      size_t min_chunk_{64u << 20};
    };
    std::vector<Entry> entries_;
    HostArena host_;
    Entry temp_{};
    device::DeviceArena *arena_{nullptr};
    device::DeviceArena *spill_{nullptr};
    size_t n_spilled_{0};
  };

  // ---- collectives
  void AllreduceImpl(void *buf, const ReduceSpec &spec, PreprocFunction prepare_fun,
                     void *prepare_arg, const char *_file, const int _line, const char *_caller,
                     const void *prep_src = nullptr, int prep_op = 0, double prep_alpha = 0);
  void CheckPointImpl(const Serializable *global_model, const Serializable *local_model,
                      bool lazy);
  /*! \brief drop the previous result unless this rank is one of its replicas */
  /*! \brief bootstrap-cache key of a call site (reference: `file::line::caller#shape`) */
  static std::string CallKey(const char *file, int line, const char *caller,
                             const std::string &shape);
  void ApplyRetention();
  /*! \brief copy an HBM result into its pinned spill slot (stream-ordered) */
  void SpillResult(void *slot, const void *src, size_t n);
  /*! \brief copy n bytes between host/device locations (synchronous w.r.t. the result) */
  void CopyAny(void *dst, bool dst_dev, const void *src, bool src_dev, size_t n);

  // ---- recovery protocol
  /*! \brief points where a rank serves another rank's recovery (fault injection) */
  enum ServePoint { kServeRouting = 1, kServeData = 2, kServeDevice = 3 };
  /*!
   * \brief called by a rank that holds or relays recovery data for a peer (result replay,
   *        checkpoint load, bootstrap cache): after the routing decision, after the first bytes
   *        of a host transfer left, before a device exchange.  The mock engine kills the rank
   *        here (mock_die_serving); no-op otherwise.
   */
  virtual void ServeHook(ServePoint where) { (void)where; }
  /*!
   * \brief run recovery actions preceding the requested one
   * \return true if the request was satisfied by recovery (buf holds the result),
   *         false if this is the newest action and must be executed
   */
  bool RecoverExec(void *buf, size_t size, int flag, int seqno, int cache_seqno,
                   const char *caller = "RecoverExec");
  /*! \brief true on success; on error repair links (tracker "recover") and return false */
  bool CheckAndRecover(Status s);
  Status TryLoadCheckPoint(bool requester);
  /*! \brief checkpoint load over the device plane (see recovery.cc); kAborted: not applicable */
  Status TryLoadDeviceCheckPoint(RecoverType role, bool *used);
  Status TryGetResult(void *buf, size_t size, int seqno, bool requester);
  /*! \brief per-rank role bits of a device recovery transfer, gathered on every rank */
  static constexpr int kReplayCapable = 1, kReplayHolder = 2, kReplayRequester = 4;
  Status GatherCodes(int mine, std::vector<int> *all);
  Status TryDecideRouting(RecoverType role, size_t *p_size, int *p_recvlink,
                          std::vector<bool> *p_req_in);
  Status TryRecoverData(RecoverType role, void *buf, size_t size, int recv_link,
                        const std::vector<bool> &req_in);
  Status TryRestoreCache(bool requester, int min_seq, int max_seq);
  /*!
   * \brief local state of version v (engine/local_recovery.cc): every rank learns every rank's
   *        slot sizes over TCP, then each missing slot is copied in one hop from a rank that
   *        holds that state (device store: one xGMI exchange; host store: routed over the tree)
   */
  Status TryRecoverLocalState(int v);
  /*! \brief replicate this rank's slot 0 of version v to its num_local_replica successors */
  Status TryCheckinLocalState(int v);
  /*! \brief n x (nslot + 1) table: slot sizes of version v per rank, then the store kind */
  Status GatherLocalSizes(int v, std::vector<int64_t> *table);
  /*! \brief write the local model into slot 0 of version v (the other slots are dropped) */
  void SaveLocalState(int v, const Serializable *local_model);
  /*! \brief load slot 0 of version v into the local model */
  void LoadLocalState(int v, Serializable *local_model);
  /*!
   * \brief two-pass message passing over the tree: out[i] = func(node, in[others], i) is sent
   *        on link i, in[i] is what link i sent (reference allreduce_robust-inl.h:33-166)
   */
  template <typename NodeT, typename EdgeT>
  Status MsgPassing(const NodeT &node, std::vector<EdgeT> *p_in, std::vector<EdgeT> *p_out,
                    EdgeT (*func)(const NodeT &, const std::vector<EdgeT> &, size_t));
  /*! \brief fixes (first call) or checks whether checkpoints carry a local model, and sets
   *  up the replica store: HBM for device local tensors, host memory otherwise */
  void LocalModelCheck(const Serializable *local_model);

  // ---- bootstrap cache (ops issued before LoadCheckPoint)
  int SetBootstrapCache(const std::string &key, const void *buf, size_t nbytes);
  int GetBootstrapCache(const std::string &key, void *buf, size_t nbytes);

  // ---- watchdog
  void WatchdogLoop();
  void StartWatchdog();
  void StopWatchdog();

  // parameters
  int num_global_replica_{5};
  int num_local_replica_{0};
  int default_local_replica_{2};
  bool elide_consensus_{true};
  // state
  int result_buffer_round_{1};
  int cur_cache_seq_{0};
  int local_chkpt_version_{0};
  int use_local_model_{-1};
  int recover_counter_{0};
  bool checkpoint_loaded_{false};
  bool fast_mode_{false};
  ResultLog resbuf_, cachebuf_, lookupbuf_;
  std::string global_checkpoint_;
  const Serializable *global_lazycheck_{nullptr};
  // global_checkpoint_ holds only the version and header of a device-route load (the payload
  // went into the caller's tensors): this rank cannot serve the checkpoint over TCP
  bool ckpt_header_only_{false};
  LocalReplicas local_;
  // watchdog
  TimeoutHandler timeout_handler_{nullptr};
  std::thread watchdog_;
  std::mutex wd_mu_;
  std::condition_variable wd_cv_;
  bool wd_stop_{false};
  std::atomic<double> recovering_since_{0.0};
  std::atomic<bool> watchdog_fired_{false};
  std::atomic<int> wd_rank_{-1};  // rank as seen by the watchdog thread (rank_ is not atomic)
  double hang_timeout_sec_{0};    // rabit_hang_timeout_sec (0: off)
  double attempt_start_{0};       // start of the current op attempt (recovery phase "detect")
  double recover_stagger_ms_{2};  // rabit_recover_stagger_ms: reconnect delay per rank (the
                                  // reference: 10; our tracker serves reconnects concurrently)
};
}  // namespace engine
}  // namespace rabit
#endif  // XRABIT_ENGINE_ENGINE_ROBUST_H_
