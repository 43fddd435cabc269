/*!
 * \file engine_base.h
 * \brief Non-fault-tolerant engine: tracker client + host TCP plane + device RCCL plane.
 *
 * Parity: reference AllreduceBase (`src/allreduce_base.{h,cc}`).  The data path is chosen
 * per call from the buffer's memory kind: host buffers use the TCP algorithms of
 * coll::HostCollectives, HBM buffers use device::DevicePlane (RCCL over xGMI + gfx950
 * kernels).  Every primitive returns a net::Status so the robust engine can retry.
 */
#ifndef XRABIT_ENGINE_ENGINE_BASE_H_
#define XRABIT_ENGINE_ENGINE_BASE_H_

#include <atomic>
#include <memory>
#include <string>
#include <vector>

#include "coll/host_coll.h"
#include "coll/shm_coll.h"
#include "device/device_checkpoint.h"
#include "device/device_plane.h"
#include "net/links.h"
#include "net/tracker_client.h"
#include "rabit/internal/engine.h"

namespace rabit {
namespace engine {

using net::Status;
typedef IEngine::ReduceFunction *ReduceFn;

/*! \brief per-engine counters exported by RabitGetStats */
/*!
 * \brief mock kills end the process immediately (print, then _Exit as the C API's fatal-error
 *        path does) instead of throwing.  Set by the C API for processes that exit on errors
 *        anyway: the throw would only unwind the stack first, which costs ~0.3 s in a process
 *        with torch's libraries loaded and delays the survivors' detection.  C++ programs and the
 *        unit tests keep the reference's throw (`src/allreduce_mock.h:196-202`).
 */
void SetMockKillsExit(bool v);
bool MockKillsExit();

struct EngineStats {
  uint64_t n_allreduce{0}, n_broadcast{0}, n_allgather{0}, n_checkpoint{0};
  uint64_t n_device_ops{0}, n_recovered_ops{0}, n_recover_events{0}, n_consensus{0};
  uint64_t n_shm_ops{0};
  uint64_t n_consensus_elided{0};
  uint64_t n_device_replays{0};
  uint64_t n_device_ckpt_loads{0};  // checkpoint loads served over the device plane
  uint64_t n_spilled_results{0};    // HBM results logged in pinned host memory (log cap hit)
  uint64_t n_spilled_replays{0};    // replays served from a spilled result
  double bytes_spilled{0};
  double bytes_local_in{0};   // local-checkpoint replica bytes received over the device plane
  double bytes_replay_in{0};  // recovered result bytes received over the device plane
  double bytes_ckpt_in{0};    // global-checkpoint bytes received over the device plane
  double bytes_allreduce{0}, bytes_broadcast{0}, bytes_allgather{0};
  double t_allreduce{0}, t_broadcast{0}, t_allgather{0}, t_checkpoint{0}, t_consensus{0};
  double t_recover{0};
  /*!
   * \brief where recovery time goes (seconds, summed over the job), survivor and restarted side:
   *        detect: from the start of the failed op attempt to the failure seen; drop_links:
   *        closing links and the reconnect stagger; relink: the tracker round; then the device
   *        bring-up of the next epoch (records: GPU records over the host ring; peer_open:
   *        preflight + IPC mapping of the direct transport; rccl: communicator bring-up; tune:
   *        RCCL channel tuning; calibration: full start-up calibration; adopt: adopting the
   *        survivors' calibration + one verified op per transport); load_checkpoint (the
   *        restarted rank's LoadCheckPoint), replay (its result catch-up), serve_load /
   *        serve_replay (survivors serving them)
   */
  struct Phases {
    double detect{0}, drop_links{0}, relink{0};
    double records{0}, peer_open{0}, rccl{0}, tune{0}, calibration{0}, adopt{0};
    double load_checkpoint{0}, replay{0}, serve_load{0}, serve_replay{0};
    uint64_t bringups{0}, calibrations{0}, adoptions{0}, replays{0}, serves{0};
  } phases;
  double t_process_start_to_init{0};  // this process: start to Init done (restart cost)
};

class EngineBase : public IEngine {
 public:
  EngineBase();
  ~EngineBase() override;
  /*! \brief parse params, connect to the tracker, bring up links and (lazily) the device */
  virtual bool Init(int argc, char *argv[]);
  /*! \brief close links, tell the tracker */
  virtual bool Shutdown();
  /*! \brief set one parameter (subclasses chain to the parent) */
  virtual void SetParam(const char *name, const char *val);

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
  void Broadcast(void *sendrecvbuf_, size_t size, int root, const char *_file, const int _line,
                 const char *_caller) override;
  void InitAfterException() override {}
  int LoadCheckPoint(Serializable *global_model, Serializable *local_model) override;
  void CheckPoint(const Serializable *global_model, const Serializable *local_model) override;
  void LazyCheckPoint(const Serializable *global_model) override;
  int VersionNumber() const override { return version_number_; }
  int GetRingPrevRank() const override;
  int GetRank() const override { return rank_; }
  int GetWorldSize() const override { return world_size_ == -1 ? 1 : world_size_; }
  bool IsDistributed() const override { return tracker_.uri != "NULL"; }
  std::string GetHost() const override { return host_uri_; }
  void TrackerPrint(const std::string &msg) override;
  void SetStream(void *stream) override;
  int GetDevice() const override { return dev_ ? dev_->device() : -1; }
  bool IsDevicePointer(const void *ptr) const override { return OnDevice(ptr); }
  const char *EngineName() const override { return "base"; }

  /*!
   * \brief fused lazy-prepare allreduce of a device buffer: dst = prep(src) then
   *        allreduce(dst).  The base engine always runs the prepare kernel.
   */
  virtual void DevAllreducePrepared(void *dst, const void *src, size_t count, int dtype, int op,
                                    int prep, double alpha, const char *_file, const int _line,
                                    const char *_caller);
  /*!
   * \brief the fault-tolerance tax, measured (RabitDevProbeAllreduce): the same device
   *        allreduce the robust engine runs, on the same transports, but outside the result log
   *        and the sequence numbering -- a collective every rank calls between the same ops, like
   *        the link probe.  mode 0: in place with the host wait (what the base engine runs);
   *        1: into a scratch slot and the user buffer (the robust engine's dual store), host
   *        wait; 2: in place, stream-ordered (no host wait).  0 on success, -1 on failure,
   *        -2 without the device plane.
   */
  int DevProbeAllreduce(void *buf, size_t count, int dtype, int op, int mode);
  /*!
   * \brief capturable in-place RCCL allreduce (RabitDevGraphAllreduce): brings the device
   *        communicator up on first use (a collective: make the first call eagerly, on every
   *        rank), then only enqueues ncclAllReduce on `stream`.  0 or a negative code (c_api.h)
   */
  int DevGraphAllreduce(void *buf, size_t count, int dtype, int op, hipStream_t stream,
                        std::string *why);
  /*!
   * \brief xGMI link probe (DevicePlane::LinkProbe) after bringing the device transports up;
   *        out receives 5 GB/s values of this rank.  0, -1 when it failed, -2 without a
   *        direct transport (world 1, or ranks on several hosts).
   */
  int DevLinkProbe(size_t bytes, double *out);
  /*! \brief copy engine of the checkpoint host mirrors (rabit_device_mirror_engine; a
   *         rabit_device_mirror_ctas > 0 alone selects the kernel engine) */
  int MirrorEngine() const {
    if (mirror_engine_ >= 0) return mirror_engine_;
    return mirror_ctas_ > 0 ? device::DeviceCheckpoint::kEngineKernel
                            : device::DeviceCheckpoint::kEngineHip;
  }
  /*!
   * \brief checkpoint HBM buffers: HBM snapshot + async pinned mirror, registered as a lazy
   *        global checkpoint (see device/device_checkpoint.h).  nl > 0: lptrs are this rank's
   *        local model (per-rank state): the robust engine keeps it, and the replicas of its
   *        ring predecessors, in HBM and replicates it over xGMI.
   */
  void DevCheckPoint(int n, void *const *ptrs, const size_t *nbytes, const std::string &meta,
                     int nl = 0, void *const *lptrs = nullptr, const size_t *lnbytes = nullptr);
  /*! \brief load the latest device checkpoint into HBM buffers (and the local model into
   *         lptrs when nl > 0); returns the version */
  int DevLoadCheckPoint(int n, void *const *ptrs, const size_t *nbytes, std::string *meta,
                        int nl = 0, void *const *lptrs = nullptr, const size_t *lnbytes = nullptr);
  /*! \brief register a device checkpoint (global snapshot, optional device local model) */
  virtual void CheckPointDevice(const Serializable *global_model, const Serializable *local_model) {
    (void)local_model;
    this->LazyCheckPoint(global_model);
  }
  /*! \brief mock engine's force_local: global tensors are checkpointed as local state too */
  virtual bool ForceLocal() const { return false; }
  /*! \brief engine statistics as JSON */
  virtual std::string StatsJson() const;
  device::DevicePlane *device_plane() { return dev_.get(); }

 protected:
  /*! \brief how to reduce: element size/count plus either a built-in (dtype, op) or a
   *  host reduce function */
  struct ReduceSpec {
    size_t type_nbytes{1};
    size_t count{0};
    ReduceFn host_red{nullptr};
    DeviceReduceLauncher *dev_red{nullptr};  // user device reduction (AllreduceDevice)
    int dtype{-1};
    int op{-1};
    size_t bytes() const { return type_nbytes * count; }
    bool builtin() const { return dtype >= 0 && op >= 0; }
  };
  bool OnDevice(const void *p) const;
  /*! \brief in-place allreduce over the host plane */
  /*! \brief host-buffer allreduce into buf; src != nullptr: inputs read from src (out of
   *  place, src untouched, so a failed attempt can be retried) */
  Status TryAllreduceHost(void *buf, const ReduceSpec &spec, const void *src = nullptr);
  /*!
   * \brief device allreduce dst = reduce(src) (src may equal dst); custom host reducers are
   *        staged through host memory
   */
  /*!
   * \brief dst = allreduce(prep(src)); also written to dst2 (if given) once the op succeeded
   *        on this rank.  prep is a device::PrepOp (kPrepCopy: none).
   */
  Status TryAllreduceDevice(const void *src, void *dst, const ReduceSpec &spec,
                            void *dst2 = nullptr, int prep = 0, double alpha = 1.0,
                            bool host_wait = true);
  /*! \brief dev_log (HBM buffers only): on success the result is also in dev_log, stored by
   *  the transport itself (no copy after the collective on the direct path) */
  Status TryBroadcast(void *buf, size_t size, int root, void *dev_log = nullptr);
  Status TryAllgather(void *buf, size_t total, size_t begin, size_t end, size_t prev_size,
                      void *dev_log = nullptr);
  /*! \brief build the device transports if missing (collective): exchange GPU records, map
   *  the peers' buffers for the direct transport, build the RCCL communicator */
  Status EnsureDeviceComm();
  /*! \brief true if a host-buffer op of this size goes through shared memory */
  bool UseShm(size_t bytes) const { return shm_enabled_ && world_size_ > 1 && bytes >= shm_min_; }
  /*! \brief build the shared-memory group (collective; uniform outcome: usable on every rank
   *  or off for this epoch) */
  Status EnsureShm();
  /*! \brief forget the group (after a failure every rank rebuilds it) */
  void ResetShm() {
    shm_.reset();
    shm_decided_ = false;
  }
  /*! \brief auto mode: time RCCL and the direct transport at two sizes, verify the direct
   *  result, and set the size from which ops go direct (collective) */
  Status CalibrateDevice();
  /*! \brief auto mode, after CalibrateDevice: time the broadcast (root 0, result-log slot
   *  included) on both transports at two sizes, verify the direct result, and route broadcasts
   *  by their own crossover (collective) */
  Status CalibrateBroadcast();
  /*! \brief collective: time the 128 MiB RCCL allreduce with RCCL's own channel count and
   *  with fixed CTA counts (rabit_rccl_tune_ctas), keep the fastest communicator */
  Status TuneRcclChannels();
  /*! \brief collective: (re)build the RCCL communicator of this epoch with the current CTA
   *  bounds; false on every rank if it did not come up on every rank */
  Status BuildRccl(bool *up);
  /*! \brief (re)connect peer links through the tracker */
  bool ReconnectLinks(const char *cmd);
  /*! \brief true if any peer link hung up (used while waiting on device ops) */
  bool PeerFailureProbe() const;
  /*! \brief Hadoop status line */
  void ReportStatus() const;
  /*! \brief mock_dev_hang: wedge this rank's stream before the next device collective;
   *  mock_die_mid: leave the process in the middle of the next multi-chunk direct allreduce */
  void MaybeInjectDeviceHang() {
    if (die_mid_armed_) {
      die_mid_armed_ = false;
      dev_->ArmDieMidOp();
    }
    if (!dev_hang_armed_) return;
    dev_hang_armed_ = false;
    dev_->InjectHang(dev_hang_max_sec_);
  }
  device::FailureProbe MakeProbe() const {
    return [this]() { return this->PeerFailureProbe(); };
  }

  /*!
   * \brief HBM tensors that form this rank's local model in a device checkpoint.  The robust
   *        engine recognises this object and moves its bytes HBM to HBM; Save/Load (host
   *        staging) serve engines that keep local state in host memory.
   */
  struct DeviceLocalModel : public Serializable {
    EngineBase *owner{nullptr};
    std::vector<void *> ptrs;
    std::vector<size_t> nbytes;
    size_t total() const {
      size_t t = 0;
      for (size_t b : nbytes) t += b;
      return t;
    }
    void Set(int n, void *const *p, const size_t *b) {
      ptrs.assign(p, p + n);
      nbytes.assign(b, b + n);
    }
    void Load(Stream *fi) override;
    void Save(Stream *fo) const override;
  };
  DeviceLocalModel dev_local_;

  // parameters / configuration
  std::vector<std::string> env_vars_;
  net::TrackerConfig tracker_;
  coll::HostCollConfig hcfg_;
  device::DeviceConfig dcfg_;
  int device_plane_mode_{1};  // 0: never, 1: when a GPU is visible
  std::string dmlc_role_{"worker"};
  std::string host_uri_;
  bool hadoop_mode_{false};
  bool debug_{false};
  bool bootstrap_cache_{false};
  bool timeout_enabled_{false};
  int timeout_sec_{1800};
  bool world1_fastpath_{true};
  // robust engine, host buffers: reduce out of place from the user buffer into the result log
  // (one copy per op instead of two)
  bool host_out_of_place_{true};
  // test hook: world-1 device ops go through the transports (a one-rank RCCL communicator, a
  // one-peer direct group) instead of the local short-cut, so their API paths run on one GPU
  bool world1_transport_{false};
  bool shm_enabled_{true};          // rabit_host_shm
  int ckpt_mirror_mode_{0};          // rabit_device_ckpt_mirror: 0 idle, 1 always, 2 off
  int ckpt_slots_{0};                // rabit_device_ckpt_slots: 2, 3, 0 = by size
  bool mirror_low_prio_{false};      // rabit_device_mirror_priority=low
  int mirror_ctas_{0};     // rabit_device_mirror_ctas: D2H mirror kernel width (> 0: kernel)
  int mirror_engine_{-1};  // rabit_device_mirror_engine: hip / kernel / sdma (-1: by ctas)
  size_t ckpt_3slot_max_{size_t(4) << 30};  // by size: 3 slots below this many bytes
  size_t shm_min_{1u << 20};        // rabit_host_shm_min
  size_t shm_stage_{32u << 20};     // rabit_host_shm_buffer (per stage, two per rank)
  bool calibrate_{true};
  bool calibrate_test_{false};  // run the calibration without RCCL (tests on a shared GPU)
  bool device_replay_{true};       // recover HBM results with a device broadcast
  bool host_via_device_{false};     // stage large host-buffer allreduces through HBM
  size_t host_dev_min_{1u << 20};
  // staged host allreduces of >= 2 chunks: 0 whole copies, 1 pipelined (host_stager.h),
  // 2 auto: after one untimed warm-up op, one such op is timed whole and the next pipelined,
  // and the faster (slowest rank's rate, agreed over the host plane) is kept for the job
  int host_stage_mode_{2};
  int host_stage_trial_{0};          // auto: eligible ops so far (3 = decided)
  bool host_stage_pipe_{false};      // auto's decision
  double host_stage_rate_[2]{0, 0};  // auto: whole / pipelined GB/s (slowest rank)
  /*! \brief last calibration: rccl small/big, direct small/big (s; direct big = the chosen
   *  variant), small/big bytes, push variant at the big size */
  struct {
    double rccl_small, rccl_big, direct_small, direct_big, small_bytes, big_bytes, push_big;
  } calib_{0, 0, 0, 0, 0, 0, 0};
  /*! \brief forms of the direct two-shot path the calibration times at its large size:
   *  {configured, other fused/classic, push configured-fused, push other}; us, -1 = not run */
  // forms of the direct two-shot path: pull / push x classic / fused, and the pipelined push
  static constexpr int kCalibForms = 5;
  double calib_form_us_[kCalibForms]{-1, -1, -1, -1, -1};
  bool calib_heap_src_{false};  // the last calibration read its inputs from the symmetric heap
  bool calib_valid_{false};     // this process holds a calibration of this job (adoptable)
  std::string calib_matrix_json_{"{}"};  // the last calibration's times and bands (stats)
  bool allgather_resolve_{true};  // rabit_device_allgather_resolve: direct allgathers resolve
                                  // the slice layout on the device (0: a host round first)
  bool adopt_calibration_{true};  // rabit_device_calibration_adopt: recovery epochs adopt the
                                  // survivors' calibration instead of re-measuring
  /*! \brief collective: if some rank holds this job's calibration (a recovery epoch), every rank
   *  takes the lowest such rank's routing and direct form, and one small op per transport is
   *  verified on the host; *adopted false: calibrate from scratch */
  Status AdoptCalibration(bool *adopted);
  /*! \brief this rank's routing and calibration results, serialized (AdoptCalibration) */
  std::string SerializeCalibration() const;
  void ApplyCalibration(const std::string &blob);
  /*! \brief one host-verified allreduce per transport of the routing (direct: 1 MiB, RCCL:
   *  64 KiB); *good false on a wrong result, a non-success status on a failed op */
  Status VerifyTransports(bool *good);
  /*! \brief the recovery phase breakdown as JSON */
  std::string PhasesJson() const;
  /*! \brief last broadcast calibration: rccl small/big, direct small/big (s; 0 = not run) */
  double calib_bcast_[4]{0, 0, 0, 0};
  bool mock_rccl_fail_{false};  // test hook: the RCCL communicator never comes up
  int rccl_failed_{0};
  bool rccl_tune_{false};          // rabit_rccl_tune: time RCCL channel counts at start-up
  bool rccl_tuned_{false};         // this process took part in (or adopted) a tuning
  std::string rccl_tune_ctas_{"64,112"};  // candidate CTA counts besides RCCL's own choice
  std::string rccl_tune_json_{"{}"};      // what the tuning measured (stats)
  bool dev_hang_armed_{false};     // set by the mock engine's mock_dev_hang
  bool die_mid_armed_{false};      // set by the mock engine's mock_die_mid
  double dev_hang_max_sec_{90};     // an injected hang ends by itself after this long
  double dev_wait_limit_sec_{600};  // watchdog: a wait on this rank's GPU may last this long
  bool trace_spans_{false};
  bool trace_roctx_{false};
  size_t trace_capacity_{1 << 16};
  // runtime state
  net::Topology topo_;
  std::unique_ptr<coll::HostCollectives> host_;
  /*! \brief shared-memory transport for large host buffers of co-located ranks (built on
   *  first use after every (re)connect, like a device epoch; nullptr while undecided or off) */
  std::unique_ptr<coll::ShmGroup> shm_;
  bool shm_decided_{false};
  std::unique_ptr<device::DevicePlane> dev_;
  std::unique_ptr<device::DeviceCheckpoint> dev_ckpt_;
  void *user_stream_{nullptr};
  std::atomic<bool> abort_flag_{false};
  int rank_{0};
  int world_size_{-1};
  int version_number_{0};
  int seq_counter_{0};
  EngineStats stats_;
};
}  // namespace engine
}  // namespace rabit
#endif  // XRABIT_ENGINE_ENGINE_BASE_H_
