/*!
 * \file engine_base.cc
 * \brief Non-fault-tolerant engine (see engine_base.h).
 */
#include "engine/engine_base.h"

#include <unistd.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <sstream>

#include "core/params.h"
#include "core/trace.h"
#include "device/kernels.h"
#include "rabit/internal/timer.h"
#include "rabit/internal/utils.h"

extern char **environ;

namespace rabit {
namespace engine {

EngineBase::EngineBase() {
  env_vars_ = {"DMLC_TASK_ID",      "DMLC_ROLE",         "DMLC_NUM_ATTEMPT",
               "DMLC_TRACKER_URI",  "DMLC_TRACKER_PORT", "DMLC_WORKER_CONNECT_RETRY"};
  tracker_.tcp_nodelay = true;  // the control plane is latency bound (consensus per op)
  host_.reset(new coll::HostCollectives(&topo_, &hcfg_, &rank_, &world_size_));
  host_->SetAbortFlag(&abort_flag_);
}

EngineBase::~EngineBase() = default;

void EngineBase::SetParam(const char *name, const char *val) {
  auto is = [name](const char *k) { return strcmp(name, k) == 0; };
  if (is("rabit_tracker_uri") || is("DMLC_TRACKER_URI")) tracker_.uri = val;
  if (is("rabit_tracker_port") || is("DMLC_TRACKER_PORT")) tracker_.port = atoi(val);
  if (is("rabit_task_id") || is("DMLC_TASK_ID")) tracker_.task_id = val;
  if (is("DMLC_ROLE")) dmlc_role_ = val;
  if (is("rabit_world_size")) world_size_ = atoi(val);
  if (is("rabit_hadoop_mode")) hadoop_mode_ = utils::StringToBool(val);
  if (is("rabit_tree_reduce_minsize")) hcfg_.tree_reduce_minsize = core::ParseUnit(name, val);
  if (is("rabit_reduce_ring_mincount")) {
    long v = atol(val);  // NOLINT(*)
    utils::Check(v > 0, "rabit_reduce_ring_mincount should be greater than 0");
    hcfg_.reduce_ring_mincount = static_cast<size_t>(v);
  }
  if (is("rabit_reduce_buffer")) {
    hcfg_.reduce_buffer_bytes = std::max<size_t>(core::ParseUnit(name, val), 8);
  }
  if (is("DMLC_WORKER_CONNECT_RETRY")) tracker_.connect_retry = atoi(val);
  if (is("rabit_bootstrap_cache")) bootstrap_cache_ = utils::StringToBool(val);
  if (is("rabit_debug")) debug_ = utils::StringToBool(val);
  if (is("rabit_timeout")) timeout_enabled_ = utils::StringToBool(val);
  if (is("rabit_timeout_sec")) {
    timeout_sec_ = atoi(val);
    utils::Check(timeout_sec_ >= 0, "rabit_timeout_sec should be non negative second");
  }
  if (is("rabit_enable_tcp_no_delay")) tracker_.tcp_nodelay = utils::StringToBool(val);
  if (is("rabit_slave_port") || is("rabit_worker_port")) tracker_.worker_port = atoi(val);
  if (is("rabit_nport_trial")) tracker_.nport_trial = atoi(val);
  // ---- xrabit extensions
  if (is("rabit_device")) dcfg_.device = atoi(val);
  if (is("rabit_device_plane")) device_plane_mode_ = utils::StringToBool(val) ? 1 : 0;
  if (is("rabit_device_sync")) dcfg_.sync = utils::StringToBool(val);
  if (is("rabit_device_timeout_sec")) {
    // "auto" (default): 60 s + 1 s per GB of the op; 0: no deadline
    dcfg_.op_timeout_sec = strcmp(val, "auto") == 0 ? -1.0 : atof(val);
  }
  if (is("rabit_device_drain_timeout_sec")) dcfg_.drain_timeout_sec = atof(val);
  if (is("rabit_device_wait_limit_sec")) dev_wait_limit_sec_ = atof(val);
  if (is("rabit_mock_dev_hang_sec")) dev_hang_max_sec_ = atof(val);
  if (is("rabit_device_spin_us")) dcfg_.spin_us = atoi(val);
  if (is("rabit_device_log_cap")) dcfg_.arena_cap = core::ParseUnit(name, val);
  if (is("rabit_device_spill_cap")) dcfg_.spill_cap = core::ParseUnit(name, val);
  if (is("rabit_device_log_chunk")) dcfg_.arena_chunk = core::ParseUnit(name, val);
  if (is("rabit_device_log_reserve")) dcfg_.arena_reserve = core::ParseUnit(name, val);
  if (is("rabit_device_algo")) {
    const std::string v(val);
    if (v == "auto") {
      dcfg_.algo = 0;
    } else if (v == "rccl") {
      dcfg_.algo = 1;
    } else if (v == "direct") {
      dcfg_.algo = 2;
    } else {
      utils::Error("rabit_device_algo must be auto, rccl or direct (got %s)", val);
    }
  }
  if (is("rabit_device_peer_buffer")) dcfg_.peer_stage = core::ParseUnit(name, val);
  if (is("rabit_device_peer_timeout_sec")) dcfg_.peer_deadline_sec = atof(val);
  if (is("rabit_device_direct_min")) {
    dcfg_.direct_min_bytes = core::ParseUnit(name, val);
    calibrate_ = false;  // an explicit threshold wins over the measured one
  }
  if (is("rabit_device_calibrate")) calibrate_ = utils::StringToBool(val);
  if (is("rabit_device_calibrate_test")) calibrate_test_ = utils::StringToBool(val);
  if (is("rabit_device_calibration_adopt")) adopt_calibration_ = utils::StringToBool(val);
  if (is("rabit_device_allgather_resolve")) allgather_resolve_ = utils::StringToBool(val);
  if (is("rabit_device_replay")) device_replay_ = utils::StringToBool(val);
  if (is("rabit_host_via_device")) host_via_device_ = utils::StringToBool(val);
  if (is("rabit_host_via_device_min")) host_dev_min_ = core::ParseUnit(name, val);
  if (is("rabit_device_oneshot_max")) dcfg_.oneshot_max = core::ParseUnit(name, val);
  if (is("rabit_device_fused")) {
    // auto: the calibration picks (without a calibration: the classic form)
    dcfg_.fused_mode = !strcmp(val, "auto") ? 2 : (utils::StringToBool(val) ? 1 : 0);
  }
  if (is("rabit_device_fused_grid")) dcfg_.fused_grid = atoi(val);
  if (is("rabit_device_fused_oneshot")) {
    // a size (one-shot ops up to it in one launch), or a boolean (0: never, 1: the default 64K)
    const size_t v = core::ParseUnit(name, val);
    dcfg_.fused_oneshot_max = v == 1 ? (64u << 10) : v;
  }
  if (is("rabit_rccl_min_ctas")) dcfg_.rccl_min_ctas = atoi(val);
  if (is("rabit_device_calibrate_bytes")) dcfg_.calib_big = core::ParseUnit(name, val);
  if (is("rabit_device_bcast_chunk")) dcfg_.bcast_chunk = core::ParseUnit(name, val);
  if (is("rabit_host_stage_chunk")) dcfg_.host_stage_chunk = core::ParseUnit(name, val);
  if (is("rabit_host_stage_threads")) dcfg_.host_stage_threads = atoi(val);
  if (is("rabit_host_stage_streams")) dcfg_.host_stage_streams = atoi(val) == 1 ? 1 : 3;
  if (is("rabit_host_stage")) {
    host_stage_mode_ = !strcmp(val, "auto") ? 2 : (utils::StringToBool(val) ? 1 : 0);
  }
  if (is("rabit_rccl_max_ctas")) dcfg_.rccl_max_ctas = atoi(val);
  if (is("rabit_rccl_tune")) rccl_tune_ = utils::StringToBool(val);
  if (is("rabit_rccl_init_timeout_sec")) dcfg_.comm_init_timeout_sec = atof(val);
  if (is("rabit_rccl_max_failures")) dcfg_.rccl_max_failures = atoi(val);
  if (is("rabit_mock_rccl_error")) dcfg_.mock_rccl_error = atoi(val);
  if (is("rabit_device_done_word")) dcfg_.done_word = utils::StringToBool(val);
  if (is("rabit_device_peer_abort")) dcfg_.peer_abort = utils::StringToBool(val);
  if (is("rabit_rccl_tune_ctas")) rccl_tune_ctas_ = val;
  if (is("rabit_device_fused_min")) dcfg_.fused_min_bytes = core::ParseUnit(name, val);
  if (is("rabit_device_direct_mode")) {
    if (!strcmp(val, "auto")) {
      dcfg_.direct_mode = 0;
    } else if (!strcmp(val, "pull")) {
      dcfg_.direct_mode = 1;
    } else if (!strcmp(val, "push")) {
      dcfg_.direct_mode = 2;
    } else if (!strcmp(val, "pipelined")) {
      dcfg_.direct_mode = 2;  // the pipelined form is a push form
      dcfg_.pipeline_mode = 1;
    } else {
      utils::Error("rabit_device_direct_mode must be auto, pull, push or pipelined (got %s)", val);
    }
  }
  if (is("rabit_device_pipeline")) {
    // auto: the calibration times the pipelined push form against the others
    dcfg_.pipeline_mode = !strcmp(val, "auto") ? 2 : (utils::StringToBool(val) ? 1 : 0);
  }
  if (is("rabit_device_pipeline_chunk")) dcfg_.pipeline_chunk = core::ParseUnit(name, val);
  if (is("rabit_device_defer_second")) dcfg_.defer_second = utils::StringToBool(val);
  if (is("rabit_device_symmetric_heap")) dcfg_.sym_heap = core::ParseUnit(name, val);
  if (is("rabit_device_zero_copy")) {
    // a size (ordinary HBM inputs from it on are registered for in-place reads), or a boolean
    // (0: never, 1: the default 1 MiB)
    const size_t v = core::ParseUnit(name, val);
    dcfg_.zero_copy_min = v == 1 ? (1u << 20) : v;
  }
  if (is("rabit_device_user_stream")) dcfg_.ops_on_user_stream = utils::StringToBool(val);
  if (is("rabit_device_phase_timing")) dcfg_.phase_timing = utils::StringToBool(val);
  if (is("rabit_world1_fastpath")) world1_fastpath_ = utils::StringToBool(val);
  if (is("rabit_host_out_of_place")) host_out_of_place_ = utils::StringToBool(val);
  if (is("rabit_device_world1_transport")) world1_transport_ = utils::StringToBool(val);
  if (is("rabit_mock_rccl_init_fail")) mock_rccl_fail_ = utils::StringToBool(val);
  if (is("rabit_host_shm")) shm_enabled_ = utils::StringToBool(val);
  if (is("rabit_device_ckpt_mirror")) {
    if (!strcmp(val, "always")) {
      ckpt_mirror_mode_ = device::DeviceCheckpoint::kMirrorAlways;
    } else if (!strcmp(val, "idle")) {
      ckpt_mirror_mode_ = device::DeviceCheckpoint::kMirrorIdle;
    } else if (!strcmp(val, "off")) {
      ckpt_mirror_mode_ = device::DeviceCheckpoint::kMirrorOff;
    } else {
      utils::Error("rabit_device_ckpt_mirror must be always, idle or off (got %s)", val);
    }
  }
  if (is("rabit_device_mirror_priority")) {
    utils::Check(!strcmp(val, "low") || !strcmp(val, "normal"),
                 "rabit_device_mirror_priority must be low or normal (got %s)", val);
    mirror_low_prio_ = !strcmp(val, "low");
  }
  if (is("rabit_device_mirror_engine")) {
    if (!strcmp(val, "hip")) {
      mirror_engine_ = device::DeviceCheckpoint::kEngineHip;
    } else if (!strcmp(val, "kernel")) {
      mirror_engine_ = device::DeviceCheckpoint::kEngineKernel;
    } else if (!strcmp(val, "sdma")) {
      mirror_engine_ = device::DeviceCheckpoint::kEngineSdma;
    } else {
      utils::Error("rabit_device_mirror_engine must be hip, kernel or sdma (got %s)", val);
    }
  }
  if (is("rabit_device_mirror_ctas")) {
    mirror_ctas_ = atoi(val);
    utils::Check(mirror_ctas_ >= 0 && mirror_ctas_ <= 4096,
                 "rabit_device_mirror_ctas must be 0 (hipMemcpyAsync) or 1..4096");
  }
  if (is("rabit_device_ckpt_slots")) {
    ckpt_slots_ = atoi(val);
    utils::Check(ckpt_slots_ == 0 || ckpt_slots_ == 2 || ckpt_slots_ == 3,
                 "rabit_device_ckpt_slots must be 2, 3 or 0 (by size)");
  }
  if (is("rabit_device_ckpt_3slot_max")) ckpt_3slot_max_ = core::ParseUnit(name, val);

  if (is("rabit_host_shm_min")) shm_min_ = core::ParseUnit(name, val);
  if (is("rabit_host_shm_buffer")) shm_stage_ = core::ParseUnit(name, val);
  if (is("rabit_poll_interval_ms")) hcfg_.poll_interval_ms = std::max(1, atoi(val));
  if (is("rabit_trace")) trace_spans_ = utils::StringToBool(val);
  if (is("rabit_trace_roctx")) trace_roctx_ = utils::StringToBool(val);
  if (is("rabit_trace_capacity")) trace_capacity_ = static_cast<size_t>(atol(val));
}

namespace {
/*! \brief seconds since this process started (/proc/self/stat field 22 against /proc/uptime;
 *  0 when unavailable): a restarted worker's start-up cost in the recovery breakdown */
double ProcessAgeSeconds() {
  FILE *f = fopen("/proc/self/stat", "r");
  if (f == nullptr) return 0;
  char buf[1024];
  const size_t k = fread(buf, 1, sizeof(buf) - 1, f);
  fclose(f);
  buf[k] = '\0';
  const char *p = strrchr(buf, ')');  // the command name may contain spaces
  if (p == nullptr) return 0;
  unsigned long long start = 0;
  // fields after the name: state (3) ... starttime (22)
  int field = 2;
  for (const char *q = p + 1; *q != '\0'; ++q) {
    if (*q == ' ') {
      ++field;
      if (field == 22) {
        start = strtoull(q + 1, nullptr, 10);
        break;
      }
    }
  }
  double up = 0;
  f = fopen("/proc/uptime", "r");
  if (f == nullptr) return 0;
  if (fscanf(f, "%lf", &up) != 1) up = 0;
  fclose(f);
  const long hz = sysconf(_SC_CLK_TCK);
  if (up <= 0 || hz <= 0 || start == 0) return 0;
  return std::max(0.0, up - static_cast<double>(start) / static_cast<double>(hz));
}
}  // namespace

bool EngineBase::Init(int argc, char *argv[]) {
  // before this engine starts any thread (watchdog, copier, bring-up helpers)
  device::DevicePlane::ConfigureRcclEnv();
  // every rabit_* environment variable is a parameter too (the reference only reads a fixed
  // list, which is kept: DMLC_* names above)
  std::vector<std::string> names = env_vars_;
  for (char **e = environ; e != nullptr && *e != nullptr; ++e) {
    const char *eq = strchr(*e, '=');
    if (eq != nullptr && strncmp(*e, "rabit_", 6) == 0) names.emplace_back(*e, eq - *e);
  }
  for (const auto &kv : core::CollectParams(argc, argv, names)) {
    this->SetParam(kv.first.c_str(), kv.second.c_str());
  }
  // Hadoop / YARN streaming environment
  const char *task_id = getenv("mapred_tip_id");
  if (task_id == nullptr) task_id = getenv("mapreduce_task_id");
  if (hadoop_mode_) utils::Check(task_id != nullptr, "hadoop_mode is set but no task id found");
  if (task_id != nullptr) {
    this->SetParam("rabit_task_id", task_id);
    this->SetParam("rabit_hadoop_mode", "1");
  }
  const char *attempt_id = getenv("mapred_task_id");
  if (attempt_id != nullptr) {
    const char *att = strrchr(attempt_id, '_');
    int trial;
    if (att != nullptr && sscanf(att + 1, "%d", &trial) == 1) {
      this->SetParam("rabit_num_trial", att + 1);
    }
  }
  const char *num_task = getenv("mapred_map_tasks");
  if (num_task == nullptr) num_task = getenv("mapreduce_job_maps");
  if (hadoop_mode_) utils::Check(num_task != nullptr, "hadoop_mode is set but no task count");
  if (num_task != nullptr) this->SetParam("rabit_world_size", num_task);

  if (dmlc_role_ != "worker") {
    fprintf(stderr, "xrabit only runs as a dmlc worker (DMLC_ROLE=%s), exiting\n",
            dmlc_role_.c_str());
    exit(0);
  }
  utils::Check(topo_.links.empty(), "can only call Init once");
  trace::Tracer::Get().Configure(trace_spans_, trace_roctx_, trace_capacity_);
  rank_ = -1;
  host_uri_ = net::HostName();
  if (!ReconnectLinks("start")) return false;
  if (device_plane_mode_ != 0 && device::DevicePlane::DeviceCount() > 0) {
    dev_.reset(new device::DevicePlane(dcfg_, rank_));
    if (user_stream_ != nullptr) dev_->SetUserStream(static_cast<hipStream_t>(user_stream_));
  }
  stats_.t_process_start_to_init = ProcessAgeSeconds();
  return true;
}

bool EngineBase::Shutdown() {
  try {
    ResetShm();
    if (dev_) {
      dev_->Synchronize();
      dev_ckpt_.reset();
      dev_.reset();
    }
    topo_.CloseAll();
    topo_.links.clear();
    topo_.tree.clear();
    topo_.ring_prev = topo_.ring_next = nullptr;
    if (tracker_.uri == "NULL") return true;
    net::TrackerClient(&tracker_).Shutdown(rank_, world_size_);
    return true;
  } catch (const std::exception &e) {
    fprintf(stderr, "xrabit: shutdown failed: %s\n", e.what());
    return false;
  }
}

bool EngineBase::ReconnectLinks(const char *cmd) {
  if (tracker_.uri == "NULL") {
    rank_ = 0;
    world_size_ = 1;
    return true;
  }
  try {
    net::TrackerClient(&tracker_).Relink(cmd, &rank_, &world_size_, &topo_);
    if (debug_) {
      utils::HandleLogInfo("[%d] %s: links ready (world %d, tree %zu, ring %d<-%d->%d)\n", rank_,
                           cmd, world_size_, topo_.tree.size(),
                           topo_.ring_prev ? topo_.ring_prev->rank : -1, rank_,
                           topo_.ring_next ? topo_.ring_next->rank : -1);
    }
    return true;
  } catch (const std::exception &e) {
    fprintf(stderr, "xrabit: ReconnectLinks(%s) failed: %s\n", cmd, e.what());
    return false;
  }
}

int EngineBase::GetRingPrevRank() const {
  return topo_.ring_prev != nullptr ? topo_.ring_prev->rank : -1;
}

void EngineBase::TrackerPrint(const std::string &msg) {
  if (tracker_.uri == "NULL") {
    utils::Printf("%s", msg.c_str());
    return;
  }
  net::TrackerClient(&tracker_).Print(rank_, world_size_, msg);
}

void EngineBase::SetStream(void *stream) {
  user_stream_ = stream;
  if (dev_) dev_->SetUserStream(static_cast<hipStream_t>(stream));
}

bool EngineBase::OnDevice(const void *p) const { return dev_ && dev_->IsDevicePtr(p); }

bool EngineBase::PeerFailureProbe() const {
  for (const auto &l : topo_.links) {
    if (!l->sock.IsClosed() && l->sock.PeerHungUp()) return true;
  }
  return false;
}

void EngineBase::ReportStatus() const {
  if (hadoop_mode_) {
    fprintf(stderr, "reporter:status:Rabit Phase[%03d] Operation %03d\n", version_number_,
            seq_counter_);
  }
}

Status EngineBase::TryAllreduceHost(void *buf, const ReduceSpec &spec, const void *src) {
  const size_t bytes = spec.bytes();
  if (host_via_device_ && dev_ && GetWorldSize() > 1 && spec.builtin() && bytes >= host_dev_min_ &&
      !(spec.op == mpi::kBitwiseOR && mpi::IsFloating(spec.dtype))) {
    // large host buffer on a GPU node: stage through HBM and use the device transports (the
    // role of the reference's MPI engine: vendor collectives instead of TCP)
    device::DeviceGuard dg(dev_->device());
    Status s = EnsureDeviceComm();
    if (s != Status::kSuccess) return s;
    const bool eligible = host_stage_mode_ != 0 && dcfg_.host_stage_chunk != 0 &&
                          bytes >= 2 * dcfg_.host_stage_chunk;
    bool pipe = eligible && (host_stage_mode_ == 1 || host_stage_pipe_);
    const bool trial = eligible && host_stage_mode_ == 2 && host_stage_trial_ < 3;
    if (trial) {
      // auto: which form is faster depends on the host (memcpy threads, PCIe sharing), so time
      // one op of each after one untimed warm-up op (first touches, first transfers); every
      // rank sees the same op sequence, so the decision is collective
      pipe = host_stage_trial_ == 2;
      dev_->Scratch(bytes, 2);
      dev_->PrepareHostStager();  // allocations outside the timed op
    }
    const double t0 = utils::GetTime();
    if (pipe) {
      // pipelined: H2D, device allreduce and D2H of consecutive chunks overlap
      stats_.n_device_ops += 1;
      s = dev_->AllreduceHostStaged(buf, src != nullptr ? src : buf, spec.count, spec.dtype,
                                    spec.op, MakeProbe());
    } else {
      void *d = dev_->Scratch(bytes, 2);
      dev_->StageToDevice(d, src != nullptr ? src : buf, bytes);
      stats_.n_device_ops += 1;
      s = dev_->Allreduce(d, d, nullptr, spec.count, spec.dtype, spec.op, device::kPrepCopy, 1.0,
                          MakeProbe());
      if (s == Status::kSuccess) s = dev_->Finish(MakeProbe());
      if (s == Status::kSuccess) dev_->StageToHost(buf, d, bytes);
    }
    if (s != Status::kSuccess || !trial) return s;
    if (host_stage_trial_ >= 1) {
      host_stage_rate_[host_stage_trial_ - 1] =
          static_cast<double>(bytes) / (utils::GetTime() - t0) / 1e9;
    }
    if (++host_stage_trial_ == 3) {
      // the slowest rank's rate of each form decides, the same way everywhere
      double inv[2] = {1.0 / host_stage_rate_[0], 1.0 / host_stage_rate_[1]};
      s = host_->Allreduce(inv, sizeof(double), 2, coll::HostReducer(mpi::kDouble, mpi::kMax));
      if (s != Status::kSuccess) {
        host_stage_trial_ = 0;  // decide again after the recovery
        return s;
      }
      host_stage_rate_[0] = 1.0 / inv[0];
      host_stage_rate_[1] = 1.0 / inv[1];
      host_stage_pipe_ = inv[1] < inv[0];
      if (debug_ || rank_ == 0) {
        utils::HandleLogInfo("[xrabit] host staging: whole copies %.2f GB/s, pipelined %.2f GB/s "
                             "-> %s\n", host_stage_rate_[0], host_stage_rate_[1],
                             host_stage_pipe_ ? "pipelined" : "whole copies");
      }
    }
    return Status::kSuccess;
  }
  ReduceFn red = spec.host_red;
  if (spec.builtin()) {
    ReduceFn fast = coll::HostReducer(static_cast<mpi::DataType>(spec.dtype),
                                      static_cast<mpi::OpType>(spec.op));
    if (fast != nullptr) red = fast;
  }
  utils::Check(red != nullptr, "Allreduce: no reducer for dtype %d op %d", spec.dtype, spec.op);
  if (UseShm(bytes)) {
    Status s = EnsureShm();
    if (s != Status::kSuccess) return s;
    if (shm_ != nullptr) {
      stats_.n_shm_ops += 1;
      return shm_->Allreduce(src != nullptr ? src : buf, buf, spec.type_nbytes, spec.count, red,
                             MakeProbe());
    }
  }
  return host_->Allreduce(buf, spec.type_nbytes, spec.count, red, src);
}

Status EngineBase::EnsureShm() {
  if (shm_decided_) return Status::kSuccess;
  const int n = GetWorldSize();
  std::unique_ptr<coll::ShmGroup> g(
      new coll::ShmGroup(shm_stage_, timeout_enabled_ ? timeout_sec_ : 1800.0));
  const size_t rb = sizeof(coll::ShmRecord);
  std::vector<coll::ShmRecord> all(n);
  std::memset(all.data(), 0, rb * n);
  all[rank_] = g->local();
  Status s = host_->RingAllgather(all.data(), rb * n, rb * rank_, rb * (rank_ + 1), rb);
  if (s != Status::kSuccess) return s;
  std::string why;
  int ok = n <= coll::kMaxShmRanks && g->ok() && g->Open(all, rank_, &why) ? 1 : 0;
  s = host_->Allreduce(&ok, sizeof(int), 1, coll::HostReducer(mpi::kInt, mpi::kMin));
  if (s != Status::kSuccess) return s;
  if (ok) {
    s = g->Seal(MakeProbe());
    if (s != Status::kSuccess) return s;
    shm_ = std::move(g);
  } else if (debug_) {
    utils::HandleLogInfo("[%d] shared-memory transport off for this epoch%s%s\n", rank_,
                         why.empty() ? "" : ": ", why.c_str());
  }
  shm_decided_ = true;
  return Status::kSuccess;
}

Status EngineBase::TryAllreduceDevice(const void *src, void *dst, const ReduceSpec &spec,
                                      void *dst2, int prep, double alpha, bool host_wait) {
  const size_t bytes = spec.bytes();
  if (bytes == 0) return Status::kSuccess;
  if (dst2 == dst) dst2 = nullptr;
  device::DeviceGuard dg(dev_->device());
  bool rccl_ok = spec.builtin() && spec.dtype <= mpi::kBFloat16;
  if (spec.builtin() && spec.op == mpi::kBitwiseOR &&
      mpi::IsFloating(spec.dtype)) {
    utils::Error("BitOR is not defined for floating point types");
  }
  dev_->EnterFromUser();
  if (spec.dev_red != nullptr) {
    // user-defined device reduction: same transports, the user's kernel reduces
    utils::Check(prep == device::kPrepCopy, "fused prepare needs a built-in reduction");
    stats_.n_device_ops += 1;
    trace::Scope ts("device_allreduce", rank_, version_number_, seq_counter_, bytes, 1);
    if (GetWorldSize() == 1 && !world1_transport_) {
      dev_->CopyDeviceAsync(dst, src, bytes);
      if (dst2 != nullptr && dst2 != src) dev_->CopyDeviceAsync(dst2, src, bytes);
      return dev_->Finish(MakeProbe(), false);  // no peer can fail: stream-ordered, no host wait
    }
    Status s = EnsureDeviceComm();
    if (s != Status::kSuccess) return s;
    MaybeInjectDeviceHang();
    s = dev_->AllreduceCustom(src, dst, dst2, spec.count, spec.type_nbytes, spec.dev_red,
                              MakeProbe());
    if (s != Status::kSuccess) return s;
    return dev_->Finish(MakeProbe());
  }
  if (!rccl_ok) {
    // user-defined reducer (host function): stage through the plane's reusable page-locked
    // buffer (DMA at PCIe rate, no allocation per op), reduce on the host, copy back
    utils::Check(prep == device::kPrepCopy, "fused prepare needs a built-in reduction");
    void *tmp = dev_->PinnedScratch(bytes);
    dev_->StageToHost(tmp, src, bytes);
    Status s = TryAllreduceHost(tmp, spec);
    if (s != Status::kSuccess) return s;
    dev_->StageToDevice(dst, tmp, bytes);
    if (dst2 != nullptr) dev_->CopyDeviceAsync(dst2, dst, bytes);
    return dev_->Finish(MakeProbe());
  }
  stats_.n_device_ops += 1;
  trace::Scope ts("device_allreduce", rank_, version_number_, seq_counter_, bytes, 1);
  if (GetWorldSize() == 1 && !world1_transport_) {
    // a one-rank reduction is the identity: only materialise it where it was asked for
    if (prep != device::kPrepCopy) {
      device::CheckHip(device::LaunchPrepare(dst, dst2, src, spec.count, spec.dtype, prep, alpha,
                                             dev_->stream()),
                       "LaunchPrepare");
    } else {
      dev_->CopyDeviceAsync(dst, src, bytes);
      if (dst2 != nullptr && dst2 != src) dev_->CopyDeviceAsync(dst2, src, bytes);
    }
    // one rank: nothing can fail remotely, so the op is stream-ordered like any HIP library
    // call (the host does not wait; later work on the caller's stream sees the result)
    return dev_->Finish(MakeProbe(), false);
  }
  Status s = EnsureDeviceComm();
  if (s != Status::kSuccess) return s;
  MaybeInjectDeviceHang();
  s = dev_->Allreduce(src, dst, dst2, spec.count, spec.dtype, spec.op, prep, alpha, MakeProbe());
  if (s != Status::kSuccess) return s;
  return dev_->Finish(MakeProbe(), host_wait);
}

Status EngineBase::TryBroadcast(void *buf, size_t size, int root, void *dev_log) {
  if (size == 0) return Status::kSuccess;
  if (!OnDevice(buf)) {
    if (GetWorldSize() == 1) return Status::kSuccess;
    if (UseShm(size)) {
      Status s = EnsureShm();
      if (s != Status::kSuccess) return s;
      if (shm_ != nullptr) {
        stats_.n_shm_ops += 1;
        return shm_->Broadcast(buf, size, root, MakeProbe());
      }
    }
    return host_->TreeBroadcast(buf, size, root);
  }
  device::DeviceGuard dg(dev_->device());
  if (GetWorldSize() == 1 && !world1_transport_) {
    if (dev_log != nullptr) {
      dev_->EnterFromUser();
      dev_->CopyDeviceAsync(dev_log, buf, size);
      return dev_->Finish(MakeProbe(), false);
    }
    return Status::kSuccess;
  }
  Status s = EnsureDeviceComm();
  if (s != Status::kSuccess) return s;
  stats_.n_device_ops += 1;
  dev_->EnterFromUser();
  MaybeInjectDeviceHang();
  s = dev_->Broadcast(buf, size, root, MakeProbe(), dev_log);
  if (s != Status::kSuccess) return s;
  return dev_->Finish(MakeProbe());
}

Status EngineBase::TryAllgather(void *buf, size_t total, size_t begin, size_t end,
                                size_t prev_size, void *dev_log) {
  if (total == 0) return Status::kSuccess;
  if (!OnDevice(buf)) {
    if (GetWorldSize() == 1) return Status::kSuccess;
    if (UseShm(total)) {
      Status s = EnsureShm();
      if (s != Status::kSuccess) return s;
      if (shm_ != nullptr) {
        // every rank needs every slice: exchange (begin, size) pairs over the host ring first
        const int n = GetWorldSize();
        std::vector<uint64_t> meta(2 * n, 0);
        meta[2 * rank_] = begin;
        meta[2 * rank_ + 1] = end - begin;
        s = host_->RingAllgather(meta.data(), meta.size() * 8, 16 * rank_, 16 * rank_ + 16, 16);
        if (s != Status::kSuccess) return s;
        std::vector<size_t> b(n), z(n);
        for (int r = 0; r < n; ++r) {
          b[r] = static_cast<size_t>(meta[2 * r]);
          z[r] = static_cast<size_t>(meta[2 * r + 1]);
        }
        stats_.n_shm_ops += 1;
        return shm_->AllgatherV(buf, total, b, z, MakeProbe());
      }
    }
    return host_->RingAllgather(buf, total, begin, end, prev_size);
  }
  device::DeviceGuard dg(dev_->device());
  if (GetWorldSize() == 1 && !world1_transport_) {
    if (dev_log != nullptr) {
      dev_->EnterFromUser();
      dev_->CopyDeviceAsync(dev_log, buf, total);
      return dev_->Finish(MakeProbe(), false);
    }
    return Status::kSuccess;
  }
  Status s = EnsureDeviceComm();
  if (s != Status::kSuccess) return s;
  if (allgather_resolve_ && !dev_->AllgatherNeedsLayout(total)) {
    // the direct transport: every window's barrier publishes this rank's slice and the gather
    // kernel resolves the owners on the device -- no host round before the op
    stats_.n_device_ops += 1;
    dev_->EnterFromUser();
    MaybeInjectDeviceHang();
    s = dev_->AllgatherResolved(buf, total, begin, end - begin, dev_log);
    if (s != Status::kSuccess) return s;
    return dev_->Finish(MakeProbe());
  }
  // RCCL's grouped broadcasts need every rank's slice: exchange (begin, size) over the host ring
  const int n = GetWorldSize();
  std::vector<uint64_t> meta(2 * n, 0);
  meta[2 * rank_] = begin;
  meta[2 * rank_ + 1] = end - begin;
  s = host_->RingAllgather(meta.data(), meta.size() * 8, 16 * rank_, 16 * rank_ + 16, 16);
  if (s != Status::kSuccess) return s;
  std::vector<size_t> b(n), z(n);
  for (int r = 0; r < n; ++r) {
    b[r] = static_cast<size_t>(meta[2 * r]);
    z[r] = static_cast<size_t>(meta[2 * r + 1]);
  }
  stats_.n_device_ops += 1;
  dev_->EnterFromUser();
  MaybeInjectDeviceHang();
  s = dev_->AllgatherV(buf, total, b, z, MakeProbe(), dev_log);
  if (s != Status::kSuccess) return s;
  return dev_->Finish(MakeProbe());
}

void EngineBase::Allreduce(void *buf, size_t type_nbytes, size_t count, ReduceFunction reducer,
                           PreprocFunction prepare_fun, void *prepare_arg, const char *,
                           const int, const char *) {
  if (prepare_fun != nullptr) prepare_fun(prepare_arg);
  if (GetWorldSize() == 1 && world1_fastpath_) return;
  ReduceSpec spec;
  spec.type_nbytes = type_nbytes;
  spec.count = count;
  spec.host_red = reducer;
  const double t0 = utils::GetTime();
  Status s = OnDevice(buf) ? TryAllreduceDevice(buf, buf, spec) : TryAllreduceHost(buf, spec);
  utils::Check(s == Status::kSuccess, "Allreduce failed: %s", net::StatusName(s));
  stats_.n_allreduce += 1;
  stats_.bytes_allreduce += static_cast<double>(spec.bytes());
  stats_.t_allreduce += utils::GetTime() - t0;
}

void EngineBase::AllreduceTyped(void *buf, size_t count, mpi::DataType dtype, mpi::OpType op,
                                ReduceFunction reducer, PreprocFunction prepare_fun,
                                void *prepare_arg, const char *, const int, const char *) {
  if (prepare_fun != nullptr) prepare_fun(prepare_arg);
  if (GetWorldSize() == 1 && world1_fastpath_) return;
  ReduceSpec spec;
  spec.type_nbytes = coll::DTypeSize(dtype);
  spec.count = count;
  spec.host_red = reducer;
  spec.dtype = dtype;
  spec.op = op;
  const double t0 = utils::GetTime();
  Status s = OnDevice(buf) ? TryAllreduceDevice(buf, buf, spec) : TryAllreduceHost(buf, spec);
  utils::Check(s == Status::kSuccess, "Allreduce failed: %s", net::StatusName(s));
  stats_.n_allreduce += 1;
  stats_.bytes_allreduce += static_cast<double>(spec.bytes());
  stats_.t_allreduce += utils::GetTime() - t0;
}

void EngineBase::AllreduceDevice(void *buf, size_t type_nbytes, size_t count,
                                 DeviceReduceLauncher *dev_reducer, ReduceFunction host_reducer,
                                 PreprocFunction prepare_fun, void *prepare_arg, const char *,
                                 const int, const char *) {
  if (prepare_fun != nullptr) prepare_fun(prepare_arg);
  if (GetWorldSize() == 1 && world1_fastpath_) return;
  ReduceSpec spec;
  spec.type_nbytes = type_nbytes;
  spec.count = count;
  spec.host_red = host_reducer;
  spec.dev_red = dev_reducer;
  const double t0 = utils::GetTime();
  Status s = OnDevice(buf) ? TryAllreduceDevice(buf, buf, spec) : TryAllreduceHost(buf, spec);
  utils::Check(s == Status::kSuccess, "Allreduce failed: %s", net::StatusName(s));
  stats_.n_allreduce += 1;
  stats_.bytes_allreduce += static_cast<double>(spec.bytes());
  stats_.t_allreduce += utils::GetTime() - t0;
}

void EngineBase::DevAllreducePrepared(void *dst, const void *src, size_t count, int dtype,
                                      int op, int prep, double alpha, const char *, const int,
                                      const char *) {
  utils::Check(OnDevice(dst) && OnDevice(src), "DevAllreducePrepared needs device buffers");
  if (GetWorldSize() == 1 && world1_fastpath_) {
    dev_->EnterFromUser();
    device::CheckHip(device::LaunchPrepare(dst, nullptr, src, count, dtype, prep, alpha,
                                           dev_->stream()),
                     "LaunchPrepare");
    utils::Check(dev_->Finish(MakeProbe()) == Status::kSuccess, "prepare failed");
    return;
  }
  ReduceSpec spec;
  spec.type_nbytes = coll::DTypeSize(static_cast<mpi::DataType>(dtype));
  spec.count = count;
  spec.dtype = dtype;
  spec.op = op;
  // the prepare pass is fused into the transport (direct: it writes the stage buffer)
  Status s = TryAllreduceDevice(src, dst, spec, nullptr, prep, alpha);
  utils::Check(s == Status::kSuccess, "Allreduce failed: %s", net::StatusName(s));
  stats_.n_allreduce += 1;
}

void EngineBase::Broadcast(void *buf, size_t size, int root, const char *, const int,
                           const char *) {
  if (GetWorldSize() == 1) return;
  const double t0 = utils::GetTime();
  Status s = TryBroadcast(buf, size, root);
  utils::Check(s == Status::kSuccess, "Broadcast failed: %s", net::StatusName(s));
  stats_.n_broadcast += 1;
  stats_.bytes_broadcast += static_cast<double>(size);
  stats_.t_broadcast += utils::GetTime() - t0;
}

void EngineBase::Allgather(void *buf, size_t total, size_t begin, size_t end, size_t prev_size,
                           const char *, const int, const char *) {
  if (GetWorldSize() == 1) return;
  const double t0 = utils::GetTime();
  Status s = TryAllgather(buf, total, begin, end, prev_size);
  utils::Check(s == Status::kSuccess, "Allgather failed: %s", net::StatusName(s));
  stats_.n_allgather += 1;
  stats_.bytes_allgather += static_cast<double>(total);
  stats_.t_allgather += utils::GetTime() - t0;
}

int EngineBase::LoadCheckPoint(Serializable *, Serializable *) { return 0; }

namespace {
/*! \brief force_local: the global tensors join the local model, the global checkpoint keeps
 *  only the metadata (the mock engine's stress test of local replication) */
void FoldIntoLocal(int *n, void *const **ptrs, const size_t **nbytes, int *nl,
                   void *const **lptrs, const size_t **lnbytes, std::vector<void *> *pbuf,
                   std::vector<size_t> *sbuf) {
  pbuf->assign(*ptrs, *ptrs + *n);
  sbuf->assign(*nbytes, *nbytes + *n);
  pbuf->insert(pbuf->end(), *lptrs, *lptrs + *nl);
  sbuf->insert(sbuf->end(), *lnbytes, *lnbytes + *nl);
  *nl = static_cast<int>(pbuf->size());
  *lptrs = pbuf->data();
  *lnbytes = sbuf->data();
  *n = 0;
}
}  // namespace

int EngineBase::DevGraphAllreduce(void *buf, size_t count, int dtype, int op,
                                  hipStream_t stream, std::string *why) {
  if (dev_ == nullptr) {
    *why = "graph allreduce needs the device plane";
    return -1;
  }
  if (GetWorldSize() == 1 && !world1_transport_) return 0;  // a one-rank reduction is identity
  device::DeviceGuard dg(dev_->device());
  if (!dev_->ready()) {
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(stream, &cs) == hipSuccess && cs != hipStreamCaptureStatusNone) {
      *why = "graph allreduce: make one eager call before capturing (it brings the device "
             "transports up)";
      return -2;
    }
    if (EnsureDeviceComm() != Status::kSuccess || !dev_->ready()) {
      *why = "graph allreduce needs a device transport (RCCL or direct)";
      return -2;
    }
  }
  const int r = dev_->GraphAllreduce(buf, count, dtype, op, stream);
  if (r == -3) *why = "graph allreduce: dtype/op not supported (BitOR)";
  if (r == -5) *why = "graph allreduce: the enqueue failed";
  if (r == 0) stats_.n_device_ops += 1;
  return r;
}

int EngineBase::DevProbeAllreduce(void *buf, size_t count, int dtype, int op, int mode) {
  if (dev_ == nullptr) return -2;
  utils::Check(mode >= 0 && mode <= 2, "probe allreduce: mode %d not in [0, 2]", mode);
  utils::Check(OnDevice(buf), "probe allreduce: the buffer must be in HBM");
  ReduceSpec spec;
  spec.type_nbytes = coll::DTypeSize(static_cast<mpi::DataType>(dtype));
  spec.count = count;
  spec.dtype = dtype;
  spec.op = op;
  void *dst = buf, *dst2 = nullptr;
  if (mode == 1) {
    dst = dev_->Scratch(spec.bytes(), device::DevicePlane::kCalibScratch);
    dst2 = buf;
  }
  const Status s = TryAllreduceDevice(buf, dst, spec, dst2, device::kPrepCopy, 1.0, mode != 2);
  return s == Status::kSuccess ? 0 : -1;
}

int EngineBase::DevLinkProbe(size_t bytes, double *out) {
  if (dev_ == nullptr || GetWorldSize() < 2) return -2;
  device::DeviceGuard dg(dev_->device());
  if (EnsureDeviceComm() != Status::kSuccess) return -1;
  if (!dev_->has_peers()) return -2;
  return dev_->LinkProbe(bytes, out) == Status::kSuccess ? 0 : -1;
}

void EngineBase::DevCheckPoint(int n, void *const *ptrs, const size_t *nbytes,
                               const std::string &meta, int nl, void *const *lptrs,
                               const size_t *lnbytes) {
  utils::Check(dev_ != nullptr, "device checkpoint needs the device plane");
  std::vector<void *> pbuf;
  std::vector<size_t> sbuf;
  if (ForceLocal()) FoldIntoLocal(&n, &ptrs, &nbytes, &nl, &lptrs, &lnbytes, &pbuf, &sbuf);
  for (int i = 0; i < n; ++i) {
    utils::Check(nbytes[i] == 0 || OnDevice(ptrs[i]), "device checkpoint: buffer %d not in HBM", i);
  }
  for (int i = 0; i < nl; ++i) {
    utils::Check(lnbytes[i] == 0 || OnDevice(lptrs[i]),
                 "device checkpoint: local buffer %d not in HBM", i);
  }
  device::DeviceGuard dg(dev_->device());
  if (!dev_ckpt_) {
    dev_ckpt_.reset(new device::DeviceCheckpoint(dev_.get()));
    dev_ckpt_->set_mirror_mode(ckpt_mirror_mode_);
    dev_ckpt_->set_mirror_engine(MirrorEngine(), mirror_ctas_);
    dev_ckpt_->set_mirror_low_priority(mirror_low_prio_);
    dev_ckpt_->set_slots(ckpt_slots_, ckpt_3slot_max_);
  }
  trace::Scope ts("device_snapshot", rank_, version_number_, seq_counter_, 0, 1);
  const Serializable *snap = dev_ckpt_->Snapshot(n, ptrs, nbytes, meta);
  dev_local_.owner = this;
  dev_local_.Set(nl, lptrs, lnbytes);
  this->CheckPointDevice(snap, nl > 0 ? &dev_local_ : nullptr);
}

int EngineBase::DevLoadCheckPoint(int n, void *const *ptrs, const size_t *nbytes,
                                  std::string *meta, int nl, void *const *lptrs,
                                  const size_t *lnbytes) {
  utils::Check(dev_ != nullptr, "device checkpoint needs the device plane");
  std::vector<void *> pbuf;
  std::vector<size_t> sbuf;
  if (ForceLocal()) FoldIntoLocal(&n, &ptrs, &nbytes, &nl, &lptrs, &lnbytes, &pbuf, &sbuf);
  device::DeviceGuard dg(dev_->device());
  if (!dev_ckpt_) {
    dev_ckpt_.reset(new device::DeviceCheckpoint(dev_.get()));
    dev_ckpt_->set_mirror_mode(ckpt_mirror_mode_);
    dev_ckpt_->set_mirror_engine(MirrorEngine(), mirror_ctas_);
    dev_ckpt_->set_mirror_low_priority(mirror_low_prio_);
    dev_ckpt_->set_slots(ckpt_slots_, ckpt_3slot_max_);
  }
  dev_local_.owner = this;
  dev_local_.Set(nl, lptrs, lnbytes);
  const int version =
      this->LoadCheckPoint(dev_ckpt_->Loader(n, ptrs, nbytes), nl > 0 ? &dev_local_ : nullptr);
  if (version > 0 && meta != nullptr) *meta = dev_ckpt_->loaded_meta();
  return version;
}

void EngineBase::DeviceLocalModel::Save(Stream *fo) const {
  // host staging (engines without an HBM replica store)
  std::vector<char> tmp;
  for (size_t i = 0; i < ptrs.size(); ++i) {
    tmp.resize(nbytes[i]);
    if (nbytes[i] != 0) owner->dev_->StageToHost(tmp.data(), ptrs[i], nbytes[i]);
    fo->Write(tmp.data(), nbytes[i]);
  }
}

void EngineBase::DeviceLocalModel::Load(Stream *fi) {
  std::vector<char> tmp;
  for (size_t i = 0; i < ptrs.size(); ++i) {
    tmp.resize(nbytes[i]);
    utils::Check(fi->Read(tmp.data(), nbytes[i]) == nbytes[i], "device local model: short read");
    if (nbytes[i] != 0) owner->dev_->StageToDevice(ptrs[i], tmp.data(), nbytes[i]);
  }
}

void EngineBase::CheckPoint(const Serializable *, const Serializable *) {
  version_number_ += 1;
  stats_.n_checkpoint += 1;
}

void EngineBase::LazyCheckPoint(const Serializable *) {
  version_number_ += 1;
  stats_.n_checkpoint += 1;
}

std::string EngineBase::PhasesJson() const {
  const EngineStats::Phases &p = stats_.phases;
  std::ostringstream os;
  os << "{\"detect\":" << p.detect << ",\"drop_links\":" << p.drop_links
     << ",\"relink\":" << p.relink << ",\"records\":" << p.records
     << ",\"peer_open\":" << p.peer_open << ",\"rccl\":" << p.rccl << ",\"tune\":" << p.tune
     << ",\"calibration\":" << p.calibration << ",\"adopt\":" << p.adopt
     << ",\"load_checkpoint\":" << p.load_checkpoint << ",\"replay\":" << p.replay
     << ",\"serve_load\":" << p.serve_load << ",\"serve_replay\":" << p.serve_replay
     << ",\"bringups\":" << p.bringups << ",\"calibrations\":" << p.calibrations
     << ",\"adoptions\":" << p.adoptions << ",\"replays\":" << p.replays
     << ",\"serves\":" << p.serves
     << ",\"process_start_to_init\":" << stats_.t_process_start_to_init << "}";
  return os.str();
}

std::string EngineBase::StatsJson() const {
  std::ostringstream os;
  const EngineStats &s = stats_;
  os << "{\"engine\":\"" << EngineName() << "\",\"rank\":" << rank_
     << ",\"world_size\":" << GetWorldSize() << ",\"version\":" << version_number_
     << ",\"device\":" << GetDevice() << ",\"device_epoch\":" << (dev_ ? dev_->epoch() : 0)
     << ",\"device_rccl\":" << (dev_ && dev_->has_comm() ? 1 : 0)
     << ",\"device_direct\":" << (dev_ && dev_->has_peers() ? 1 : 0)
     << ",\"zero_copy_chunks\":" << (dev_ ? dev_->zero_copy_chunks() : 0)
     << ",\"zero_copy_registry\":" << (dev_ ? dev_->RegistryJson() : std::string("{}"))
     << ",\"resolved_allgathers\":" << (dev_ ? dev_->resolved_allgathers() : 0)
     << ",\"recovery_phases_s\":" << PhasesJson()
     << ",\"calib_matrix\":" << calib_matrix_json_
     << ",\"rccl_init_refused\":" << (dev_ ? dev_->init_refused() : 0)
     << ",\"rccl_live_abandoned\":" << device::DevicePlane::LiveAbandonedInits()
     << ",\"oneshot_ops\":" << (dev_ ? dev_->oneshot_ops() : 0)
     << ",\"fused_chunks\":" << (dev_ ? dev_->fused_chunks() : 0)
     << ",\"fused_oneshots\":" << (dev_ ? dev_->fused_oneshots() : 0)
     << ",\"fused_grid\":" << (dev_ ? dev_->fused_grid() : 0)
     << ",\"symmetric_heap_used\":" << (dev_ ? dev_->sym_heap_used() : 0)
     << ",\"device_direct_min\":"
     << (dev_ && dev_->has_peers() ? static_cast<double>(dev_->direct_min_bytes()) : -1.0)
     << ",\"device_direct_below\":" << (dev_ ? dev_->direct_below_bytes() : 0)
     << ",\"calib_us\":[" << calib_.rccl_small * 1e6 << "," << calib_.rccl_big * 1e6 << ","
     << calib_.direct_small * 1e6 << "," << calib_.direct_big * 1e6 << "]"
     << ",\"calib_push_us\":" << calib_.push_big * 1e6
     << ",\"calib_bcast_us\":[" << calib_bcast_[0] * 1e6 << "," << calib_bcast_[1] * 1e6 << ","
     << calib_bcast_[2] * 1e6 << "," << calib_bcast_[3] * 1e6 << "]"
     << ",\"bcast_routed\":" << (dev_ && dev_->bcast_routed() ? 1 : 0)
     << ",\"bcast_direct_min\":"
     << (dev_ && dev_->bcast_routed() ? static_cast<double>(dev_->bcast_min_bytes()) : -1.0)
     << ",\"bcast_direct_below\":" << (dev_ ? dev_->bcast_below_bytes() : 0)
     << ",\"direct_bcast_ops\":" << (dev_ ? dev_->bcast_ops() : 0)
     << ",\"direct_bcast_chunks\":" << (dev_ ? dev_->bcast_chunks() : 0)
     << ",\"host_staged_ops\":" << (dev_ ? dev_->host_staged_ops() : 0)
     << ",\"host_stage_threads\":" << (dev_ ? dev_->host_stage_threads() : 0)
     << ",\"host_stage\":" << (dev_ ? dev_->HostStageJson() : std::string("{}"))
     << ",\"host_stage_choice\":\""
     << (host_stage_mode_ == 0 ? "whole"
                               : (host_stage_mode_ == 1 ? "pipelined"
                                                        : (host_stage_trial_ < 3
                                                               ? "pending"
                                                               : (host_stage_pipe_ ? "pipelined"
                                                                                   : "whole"))))
     << "\",\"host_stage_rates_GBps\":[" << host_stage_rate_[0] << "," << host_stage_rate_[1] << "]"
     << ",\"calib_forms_us\":[" << calib_form_us_[0] << "," << calib_form_us_[1] << ","
     << calib_form_us_[2] << "," << calib_form_us_[3] << "," << calib_form_us_[4] << "]"
     << ",\"direct_pipeline\":" << (dev_ && dev_->pipeline() ? 1 : 0)
     << ",\"pipelined_ops\":" << (dev_ ? dev_->pipelined_ops() : 0)
     << ",\"pipelined_rounds\":" << (dev_ ? dev_->pipelined_rounds() : 0)
     << ",\"graph_direct_ops\":" << (dev_ ? dev_->graph_direct_ops() : 0)
     << ",\"direct_fused\":" << (dev_ && dev_->fused() ? 1 : 0)
     << ",\"calib_heap_src\":" << (calib_heap_src_ ? 1 : 0)
     << ",\"rccl_init_failed\":" << rccl_failed_
     << ",\"rccl_calls\":" << (dev_ ? dev_->rccl_calls() : 0)
     << ",\"rccl_settled\":" << (dev_ ? dev_->rccl_settled() : 0)
     << ",\"rccl_aborts\":" << (dev_ ? dev_->rccl_aborts() : 0)
     << ",\"rccl_init_abandoned\":" << (dev_ ? dev_->init_abandoned() : 0)
     << ",\"done_word_waits\":" << (dev_ ? dev_->done_words() : 0)
     << ",\"rccl_tuning\":" << rccl_tune_json_
     << ",\"direct_push\":" << (dev_ && dev_->direct_push() ? 1 : 0)
     << ",\"push_chunks\":" << (dev_ ? dev_->push_chunks() : 0)
     << ",\"peer_links\":" << (dev_ ? dev_->PeerLinksJson() : std::string("[]"));
  double phase[device::PeerGroup::kPhases];
  uint64_t nphase = 0;
  if (dev_ && dev_->DirectPhaseUs(phase, &nphase)) {
    os << ",\"direct_timed_ops\":" << nphase << ",\"direct_phase_us\":{\"stage\":" << phase[0]
       << ",\"barrier1\":" << phase[1] << ",\"reduce\":" << phase[2] << ",\"barrier2\":" << phase[3]
       << ",\"gather\":" << phase[4] << "}";
  }
  os << ",\"n_allreduce\":" << s.n_allreduce << ",\"n_broadcast\":" << s.n_broadcast
     << ",\"n_allgather\":" << s.n_allgather << ",\"n_checkpoint\":" << s.n_checkpoint
     << ",\"n_device_ops\":" << s.n_device_ops << ",\"n_shm_ops\":" << s.n_shm_ops
     << ",\"ckpt_mirrors\":" << (dev_ckpt_ ? dev_ckpt_->mirrors() : 0)
     << ",\"ckpt_mirrors_deferred\":" << (dev_ckpt_ ? dev_ckpt_->mirrors_deferred() : 0)
     << ",\"ckpt_mirror_engine\":" << (dev_ckpt_ ? dev_ckpt_->mirror_engine() : MirrorEngine())
     << ",\"ckpt_slots\":" << (dev_ckpt_ ? dev_ckpt_->slots() : 0)
     << ",\"ckpt_hbm_bytes\":" << (dev_ckpt_ ? dev_ckpt_->reserved_bytes() : 0)
     << ",\"ckpt_pinned_bytes\":" << (dev_ckpt_ ? dev_ckpt_->pinned_bytes() : 0)
     << ",\"n_recovered_ops\":" << s.n_recovered_ops
     << ",\"n_recover_events\":" << s.n_recover_events << ",\"n_consensus\":" << s.n_consensus
     << ",\"n_consensus_elided\":" << s.n_consensus_elided
     << ",\"n_device_replays\":" << s.n_device_replays
     << ",\"n_device_ckpt_loads\":" << s.n_device_ckpt_loads
     << ",\"bytes_local_in\":" << s.bytes_local_in << ",\"bytes_replay_in\":" << s.bytes_replay_in
     << ",\"bytes_ckpt_in\":" << s.bytes_ckpt_in
     << ",\"bytes_allreduce\":" << s.bytes_allreduce
     << ",\"bytes_broadcast\":" << s.bytes_broadcast
     << ",\"bytes_allgather\":" << s.bytes_allgather << ",\"t_allreduce\":" << s.t_allreduce
     << ",\"t_broadcast\":" << s.t_broadcast << ",\"t_allgather\":" << s.t_allgather
     << ",\"t_checkpoint\":" << s.t_checkpoint << ",\"t_consensus\":" << s.t_consensus
     << ",\"t_recover\":" << s.t_recover
     << ",\"n_spilled_results\":" << s.n_spilled_results
     << ",\"n_spilled_replays\":" << s.n_spilled_replays
     << ",\"bytes_spilled\":" << s.bytes_spilled
     << ",\"device_log_bytes\":" << (dev_ ? dev_->arena()->used() : 0)
     << ",\"device_spill_bytes\":"
     << (dev_ && dev_->spill_arena() ? dev_->spill_arena()->used() : 0) << "}";
  return os.str();
}
}  // namespace engine
}  // namespace rabit
