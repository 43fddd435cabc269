/*!
 * \file engine_robust.cc
 * \brief Fault-tolerant engine: collectives, checkpoints, result log, bootstrap cache,
 *        watchdog.  The recovery protocol itself is in recovery.cc.
 */
#include "engine/engine_robust.h"

#include <sys/mman.h>

#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <cstdlib>
#include <cstring>

#include "core/exit.h"
#include "core/trace.h"
#include "core/wait_state.h"
#include "device/kernels.h"
#include "rabit/internal/io.h"
#include "rabit/internal/timer.h"
#include "rabit/internal/utils.h"

namespace rabit {
namespace engine {

// ------------------------------------------------------------------ ResultLog
EngineRobust::ResultLog::HostArena::~HostArena() {
  for (auto &c : chunks_) std::free(c.base);
}

void *EngineRobust::ResultLog::HostArena::Alloc(size_t bytes) {
  const size_t need = (bytes + 63) & ~static_cast<size_t>(63);
  while (cur_ < chunks_.size()) {
    Chunk &c = chunks_[cur_];
    if (c.size - c.used >= need) {
      void *p = c.base + c.used;
      c.used += need;
      return p;
    }
    if (cur_ + 1 == chunks_.size()) break;
    ++cur_;
  }
  Chunk c;
  // big chunks are 2 MiB aligned and backed by transparent huge pages where the kernel allows
  // it: a result log chunk is written once per op in full, and 4 KiB first-touch faults on
  // fresh chunks cost as much as the copy itself.  Logs of short keys use small chunks.
  constexpr size_t kHuge = 2u << 20;
  const size_t want = std::max(need, min_chunk_);
  if (want >= kHuge) {
    c.size = (want + kHuge - 1) & ~(kHuge - 1);
    c.base = static_cast<char *>(std::aligned_alloc(kHuge, c.size));
    if (c.base != nullptr) (void)madvise(c.base, c.size, MADV_HUGEPAGE);
  } else {
    c.size = (want + 63) & ~static_cast<size_t>(63);
    c.base = static_cast<char *>(std::aligned_alloc(64, c.size));
  }
  utils::Check(c.base != nullptr, "out of host memory for the result log (%zu bytes)", c.size);
  c.used = need;
  chunks_.push_back(c);
  cur_ = chunks_.size() - 1;
  return c.base;
}

void EngineRobust::ResultLog::HostArena::PopTo(void *ptr) {
  char *p = static_cast<char *>(ptr);
  for (size_t i = 0; i < chunks_.size(); ++i) {
    Chunk &c = chunks_[i];
    if (p >= c.base && p < c.base + c.size) {
      c.used = static_cast<size_t>(p - c.base);
      for (size_t j = i + 1; j < chunks_.size(); ++j) chunks_[j].used = 0;
      cur_ = i;
      return;
    }
  }
}

void EngineRobust::ResultLog::HostArena::Reset() {
  for (auto &c : chunks_) c.used = 0;
  cur_ = 0;
}

void EngineRobust::ResultLog::Clear() {
  entries_.clear();
  host_.Reset();
  if (arena_ != nullptr) arena_->Reset();
  if (spill_ != nullptr) spill_->Reset();
}

void *EngineRobust::ResultLog::AllocTemp(size_t size, bool device) {
  utils::Assert(size != 0, "cannot log a zero-size result");
  temp_ = Entry{-1, size, device, nullptr, false};
  if (device) {
    utils::Check(arena_ != nullptr, "device result without a device arena");
    void *p = arena_->Alloc(size);
    if (p == nullptr && spill_ != nullptr) {
      // the HBM log reached rabit_device_log_cap (or HBM is full): keep this result in pinned
      // host memory, like the reference's unbounded host log (allreduce_robust.h:324-388)
      p = spill_->Alloc(size);
      if (p != nullptr) {
        temp_.on_device = false;
        temp_.spilled = true;
        n_spilled_ += 1;
      }
    }
    utils::Check(p != nullptr,
                 "device result log is full (%zu bytes in HBM since the last checkpoint, %zu "
                 "spilled to host); checkpoint more often or raise rabit_device_log_cap / "
                 "rabit_device_spill_cap",
                 arena_->used(), spill_ != nullptr ? spill_->used() : size_t(0));
    temp_.ptr = p;
    return p;
  }
  temp_.ptr = host_.Alloc(size);
  return temp_.ptr;
}

void EngineRobust::ResultLog::PushTemp(int seqno, size_t size) {
  utils::Assert(size == temp_.size, "PushTemp: size differs from AllocTemp");
  if (!entries_.empty()) {
    utils::Assert(entries_.back().seqno < seqno, "PushTemp: sequence numbers must increase");
  }
  temp_.seqno = seqno;
  entries_.push_back(temp_);
}

const EngineRobust::ResultLog::Entry *EngineRobust::ResultLog::Query(int seqno) const {
  auto it = std::lower_bound(entries_.begin(), entries_.end(), seqno,
                             [](const Entry &e, int s) { return e.seqno < s; });
  if (it == entries_.end() || it->seqno != seqno) return nullptr;
  return &*it;
}

void EngineRobust::ResultLog::DropLast() {
  utils::Assert(!entries_.empty(), "nothing to drop");
  const Entry e = entries_.back();
  entries_.pop_back();
  if (e.spilled) {
    if (spill_ != nullptr) spill_->PopTo(e.ptr);
  } else if (e.on_device) {
    if (arena_ != nullptr) arena_->PopTo(e.ptr);
  } else {
    host_.PopTo(e.ptr);
  }
}

// ------------------------------------------------------------------ consensus reducer
void EngineRobust::ActionSummary::Reducer(const void *src_, void *dst_, int len,
                                          const MPI::Datatype &) {
  const ActionSummary *src = static_cast<const ActionSummary *>(src_);
  ActionSummary *dst = static_cast<ActionSummary *>(dst_);
  for (int i = 0; i < len; ++i) {
    const uint32_t min_seq = std::min(src[i].seqno(), dst[i].seqno());
    const uint32_t max_cache = std::max(src[i].seqno(kCache), dst[i].seqno(kCache));
    const int flags = src[i].flag() | dst[i].flag() |
                      (src[i].seqno() != dst[i].seqno() ? kDiffSeq : 0);
    const int role = src[i].flag(kCache) & dst[i].flag(kCache);
    dst[i] = ActionSummary(flags, role, min_seq, max_cache);
  }
}

// ------------------------------------------------------------------ lifecycle
EngineRobust::EngineRobust() {
  env_vars_.push_back("rabit_global_replica");
  env_vars_.push_back("rabit_local_replica");
}

EngineRobust::~EngineRobust() { StopWatchdog(); }

void EngineRobust::SetParam(const char *name, const char *val) {
  EngineBase::SetParam(name, val);
  if (!strcmp(name, "rabit_global_replica")) num_global_replica_ = atoi(val);
  if (!strcmp(name, "rabit_local_replica")) num_local_replica_ = atoi(val);
  if (!strcmp(name, "rabit_elide_consensus")) elide_consensus_ = utils::StringToBool(val);
  if (!strcmp(name, "rabit_recover_stagger_ms")) {
    recover_stagger_ms_ = atof(val);
    utils::Check(recover_stagger_ms_ >= 0, "rabit_recover_stagger_ms should be non negative");
  }
  if (!strcmp(name, "rabit_hang_timeout_sec")) {
    hang_timeout_sec_ = atof(val);
    utils::Check(hang_timeout_sec_ >= 0, "rabit_hang_timeout_sec should be non negative");
  }
}

bool EngineRobust::Init(int argc, char *argv[]) {
  if (!EngineBase::Init(argc, argv)) return false;
  if (bootstrap_cache_) utils::HandleLogInfo("[EXPERIMENTAL] bootstrap cache enabled\n");
  checkpoint_loaded_ = false;
  result_buffer_round_ =
      num_global_replica_ == 0 ? -1 : std::max(GetWorldSize() / num_global_replica_, 1);
  if (dev_) resbuf_.SetArena(dev_->arena(), dev_->spill_arena());
  // the bootstrap cache logs keys (short strings) and small early results
  lookupbuf_.SetHostChunk(64u << 10);
  cachebuf_.SetHostChunk(1u << 20);
  if (timeout_enabled_ || hang_timeout_sec_ > 0 || (dev_ && dev_wait_limit_sec_ > 0)) {
    StartWatchdog();
  }
  return true;
}

bool EngineRobust::Shutdown() {
  try {
    if (GetWorldSize() > 1 || !world1_fastpath_) {
      // a pseudo checkpoint keeps serving late / recovering peers before everyone leaves
      utils::Check(RecoverExec(nullptr, 0, ActionSummary::kCheckPoint, ActionSummary::kSpecialOp,
                               cur_cache_seq_, "Shutdown"),
                   "Shutdown: checkpoint must return true");
      resbuf_.Clear();
      seq_counter_ = 0;
      cachebuf_.Clear();
      cur_cache_seq_ = 0;
      lookupbuf_.Clear();
      utils::Check(RecoverExec(nullptr, 0, ActionSummary::kCheckAck, ActionSummary::kSpecialOp,
                               cur_cache_seq_, "Shutdown"),
                   "Shutdown: check ack must return true");
    }
    recovering_since_.store(0.0);
    StopWatchdog();
    return EngineBase::Shutdown();
  } catch (const std::exception &e) {
    fprintf(stderr, "xrabit: shutdown failed: %s\n", e.what());
    return false;
  }
}

void EngineRobust::InitAfterException() {
  // drop every link and rejoin through the tracker, as after a failure
  for (auto &l : topo_.links) l->sock.Close();
  if (dev_) dev_->AbortComm();
  ResetShm();
  fast_mode_ = false;
  ReconnectLinks("recover");
}

// ------------------------------------------------------------------ helpers
std::string EngineRobust::CallKey(const char *file, int line, const char *caller,
                                  const std::string &shape) {
  return std::string(file) + "::" + std::to_string(line) + "::" + caller + shape;
}

void EngineRobust::ApplyRetention() {
  const int last = resbuf_.LastSeqNo();
  if (last != -1 &&
      (result_buffer_round_ == -1 || last % result_buffer_round_ != rank_ % result_buffer_round_)) {
    resbuf_.DropLast();
  }
}

void EngineRobust::CopyAny(void *dst, bool dst_dev, const void *src, bool src_dev, size_t n) {
  if (n == 0 || dst == src) return;
  if (!dst_dev && !src_dev) {
    std::memcpy(dst, src, n);
    return;
  }
  dev_->EnterFromUser();
  dev_->CopyAsync(dst, src, n);
  utils::Check(dev_->Finish(MakeProbe(), true) == Status::kSuccess, "device copy failed");
}

void EngineRobust::SpillResult(void *slot, const void *src, size_t n) {
  // stream-ordered D2H: later work on the caller's stream (which may overwrite src) runs after
  // it; a reader of the slot on the host synchronises first (TryGetResult)
  dev_->EnterFromUser();
  dev_->CopyAsync(slot, src, n);
  dev_->Finish(MakeProbe(), false);
  stats_.n_spilled_results += 1;
  stats_.bytes_spilled += static_cast<double>(n);
}

// ------------------------------------------------------------------ collectives
void EngineRobust::Allreduce(void *buf, size_t type_nbytes, size_t count,
                             ReduceFunction reducer, PreprocFunction prepare_fun,
                             void *prepare_arg, const char *_file, const int _line,
                             const char *_caller) {
  ReduceSpec spec;
  spec.type_nbytes = type_nbytes;
  spec.count = count;
  spec.host_red = reducer;
  AllreduceImpl(buf, spec, prepare_fun, prepare_arg, _file, _line, _caller);
}

void EngineRobust::AllreduceTyped(void *buf, size_t count, mpi::DataType dtype, mpi::OpType op,
                                  ReduceFunction reducer, PreprocFunction prepare_fun,
                                  void *prepare_arg, const char *_file, const int _line,
                                  const char *_caller) {
  ReduceSpec spec;
  spec.type_nbytes = coll::DTypeSize(dtype);
  spec.count = count;
  spec.host_red = reducer;
  spec.dtype = dtype;
  spec.op = op;
  AllreduceImpl(buf, spec, prepare_fun, prepare_arg, _file, _line, _caller);
}

void EngineRobust::AllreduceDevice(void *buf, size_t type_nbytes, size_t count,
                                   DeviceReduceLauncher *dev_reducer, ReduceFunction host_reducer,
                                   PreprocFunction prepare_fun, void *prepare_arg,
                                   const char *_file, const int _line, const char *_caller) {
  ReduceSpec spec;
  spec.type_nbytes = type_nbytes;
  spec.count = count;
  spec.host_red = host_reducer;
  spec.dev_red = dev_reducer;
  AllreduceImpl(buf, spec, prepare_fun, prepare_arg, _file, _line, _caller);
}

void EngineRobust::DevAllreducePrepared(void *dst, const void *src, size_t count, int dtype,
                                        int op, int prep, double alpha, const char *_file,
                                        const int _line, const char *_caller) {
  utils::Check(OnDevice(dst) && OnDevice(src), "DevAllreducePrepared needs device buffers");
  ReduceSpec spec;
  spec.type_nbytes = coll::DTypeSize(static_cast<mpi::DataType>(dtype));
  spec.count = count;
  spec.dtype = dtype;
  spec.op = op;
  AllreduceImpl(dst, spec, nullptr, nullptr, _file, _line, _caller, src, prep, alpha);
}

void EngineRobust::AllreduceImpl(void *buf, const ReduceSpec &spec, PreprocFunction prepare_fun,
                                 void *prepare_arg, const char *_file, const int _line,
                                 const char *_caller, const void *prep_src, int prep_op,
                                 double prep_alpha) {
  core::OpScope op_scope;
  const bool dev = OnDevice(buf);
  const size_t bytes = spec.bytes();
  auto run_prepare = [&]() {
    // a device prepare (prep_src) is fused into the transport below, not run here
    if (prepare_fun != nullptr) prepare_fun(prepare_arg);
  };
  if (GetWorldSize() == 1 && world1_fastpath_) {
    if (prep_src != nullptr) {
      dev_->EnterFromUser();
      device::CheckHip(device::LaunchPrepare(buf, nullptr, prep_src, spec.count, spec.dtype,
                                             prep_op, prep_alpha, dev_->stream()),
                       "LaunchPrepare");
      dev_->Finish(MakeProbe(), false);
    }
    run_prepare();
    return;
  }
  if (bytes == 0) {
    run_prepare();
    return;
  }
  // the caller-signature key only serves the bootstrap cache and the debug log: built only
  // when one of them is on (a string build per op is measurable on the small-op path)
  const bool keyed = debug_ || (bootstrap_cache_ && !checkpoint_loaded_);
  const std::string key =
      keyed ? CallKey(_file, _line, _caller,
                      "#" + std::to_string(spec.type_nbytes) + "x" + std::to_string(spec.count))
            : std::string();
  if (!checkpoint_loaded_ && bootstrap_cache_ && GetBootstrapCache(key, buf, bytes) != -1) {
    return;
  }
  const double t0 = utils::GetTime();
  trace::Scope ts("allreduce", rank_, version_number_, seq_counter_, bytes, dev);
  bool recovered = RecoverExec(buf, bytes, 0, seq_counter_, cur_cache_seq_, "Allreduce");
  ApplyRetention();
  if (!recovered) run_prepare();
  void *temp = resbuf_.AllocTemp(bytes, dev);
  const bool spilled = resbuf_.temp_spilled();
  for (;;) {
    if (recovered) {
      CopyAny(temp, dev && !spilled, buf, dev, bytes);
      stats_.n_recovered_ops += 1;
      break;
    }
    Status s;
    if (dev) {
      // the collective writes the log slot, and the user buffer only once it succeeded on this
      // rank, so a retry still finds the input (prep_src: the prepare pass runs in the
      // transport and is skipped entirely when the result is recovered).  A spilled slot is
      // host memory: the collective writes an HBM stage, copied to the slot behind it.
      void *slot = spilled ? dev_->Scratch(bytes, device::DevicePlane::kSpillScratch) : temp;
      s = TryAllreduceDevice(prep_src != nullptr ? prep_src : buf, slot, spec, buf,
                             prep_src != nullptr ? prep_op : device::kPrepCopy, prep_alpha);
      if (s == Status::kSuccess && spilled) SpillResult(temp, slot, bytes);
    } else {
      // out of place: the log slot receives the result, buf keeps the input until success
      if (host_out_of_place_) {
        s = TryAllreduceHost(temp, spec, buf);
      } else {
        std::memcpy(temp, buf, bytes);
        s = TryAllreduceHost(temp, spec);
      }
    }
    if (CheckAndRecover(s)) {
      if (!dev) std::memcpy(buf, temp, bytes);
      break;
    }
    recovered = RecoverExec(buf, bytes, 0, seq_counter_, cur_cache_seq_, "Allreduce");
  }
  const double dt = utils::GetTime() - t0;
  stats_.n_allreduce += 1;
  stats_.bytes_allreduce += static_cast<double>(bytes);
  stats_.t_allreduce += dt;
  if (debug_) {
    utils::HandleLogInfo("[%d] allreduce (%s) finished version %d, seq %d, take %f seconds\n",
                         rank_, key.c_str(), version_number_, seq_counter_, dt);
  }
  if (checkpoint_loaded_ || !bootstrap_cache_) {
    resbuf_.PushTemp(seq_counter_, bytes);
    seq_counter_ += 1;
  } else {
    resbuf_.PushTemp(seq_counter_, bytes);
    resbuf_.DropLast();
    SetBootstrapCache(key, buf, bytes);
  }
}

void EngineRobust::Broadcast(void *buf, size_t total_size, int root, const char *_file,
                             const int _line, const char *_caller) {
  core::OpScope op_scope;
  if (GetWorldSize() == 1 && world1_fastpath_) return;
  if (total_size == 0) return;
  const bool dev = OnDevice(buf);
  const bool keyed = debug_ || (bootstrap_cache_ && !checkpoint_loaded_);
  const std::string key =
      keyed ? CallKey(_file, _line, _caller,
                      "#" + std::to_string(total_size) + "@" + std::to_string(root))
            : std::string();
  if (!checkpoint_loaded_ && bootstrap_cache_ &&
      GetBootstrapCache(key, buf, total_size) != -1) {
    return;
  }
  const double t0 = utils::GetTime();
  trace::Scope ts("broadcast", rank_, version_number_, seq_counter_, total_size, dev);
  bool recovered = RecoverExec(buf, total_size, 0, seq_counter_, cur_cache_seq_, "Broadcast");
  ApplyRetention();
  void *temp = resbuf_.AllocTemp(total_size, dev);
  for (;;) {
    if (recovered) {
      CopyAny(temp, dev && !resbuf_.temp_spilled(), buf, dev, total_size);
      stats_.n_recovered_ops += 1;
      break;
    }
    // an HBM log slot is written by the collective itself (dual store), not copied after it
    const bool log_in_op = dev && !resbuf_.temp_spilled();
    if (CheckAndRecover(TryBroadcast(buf, total_size, root, log_in_op ? temp : nullptr))) {
      if (dev && resbuf_.temp_spilled()) {
        SpillResult(temp, buf, total_size);
      } else if (!dev) {
        std::memcpy(temp, buf, total_size);
      }
      break;
    }
    recovered = RecoverExec(buf, total_size, 0, seq_counter_, cur_cache_seq_, "Broadcast");
  }
  const double dt = utils::GetTime() - t0;
  stats_.n_broadcast += 1;
  stats_.bytes_broadcast += static_cast<double>(total_size);
  stats_.t_broadcast += dt;
  if (debug_) {
    utils::HandleLogInfo(
        "[%d] broadcast (%s) root %d finished version %d, seq %d, take %f seconds\n", rank_,
        key.c_str(), root, version_number_, seq_counter_, dt);
  }
  if (checkpoint_loaded_ || !bootstrap_cache_) {
    resbuf_.PushTemp(seq_counter_, total_size);
    seq_counter_ += 1;
  } else {
    resbuf_.PushTemp(seq_counter_, total_size);
    resbuf_.DropLast();
    SetBootstrapCache(key, buf, total_size);
  }
}

void EngineRobust::Allgather(void *buf, size_t total_size, size_t slice_begin, size_t slice_end,
                             size_t size_prev_slice, const char *_file, const int _line,
                             const char *_caller) {
  core::OpScope op_scope;
  if (GetWorldSize() == 1 && world1_fastpath_) return;
  if (total_size == 0) return;
  const bool dev = OnDevice(buf);
  const bool keyed = debug_ || (bootstrap_cache_ && !checkpoint_loaded_);
  const std::string key =
      keyed ? CallKey(_file, _line, _caller, "#" + std::to_string(total_size)) : std::string();
  if (!checkpoint_loaded_ && bootstrap_cache_ &&
      GetBootstrapCache(key, buf, total_size) != -1) {
    return;
  }
  const double t0 = utils::GetTime();
  trace::Scope ts("allgather", rank_, version_number_, seq_counter_, total_size, dev);
  bool recovered = RecoverExec(buf, total_size, 0, seq_counter_, cur_cache_seq_, "Allgather");
  ApplyRetention();
  void *temp = resbuf_.AllocTemp(total_size, dev);
  for (;;) {
    if (recovered) {
      CopyAny(temp, dev && !resbuf_.temp_spilled(), buf, dev, total_size);
      stats_.n_recovered_ops += 1;
      break;
    }
    // in place on the user buffer: the ring never overwrites this rank's own slice, so a
    // retry after a failure still finds its input
    const bool log_in_op = dev && !resbuf_.temp_spilled();
    if (CheckAndRecover(TryAllgather(buf, total_size, slice_begin, slice_end, size_prev_slice,
                                     log_in_op ? temp : nullptr))) {
      if (dev && resbuf_.temp_spilled()) {
        SpillResult(temp, buf, total_size);
      } else if (!dev) {
        std::memcpy(temp, buf, total_size);
      }
      break;
    }
    recovered = RecoverExec(buf, total_size, 0, seq_counter_, cur_cache_seq_, "Allgather");
  }
  const double dt = utils::GetTime() - t0;
  stats_.n_allgather += 1;
  stats_.bytes_allgather += static_cast<double>(total_size);
  stats_.t_allgather += dt;
  if (debug_) {
    utils::HandleLogInfo("[%d] allgather (%s) finished version %d, seq %d, take %f seconds\n",
                         rank_, key.c_str(), version_number_, seq_counter_, dt);
  }
  if (checkpoint_loaded_ || !bootstrap_cache_) {
    resbuf_.PushTemp(seq_counter_, total_size);
    seq_counter_ += 1;
  } else {
    resbuf_.PushTemp(seq_counter_, total_size);
    resbuf_.DropLast();
    SetBootstrapCache(key, buf, total_size);
  }
}

// ------------------------------------------------------------------ checkpoints
void EngineRobust::LocalModelCheck(const Serializable *local_model) {
  const bool with_local = local_model != nullptr;
  if (use_local_model_ == -1) {
    if (with_local) {
      use_local_model_ = 1;
      if (num_local_replica_ == 0) num_local_replica_ = default_local_replica_;
      // local tensors stay in HBM (replicated over xGMI); Serializable models in host memory
      const bool on_device = local_model == &dev_local_ && dev_ != nullptr;
      local_.Configure(num_local_replica_ + 1, on_device, on_device ? dev_->device() : -1);
      local_.set_mirror_ctas(MirrorEngine() == device::DeviceCheckpoint::kEngineKernel
                                 ? std::max(mirror_ctas_, 1) : 0);
      // the global checkpoint's mirror settings hold for the local state as well
      local_.set_mirror_off(ckpt_mirror_mode_ == device::DeviceCheckpoint::kMirrorOff);
      local_.set_mirror_sdma(on_device &&
                             MirrorEngine() == device::DeviceCheckpoint::kEngineSdma);
    } else {
      use_local_model_ = 0;
      num_local_replica_ = 0;
    }
  } else {
    utils::Check(use_local_model_ == static_cast<int>(with_local),
                 "CheckPoint/LoadCheckPoint must always be called either with or without "
                 "local_model, not both");
    if (with_local) {
      utils::Check(local_.on_device() == (local_model == &dev_local_),
                   "the local model must always be HBM tensors or always a host model");
    }
  }
}

void EngineRobust::SaveLocalState(int v, const Serializable *local_model) {
  local_.Clear(v);
  if (local_.on_device()) {
    // the tensors, back to back, into slot 0 (HBM to HBM on the plane stream)
    device::DeviceGuard dg(dev_->device());
    dev_->EnterFromUser();
    local_.BeforeWrite(v, dev_->stream());
    char *dst = static_cast<char *>(local_.Alloc(v, 0, dev_local_.total()));
    for (size_t i = 0; i < dev_local_.ptrs.size(); ++i) {
      if (dev_local_.nbytes[i] == 0) continue;
      dev_->CopyDeviceAsync(dst, dev_local_.ptrs[i], dev_local_.nbytes[i]);
      dst += dev_local_.nbytes[i];
    }
    return;
  }
  std::string *host = local_.HostSlot(v, 0);
  utils::MemoryBufferStream fs(host);
  if (local_model != nullptr) local_model->Save(&fs);
  local_.Alloc(v, 0, host->size());
}

void EngineRobust::LoadLocalState(int v, Serializable *local_model) {
  if (local_.on_device()) {
    utils::Check(static_cast<size_t>(local_.size(v, 0)) == dev_local_.total(),
                 "[%d] local checkpoint holds %lld bytes, the local tensors %zu", rank_,
                 static_cast<long long>(local_.size(v, 0)), dev_local_.total());
    device::DeviceGuard dg(dev_->device());
    dev_->EnterFromUser();
    const char *src = static_cast<const char *>(local_.Data(v, 0));
    for (size_t i = 0; i < dev_local_.ptrs.size(); ++i) {
      if (dev_local_.nbytes[i] == 0) continue;
      dev_->CopyDeviceAsync(dev_local_.ptrs[i], src, dev_local_.nbytes[i]);
      src += dev_local_.nbytes[i];
    }
    utils::Check(dev_->Finish(MakeProbe(), false) == Status::kSuccess, "local state load");
    return;
  }
  utils::MemoryFixSizeBuffer fs(local_.Data(v, 0), static_cast<size_t>(local_.size(v, 0)));
  local_model->Load(&fs);
}

int EngineRobust::LoadCheckPoint(Serializable *global_model, Serializable *local_model) {
  core::OpScope op_scope;
  checkpoint_loaded_ = true;
  if (GetWorldSize() == 1 && world1_fastpath_) return 0;
  LocalModelCheck(local_model);
  if (num_local_replica_ == 0) {
    utils::Check(local_model == nullptr,
                 "need to set rabit_local_replica larger than 1 to checkpoint local_model");
  }
  const double t0 = utils::GetTime();
  trace::Scope ts("load_checkpoint", rank_, version_number_, seq_counter_, 0, 0);
  if (RecoverExec(nullptr, 0, ActionSummary::kLoadCheck, ActionSummary::kSpecialOp,
                  cur_cache_seq_, "LoadCheckPoint")) {
    const int nlocal = local_.configured() ? local_.Count(local_chkpt_version_) : 0;
    if (local_model != nullptr) {
      if (nlocal == num_local_replica_ + 1) {
        LoadLocalState(local_chkpt_version_, local_model);
      } else {
        utils::Assert(nlocal == 0, "[%d] local model inconsistent, nlocal=%d", rank_, nlocal);
      }
    }
    resbuf_.Clear();
    seq_counter_ = 0;
    utils::MemoryBufferStream fs(&global_checkpoint_);
    if (global_checkpoint_.empty()) {
      version_number_ = 0;
    } else {
      utils::Assert(fs.Read(&version_number_, sizeof(version_number_)) ==
                        sizeof(version_number_),
                    "read in version number");
      global_model->Load(&fs);
      utils::Assert(local_model == nullptr || nlocal == num_local_replica_ + 1,
                    "local model inconsistent, nlocal=%d", nlocal);
    }
    utils::Check(RecoverExec(nullptr, 0, ActionSummary::kCheckAck, ActionSummary::kSpecialOp,
                             cur_cache_seq_, "LoadCheckPoint"),
                 "check ack must return true");
    if (!RecoverExec(nullptr, 0, ActionSummary::kLoadBootstrapCache, seq_counter_,
                     cur_cache_seq_, "LoadCheckPoint") &&
        debug_) {
      utils::HandleLogInfo("[%d] no bootstrap cache to load\n", rank_);
    }
    if (debug_) {
      utils::HandleLogInfo(
          "[%d] loadcheckpoint size %zu finished version %d, seq %d, take %f seconds\n", rank_,
          global_checkpoint_.length(), version_number_, seq_counter_, utils::GetTime() - t0);
    }
    return version_number_;
  }
  if (debug_) utils::HandleLogInfo("[%d] loadcheckpoint reset\n", rank_);
  resbuf_.Clear();
  seq_counter_ = 0;
  version_number_ = 0;
  return version_number_;
}

void EngineRobust::CheckPointImpl(const Serializable *global_model,
                                  const Serializable *local_model, bool lazy) {
  core::OpScope op_scope;
  if (GetWorldSize() == 1 && world1_fastpath_) {
    version_number_ += 1;
    return;
  }
  const double t0 = utils::GetTime();
  trace::Scope ts("checkpoint", rank_, version_number_, seq_counter_, 0, 0);
  LocalModelCheck(local_model);
  if (num_local_replica_ == 0) {
    utils::Check(local_model == nullptr,
                 "need to set rabit_local_replica larger than 1 to checkpoint local_model");
  }
  if (num_local_replica_ != 0) {
    // the new version is written next to the acknowledged one, which stays loadable until
    // every rank has passed kLocalCheckAck
    const int nv = !local_chkpt_version_;
    for (;;) {
      if (RecoverExec(nullptr, 0, 0, ActionSummary::kLocalCheckPoint, cur_cache_seq_,
                      "CheckPoint")) {
        break;
      }
      SaveLocalState(nv, local_model);
      if (CheckAndRecover(TryCheckinLocalState(nv))) break;
    }
    RecoverExec(nullptr, 0, 0, ActionSummary::kLocalCheckAck, cur_cache_seq_, "CheckPoint");
    local_chkpt_version_ = nv;
    // every rank passed kLocalCheckAck holding version nv: the superseded version can never be
    // loaded again, so its slots are marked absent now.  A stale slot must not look present
    // when the next checkpoint reuses this version (a holder picked by the recovery plan would
    // serve a model from two checkpoints ago).
    local_.Clear(!nv);
    if (local_.on_device()) local_.Mirror(nv, dev_->stream());
  }
  utils::Check(RecoverExec(nullptr, 0, ActionSummary::kCheckPoint, ActionSummary::kSpecialOp,
                           cur_cache_seq_, "CheckPoint"),
               "check point must return true");
  version_number_ += 1;
  ckpt_header_only_ = false;
  if (lazy) {
    global_lazycheck_ = global_model;
  } else {
    global_checkpoint_.clear();
    utils::MemoryBufferStream fs(&global_checkpoint_);
    fs.Write(&version_number_, sizeof(version_number_));
    global_model->Save(&fs);
    global_lazycheck_ = nullptr;
  }
  if (debug_) {
    utils::HandleLogInfo("[%d] checkpoint finished version %d, seq %d, take %f seconds\n", rank_,
                         version_number_, seq_counter_, utils::GetTime() - t0);
  }
  const double t1 = utils::GetTime();
  resbuf_.Clear();
  seq_counter_ = 0;
  utils::Check(RecoverExec(nullptr, 0, ActionSummary::kCheckAck, ActionSummary::kSpecialOp,
                           cur_cache_seq_, "CheckPoint"),
               "check ack must return true");
  if (debug_) {
    utils::HandleLogInfo("[%d] checkpoint ack finished version %d, take %f seconds\n", rank_,
                         version_number_, utils::GetTime() - t1);
  }
  stats_.n_checkpoint += 1;
  stats_.t_checkpoint += utils::GetTime() - t0;
}

// ------------------------------------------------------------------ bootstrap cache
int EngineRobust::SetBootstrapCache(const std::string &key, const void *buf, size_t nbytes) {
  utils::Assert(nbytes > 0, "can't set empty cache");
  const bool dev = OnDevice(buf);
  void *temp = cachebuf_.AllocTemp(nbytes, false);
  if (dev) {
    dev_->StageToHost(temp, buf, nbytes);
  } else {
    std::memcpy(temp, buf, nbytes);
  }
  cachebuf_.PushTemp(cur_cache_seq_, nbytes);
  void *name = lookupbuf_.AllocTemp(key.size() + 1, false);
  std::memcpy(name, key.c_str(), key.size() + 1);
  lookupbuf_.PushTemp(cur_cache_seq_, key.size() + 1);
  cur_cache_seq_ += 1;
  return 0;
}

int EngineRobust::GetBootstrapCache(const std::string &key, void *buf, size_t nbytes) {
  if (!RecoverExec(nullptr, 0, ActionSummary::kLoadBootstrapCache, seq_counter_, cur_cache_seq_,
                   "GetBootstrapCache")) {
    return -1;
  }
  int index = -1;
  for (int i = 0; i < cur_cache_seq_; ++i) {
    const ResultLog::Entry *e = lookupbuf_.Query(i);
    if (e != nullptr && e->size == key.size() + 1 &&
        strcmp(static_cast<const char *>(lookupbuf_.Data(*e)), key.c_str()) == 0) {
      index = i;
      break;
    }
  }
  if (index == -1) return -1;
  const ResultLog::Entry *e = cachebuf_.Query(index);
  utils::Assert(e != nullptr && e->size == nbytes, "cached size differs from the request");
  void *src = cachebuf_.Data(*e);
  if (OnDevice(buf)) {
    dev_->StageToDevice(buf, src, nbytes);
  } else {
    std::memcpy(buf, src, nbytes);
  }
  return 0;
}

// ------------------------------------------------------------------ watchdog
void EngineRobust::StartWatchdog() {
  if (watchdog_.joinable()) return;
  wd_stop_ = false;
  watchdog_ = std::thread([this]() { WatchdogLoop(); });
}

void EngineRobust::StopWatchdog() {
  if (!watchdog_.joinable()) return;
  {
    std::lock_guard<std::mutex> lk(wd_mu_);
    wd_stop_ = true;
  }
  wd_cv_.notify_all();
  watchdog_.join();
}

void EngineRobust::WatchdogLoop() {
  std::unique_lock<std::mutex> lk(wd_mu_);
  while (!wd_stop_) {
    // system_clock: wait_until then maps to pthread_cond_timedwait, which ThreadSanitizer
    // understands (steady-clock waits use pthread_cond_clockwait, invisible to gcc-11 TSan)
    wd_cv_.wait_until(lk, std::chrono::system_clock::now() + std::chrono::milliseconds(100));
    if (wd_stop_) break;
    // a rank stuck in its own code inside an op (a prepare function or Save that never
    // returns): its peers only wait for it, so nobody else can notice.  Leaving with a
    // restartable status turns the hang into an ordinary failure: the peers see the links
    // drop and recover, and the restarted rank replays what it missed.
    const double working = core::WorkingFor();
    if (hang_timeout_sec_ > 0 && working > hang_timeout_sec_) {
      fprintf(stderr,
              "[%d] xrabit: working inside a collective for %.1f s without waiting on peers "
              "(rabit_hang_timeout_sec=%g): exiting for a restart\n",
              wd_rank_.load(), working, hang_timeout_sec_);
      fflush(stderr);
      utils::ExitProcess(kHangExitCode);
    }
    // a wait on this rank's own GPU that outlasts every deadline (a HIP call that blocks on a
    // wedged stream): nothing in this process can unblock it, so leave for a restart
    const double on_gpu = core::DeviceWaitingFor();
    const double gpu_limit = core::EffectiveDeviceWaitLimit(
        dev_wait_limit_sec_, core::GlobalWaitState().device_op_deadline.load(),
        dcfg_.drain_timeout_sec);
    if (gpu_limit > 0 && on_gpu > gpu_limit) {
      fprintf(stderr, "[%d] xrabit: waiting on the GPU for %.1f s (limit %.1f s: "
              "rabit_device_wait_limit_sec=%g, op deadline %.1f s)\n", wd_rank_.load(), on_gpu,
              gpu_limit, dev_wait_limit_sec_, core::GlobalWaitState().device_op_deadline.load());
      device::DevicePlane::WedgedExit("watchdog");
    }
    const double since = recovering_since_.load();
    if (timeout_enabled_ && since > 0 && utils::GetTime() - since > timeout_sec_ &&
        !watchdog_fired_.load()) {
      watchdog_fired_.store(true);
      // unblock whatever this rank is waiting on, then apply the timeout action
      abort_flag_.store(true);
      const int rank = wd_rank_.load();
      if (timeout_handler_ != nullptr) {
        timeout_handler_(rank, timeout_sec_);
      } else {
        fprintf(stderr, "[%d] xrabit: recovery did not finish within %d s, exiting\n", rank,
                timeout_sec_);
        fflush(stderr);
        utils::ExitProcess(253);
      }
    }
  }
}
}  // namespace engine
}  // namespace rabit
