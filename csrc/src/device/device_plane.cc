/*!
 * \file device_plane.cc
 * \brief RCCL + HIP implementation of the device data plane.
 */
#include "device/device_plane.h"

#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <thread>

#include "core/wait_state.h"
#include "device/kernels.h"
#include "rabit/internal/utils.h"

namespace rabit {
namespace device {

void CheckHip(hipError_t e, const char *what) {
  if (e != hipSuccess) utils::Error("HIP error in %s: %s", what, hipGetErrorString(e));
}

namespace {
void CheckNccl(ncclResult_t r, const char *what) {
  if (r != ncclSuccess) utils::Error("RCCL error in %s: %s", what, ncclGetErrorString(r));
}

bool RcclType(int dtype, ncclDataType_t *out) {
  switch (dtype) {
    case 0: *out = ncclInt8; return true;
    case 1: *out = ncclUint8; return true;
    case 2: *out = ncclInt32; return true;
    case 3: *out = ncclUint32; return true;
    case 4: *out = ncclInt64; return true;
    case 5: *out = ncclUint64; return true;
    case 6: *out = ncclFloat32; return true;
    case 7: *out = ncclFloat64; return true;
    case 8: *out = ncclInt64; return true;
    case 9: *out = ncclUint64; return true;
    case 10: *out = ncclFloat16; return true;
    case 11: *out = ncclBfloat16; return true;
    default: return false;
  }
}

bool RcclOp(int op, ncclRedOp_t *out) {
  switch (op) {
    case 0: *out = ncclMax; return true;
    case 1: *out = ncclMin; return true;
    case 2: *out = ncclSum; return true;
    default: return false;  // BitOR: no RCCL equivalent
  }
}

size_t TypeBytes(int dtype) {
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
}  // namespace

// ------------------------------------------------------------------ arena
DeviceArena::~DeviceArena() {
  for (auto &c : chunks_) (void)hipFree(c.base);
}

void *DeviceArena::Alloc(size_t bytes) {
  const size_t need = (bytes + 255) & ~static_cast<size_t>(255);
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
  if (reserved() + std::max(need, chunk_) > cap_) return nullptr;
  Chunk c;
  c.size = std::max(need, chunk_);
  c.used = need;
  void *base = nullptr;
  if (hipMalloc(&base, c.size) != hipSuccess) {
    (void)hipGetLastError();
    return nullptr;
  }
  c.base = static_cast<char *>(base);
  chunks_.push_back(c);
  cur_ = chunks_.size() - 1;
  return c.base;
}

void DeviceArena::PopTo(void *ptr) {
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

void DeviceArena::Reset() {
  for (auto &c : chunks_) c.used = 0;
  cur_ = 0;
}

size_t DeviceArena::used() const {
  size_t s = 0;
  for (auto &c : chunks_) s += c.used;
  return s;
}

size_t DeviceArena::reserved() const {
  size_t s = 0;
  for (auto &c : chunks_) s += c.size;
  return s;
}

// ------------------------------------------------------------------ plane
int DevicePlane::DeviceCount() {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) {
    (void)hipGetLastError();
    return 0;
  }
  return n;
}

DevicePlane::DevicePlane(const DeviceConfig &cfg, int rank_hint) : cfg_(cfg) {
  const int ndev = DeviceCount();
  utils::Check(ndev > 0, "DevicePlane: no HIP device visible");
  int dev = cfg.device;
  if (dev < 0) {
    const char *lr = getenv("LOCAL_RANK");
    dev = lr != nullptr ? atoi(lr) : std::max(rank_hint, 0);
  }
  device_ = dev % ndev;
  CheckHip(hipSetDevice(device_), "hipSetDevice");
  CheckHip(hipStreamCreateWithFlags(&own_stream_, hipStreamNonBlocking), "hipStreamCreate");
  CheckHip(hipEventCreateWithFlags(&ev_switch_, hipEventDisableTiming), "hipEventCreate");
  stream_ = cfg_.ops_on_user_stream ? user_stream_ : own_stream_;
  CheckHip(hipEventCreateWithFlags(&ev_in_, hipEventDisableTiming), "hipEventCreate");
  CheckHip(hipEventCreateWithFlags(&ev_done_, hipEventDisableTiming), "hipEventCreate");
  arena_.Configure(cfg.arena_chunk, cfg.arena_cap);
  if (cfg.sym_heap > 0) {
    // symmetric heap: uncached like the stage buffers (peers read it over xGMI in place)
    heap_.bytes = (cfg.sym_heap + (1u << 16) - 1) & ~static_cast<size_t>((1u << 16) - 1);
    void *p = nullptr;
    CheckHip(hipExtMallocWithFlags(&p, heap_.bytes, hipDeviceMallocUncached),
             "hipExtMallocWithFlags(symmetric heap)");
    heap_.base = static_cast<char *>(p);
    hipIpcMemHandle_t h;
    CheckHip(hipIpcGetMemHandle(&h, heap_.base), "hipIpcGetMemHandle(heap)");
    std::memcpy(heap_.ipc, &h, sizeof(h));
  }
}

void *DevicePlane::SymAlloc(size_t bytes) {
  const size_t need = (bytes + 255) & ~static_cast<size_t>(255);
  if (heap_.base == nullptr || heap_used_ + need > heap_.bytes) return nullptr;
  void *p = heap_.base + heap_used_;
  heap_used_ += need;
  return p;
}

DevicePlane::~DevicePlane() {
  // the caller's stream may be gone by now: drain the device instead of that stream
  (void)hipSetDevice(device_);
  (void)hipDeviceSynchronize();
  peers_.reset();
  if (comm_ != nullptr) {
    ncclCommDestroy(comm_);
    comm_ = nullptr;
  }
  for (int i = 0; i < kScratchSlots; ++i) {
    if (scratch_[i] != nullptr) (void)hipFree(scratch_[i]);
  }
  if (pinned_ != nullptr) (void)hipHostFree(pinned_);
  if (ev_in_ != nullptr) (void)hipEventDestroy(ev_in_);
  if (ev_done_ != nullptr) (void)hipEventDestroy(ev_done_);
  peers_.reset();
  if (heap_.base != nullptr) (void)hipFree(heap_.base);
  if (ev_switch_ != nullptr) (void)hipEventDestroy(ev_switch_);
  if (own_stream_ != nullptr) (void)hipStreamDestroy(own_stream_);
}

bool DevicePlane::IsDevicePtr(const void *p) const {
  if (p == nullptr) return false;
  hipPointerAttribute_t attr;
  hipError_t e = hipPointerGetAttributes(&attr, p);
  if (e != hipSuccess) {
    (void)hipGetLastError();
    return false;
  }
  return attr.type == hipMemoryTypeDevice || attr.type == hipMemoryTypeManaged;
}

std::string DevicePlane::NewUniqueId() {
  ncclUniqueId id;
  CheckNccl(ncclGetUniqueId(&id), "ncclGetUniqueId");
  return std::string(id.internal, sizeof(id.internal));
}

Status DevicePlane::InitComm(const std::string &id_bytes, int nranks, int rank,
                             const FailureProbe &probe) {
  (void)probe;
  if (comm_ != nullptr) AbortComm();
  utils::Check(id_bytes.size() == sizeof(ncclUniqueId), "bad ncclUniqueId size");
  ncclUniqueId id;
  std::memcpy(id.internal, id_bytes.data(), sizeof(id.internal));
  CheckHip(hipSetDevice(device_), "hipSetDevice");
  ncclResult_t r = ncclCommInitRank(&comm_, nranks, id, rank);
  if (r != ncclSuccess) {
    comm_ = nullptr;
    utils::HandleLogInfo("[xrabit] ncclCommInitRank failed: %s\n", ncclGetErrorString(r));
    return Status::kAborted;
  }
  nranks_ = nranks;
  rank_ = rank;
  return Status::kSuccess;
}

void DevicePlane::AbortComm() {
  if (peers_ != nullptr) {
    peers_->SignalAbort();  // spinning barriers give up; later kernels of the group are guarded
  }
  if (comm_ != nullptr) {
    ncclCommAbort(comm_);
    comm_ = nullptr;
  }
  if (peers_ != nullptr) {
    (void)hipStreamSynchronize(stream_);
    peers_.reset();
  }
}

void DevicePlane::DescribeDevice(PeerRecord *rec) const {
  (void)hipDeviceGetPCIBusId(rec->pci, sizeof(rec->pci), device_);
  gethostname(rec->host, sizeof(rec->host) - 1);
  rec->device = device_;
  rec->pid = static_cast<int32_t>(getpid());
}

bool DevicePlane::PreparePeers(PeerRecord *rec, std::string *why) {
  DropPeers();
  try {
    peers_.reset(
        new PeerGroup(device_, cfg_.peer_stage, cfg_.peer_deadline_sec, stream_, heap_));
    if (cfg_.phase_timing) peers_->EnableTiming();
    peers_->set_oneshot_max(cfg_.oneshot_max);
    peers_->set_push(cfg_.direct_mode == 2);
  } catch (const std::exception &e) {
    peers_.reset();
    *why = e.what();
    return false;
  }
  *rec = peers_->local();
  return true;
}

bool DevicePlane::OpenPeers(const std::vector<PeerRecord> &all, int rank, std::string *why) {
  if (peers_ == nullptr) {
    *why = "no local peer buffers";
    return false;
  }
  if (!peers_->Open(all, rank, why)) {
    peers_.reset();
    return false;
  }
  return true;
}

bool DevicePlane::DirectPhaseUs(double out[PeerGroup::kPhases], uint64_t *nops) const {
  if (peers_ == nullptr || peers_->timed_ops() == 0) return false;
  *nops = peers_->timed_ops();
  for (int k = 0; k < PeerGroup::kPhases; ++k) out[k] = peers_->phase_ms()[k] * 1e3 / *nops;
  return true;
}

void DevicePlane::DropPeers() {
  if (peers_ != nullptr) {
    (void)hipStreamSynchronize(stream_);
    peers_.reset();
  }
}

void DevicePlane::SetUserStream(hipStream_t s) {
  user_stream_ = s;
  if (!cfg_.ops_on_user_stream || s == stream_) return;
  // keep collectives in issue order across a change of stream
  CheckHip(hipEventRecord(ev_switch_, stream_), "hipEventRecord(switch)");
  CheckHip(hipStreamWaitEvent(s, ev_switch_, 0), "hipStreamWaitEvent(switch)");
  stream_ = s;
  if (peers_ != nullptr) peers_->set_stream(s);
}

void DevicePlane::EnterFromUser() {
  if (user_stream_ == stream_) return;
  CheckHip(hipEventRecord(ev_in_, user_stream_), "hipEventRecord(user)");
  CheckHip(hipStreamWaitEvent(stream_, ev_in_, 0), "hipStreamWaitEvent");
}

Status DevicePlane::WaitEvent(hipEvent_t ev, const FailureProbe &probe) {
  core::WaitScope waiting;  // peers' barriers and RCCL: waiting on other ranks
  using clock = std::chrono::steady_clock;
  const auto t0 = clock::now();
  for (uint64_t iter = 0;; ++iter) {
    hipError_t e = hipEventQuery(ev);
    if (e == hipSuccess) {
      if (peers_ != nullptr && peers_->failed()) {
        utils::HandleLogInfo("[xrabit] direct transport: a peer barrier gave up\n");
        if (force_ == 1) {
          DropPeers();  // calibration probe: keep the RCCL communicator
        } else {
          AbortComm();
        }
        return Status::kAborted;
      }
      if (peers_ != nullptr) peers_->CollectTiming();
      return Status::kSuccess;
    }
    if (e != hipErrorNotReady) CheckHip(e, "device collective");
    if (comm_ != nullptr && (iter & 15) == 0) {
      ncclResult_t ae = ncclSuccess;
      if (ncclCommGetAsyncError(comm_, &ae) == ncclSuccess && ae != ncclSuccess &&
          ae != ncclInProgress) {
        utils::HandleLogInfo("[xrabit] RCCL async error: %s\n", ncclGetErrorString(ae));
        AbortComm();
        return Status::kAborted;
      }
    }
    const double waited = std::chrono::duration<double>(clock::now() - t0).count();
    if (probe && (iter & 63) == 0 && waited > 1e-3 && probe()) {
      AbortComm();
      (void)hipStreamSynchronize(stream_);
      return Status::kAborted;
    }
    if (cfg_.op_timeout_sec > 0 && waited > cfg_.op_timeout_sec) {
      utils::HandleLogInfo("[xrabit] device op exceeded %.1f s, aborting communicator\n",
                           cfg_.op_timeout_sec);
      AbortComm();
      (void)hipStreamSynchronize(stream_);
      return Status::kTimeout;
    }
    // spin first: the wake-up latency after completion sits on the critical path of every op
    if (waited * 1e6 > cfg_.spin_us) std::this_thread::sleep_for(std::chrono::microseconds(10));
  }
}

Status DevicePlane::Finish(const FailureProbe &probe, bool host_wait) {
  CheckHip(hipEventRecord(ev_done_, stream_), "hipEventRecord(done)");
  Status s = Status::kSuccess;
  if (cfg_.sync && host_wait) s = WaitEvent(ev_done_, probe);
  if (pending_dst_ != nullptr) {
    if (s == Status::kSuccess) {
      CopyDeviceAsync(pending_dst_, pending_src_, pending_bytes_);
      CheckHip(hipEventRecord(ev_done_, stream_), "hipEventRecord(done)");
    }
    pending_dst_ = nullptr;
  }
  if (user_stream_ != stream_) {
    CheckHip(hipStreamWaitEvent(user_stream_, ev_done_, 0), "hipStreamWaitEvent(user)");
  }
  return s;
}

void DevicePlane::Synchronize() {
  core::WaitScope waiting;
  CheckHip(hipStreamSynchronize(stream_), "hipStreamSynchronize");
}

void DevicePlane::CopyAsync(void *dst, const void *src, size_t bytes) {
  if (bytes == 0 || dst == src) return;
  CheckHip(hipMemcpyAsync(dst, src, bytes, hipMemcpyDefault, stream_), "hipMemcpyAsync");
}

void DevicePlane::CopyDeviceAsync(void *dst, const void *src, size_t bytes) {
  CheckHip(LaunchCopy(dst, src, bytes, stream_), "LaunchCopy");
}

void *DevicePlane::Scratch(size_t bytes, int slot) {
  if (scratch_bytes_[slot] < bytes) {
    if (scratch_[slot] != nullptr) {
      CheckHip(hipStreamSynchronize(stream_), "hipStreamSynchronize");
      (void)hipFree(scratch_[slot]);
    }
    size_t want = std::max(bytes, scratch_bytes_[slot] * 2);
    CheckHip(hipMalloc(&scratch_[slot], want), "hipMalloc(scratch)");
    scratch_bytes_[slot] = want;
  }
  return scratch_[slot];
}

void DevicePlane::StageToHost(void *host, const void *dev, size_t bytes) {
  CheckHip(hipMemcpyAsync(host, dev, bytes, hipMemcpyDeviceToHost, stream_), "D2H");
  CheckHip(hipStreamSynchronize(stream_), "hipStreamSynchronize");
}

void DevicePlane::StageToDevice(void *dev, const void *host, size_t bytes) {
  CheckHip(hipMemcpyAsync(dev, host, bytes, hipMemcpyHostToDevice, stream_), "H2D");
  CheckHip(hipStreamSynchronize(stream_), "hipStreamSynchronize");
}

Status DevicePlane::Allreduce(const void *send, void *recv, void *recv2, size_t count, int dtype,
                              int op, int prep, double alpha, const FailureProbe &probe) {
  const size_t bytes = count * TypeBytes(dtype);
  if (UseDirect(bytes)) {
    CheckHip(peers_->Allreduce(send, recv, recv2, count, dtype, op, prep, alpha),
             "direct allreduce");
    return Status::kSuccess;
  }
  utils::Check(comm_ != nullptr, "device allreduce without communicator");
  ncclDataType_t t;
  ncclRedOp_t o;
  if (!RcclType(dtype, &t)) utils::Error("unsupported dtype %d on device", dtype);
  if (prep != kPrepCopy) {
    CheckHip(LaunchPrepare(recv, nullptr, send, count, dtype, prep, alpha, stream_),
             "LaunchPrepare");
    send = recv;
  }
  if (!RcclOp(op, &o)) {
    PeerGroup::ReduceStep step = [dtype, op](void *dst, const void *const *srcs, int n, size_t c,
                                             const int *guard, const void *const *table,
                                             double post, hipStream_t st) {
      return LaunchReduceMulti(dst, srcs, n, c, dtype, op, st, guard, table, post);
    };
    Status s = AllreduceByKernel(send, recv, count, TypeBytes(dtype), step, probe);
    if (s != Status::kSuccess) return s;
  } else {
    CheckNccl(ncclAllReduce(send, recv, count, t, o, comm_, stream_), "ncclAllReduce");
  }
  // RCCL writes recv only; the second copy is enqueued by Finish once the op is known to have
  // succeeded (an aborted RCCL kernel leaves garbage in recv)
  if (recv2 != nullptr && recv2 != recv) {
    pending_dst_ = recv2;
    pending_src_ = recv;
    pending_bytes_ = bytes;
  }
  return Status::kSuccess;
}

Status DevicePlane::AllreduceCustom(const void *send, void *recv, void *recv2, size_t count,
                                    size_t type_nbytes, DeviceReduceLauncher *launcher,
                                    const FailureProbe &probe) {
  PeerGroup::ReduceStep step = [launcher](void *dst, const void *const *srcs, int n, size_t c,
                                          const int *guard, const void *const *, double,
                                          hipStream_t st) {
    return static_cast<hipError_t>(launcher(dst, srcs, n, c, guard, st));
  };
  const size_t bytes = count * type_nbytes;
  if (UseDirect(bytes)) {
    CheckHip(peers_->AllreduceCustom(send, recv, recv2, count, type_nbytes, step),
             "direct allreduce (custom)");
    return Status::kSuccess;
  }
  Status s = AllreduceByKernel(send, recv, count, type_nbytes, step, probe);
  if (s != Status::kSuccess) return s;
  if (recv2 != nullptr && recv2 != recv) {
    pending_dst_ = recv2;
    pending_src_ = recv;
    pending_bytes_ = bytes;
  }
  return Status::kSuccess;
}

Status DevicePlane::AllreduceByKernel(const void *send, void *recv, size_t count, size_t tn,
                                      const PeerGroup::ReduceStep &step,
                                      const FailureProbe &probe) {
  (void)probe;
  utils::Check(comm_ != nullptr, "device allreduce without communicator");
  const int n = nranks_;
  // all-to-all: rank k receives everyone's copy of segment k, reduces it with the
  // multi-source kernel, then an allgather distributes the reduced segments
  const size_t seg = (count + n - 1) / n;
  const size_t seg_bytes = ((seg * tn + 255) / 256) * 256;  // keep segments 256-B aligned
  char *a = static_cast<char *>(Scratch(seg_bytes * n, 0));
  char *b = static_cast<char *>(Scratch(seg_bytes * n, 1));
  // pack the input as n segments of seg_bytes
  for (int k = 0; k < n; ++k) {
    const size_t lo = std::min(count, k * seg), hi = std::min(count, (k + 1) * seg);
    if (hi > lo) {
      CheckHip(LaunchCopy(a + k * seg_bytes, static_cast<const char *>(send) + lo * tn,
                          (hi - lo) * tn, stream_),
               "pack");
    }
  }
  CheckNccl(ncclAllToAll(a, b, seg_bytes, ncclUint8, comm_, stream_), "ncclAllToAll");
  // reduce the n copies of my segment, up to 8 sources per kernel pass
  char *mine = a + static_cast<size_t>(rank_) * seg_bytes;
  std::vector<const void *> srcs;
  int done = 0;
  while (done < n) {
    srcs.clear();
    if (done > 0) srcs.push_back(mine);
    while (done < n && static_cast<int>(srcs.size()) < kMaxReduceSources) {
      srcs.push_back(b + static_cast<size_t>(done) * seg_bytes);
      ++done;
    }
    CheckHip(step(mine, srcs.data(), static_cast<int>(srcs.size()), seg, nullptr, nullptr, 0.0,
                  stream_),
             "allreduce reduce step");
  }
  CheckNccl(ncclAllGather(mine, b, seg_bytes, ncclUint8, comm_, stream_), "ncclAllGather");
  for (int k = 0; k < n; ++k) {
    const size_t lo = std::min(count, k * seg), hi = std::min(count, (k + 1) * seg);
    if (hi > lo) {
      CheckHip(LaunchCopy(static_cast<char *>(recv) + lo * tn, b + k * seg_bytes,
                          (hi - lo) * tn, stream_),
               "unpack");
    }
  }
  return Status::kSuccess;
}

Status DevicePlane::Broadcast(void *buf, size_t bytes, int root, const FailureProbe &probe) {
  (void)probe;
  if (UseDirect(bytes)) {
    CheckHip(peers_->Broadcast(buf, bytes, root), "direct broadcast");
    return Status::kSuccess;
  }
  utils::Check(comm_ != nullptr, "device broadcast without communicator");
  CheckNccl(ncclBroadcast(buf, buf, bytes, ncclUint8, root, comm_, stream_), "ncclBroadcast");
  return Status::kSuccess;
}

Status DevicePlane::AllgatherV(void *buf_, size_t total, const std::vector<size_t> &begin,
                               const std::vector<size_t> &size, const FailureProbe &probe) {
  (void)probe;
  if (UseDirect(total)) {
    CheckHip(peers_->AllgatherV(buf_, total, begin, size), "direct allgather");
    return Status::kSuccess;
  }
  utils::Check(comm_ != nullptr, "device allgather without communicator");
  char *buf = static_cast<char *>(buf_);
  const int n = nranks_;
  bool uniform = total == size[0] * n;
  for (int r = 0; r < n && uniform; ++r) uniform = begin[r] == r * size[0] && size[r] == size[0];
  if (uniform) {
    CheckNccl(ncclAllGather(buf + begin[rank_], buf, size[0], ncclUint8, comm_, stream_),
              "ncclAllGather");
    return Status::kSuccess;
  }
  CheckNccl(ncclGroupStart(), "ncclGroupStart");
  for (int r = 0; r < n; ++r) {
    size_t b = begin[r] % total, s = size[r];
    const size_t first = std::min(s, total - b);
    if (first != 0) {
      CheckNccl(ncclBroadcast(buf + b, buf + b, first, ncclUint8, r, comm_, stream_),
                "ncclBroadcast");
    }
    if (s > first) {
      CheckNccl(ncclBroadcast(buf, buf, s - first, ncclUint8, r, comm_, stream_),
                "ncclBroadcast");
    }
  }
  CheckNccl(ncclGroupEnd(), "ncclGroupEnd");
  return Status::kSuccess;
}
}  // namespace device
}  // namespace rabit
