/*!
 * \file device_plane.cc
 * \brief RCCL + HIP implementation of the device data plane.
 */
#include "device/device_plane.h"

#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <condition_variable>
#include <memory>
#include <mutex>
#include <thread>

#include "core/exit.h"
#include "core/trace.h"
#include "core/wait_state.h"
#include "device/kernels.h"
#include "rabit/internal/half.h"
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

// pinned word that ends an injected hang; process-wide so that the watchdog thread and the
// exit path can release it without touching the plane
std::atomic<int *> g_hang_release{nullptr};

// ------------------------------------------------------------------ arena
DeviceArena::~DeviceArena() {
  for (auto &c : chunks_) {
    if (pinned_) {
      (void)hipHostFree(c.base);
    } else {
      (void)hipFree(c.base);
    }
  }
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
  const size_t have = reserved();
  const size_t least = std::max(need, chunk_);
  if (have + least > cap_) return nullptr;
  size_t want = least;
  if (chunks_.empty()) {
    want = std::max(want, reserve_);
  } else if (!pinned_) {
    want = std::max(want, std::min(have, kMaxStep));  // geometric growth of the HBM log
  }
  want = std::min(want, cap_ - have);
  Chunk c;
  c.used = need;
  void *base = nullptr;
  auto try_alloc = [&](size_t size) {
    const hipError_t e =
        pinned_ ? hipHostMalloc(&base, size, hipHostMallocDefault) : hipMalloc(&base, size);
    if (e != hipSuccess) {
      (void)hipGetLastError();
      base = nullptr;
      return false;
    }
    c.size = size;
    return true;
  };
  // the larger step first; when memory is short, the smallest chunk that fits this slot
  if (!try_alloc(want) && (want == least || !try_alloc(least))) return nullptr;
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

void DevicePlane::ConfigureRcclEnv() { setenv("NCCL_RUNTIME_CONNECT", "0", 0); }

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
  arena_.Configure(cfg.arena_chunk, cfg.arena_cap, false, cfg.arena_reserve);
  spill_.Configure(std::min<size_t>(cfg.arena_chunk, 64u << 20), cfg.spill_cap, true);
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
  stager_.reset();
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

namespace {
/*!
 * \brief state shared by the thread that waits for a communicator's bring-up and the helper
 *        thread that runs it.  The helper may outlive the waiter's interest (a peer died inside
 *        RCCL's bootstrap, which waits on sockets without any deadline): the waiter then
 *        abandons it, and a helper that ever returns aborts the communicator it built itself.
 *        The warm-up stream and buffer belong to this state, not to the plane: an abandoned
 *        helper that wakes up later enqueues nothing on a stream the plane reuses or frees, and
 *        whoever drops the state last releases them (once idle).
 */
struct CommBringUp {
  std::mutex mu;
  std::condition_variable cv;
  bool done{false}, abandoned{false};
  ncclResult_t result{ncclSuccess};
  ncclComm_t comm{nullptr};
  hipStream_t stream{nullptr};
  char *buf{nullptr};
  size_t buf_bytes{0};
  ~CommBringUp() {
    // work still queued (an aborted warm-up that never drained): leak rather than free memory
    // a kernel may still touch
    const bool idle = stream == nullptr || hipStreamQuery(stream) == hipSuccess;
    (void)hipGetLastError();
    if (!idle) return;
    if (buf != nullptr) (void)hipFree(buf);
    if (stream != nullptr) (void)hipStreamDestroy(stream);
  }
};
/*! \brief helpers abandoned in RCCL's bootstrap that have not returned yet (process-wide) */
std::atomic<int> g_live_abandoned{0};
}  // namespace

int DevicePlane::LiveAbandonedInits() { return g_live_abandoned.load(); }

Status DevicePlane::InitComm(const std::string &id_bytes, int nranks, int rank,
                             const FailureProbe &probe) {
  if (comm_ != nullptr) AbortComm();
  utils::Check(id_bytes.size() == sizeof(ncclUniqueId), "bad ncclUniqueId size");
  if (nranks > 1 && g_live_abandoned.load() >= kMaxAbandonedInits) {
    // every abandoned helper holds a thread and RCCL's bootstrap sockets until its peer shows
    // up, which it may never do: beyond the cap no new multi-rank bring-up starts.  The engine
    // then runs on the direct transport, or fails for a restart when none is left.
    rccl_fail_streak_ += 1;
    utils::Check(cfg_.rccl_max_failures <= 0 || rccl_fail_streak_ <= cfg_.rccl_max_failures,
                 "RCCL bring-up failed %d times in a row; giving up", rccl_fail_streak_);
    utils::HandleLogInfo("[xrabit] RCCL bring-up refused: %d abandoned bring-ups still blocked "
                         "in RCCL's bootstrap\n", g_live_abandoned.load());
    init_refused_ += 1;
    return Status::kAborted;
  }
  ncclUniqueId id;
  std::memcpy(id.internal, id_bytes.data(), sizeof(id.internal));
  CheckHip(hipSetDevice(device_), "hipSetDevice");
  // channel (CTA) bounds for the 7 xGMI links: RCCL's own choice unless configured
  // (rabit_rccl_min_ctas / rabit_rccl_max_ctas; one CTA drives one channel)
  ncclConfig_t config = NCCL_CONFIG_INITIALIZER;
  if (cfg_.rccl_min_ctas > 0) config.minCTAs = cfg_.rccl_min_ctas;
  if (cfg_.rccl_max_ctas > 0) config.maxCTAs = cfg_.rccl_max_ctas;
  config.commName = "xrabit";
  // Blocking communicator, brought up on a helper thread.  RCCL 2.27's non-blocking mode does
  // not help here: ncclCommInitRankConfig with blocking = 0 still blocks the caller inside the
  // bootstrap while a rank is missing (measured: profiles/r3_rccl_lifecycle/).  The helper runs
  // the init and then connects every channel this job will use (eager collective connections,
  // NCCL_RUNTIME_CONNECT=0, set by the engine at start-up; plus one grouped send/recv with every
  // peer and one allreduce per size class the routing may send to RCCL), all while the ranks
  // are known to be alive.  Afterwards no RCCL call of this epoch waits on a peer on the host:
  // only kernels do, and WaitEvent aborts those.  This thread meanwhile watches the failure
  // probe and the deadline.
  config.blocking = 1;
  auto g = std::make_shared<CommBringUp>();
  CheckHip(hipStreamCreateWithFlags(&g->stream, hipStreamNonBlocking), "hipStreamCreate(warm-up)");
  // size classes of the warm-up: 64 KiB (latency algorithms), 4 MiB (gradient buckets) and the
  // large point (128 MiB by default): each reaches the protocol RCCL picks for that size
  const size_t big = std::max<size_t>(cfg_.rccl_warm_bytes, 4096) / 256 * 256;
  g->buf_bytes = nranks > 1 ? big : 4096;
  if (hipMalloc(&g->buf, g->buf_bytes) != hipSuccess) {
    (void)hipGetLastError();
    g->buf_bytes = 4096;
    CheckHip(hipMalloc(&g->buf, g->buf_bytes), "hipMalloc(rccl warm-up)");
  }
  const int dev = device_;
  std::thread([g, id, nranks, rank, config, dev]() mutable {
    (void)hipSetDevice(dev);
    ncclComm_t c = nullptr;
    ncclResult_t r = ncclCommInitRankConfig(&c, nranks, id, rank, &config);
    {
      std::lock_guard<std::mutex> lk(g->mu);
      if (g->abandoned) {
        g->done = true;
        if (c != nullptr) ncclCommAbort(c);
        g_live_abandoned.fetch_sub(1);
        return;
      }
    }
    hipStream_t ws = g->stream;
    char *wbuf = g->buf;
    if (r == ncclSuccess && nranks > 1) {
      // every p2p pair (RCCL connects send/recv channels lazily inside ncclGroupEnd) and the
      // allreduce paths, 1-byte p2p payloads
      r = ncclGroupStart();
      for (int p = 0; p < nranks && r == ncclSuccess; ++p) {
        if (p == rank) continue;
        r = ncclSend(wbuf + 64 * (p % 32), 1, ncclUint8, p, c, ws);
        if (r == ncclSuccess) r = ncclRecv(wbuf + 2048 + 64 * (p % 32), 1, ncclUint8, p, c, ws);
      }
      const ncclResult_t e = ncclGroupEnd();
      if (r == ncclSuccess) r = e;
      const size_t classes[3] = {64u << 10, 4u << 20, g->buf_bytes};
      size_t last = 0;
      for (size_t bytes : classes) {
        bytes = std::min(bytes, g->buf_bytes);
        if (r != ncclSuccess || bytes <= last) continue;
        last = bytes;
        r = ncclAllReduce(wbuf, wbuf, bytes / 4, ncclFloat32, ncclSum, c, ws);
      }
    }
    bool abandoned;
    {
      std::lock_guard<std::mutex> lk(g->mu);
      g->comm = c;
      g->result = r;
      g->done = true;
      abandoned = g->abandoned;
    }
    g->cv.notify_all();
    if (abandoned) {
      if (c != nullptr) ncclCommAbort(c);  // nobody else will ever use it
      g_live_abandoned.fetch_sub(1);
    }
  }).detach();
  core::WaitScope waiting;  // the bootstrap waits on every peer
  using clock = std::chrono::steady_clock;
  const auto t0 = clock::now();
  const double limit = cfg_.comm_init_timeout_sec;
  bool done = false;
  Status fail = Status::kSuccess;
  {
    std::unique_lock<std::mutex> lk(g->mu);
    for (;;) {
      g->cv.wait_for(lk, std::chrono::milliseconds(2), [&]() { return g->done; });
      if (g->done) {
        done = true;
        break;
      }
      const double waited = std::chrono::duration<double>(clock::now() - t0).count();
      if (probe && waited > 1e-3) {
        lk.unlock();
        const bool dead = probe();
        lk.lock();
        if (g->done) {
          done = true;
          break;
        }
        if (dead) {
          fail = Status::kAborted;
          break;
        }
      }
      if (limit > 0 && waited > limit) {
        fail = Status::kTimeout;
        break;
      }
    }
    if (!done) {
      g->abandoned = true;  // the helper aborts what it built, if it ever returns
      g_live_abandoned.fetch_add(1);
    }
  }
  if (!done) {
    rccl_aborts_ += 1;
    init_abandoned_ += 1;
    // an abandoned bring-up counts like an aborted op: a job whose communicators never come up
    // stops after rccl_max_failures of them instead of leaking helpers forever
    rccl_fail_streak_ += 1;
    utils::HandleLogInfo("[xrabit] RCCL communicator bring-up %s after %.1f s: abandoned (the "
                         "helper thread stays blocked in RCCL's bootstrap; %d live)\n",
                         fail == Status::kTimeout ? "timed out" : "lost a peer",
                         std::chrono::duration<double>(clock::now() - t0).count(),
                         g_live_abandoned.load());
    utils::Check(cfg_.rccl_max_failures <= 0 || rccl_fail_streak_ <= cfg_.rccl_max_failures,
                 "RCCL bring-up failed %d times in a row; giving up", rccl_fail_streak_);
    return fail;
  }
  comm_ = g->comm;
  if (g->result != ncclSuccess) {
    utils::HandleLogInfo("[xrabit] RCCL communicator bring-up failed: %s\n",
                         ncclGetErrorString(g->result));
    rccl_fail_streak_ += 1;
    if (comm_ != nullptr) {
      rccl_aborts_ += 1;
      AbortComm();
    }
    comm_ = nullptr;
    // the warm-up kernels were aborted with the communicator: let them leave the stream
    DrainBringUp(g->stream);
    utils::Check(cfg_.rccl_max_failures <= 0 || rccl_fail_streak_ <= cfg_.rccl_max_failures,
                 "RCCL bring-up failed %d times in a row; giving up", rccl_fail_streak_);
    return Status::kAborted;
  }
  nranks_ = nranks;
  rank_ = rank;
  if (nranks > 1) {
    // the warm-up kernels need every peer as well: wait like for any collective (probe,
    // deadline, abort on failure)
    hipEvent_t ev = nullptr;
    CheckHip(hipEventCreateWithFlags(&ev, hipEventDisableTiming), "hipEventCreate(warm-up)");
    CheckHip(hipEventRecord(ev, g->stream), "hipEventRecord(warm-up)");
    op_bytes_ = g->buf_bytes;
    const Status s = WaitEvent(ev, probe);
    (void)hipEventDestroy(ev);
    if (s != Status::kSuccess) {
      DrainBringUp(g->stream);
      return s;  // WaitEvent aborted the communicator
    }
  }
  return Status::kSuccess;
}

void DevicePlane::DrainBringUp(hipStream_t s) {
  using clock = std::chrono::steady_clock;
  const auto t0 = clock::now();
  while (hipStreamQuery(s) == hipErrorNotReady &&
         std::chrono::duration<double>(clock::now() - t0).count() < cfg_.drain_timeout_sec) {
    std::this_thread::sleep_for(std::chrono::milliseconds(1));
  }
  (void)hipGetLastError();
}

bool DevicePlane::MockRcclFault() {
  rccl_calls_ += 1;
  if (cfg_.mock_rccl_error > 0 && rccl_calls_ == static_cast<uint64_t>(cfg_.mock_rccl_error)) {
    utils::HandleLogInfo("[xrabit] mock: RCCL call %llu fails with ncclRemoteError\n",
                         static_cast<unsigned long long>(rccl_calls_));
    return true;
  }
  return false;
}

Status DevicePlane::FailRccl(const char *what, int result) {
  const ncclResult_t r = static_cast<ncclResult_t>(result);
  if (ClassifyRccl(result) == RcclOutcome::kFatal) {
    utils::Error("RCCL error in %s: %s", what, ncclGetErrorString(r));
  }
  rccl_aborts_ += 1;
  rccl_fail_streak_ += 1;
  utils::Check(cfg_.rccl_max_failures <= 0 || rccl_fail_streak_ <= cfg_.rccl_max_failures,
               "RCCL failed %d times in a row (last: %s in %s); giving up", rccl_fail_streak_,
               ncclGetErrorString(r), what);
  utils::HandleLogInfo("[xrabit] RCCL %s in %s: aborting the communicator, recovering\n",
                       ncclGetErrorString(r), what);
  AbortComm();
  return Status::kAborted;
}

Status DevicePlane::Settle(const char *what, const FailureProbe &probe, double limit_sec) {
  core::WaitScope waiting;  // RCCL init / lazy connection setup waits on the peers
  using clock = std::chrono::steady_clock;
  const auto t0 = clock::now();
  rccl_settled_ += 1;
  for (uint64_t iter = 0;; ++iter) {
    ncclResult_t st = ncclInProgress;
    const ncclResult_t q = ncclCommGetAsyncError(comm_, &st);
    if (q != ncclSuccess) st = q;
    if (st == ncclSuccess) return Status::kSuccess;
    if (st != ncclInProgress) return FailRccl(what, st);
    const double waited = std::chrono::duration<double>(clock::now() - t0).count();
    if (probe && (iter & 7) == 0 && waited > 1e-3 && probe()) {
      utils::HandleLogInfo("[xrabit] a peer failed during %s: aborting the communicator\n", what);
      rccl_aborts_ += 1;
      AbortComm();
      return Status::kAborted;
    }
    if (limit_sec > 0 && waited > limit_sec) {
      utils::HandleLogInfo("[xrabit] %s did not complete within %.1f s: aborting the "
                           "communicator\n", what, limit_sec);
      rccl_aborts_ += 1;
      AbortComm();
      return Status::kTimeout;
    }
    // lazy connection setup takes milliseconds: spin briefly, then poll every 100 us
    if (waited > 2e-4) std::this_thread::sleep_for(std::chrono::microseconds(100));
  }
}

Status DevicePlane::Rccl(int result, const char *what, const FailureProbe &probe) {
  switch (ClassifyRccl(result)) {
    case RcclOutcome::kOk: return Status::kSuccess;
    case RcclOutcome::kPending: {
      const double limit =
          cfg_.op_timeout_sec < 0 ? AutoOpDeadline(op_bytes_) : cfg_.op_timeout_sec;
      return Settle(what, probe, limit);
    }
    default: return FailRccl(what, result);
  }
}

Status DevicePlane::RunP2P(const std::vector<P2POp> &ops,
                           const std::function<char *(size_t, const P2POp &)> &at,
                           const char *what, const FailureProbe &probe) {
  if (ops.empty()) return Status::kSuccess;
  if (MockRcclFault()) return FailRccl(what, ncclRemoteError);
  ncclResult_t r = ncclGroupStart();
  if (r != ncclSuccess) return Rccl(r, what, probe);
  for (size_t i = 0; i < ops.size() && r == ncclSuccess; ++i) {
    const P2POp &o = ops[i];
    char *p = at(i, o);
    r = o.send ? ncclSend(p, o.bytes, ncclUint8, o.peer, comm_, stream_)
               : ncclRecv(p, o.bytes, ncclUint8, o.peer, comm_, stream_);
  }
  // the group is always closed (a failed call inside it is reported by ncclGroupEnd too)
  const ncclResult_t e = ncclGroupEnd();
  return Rccl(r != ncclSuccess ? r : e, what, probe);
}

void DevicePlane::AbortComm() {
  if (peers_ != nullptr) {
    peers_->SignalAbort();  // spinning barriers give up; later kernels of the group are guarded
  }
  if (comm_ != nullptr) {
    ncclCommAbort(comm_);
    comm_ = nullptr;
  }
  // whatever was in flight must now end: aborted RCCL kernels and barriers return promptly;
  // a stream that does not drain holds work of this rank that will never finish
  if (!DrainStream(cfg_.drain_timeout_sec)) {
    WedgedExit("the device stream did not drain after the communicators were aborted");
  }
  peers_.reset();
}

void DevicePlane::DropComm() {
  if (comm_ != nullptr) {
    ncclCommAbort(comm_);
    comm_ = nullptr;
  }
}

void DevicePlane::InjectHang(double max_sec) {
  int *w = g_hang_release.load();
  if (w == nullptr) {
    void *p = nullptr;
    CheckHip(hipHostMalloc(&p, 64, hipHostMallocCoherent | hipHostMallocMapped),
             "hipHostMalloc(hang word)");
    w = static_cast<int *>(p);
    g_hang_release.store(w);
  }
  __atomic_store_n(w, 0, __ATOMIC_SEQ_CST);
  int khz = 100000;
  (void)hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, device_);
  const long long ticks = static_cast<long long>(max_sec * khz * 1000.0);
  CheckHip(LaunchHang(w, ticks, stream_), "LaunchHang");
}

void DevicePlane::ReleaseHang() {
  int *w = g_hang_release.load();
  if (w != nullptr) __atomic_store_n(w, 1, __ATOMIC_SEQ_CST);
}

bool DevicePlane::DrainStream(double sec) {
  using clock = std::chrono::steady_clock;
  const auto t0 = clock::now();
  for (;;) {
    const hipError_t e = hipStreamQuery(stream_);
    if (e == hipSuccess) return true;
    if (e != hipErrorNotReady) {
      (void)hipGetLastError();
      return true;  // a failed stream is not a hung one: the error surfaces on its next use
    }
    if (std::chrono::duration<double>(clock::now() - t0).count() > sec) return false;
    std::this_thread::sleep_for(std::chrono::milliseconds(1));
  }
}

void DevicePlane::WedgedExit(const char *why) {
  fprintf(stderr, "xrabit: %s: device stream wedged, exiting for a restart\n", why);
  fflush(stderr);
  ReleaseHang();
  // a released injected hang and the guarded kernels behind it retire within microseconds;
  // give them that time before the process and its queues go away (no blocking HIP call here:
  // a really wedged stream would never return from it)
  std::this_thread::sleep_for(std::chrono::milliseconds(200));
  utils::ExitProcess(kDeviceHangExitCode);
}

bool DevicePlane::Preflight(const std::vector<PeerRecord> &all, int rank, std::string *why) {
  links_.clear();
  char mine[32] = {0};
  (void)hipDeviceGetPCIBusId(mine, sizeof(mine), device_);
  bool ok = true;
  for (int r = 0; r < static_cast<int>(all.size()); ++r) {
    if (r == rank) continue;
    PeerLinkInfo li;
    li.rank = r;
    char pci[sizeof(all[r].pci) + 1] = {0};
    std::memcpy(pci, all[r].pci, sizeof(all[r].pci));
    li.same_gpu = std::strncmp(pci, mine, sizeof(mine)) == 0;
    int ord = -1;
    if (pci[0] != '\0' && hipDeviceGetByPCIBusId(&ord, pci) == hipSuccess) {
      li.ordinal = ord;
    } else {
      (void)hipGetLastError();
    }
    if (li.ordinal >= 0 && !li.same_gpu) {
      int can = 0;
      if (hipDeviceCanAccessPeer(&can, device_, li.ordinal) == hipSuccess) {
        li.can_access = can;
      } else {
        (void)hipGetLastError();
      }
      uint32_t type = 0, hops = 0;
      if (hipExtGetLinkTypeAndHopCount(device_, li.ordinal, &type, &hops) == hipSuccess) {
        li.link_type = static_cast<int>(type);
        li.hops = static_cast<int>(hops);
      } else {
        (void)hipGetLastError();
      }
      if (li.can_access == 0 && ok) {
        ok = false;
        *why = "GPU " + std::to_string(device_) + " cannot access the GPU of rank " +
               std::to_string(r) + " (" + pci + ")";
      }
      if (li.can_access == 1) {
        // kernels of this process read and write the peer's mapped buffers directly (the IPC
        // mapping's lazy flag covers the same; enabling it here makes the order explicit)
        DeviceGuard dg(device_);
        const hipError_t e = hipDeviceEnablePeerAccess(li.ordinal, 0);
        if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled) {
          utils::HandleLogInfo("[xrabit] hipDeviceEnablePeerAccess(%d -> %d): %s\n", device_,
                               li.ordinal, hipGetErrorString(e));
        }
        (void)hipGetLastError();
      }
    }
    links_.push_back(li);
  }
  return ok;
}

std::string DevicePlane::PeerLinksJson() const {
  std::string out = "[";
  for (size_t i = 0; i < links_.size(); ++i) {
    const PeerLinkInfo &l = links_[i];
    const char *type = l.same_gpu ? "same_gpu"
                                  : (l.link_type == 4 ? "xgmi"
                                                      : (l.link_type == 2 ? "pcie" : "unknown"));
    char buf[192];
    snprintf(buf, sizeof(buf),
             "%s{\"rank\":%d,\"ordinal\":%d,\"can_access\":%d,\"link\":\"%s\",\"hops\":%d}",
             i ? "," : "", l.rank, l.ordinal, l.can_access, type, l.hops);
    out += buf;
  }
  return out + "]";
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
    peers_->set_fused(cfg_.fused_mode == 1);  // auto: classic until the calibration decides
    peers_->set_fused_grid(cfg_.fused_grid);
    peers_->set_fused_oneshot_max(cfg_.fused_oneshot_max);
    peers_->set_fused_min_bytes(cfg_.fused_min_bytes);
    peers_->set_done_signal(cfg_.done_word);
    peers_->set_peer_abort(cfg_.peer_abort);
    peers_->set_bcast_chunk(cfg_.bcast_chunk);
    // pipelined push form: forced on (with push), or off until the calibration decides
    peers_->set_pipeline(cfg_.pipeline_mode == 1);
    peers_->set_pipeline_chunk(cfg_.pipeline_chunk);
    peers_->set_defer_second(cfg_.defer_second);
    peers_->set_zero_copy_min(cfg_.zero_copy_min);
    // a new group starts from the configured form; a calibration (or its adoption) replaces it
    SetDefaultForm(cfg_.direct_mode == 2, cfg_.pipeline_mode == 1, cfg_.fused_mode == 1);
    transport_bands_.clear();
    form_bands_.clear();
    form_forced_ = false;
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

std::string DevicePlane::RegistryJson() const {
  if (peers_ == nullptr) return "{}";
  const PeerRegistry &r = peers_->registry();
  return "{\"exports\":" + std::to_string(r.exports()) + ",\"imports\":" +
         std::to_string(r.imports()) + ",\"pending\":" + std::to_string(r.pending()) +
         ",\"unexportable\":" + std::to_string(r.unexportable()) + ",\"zero_copy_chunks\":" +
         std::to_string(peers_->reg_zero_copy_chunks()) + ",\"opened\":" +
         (r.opened() ? "true" : "false") + "}";
}

bool DevicePlane::DirectPhaseUs(double out[PeerGroup::kPhases], uint64_t *nops) const {
  if (peers_ == nullptr || peers_->timed_ops() == 0) return false;
  *nops = peers_->timed_ops();
  for (int k = 0; k < PeerGroup::kPhases; ++k) out[k] = peers_->phase_ms()[k] * 1e3 / *nops;
  return true;
}

void DevicePlane::DropPeers() {
  if (peers_ != nullptr) {
    if (!DrainStream(cfg_.drain_timeout_sec)) {
      peers_->SignalAbort();
      if (!DrainStream(cfg_.drain_timeout_sec)) WedgedExit("dropping the direct transport");
    }
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
  return WaitUntil([ev]() { return hipEventQuery(ev); }, probe);
}

Status DevicePlane::WaitWord(const volatile unsigned long long *word, unsigned long long epoch,
                             const FailureProbe &probe) {
  return WaitUntil(
      [word, epoch]() {
        return __atomic_load_n(word, __ATOMIC_ACQUIRE) >= epoch ? hipSuccess : hipErrorNotReady;
      },
      probe);
}

template <typename Poll>
Status DevicePlane::WaitUntil(const Poll &poll, const FailureProbe &probe) {
  trace::Scope ts("device_wait", rank_, -1, -1, op_bytes_, 1);
  core::WaitScope waiting;  // peers' barriers and RCCL: waiting on other ranks
  core::DeviceWaitScope on_gpu;
  using clock = std::chrono::steady_clock;
  const auto t0 = clock::now();
  const double limit = cfg_.op_timeout_sec < 0 ? AutoOpDeadline(op_bytes_) : cfg_.op_timeout_sec;
  core::DeviceDeadlineScope deadline(limit);  // the watchdog leaves this wait to the deadline
  for (uint64_t iter = 0;; ++iter) {
    hipError_t e = poll();
    if (e == hipSuccess) {
      if (peers_ != nullptr && peers_->failed()) {
        const int why = peers_->fail_reason();
        utils::HandleLogInfo("[xrabit] direct transport: a peer barrier gave up "
                             "(%s; registry %s)\n",
                             why == 1   ? "abort raised"
                             : why == 2 ? "a zero-copy source was not mapped"
                             : why == 3 ? "deadline"
                             : why == 4 ? "a peer aborted the group"
                                        : "unknown",
                             RegistryJson().c_str());
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
    // the host's view of the peers (their links), about once a millisecond once the op has
    // waited that long: the rank that notices a death first aborts every rank's kernels
    // (PeerGroup::SignalAbort), so this interval is most of the job's detection latency
    if (probe && (iter & 15) == 0 && waited > 1e-3 && probe()) {
      AbortComm();  // drains the stream, or ends the process if this rank's work is wedged
      return Status::kAborted;
    }
    if (limit > 0 && waited > limit) {
      utils::HandleLogInfo("[xrabit] device op (%zu B) exceeded its %.1f s deadline, aborting "
                           "the communicators\n", op_bytes_, limit);
      AbortComm();
      return Status::kTimeout;
    }
    // spin first: the wake-up latency after completion sits on the critical path of every op
    const int spin = spin_us_override_ >= 0 ? spin_us_override_ : cfg_.spin_us;
    if (waited * 1e6 > spin) std::this_thread::sleep_for(std::chrono::microseconds(10));
  }
}

Status DevicePlane::Finish(const FailureProbe &probe, bool host_wait) {
  // the "done" event is recorded only where something waits on it: a record costs ~3 us of
  // release fence between back-to-back ops (tools/event_fence_probe.hip), and an op on the
  // caller's stream with no host wait needs none (stream order is the dependency)
  Status s = Status::kSuccess;
  const volatile unsigned long long *word = nullptr;
  unsigned long long epoch = 0;
  const bool signalled = peers_ != nullptr && peers_->TakeDoneSignal(&word, &epoch);
  if (cfg_.sync && host_wait) {
    if (signalled && pending_dst_ == nullptr) {
      // the op's last kernel stores its completion into pinned host memory: poll that word
      // (no event record / query round trips on the small-op path)
      s = WaitWord(word, epoch, probe);
      done_words_ += 1;
    } else {
      CheckHip(hipEventRecord(ev_done_, stream_), "hipEventRecord(done)");
      s = WaitEvent(ev_done_, probe);
    }
  }
  op_bytes_ = 0;
  if (s == Status::kSuccess) rccl_fail_streak_ = 0;
  if (pending_dst_ != nullptr) {
    if (s == Status::kSuccess) CopyDeviceAsync(pending_dst_, pending_src_, pending_bytes_);
    pending_dst_ = nullptr;
  }
  if (user_stream_ != stream_) {
    CheckHip(hipEventRecord(ev_done_, stream_), "hipEventRecord(done)");
    CheckHip(hipStreamWaitEvent(user_stream_, ev_done_, 0), "hipStreamWaitEvent(user)");
  }
  return s;
}

void DevicePlane::Synchronize() {
  core::WaitScope waiting;
  core::DeviceWaitScope on_gpu;
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

void *DevicePlane::PinnedScratch(size_t bytes) {
  if (bytes > pinned_bytes_) {
    if (pinned_ != nullptr) {
      CheckHip(hipStreamSynchronize(stream_), "hipStreamSynchronize");  // (no copy in flight)
      (void)hipHostFree(pinned_);
      pinned_ = nullptr;
      pinned_bytes_ = 0;
    }
    const size_t want = std::max<size_t>(bytes, 1u << 20);
    CheckHip(hipHostMalloc(&pinned_, want, hipHostMallocDefault), "hipHostMalloc(staging)");
    pinned_bytes_ = want;
  }
  return pinned_;
}

void DevicePlane::StageToHost(void *host, const void *dev, size_t bytes) {
  core::DeviceWaitScope on_gpu;
  CheckHip(hipMemcpyAsync(host, dev, bytes, hipMemcpyDeviceToHost, stream_), "D2H");
  CheckHip(hipStreamSynchronize(stream_), "hipStreamSynchronize");
}

void DevicePlane::StageToDevice(void *dev, const void *host, size_t bytes) {
  core::DeviceWaitScope on_gpu;
  CheckHip(hipMemcpyAsync(dev, host, bytes, hipMemcpyHostToDevice, stream_), "H2D");
  CheckHip(hipStreamSynchronize(stream_), "hipStreamSynchronize");
}

void DevicePlane::PrepareHostStager() {
  if (stager_ != nullptr) return;
  // the pool's share of the host: its threads (OMP_NUM_THREADS or the CPU affinity) divided
  // among this host's ranks, when no count is configured
  int threads = cfg_.host_stage_threads;
  if (threads <= 0 && local_ranks_ > 0) threads = CopyPool::AutoThreads(local_ranks_);
  stager_.reset(new HostStager(device_, cfg_.host_stage_chunk, threads));
  stager_->set_single_stream(cfg_.host_stage_streams == 1);
}

std::string DevicePlane::HostStageJson() const {
  if (stager_ == nullptr) return "{}";
  const HostStager::Times &t = stager_->times();
  char buf[256];
  snprintf(buf, sizeof(buf),
           "{\"runs\":%llu,\"total_ms\":%.3f,\"copy_in_ms\":%.3f,\"copy_out_ms\":%.3f,"
           "\"wait_in_ms\":%.3f,\"wait_out_ms\":%.3f,\"enqueue_ms\":%.3f,\"chunk\":%zu,"
           "\"threads\":%d,\"streams\":%d}",
           static_cast<unsigned long long>(t.runs), t.total * 1e3, t.copy_in * 1e3,
           t.copy_out * 1e3, t.wait_in * 1e3, t.wait_out * 1e3, t.enqueue * 1e3, stager_->chunk(),
           stager_->threads(), stager_->single_stream() ? 1 : 3);
  return buf;
}

Status DevicePlane::LinkProbe(size_t bytes, double out[PeerGroup::kLinkProbeValues]) {
  utils::Check(peers_ != nullptr, "link probe needs the direct transport");
  DeviceGuard dg(device_);
  // a peer that never arrives costs seconds, not the op deadline
  peers_->set_deadline_sec(std::min(cfg_.peer_deadline_sec, 10.0));
  const hipError_t e = peers_->LinkProbe(bytes, out);
  CheckHip(e, "link probe");
  CheckHip(hipStreamSynchronize(stream_), "link probe");
  const bool failed = peers_->failed();
  peers_->set_deadline_sec(cfg_.peer_deadline_sec);
  if (failed) {
    AbortComm();
    return Status::kAborted;
  }
  return Status::kSuccess;
}

Status DevicePlane::AllreduceHostStaged(void *host_out, const void *host_in, size_t count,
                                        int dtype, int op, const FailureProbe &probe) {
  const size_t tn = TypeBytes(dtype), bytes = count * tn;
  char *d = static_cast<char *>(Scratch(bytes, 2));
  PrepareHostStager();
  host_staged_ops_ += 1;
  HostStager::ChunkOp chunk_op = [&](size_t off, size_t len) {
    return Allreduce(d + off, d + off, nullptr, len / tn, dtype, op, kPrepCopy, 1.0, probe);
  };
  // the host copies of the other chunks need the CPUs this wait would spin on: poll with
  // short sleeps instead (a chunk takes milliseconds, the 10 us wake-up granularity is noise)
  HostStager::EventWait wait = [&](hipEvent_t ev) {
    spin_us_override_ = 0;
    const Status w = WaitEvent(ev, probe);
    spin_us_override_ = -1;
    return w;
  };
  op_bytes_ = bytes;
  const Status s = stager_->Run(host_out, host_in, bytes, tn, d, stream_, chunk_op, wait);
  // a small tail chunk may have taken the one-kernel path, whose completion word nobody polls
  // here (the D2H after it was waited for instead)
  const volatile unsigned long long *word = nullptr;
  unsigned long long epoch = 0;
  if (peers_ != nullptr) (void)peers_->TakeDoneSignal(&word, &epoch);
  op_bytes_ = 0;
  if (s == Status::kSuccess) rccl_fail_streak_ = 0;
  return s;
}

Status DevicePlane::Allreduce(const void *send, void *recv, void *recv2, size_t count, int dtype,
                              int op, int prep, double alpha, const FailureProbe &probe) {
  const size_t bytes = count * TypeBytes(dtype);
  op_bytes_ = bytes;
  if (UseDirect(bytes)) {
    ApplyForm(bytes);
    CheckHip(peers_->Allreduce(send, recv, recv2, count, dtype, op, prep, alpha),
             "direct allreduce");
    return Status::kSuccess;
  }
  utils::Check(comm_ != nullptr, "device allreduce without communicator");
  ncclDataType_t t;
  ncclRedOp_t o;
  if (!RcclType(dtype, &t)) utils::Error("unsupported dtype %d on device", dtype);
  // a scaling prepare of a floating sum rides on RCCL's pre-multiplied sum (no extra pass)
  const bool premul = prep == kPrepScale && op == 2 &&
                      (dtype == 6 || dtype == 7 || dtype == 10 || dtype == 11);
  if ((prep != kPrepCopy && !premul) || !RcclOp(op, &o)) {
    // ops RCCL cannot express (BitOR) and prepares it cannot fuse (g*g, |g|): reduce-scatter
    // by grouped point-to-point copies, our reduce kernel applying the prepare as it loads
    // each rank's segment (no separate prepare pass), then the allgather
    const int p = premul ? kPrepCopy : prep;
    PassFn pass = [dtype, op, p, alpha](void *dst, const void *const *srcs, int n, size_t c,
                                        bool acc_first, hipStream_t st) {
      return LaunchReduceMulti(dst, srcs, n, c, dtype, op, st, nullptr, nullptr, 0.0, nullptr, p,
                               alpha, acc_first ? 1 : 0);
    };
    Status s = AllreduceByKernel(send, recv, count, TypeBytes(dtype), pass, probe);
    if (s != Status::kSuccess) return s;
  } else if (premul) {
    ncclRedOp_t pm;
    double a64 = alpha;
    float a32 = static_cast<float>(alpha);
    // fp16/bf16 scalars are passed as the element type by RCCL: convert on the host
    uint16_t a16 = 0;
    void *scalar = &a32;
    if (dtype == 7) {
      scalar = &a64;
    } else if (dtype == 10) {
      a16 = half_t::FromFloat(a32);
      scalar = &a16;
    } else if (dtype == 11) {
      a16 = bf16_t::FromFloat(a32);
      scalar = &a16;
    }
    Status s = Rccl(ncclRedOpCreatePreMulSum(&pm, scalar, t, ncclScalarHostImmediate, comm_),
                    "ncclRedOpCreatePreMulSum", probe);
    if (s != Status::kSuccess) return s;
    s = Rccl(MockRcclFault() ? ncclRemoteError
                             : ncclAllReduce(send, recv, count, t, pm, comm_, stream_),
             "ncclAllReduce", probe);
    if (s != Status::kSuccess) return s;  // the aborted communicator took the op with it
    s = Rccl(ncclRedOpDestroy(pm, comm_), "ncclRedOpDestroy", probe);
    if (s != Status::kSuccess) return s;
  } else {
    Status s = Rccl(MockRcclFault() ? ncclRemoteError
                                    : ncclAllReduce(send, recv, count, t, o, comm_, stream_),
                    "ncclAllReduce", probe);
    if (s != Status::kSuccess) return s;
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

int DevicePlane::GraphAllreduce(void *buf, size_t count, int dtype, int op, hipStream_t stream) {
  ncclDataType_t t;
  ncclRedOp_t o;
  if (!RcclType(dtype, &t) || !RcclOp(op, &o)) return -3;
  if (count == 0) return 0;
  DeviceGuard dg(device_);
  if (peers_ != nullptr && (comm_ == nullptr || UseDirect(count * TypeBytes(dtype)))) {
    ApplyForm(count * TypeBytes(dtype));
    // the direct transport's classic form, barriers numbered on the device (replayable)
    graph_direct_ops_ += 1;
    return peers_->AllreduceGraphable(buf, count, dtype, op, stream) == hipSuccess ? 0 : -5;
  }
  if (comm_ == nullptr) return -2;
  rccl_calls_ += 1;
  ncclResult_t r = ncclAllReduce(buf, buf, count, t, o, comm_, stream);
  if (r == ncclInProgress) {
    // non-blocking communicator: the enqueue completes on RCCL's side (host-side polling only,
    // so this is legal while `stream` is being captured)
    ncclResult_t st = ncclInProgress;
    while (ncclCommGetAsyncError(comm_, &st) == ncclSuccess && st == ncclInProgress) {
      std::this_thread::sleep_for(std::chrono::microseconds(50));
    }
    r = st;
  }
  return r == ncclSuccess ? 0 : -5;
}

Status DevicePlane::AllreduceCustom(const void *send, void *recv, void *recv2, size_t count,
                                    size_t type_nbytes, DeviceReduceLauncher *launcher,
                                    const FailureProbe &probe) {
  const size_t bytes = count * type_nbytes;
  op_bytes_ = bytes;
  if (UseDirect(bytes)) {
    ApplyForm(bytes);
    PeerGroup::ReduceStep step = [launcher](void *dst, const void *const *srcs, int n, size_t c,
                                            const int *guard, const void *const *, double,
                                            hipStream_t st) {
      return static_cast<hipError_t>(launcher(dst, srcs, n, c, guard, st));
    };
    CheckHip(peers_->AllreduceCustom(send, recv, recv2, count, type_nbytes, step),
             "direct allreduce (custom)");
    return Status::kSuccess;
  }
  PassFn pass = [launcher](void *dst, const void *const *srcs, int n, size_t c, bool,
                           hipStream_t st) {
    return static_cast<hipError_t>(launcher(dst, srcs, n, c, nullptr, st));
  };
  Status s = AllreduceByKernel(send, recv, count, type_nbytes, pass, probe);
  if (s != Status::kSuccess) return s;
  if (recv2 != nullptr && recv2 != recv) {
    pending_dst_ = recv2;
    pending_src_ = recv;
    pending_bytes_ = bytes;
  }
  return Status::kSuccess;
}

Status DevicePlane::AllreduceByKernel(const void *send, void *recv, size_t count, size_t tn,
                                      const PassFn &pass, const FailureProbe &probe) {
  utils::Check(comm_ != nullptr, "device allreduce without communicator");
  // reduce-scatter + allgather as two rounds of grouped point-to-point copies that read and
  // write the buffers in place (p2p_plan.h: segments are whole 256-element blocks, so every
  // segment start is as aligned as the buffer): no packing into scratch, no unpacking
  const SegmentPlan plan(count, tn, nranks_);
  const char *in = static_cast<const char *>(send);
  char *out = static_cast<char *>(recv);
  char *inbox = static_cast<char *>(Scratch(plan.inbox_bytes(rank_), 1));
  char *bufs[3] = {const_cast<char *>(in), out, inbox};
  auto at = [&bufs](size_t, const P2POp &o) { return bufs[o.buf] + o.offset; };
  // 1. segment k of every rank's input goes to rank k
  Status s = RunP2P(plan.ScatterOps(rank_), at, "allreduce reduce-scatter", probe);
  if (s != Status::kSuccess) return s;
  // 2. reduce the n copies of my segment (rank order, up to 8 sources per pass) into place
  char *dst = out + plan.lo(rank_) * tn;
  std::vector<const void *> srcs;
  for (const std::vector<int> &p : plan.ReducePasses(rank_, kMaxReduceSources)) {
    srcs.clear();
    for (int k : p) {
      const void *own = in + plan.lo(rank_) * tn;
      const void *slot = inbox + static_cast<size_t>(k) * plan.slot_bytes(rank_);
      srcs.push_back(k < 0 ? static_cast<const void *>(dst) : (k == rank_ ? own : slot));
    }
    CheckHip(pass(dst, srcs.data(), static_cast<int>(srcs.size()), plan.elems(rank_), p[0] < 0,
                  stream_),
             "allreduce reduce step");
  }
  // 3. every reduced segment to every rank, straight into its place in recv
  return RunP2P(plan.GatherOps(rank_), at, "allreduce allgather", probe);
}

Status DevicePlane::Broadcast(void *buf, size_t bytes, int root, const FailureProbe &probe,
                              void *log) {
  op_bytes_ = bytes;
  if (UseDirectBcast(bytes)) {
    CheckHip(peers_->Broadcast(buf, bytes, root, log), "direct broadcast");
    return Status::kSuccess;
  }
  utils::Check(comm_ != nullptr, "device broadcast without communicator");
  Status s = Rccl(MockRcclFault() ? ncclRemoteError
                                  : ncclBroadcast(buf, buf, bytes, ncclUint8, root, comm_, stream_),
                  "ncclBroadcast", probe);
  if (s == Status::kSuccess && log != nullptr && log != buf) {
    pending_dst_ = log;  // copied by Finish once the op is known to have succeeded
    pending_src_ = buf;
    pending_bytes_ = bytes;
  }
  return s;
}

Status DevicePlane::Exchange(const std::vector<ExchangeItem> &plan, size_t *bytes_in,
                             const FailureProbe &probe) {
  *bytes_in = 0;
  op_bytes_ = 0;
  for (const ExchangeItem &x : plan) op_bytes_ += x.bytes;
  const bool direct = peers_ != nullptr && (comm_ == nullptr || force_ == 1);
  if (direct) {
    CheckHip(peers_->Exchange(plan, bytes_in), "direct exchange");
    return Status::kSuccess;
  }
  // a copy to itself is a local kernel; the rest pairs up as ncclSend / ncclRecv (p2p_plan.h:
  // every rank walks the same plan in the same order, so the k-th send from s to d meets the
  // k-th receive at d from s)
  std::vector<size_t> item_of, local;
  const std::vector<P2POp> ops = ExchangeOps(plan, rank_, &item_of, &local);
  for (size_t i : local) CopyDeviceAsync(plan[i].dst_ptr, plan[i].src_ptr, plan[i].bytes);
  if (ops.empty()) return Status::kSuccess;
  utils::Check(comm_ != nullptr, "device exchange without a transport");
  for (const P2POp &o : ops) {
    if (!o.send) *bytes_in += o.bytes;
  }
  auto at = [&plan, &item_of](size_t i, const P2POp &o) {
    const ExchangeItem &x = plan[item_of[i]];
    return o.send ? static_cast<char *>(const_cast<void *>(x.src_ptr))
                  : static_cast<char *>(x.dst_ptr);
  };
  return RunP2P(ops, at, "exchange", probe);
}

Status DevicePlane::AllgatherResolved(void *buf, size_t total, size_t begin, size_t size,
                                      void *log) {
  utils::Check(peers_ != nullptr && UseDirect(total), "resolved allgather needs the direct path");
  op_bytes_ = total;
  CheckHip(peers_->AllgatherResolved(buf, total, begin, size, log), "direct allgather");
  return Status::kSuccess;
}

Status DevicePlane::AllgatherV(void *buf_, size_t total, const std::vector<size_t> &begin,
                               const std::vector<size_t> &size, const FailureProbe &probe,
                               void *log) {
  op_bytes_ = total;
  if (UseDirect(total)) {
    CheckHip(peers_->AllgatherV(buf_, total, begin, size, log), "direct allgather");
    return Status::kSuccess;
  }
  utils::Check(comm_ != nullptr, "device allgather without communicator");
  char *buf = static_cast<char *>(buf_);
  Status s;
  if (AllgatherUniform(total, begin, size)) {
    s = Rccl(MockRcclFault() ? ncclRemoteError
                             : ncclAllGather(buf + begin[rank_], buf, size[0], ncclUint8, comm_,
                                             stream_),
             "ncclAllGather", probe);
  } else if (MockRcclFault()) {
    s = FailRccl("allgather", ncclRemoteError);
  } else {
    // variable, wrapping slices: one broadcast per piece (p2p_plan.h), in one group
    ncclResult_t r = ncclGroupStart();
    if (r != ncclSuccess) return Rccl(r, "allgather", probe);
    for (const BcastPiece &p : AllgatherPieces(total, begin, size)) {
      if (r != ncclSuccess) break;
      r = ncclBroadcast(buf + p.offset, buf + p.offset, p.bytes, ncclUint8, p.root, comm_,
                        stream_);
    }
    const ncclResult_t e = ncclGroupEnd();
    s = Rccl(r != ncclSuccess ? r : e, "allgather", probe);
  }
  if (s == Status::kSuccess && log != nullptr && log != buf) {
    pending_dst_ = log;
    pending_src_ = buf;
    pending_bytes_ = total;
  }
  return s;
}
}  // namespace device
}  // namespace rabit
