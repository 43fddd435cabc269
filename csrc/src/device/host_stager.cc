/*!
 * \file host_stager.cc
 * \brief Pipelined host <-> HBM staging of host-buffer collectives (see host_stager.h).
 */
#include "device/host_stager.h"

#include <sched.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>

#include "device/device_plane.h"
#include "rabit/internal/timer.h"
#include "rabit/internal/utils.h"

namespace rabit {
namespace device {

// ---------------------------------------------------------------- CopyPool
CopyPool::CopyPool(int threads) {
  for (int i = 1; i < std::max(threads, 1); ++i) workers_.emplace_back([this]() { Work(); });
}

CopyPool::~CopyPool() {
  {
    std::lock_guard<std::mutex> lk(mu_);
    stop_ = true;
  }
  cv_.notify_all();
  for (auto &t : workers_) t.join();
}

int CopyPool::HostShare() {
  int share = 0;
  if (const char *omp = getenv("OMP_NUM_THREADS")) share = atoi(omp);
  if (share <= 0) {
    cpu_set_t set;
    CPU_ZERO(&set);
    share = sched_getaffinity(0, sizeof(set), &set) == 0 ? CPU_COUNT(&set) : 1;
  }
  return std::max(1, share);
}

int CopyPool::AutoThreads(int local) {
  if (local <= 0) {
    local = 1;
    if (const char *l = getenv("LOCAL_WORLD_SIZE")) local = std::max(1, atoi(l));
  }
  return std::min(8, std::max(1, HostShare() / local));
}

bool CopyPool::TakePiece(uint64_t gen) {
  char *dst;
  const char *src;
  size_t lo, hi;
  {
    std::lock_guard<std::mutex> lk(mu_);
    if (gen != gen_ || next_ >= pieces_) return false;
    const int p = next_++;
    lo = static_cast<size_t>(p) * piece_;
    hi = std::min(n_, lo + piece_);
    dst = dst_;
    src = src_;
  }
  // pieces are >= 64 KiB: two lock round trips per piece are noise next to the memcpy
  if (hi > lo) std::memcpy(dst + lo, src + lo, hi - lo);
  bool last;
  {
    std::lock_guard<std::mutex> lk(mu_);
    last = ++done_ == pieces_;
  }
  if (last) done_cv_.notify_all();
  return true;
}

void CopyPool::Work() {
  uint64_t seen = 0;
  for (;;) {
    {
      std::unique_lock<std::mutex> lk(mu_);
      cv_.wait(lk, [&]() { return stop_ || gen_ != seen; });
      if (stop_) return;
      seen = gen_;
    }
    while (TakePiece(seen)) {
    }
  }
}

void CopyPool::Copy(void *dst, const void *src, size_t n) {
  if (n == 0) return;
  const int t = threads();
  if (t == 1 || n < (size_t(1) << 20)) {
    std::memcpy(dst, src, n);
    return;
  }
  uint64_t gen;
  {
    std::lock_guard<std::mutex> lk(mu_);
    dst_ = static_cast<char *>(dst);
    src_ = static_cast<const char *>(src);
    n_ = n;
    // 2 pieces per thread, 64 KiB aligned, so a late-waking helper does not hold up the rest
    piece_ = ((n + 2 * t - 1) / (2 * t) + (64u << 10) - 1) / (64u << 10) * (64u << 10);
    pieces_ = static_cast<int>((n + piece_ - 1) / piece_);
    next_ = 0;
    done_ = 0;
    gen = ++gen_;
  }
  cv_.notify_all();
  while (TakePiece(gen)) {
  }
  std::unique_lock<std::mutex> lk(mu_);
  done_cv_.wait(lk, [&]() { return done_ == pieces_; });
}

// ---------------------------------------------------------------- HostStager
HostStager::HostStager(int device, size_t chunk, int threads)
    : device_(device),
      chunk_(std::max<size_t>(chunk, 1u << 20) / 4096 * 4096),
      pool_(threads > 0 ? threads : CopyPool::AutoThreads()) {
  DeviceGuard dg(device_);
  CheckHip(hipStreamCreateWithFlags(&h2d_, hipStreamNonBlocking), "hipStreamCreate(h2d)");
  CheckHip(hipStreamCreateWithFlags(&d2h_, hipStreamNonBlocking), "hipStreamCreate(d2h)");
  for (int s = 0; s < 2; ++s) {
    CheckHip(hipHostMalloc(reinterpret_cast<void **>(&pin_in_[s]), chunk_), "hipHostMalloc(in)");
    CheckHip(hipHostMalloc(reinterpret_cast<void **>(&pin_out_[s]), chunk_), "hipHostMalloc(out)");
    for (hipEvent_t *e : {&ev_in_[s], &ev_op_[s], &ev_out_[s]}) {
      CheckHip(hipEventCreateWithFlags(e, hipEventDisableTiming), "hipEventCreate(stage)");
    }
  }
}

HostStager::~HostStager() {
  DeviceGuard dg(device_);
  (void)hipStreamSynchronize(h2d_);
  (void)hipStreamSynchronize(d2h_);
  for (int s = 0; s < 2; ++s) {
    (void)hipHostFree(pin_in_[s]);
    (void)hipHostFree(pin_out_[s]);
    (void)hipEventDestroy(ev_in_[s]);
    (void)hipEventDestroy(ev_op_[s]);
    (void)hipEventDestroy(ev_out_[s]);
  }
  (void)hipStreamDestroy(h2d_);
  (void)hipStreamDestroy(d2h_);
}

net::Status HostStager::Run(void *host_out, const void *host_in, size_t bytes, size_t align,
                            char *dev, hipStream_t plane, const ChunkOp &op,
                            const EventWait &wait) {
  DeviceGuard dg(device_);
  char *out = static_cast<char *>(host_out);
  const char *in = static_cast<const char *>(host_in);
  const size_t step = std::max<size_t>(chunk_ / std::max<size_t>(align, 1) * align, align);
  const size_t nchunks = (bytes + step - 1) / step;
  auto off_of = [step](size_t k) { return k * step; };
  auto len_of = [step, bytes](size_t k) { return std::min(step, bytes - k * step); };
  net::Status st = net::Status::kSuccess;
  const double t_start = utils::GetTime();
  // the CPU copy of chunk k's result out of its pinned slot (its D2H waited for first)
  auto drain_out = [&](size_t k) {
    const int s = static_cast<int>(k & 1);
    double t0 = utils::GetTime();
    const net::Status w = wait(ev_out_[s]);
    const double t1 = utils::GetTime();
    times_.wait_out += t1 - t0;
    if (w != net::Status::kSuccess) return w;
    pool_.Copy(out + off_of(k), pin_out_[s], len_of(k));
    times_.copy_out += utils::GetTime() - t1;
    return net::Status::kSuccess;
  };
  for (size_t k = 0; k < nchunks && st == net::Status::kSuccess; ++k) {
    const int s = static_cast<int>(k & 1);
    const size_t off = off_of(k), len = len_of(k);
    // 1. the slot's previous H2D (chunk k-2) has read it: refill it from pageable memory
    const double t0 = utils::GetTime();
    CheckHip(hipEventSynchronize(ev_in_[s]), "stage slot (in)");
    const double t1 = utils::GetTime();
    pool_.Copy(pin_in_[s], in + off, len);
    const double t2 = utils::GetTime();
    times_.wait_in += t1 - t0;
    times_.copy_in += t2 - t1;
    hipStream_t in_stream = single_stream_ ? plane : h2d_;
    hipStream_t out_stream = single_stream_ ? plane : d2h_;
    CheckHip(hipMemcpyAsync(dev + off, pin_in_[s], len, hipMemcpyHostToDevice, in_stream),
             "H2D chunk");
    CheckHip(hipEventRecord(ev_in_[s], in_stream), "hipEventRecord(in)");
    // 2. the collective on the chunk once it has landed
    if (!single_stream_) {
      CheckHip(hipStreamWaitEvent(plane, ev_in_[s], 0), "hipStreamWaitEvent(plane)");
    }
    st = op(off, len);
    if (st != net::Status::kSuccess) break;
    // 3. its result back into the slot's pinned output (the slot's previous content, chunk
    //    k-2, was copied out by iteration k-1 before this enqueue)
    if (!single_stream_) {
      CheckHip(hipEventRecord(ev_op_[s], plane), "hipEventRecord(op)");
      CheckHip(hipStreamWaitEvent(d2h_, ev_op_[s], 0), "hipStreamWaitEvent(d2h)");
    }
    CheckHip(hipMemcpyAsync(pin_out_[s], dev + off, len, hipMemcpyDeviceToHost, out_stream),
             "D2H chunk");
    CheckHip(hipEventRecord(ev_out_[s], out_stream), "hipEventRecord(out)");
    times_.enqueue += utils::GetTime() - t2;
    // 4. meanwhile on the host: the previous chunk's result to the user buffer
    if (k >= 1) st = drain_out(k - 1);
  }
  if (st == net::Status::kSuccess && nchunks > 0) st = drain_out(nchunks - 1);
  times_.total += utils::GetTime() - t_start;
  times_.runs += 1;
  if (st != net::Status::kSuccess) {
    // the failed op aborted the plane's stream, which releases every copy waiting behind it
    (void)hipStreamSynchronize(h2d_);
    (void)hipStreamSynchronize(d2h_);
  }
  return st;
}

}  // namespace device
}  // namespace rabit
