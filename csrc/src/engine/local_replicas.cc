/*!
 * \file local_replicas.cc
 * \brief Slot storage of the replicated local checkpoint state (see local_replicas.h).
 */
#include "engine/local_replicas.h"

#include <algorithm>

#include "device/device_plane.h"
#include "device/dma_copier.h"
#include "device/kernels.h"
#include "rabit/internal/utils.h"

namespace rabit {
namespace engine {

LocalReplicas::~LocalReplicas() {
  if (!on_device_) return;
  (void)hipSetDevice(device_);
  if (dma_) {
    (void)dma_->WaitAll();  // the copier reads slot 0 and writes pinned_
    dma_.reset();
  }
  if (side_ != nullptr) (void)hipStreamSynchronize(side_);
  for (auto &v : slots_) {
    for (auto &s : v) {
      if (s.dev != nullptr) (void)hipFree(s.dev);
    }
  }
  if (pinned_ != nullptr) (void)hipHostFree(pinned_);
  if (ready_ != nullptr) (void)hipEventDestroy(ready_);
  if (done_ != nullptr) (void)hipEventDestroy(done_);
  if (side_ != nullptr) (void)hipStreamDestroy(side_);
}

void LocalReplicas::Configure(int nslot, bool on_device, int device) {
  utils::Check(!configured(), "local replica store configured twice");
  utils::Check(nslot >= 1, "local replica store needs at least one slot");
  nslot_ = nslot;
  on_device_ = on_device;
  device_ = device;
  for (auto &v : slots_) v.assign(nslot, Slot());
  if (on_device_) {
    device::DeviceGuard dg(device_);
    device::CheckHip(hipStreamCreateWithFlags(&side_, hipStreamNonBlocking), "hipStreamCreate");
    device::CheckHip(hipEventCreateWithFlags(&ready_, hipEventDisableTiming), "hipEventCreate");
    device::CheckHip(hipEventCreateWithFlags(&done_, hipEventDisableTiming), "hipEventCreate");
  }
}

int LocalReplicas::Count(int v) const {
  int c = 0;
  for (const auto &s : slots_[v]) c += s.size != kAbsent ? 1 : 0;
  return c;
}

std::vector<int64_t> LocalReplicas::Sizes(int v) const {
  std::vector<int64_t> out(nslot_);
  for (int k = 0; k < nslot_; ++k) out[k] = slots_[v][k].size;
  return out;
}

void LocalReplicas::Clear(int v) {
  for (auto &s : slots_[v]) {
    s.size = kAbsent;
    if (!on_device_) s.host.clear();
  }
}

void *LocalReplicas::Alloc(int v, int k, size_t bytes) {
  utils::Assert(k >= 0 && k < nslot_, "local replica slot %d out of range", k);
  Slot &s = slots_[v][k];
  s.size = static_cast<int64_t>(bytes);
  if (!on_device_) {
    s.host.resize(bytes);
    return &s.host[0];
  }
  if (s.cap < bytes) {
    device::DeviceGuard dg(device_);
    if (s.dev != nullptr) {
      // the old buffer may still be read by queued copies of the plane stream
      device::CheckHip(hipDeviceSynchronize(), "hipDeviceSynchronize");
      device::CheckHip(hipFree(s.dev), "hipFree(local slot)");
      s.dev = nullptr;
    }
    // 2 MiB granules: steady checkpoints of a slowly growing state do not reallocate
    const size_t granule = size_t(2) << 20;
    const size_t cap = std::max<size_t>((bytes + granule - 1) & ~(granule - 1), granule);
    device::CheckHip(hipMalloc(&s.dev, cap), "hipMalloc(local slot)");
    s.cap = cap;
  }
  return s.dev;
}

size_t LocalReplicas::Bytes(int v) const {
  size_t b = 0;
  for (const auto &s : slots_[v]) b += s.size > 0 ? static_cast<size_t>(s.size) : 0;
  return b;
}

void LocalReplicas::set_mirror_sdma(bool sdma) {
  dma_.reset();
  if (!sdma || !on_device_) return;
  std::unique_ptr<device::DmaCopier> d(new device::DmaCopier(device_));
  if (d->ok()) {
    dma_ = std::move(d);
  } else {
    utils::HandleLogInfo("[xrabit] SDMA local mirror unavailable (%s): using hipMemcpyAsync\n",
                         d->why().c_str());
  }
}

void LocalReplicas::Mirror(int v, hipStream_t stream) {
  if (!on_device_ || mirror_off_ || !valid(v, 0) || slots_[v][0].size == 0) return;
  device::DeviceGuard dg(device_);
  if (mirror_pending_) {
    if (dma_) {
      if (!dma_->Done(dma_ticket_)) {
        ++mirrors_skipped_;
        return;
      }
      (void)dma_->Wait(dma_ticket_);  // a failed mirror is simply superseded by this one
    } else {
      const hipError_t e = hipEventQuery(done_);
      if (e == hipErrorNotReady) {
        ++mirrors_skipped_;
        return;
      }
      device::CheckHip(e, "local mirror");
    }
    mirror_pending_ = false;
  }
  const size_t bytes = static_cast<size_t>(slots_[v][0].size);
  if (pinned_cap_ < bytes) {
    if (pinned_ != nullptr) device::CheckHip(hipHostFree(pinned_), "hipHostFree");
    pinned_ = nullptr;
    device::CheckHip(hipHostMalloc(&pinned_, bytes, hipHostMallocDefault), "hipHostMalloc(mirror)");
    pinned_cap_ = bytes;
  }
  device::CheckHip(hipEventRecord(ready_, stream), "hipEventRecord");
  if (dma_) {
    // the copier's thread waits for ready_ and runs the copy on an SDMA engine (no CU time)
    dma_ticket_ = dma_->Submit(pinned_, slots_[v][0].dev, bytes, ready_);
    mirror_pending_ = true;
    mirror_version_ = v;
    ++mirrors_;
    return;
  }
  device::CheckHip(hipStreamWaitEvent(side_, ready_, 0), "hipStreamWaitEvent");
  device::CheckHip(mirror_ctas_ > 0
                       ? device::LaunchCopyNarrow(pinned_, slots_[v][0].dev, bytes, mirror_ctas_,
                                                  side_)
                       : hipMemcpyAsync(pinned_, slots_[v][0].dev, bytes, hipMemcpyDeviceToHost,
                                        side_),
                   "D2H local mirror");
  device::CheckHip(hipEventRecord(done_, side_), "hipEventRecord");
  mirror_pending_ = true;
  mirror_version_ = v;
  ++mirrors_;
}
void LocalReplicas::BeforeWrite(int v, hipStream_t stream) {
  if (!on_device_ || !mirror_pending_ || mirror_version_ != v) return;
  device::DeviceGuard dg(device_);
  if (dma_) {
    // an SDMA job is not on any stream: the host waits until it has read the slot
    (void)dma_->Wait(dma_ticket_);
    mirror_pending_ = false;
    return;
  }
  device::CheckHip(hipStreamWaitEvent(stream, done_, 0), "hipStreamWaitEvent(mirror)");
}
}  // namespace engine
}  // namespace rabit
