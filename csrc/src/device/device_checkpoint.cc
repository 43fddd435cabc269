/*!
 * \file device_checkpoint.cc
 * \brief HBM snapshot checkpoints (see device_checkpoint.h).
 */
#include "device/device_checkpoint.h"

#include <algorithm>
#include <cstring>

#include "device/kernels.h"
#include "rabit/internal/utils.h"

namespace rabit {
namespace device {

DeviceCheckpoint::DeviceCheckpoint(DevicePlane *plane) : plane_(plane) {
  CheckHip(hipStreamCreateWithFlags(&side_, hipStreamNonBlocking), "hipStreamCreate(ckpt)");
  for (auto &h : half_) {
    h.owner = this;
    CheckHip(hipEventCreateWithFlags(&h.d2h_done, hipEventDisableTiming), "hipEventCreate");
    CheckHip(hipEventCreateWithFlags(&h.snap_done, hipEventDisableTiming), "hipEventCreate");
  }
  loader_.owner = this;
}

void DeviceCheckpoint::set_mirror_low_priority(bool low) {
  if (!low) return;
  int least = 0, greatest = 0;
  CheckHip(hipDeviceGetStreamPriorityRange(&least, &greatest), "hipDeviceGetStreamPriorityRange");
  CheckHip(hipStreamSynchronize(side_), "hipStreamSynchronize(ckpt)");
  CheckHip(hipStreamDestroy(side_), "hipStreamDestroy(ckpt)");
  CheckHip(hipStreamCreateWithPriority(&side_, hipStreamNonBlocking, least),
           "hipStreamCreateWithPriority(ckpt)");
}

void DeviceCheckpoint::set_mirror_engine(int engine, int ctas) {
  mirror_engine_ = engine;
  if (ctas > 0) mirror_ctas_ = ctas;
  dma_.reset();
  if (engine == kEngineSdma) {
    std::unique_ptr<DmaCopier> d(new DmaCopier(plane_->device()));
    if (d->ok()) {
      dma_ = std::move(d);
    } else {
      utils::HandleLogInfo("[xrabit] SDMA mirror unavailable (%s): using hipMemcpyAsync\n",
                           d->why().c_str());
      mirror_engine_ = kEngineHip;
    }
  }
}

bool DeviceCheckpoint::MirrorDone(const Half &h) const {
  if (dma_) return dma_->Done(h.ticket);
  const hipError_t q = hipEventQuery(h.d2h_done);
  if (q != hipErrorNotReady) CheckHip(q, "checkpoint mirror query");
  return q == hipSuccess;
}

void DeviceCheckpoint::WaitMirror(const Half &h) const {
  if (dma_) {
    if (!dma_->Wait(h.ticket) && pinned_owner_ == &h) {
      // the copier could not deliver this mirror: redo it synchronously on the side stream so
      // a Save of these bytes reads a complete host copy
      utils::HandleLogInfo("[xrabit] checkpoint mirror failed on the SDMA path: redone with "
                           "hipMemcpyAsync\n");
      size_t off = 0;
      for (size_t i = 0; i < h.sizes.size(); ++i) {
        if (h.sizes[i] != 0) {
          CheckHip(hipMemcpyAsync(pinned_ + off, h.dev[i], h.sizes[i], hipMemcpyDeviceToHost,
                                  side_),
                   "D2H mirror (redo)");
        }
        off += h.sizes[i];
      }
      CheckHip(hipStreamSynchronize(side_), "checkpoint mirror redo");
    }
    return;
  }
  CheckHip(hipEventSynchronize(h.d2h_done), "checkpoint mirror wait");
}

DeviceCheckpoint::~DeviceCheckpoint() {
  if (dma_) (void)dma_->WaitAll();
  dma_.reset();
  (void)hipStreamSynchronize(side_);
  for (auto &h : half_) {
    for (void *p : h.dev) (void)hipFree(p);
    (void)hipEventDestroy(h.d2h_done);
    (void)hipEventDestroy(h.snap_done);
  }
  if (pinned_ != nullptr) (void)hipHostFree(pinned_);
  (void)hipStreamDestroy(side_);
}

size_t DeviceCheckpoint::reserved_bytes() const {
  size_t s = 0;
  for (const auto &h : half_) {
    for (size_t c : h.cap) s += c;
  }
  return s;
}

const Serializable *DeviceCheckpoint::Snapshot(int n, void *const *ptrs, const size_t *nbytes,
                                               const std::string &meta) {
  size_t total = 0;
  for (int i = 0; i < n; ++i) total += nbytes[i];
  if (nslots_ == 0) {
    nslots_ = slots_req_ == 2 || slots_req_ == 3 ? slots_req_
                                                 : (total < three_slot_max_ ? 3 : 2);
  }
  // the oldest slot: the newest version (and, with 3 slots, the one before) stays intact
  cur_ = (cur_ + 1) % nslots_;
  Half &h = half_[cur_];
  // a mirror still reading this slot must finish before its buffers are reused
  WaitMirror(h);
  if (pinned_owner_ == &h) pinned_owner_ = nullptr;  // its bytes are about to change
  h.dev.resize(n, nullptr);
  h.cap.resize(n, 0);
  h.sizes.assign(nbytes, nbytes + n);
  h.meta = meta;
  for (int i = 0; i < n; ++i) {
    if (h.cap[i] < nbytes[i]) {
      if (h.dev[i] != nullptr) (void)hipFree(h.dev[i]);
      CheckHip(hipMalloc(&h.dev[i], std::max<size_t>(nbytes[i], 256)), "hipMalloc(snapshot)");
      h.cap[i] = std::max<size_t>(nbytes[i], 256);
    }
  }
  // 1. HBM snapshot on the plane stream, ordered after the caller's stream
  plane_->EnterFromUser();
  for (int i = 0; i < n; ++i) plane_->CopyDeviceAsync(h.dev[i], ptrs[i], nbytes[i]);
  CheckHip(hipEventRecord(h.snap_done, plane_->stream()), "hipEventRecord(snapshot)");
  // the caller may overwrite its tensors only after the snapshot read them
  plane_->Finish(FailureProbe(), false);
  // 2. pinned host mirror on the side stream: always, or when the previous one is done
  const bool idle = last_mirror_ == nullptr || MirrorDone(*last_mirror_);
  if (mirror_mode_ == kMirrorAlways || (mirror_mode_ == kMirrorIdle && idle)) {
    h.StartMirror();
    mirrors_ += 1;
  } else {
    mirrors_deferred_ += 1;  // copied on demand by Save if a peer asks for these bytes
  }
  return &h;
}

void DeviceCheckpoint::Half::StartMirror() const {
  DeviceCheckpoint *o = owner;
  size_t total = 0;
  for (size_t s : sizes) total += s;
  if (o->pinned_cap_ < total) {
    // the side stream (or the SDMA queue) holds the only readers and writers of the old buffer
    if (o->dma_) (void)o->dma_->WaitAll();  // the old buffer is dropped: failures do not matter
    CheckHip(hipStreamSynchronize(o->side_), "checkpoint mirror drain");
    if (o->pinned_ != nullptr) (void)hipHostFree(o->pinned_);
    o->pinned_ = nullptr;
    o->pinned_cap_ = 0;
    CheckHip(hipHostMalloc(reinterpret_cast<void **>(&o->pinned_), std::max<size_t>(total, 1)),
             "hipHostMalloc(mirror)");
    o->pinned_cap_ = std::max<size_t>(total, 1);
  }
  if (o->dma_) {
    // SDMA: jobs wait for the snapshot and run in order in the copier's thread
    size_t at = 0;
    ticket = 0;
    for (size_t i = 0; i < sizes.size(); ++i) {
      if (sizes[i] != 0) ticket = o->dma_->Submit(o->pinned_ + at, dev[i], sizes[i], snap_done);
      at += sizes[i];
    }
    o->pinned_owner_ = this;
    o->last_mirror_ = this;
    return;
  }
  // queued behind any earlier mirror on the same stream, so copies into the shared buffer
  // never overlap
  CheckHip(hipStreamWaitEvent(o->side_, snap_done, 0), "hipStreamWaitEvent(mirror)");
  size_t off = 0;
  for (size_t i = 0; i < sizes.size(); ++i) {
    if (sizes[i] != 0) {
      CheckHip(o->mirror_engine_ == kEngineKernel
                   ? LaunchCopyNarrow(o->pinned_ + off, dev[i], sizes[i], o->mirror_ctas_, o->side_)
                   : hipMemcpyAsync(o->pinned_ + off, dev[i], sizes[i], hipMemcpyDeviceToHost,
                                    o->side_),
               "D2H mirror");
    }
    off += sizes[i];
  }
  CheckHip(hipEventRecord(d2h_done, o->side_), "hipEventRecord(mirror)");
  o->pinned_owner_ = this;
  o->last_mirror_ = this;
}

void DeviceCheckpoint::Half::Save(Stream *fo) const {
  if (!mirrored()) StartMirror();  // deferred mirror: a peer needs the bytes now
  owner->WaitMirror(*this);
  uint64_t ml = meta.size();
  fo->Write(&ml, sizeof(ml));
  if (ml != 0) fo->Write(meta.data(), ml);
  uint64_t n = sizes.size();
  fo->Write(&n, sizeof(n));
  for (size_t s : sizes) {
    uint64_t v = s;
    fo->Write(&v, sizeof(v));
  }
  size_t total = 0;
  for (size_t s : sizes) total += s;
  if (total != 0) fo->Write(owner->pinned_, total);
}

void DeviceCheckpoint::Half::Load(Stream *) { utils::Error("snapshot halves are save-only"); }

Serializable *DeviceCheckpoint::Loader(int n, void *const *ptrs, const size_t *nbytes) {
  loader_.ptrs.assign(ptrs, ptrs + n);
  loader_.nbytes.assign(nbytes, nbytes + n);
  loaded_meta_.clear();
  loader_active_ = true;
  payload_delivered_ = false;
  return &loader_;
}

void DeviceCheckpoint::SaveHeader(const Serializable *snapshot, Stream *fo) const {
  const Half &h = *static_cast<const Half *>(snapshot);
  uint64_t ml = h.meta.size();
  fo->Write(&ml, sizeof(ml));
  if (ml != 0) fo->Write(h.meta.data(), ml);
  uint64_t n = h.sizes.size();
  fo->Write(&n, sizeof(n));
  for (size_t s : h.sizes) {
    uint64_t v = s;
    fo->Write(&v, sizeof(v));
  }
}

void *DeviceCheckpoint::SnapshotBuffer(const Serializable *snapshot, size_t i) const {
  const Half &h = *static_cast<const Half *>(snapshot);
  utils::Check(i < h.dev.size(), "snapshot buffer %zu out of range", i);
  return h.dev[i];
}

void DeviceCheckpoint::LoaderImpl::Load(Stream *fi) {
  uint64_t ml = 0;
  utils::Check(fi->Read(&ml, sizeof(ml)) == sizeof(ml), "device checkpoint: meta length");
  owner->loaded_meta_.resize(ml);
  if (ml != 0) {
    utils::Check(fi->Read(&owner->loaded_meta_[0], ml) == ml, "device checkpoint: meta");
  }
  uint64_t n = 0;
  utils::Check(fi->Read(&n, sizeof(n)) == sizeof(n), "device checkpoint: count");
  utils::Check(n == ptrs.size(), "device checkpoint holds %llu buffers, %zu given",
               static_cast<unsigned long long>(n), ptrs.size());
  std::vector<uint64_t> sizes(n);
  for (auto &s : sizes) {
    utils::Check(fi->Read(&s, sizeof(s)) == sizeof(s), "device checkpoint: size");
  }
  owner->loader_active_ = false;
  if (owner->payload_delivered_) {
    // the engine already broadcast the payloads into ptrs on the device
    owner->payload_delivered_ = false;
    for (size_t i = 0; i < n; ++i) {
      utils::Check(sizes[i] == nbytes[i], "device checkpoint buffer %zu: %llu bytes, %zu given", i,
                   static_cast<unsigned long long>(sizes[i]), nbytes[i]);
    }
    return;
  }
  std::vector<char> host;
  for (size_t i = 0; i < n; ++i) {
    utils::Check(sizes[i] == nbytes[i],
                 "device checkpoint buffer %zu: %llu bytes stored, %zu given",
                 i, static_cast<unsigned long long>(sizes[i]), nbytes[i]);
    host.resize(sizes[i]);
    if (sizes[i] == 0) continue;
    utils::Check(fi->Read(host.data(), sizes[i]) == sizes[i], "device checkpoint: payload");
    owner->plane_->StageToDevice(ptrs[i], host.data(), sizes[i]);
  }
}

void DeviceCheckpoint::LoaderImpl::Save(Stream *) const {
  utils::Error("the checkpoint loader is load-only");
}
}  // namespace device
}  // namespace rabit
