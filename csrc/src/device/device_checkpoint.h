/*!
 * \file device_checkpoint.h
 * \brief Checkpoints of HBM-resident model state (SURVEY §5.4 MI355X plan).
 *
 * The reference serialises the global model into a host string at every CheckPoint.  For
 * device tensors that means a synchronous D2H of the whole model on the critical path.  Here
 * a checkpoint is:
 *   1. an HBM-to-HBM snapshot of the tensors (gfx950 copy kernel, ~6 TB/s) into the oldest of
 *      2 or 3 snapshot slots.  Two are required: the previous version must stay intact until
 *      the new checkpoint is acknowledged (peers may still be loading it) — the same 2x model
 *      size the reference holds while it serialises a new checkpoint next to the old one.  A
 *      third slot lets the host mirror of a slot still be in flight when that slot comes round
 *      again; it is used for models below rabit_device_ckpt_3slot_max (default 4 GiB), where a
 *      third copy is cheap and checkpoints may come faster than a PCIe copy of the model;
 *      rabit_device_ckpt_slots=2|3 forces either,
 *   2. an asynchronous D2H copy of the snapshot into ONE pinned host buffer on a side stream
 *      (overlaps the next iterations; host-DRAM durability).  In the default "idle" mode a
 *      mirror starts only when the previous one has finished, so iterations shorter than a
 *      PCIe copy of the model are never throttled by it; a snapshot that was not mirrored is
 *      copied on demand if a peer asks for its bytes.  "always" mirrors every checkpoint,
 *      "off" only on demand (rabit_device_ckpt_mirror=always|idle|off),
 *   3. registration with the robust engine as a *lazy* checkpoint: bytes are produced (from the
 *      pinned mirror, after its event) only if a recovering peer requests them.
 * Wire format of the global checkpoint: uint64 meta_len, meta, uint64 n, n x uint64 size,
 * then the n payloads.  A recovering worker that loads into HBM gets the header over TCP and
 * the payloads by device broadcasts from a survivor's snapshot (EngineRobust::TryLoadCheckPoint).
 */
#ifndef XRABIT_DEVICE_DEVICE_CHECKPOINT_H_
#define XRABIT_DEVICE_DEVICE_CHECKPOINT_H_

#include <hip/hip_runtime_api.h>

#include <memory>
#include <string>
#include <vector>

#include "device/device_plane.h"
#include "device/dma_copier.h"
#include "rabit/serializable.h"

namespace rabit {
namespace device {

class DeviceCheckpoint {
 public:
  explicit DeviceCheckpoint(DevicePlane *plane);
  ~DeviceCheckpoint();
  /*!
   * \brief snapshot n HBM buffers plus a host metadata blob into the next half and start its
   *        D2H mirror; returns the Serializable to register as the (lazy) global checkpoint
   */
  const Serializable *Snapshot(int n, void *const *ptrs, const size_t *nbytes,
                               const std::string &meta);
  /*! \brief Serializable that loads a checkpoint into the given HBM buffers */
  Serializable *Loader(int n, void *const *ptrs, const size_t *nbytes);
  /*! \brief metadata of the last Load */
  const std::string &loaded_meta() const { return loaded_meta_; }

  // ---- device-side recovery (the robust engine broadcasts snapshot buffers over xGMI)
  /*! \brief true if s is one of this checkpoint's snapshot slots */
  bool IsSnapshot(const Serializable *s) const {
    for (const auto &h : half_) {
      if (s == &h) return true;
    }
    return false;
  }
  /*! \brief mirror policy */
  enum MirrorMode { kMirrorIdle = 0, kMirrorAlways = 1, kMirrorOff = 2 };
  void set_mirror_mode(int m) { mirror_mode_ = m; }
  /*! \brief copy engine of the host mirror: hipMemcpyAsync, a narrow copy kernel, or an SDMA
   *         engine driven through ROCr (dma_copier.h) */
  enum MirrorEngine { kEngineHip = 0, kEngineKernel = 1, kEngineSdma = 2 };
  /*! \brief choose the engine (before the first snapshot); ctas: the kernel's workgroups.
   *         An SDMA copier that cannot start falls back to hipMemcpyAsync (logged). */
  void set_mirror_engine(int engine, int ctas);
  int mirror_engine() const { return dma_ ? kEngineSdma : mirror_engine_; }
  /*! \brief run the mirrors on a stream of the lowest priority (before the first snapshot) */
  void set_mirror_low_priority(bool low);
  /*! \brief snapshot slots: 2, 3, or 0 = by size (3 below three_slot_max bytes) */
  void set_slots(int n, size_t three_slot_max) {
    slots_req_ = n;
    three_slot_max_ = three_slot_max;
  }
  int slots() const { return nslots_; }
  /*! \brief bytes of pinned host memory held by the mirror */
  size_t pinned_bytes() const { return pinned_cap_; }
  /*! \brief checkpoints whose host mirror was started at snapshot time / deferred */
  uint64_t mirrors() const { return mirrors_; }
  uint64_t mirrors_deferred() const { return mirrors_deferred_; }
  /*! \brief the header of a snapshot: meta_len, meta, n, sizes (the payload format minus data) */
  void SaveHeader(const Serializable *snapshot, Stream *fo) const;
  /*! \brief HBM buffer i of a snapshot */
  void *SnapshotBuffer(const Serializable *snapshot, size_t i) const;
  /*! \brief a Loader is waiting for data (set by Loader(), cleared by its Load) */
  bool loader_active() const { return loader_active_; }
  const std::vector<void *> &loader_targets() const { return loader_.ptrs; }
  const std::vector<size_t> &loader_sizes() const { return loader_.nbytes; }
  /*! \brief the payload already reached the loader's buffers: its Load reads the header only */
  void MarkPayloadDelivered() { payload_delivered_ = true; }
  /*! \brief bytes of HBM reserved by the snapshot slots */
  size_t reserved_bytes() const;

 private:
  struct Half : public Serializable {
    DeviceCheckpoint *owner{nullptr};
    std::vector<void *> dev;      // HBM snapshot buffers
    std::vector<size_t> cap;      // their capacities
    std::vector<size_t> sizes;    // payload sizes of the current snapshot
    std::string meta;
    hipEvent_t d2h_done{nullptr};
    mutable uint64_t ticket{0};     // SDMA engine: the mirror's last copy job (0: none)
    hipEvent_t snap_done{nullptr};  // the HBM snapshot of this slot is complete
    /*! \brief queue the D2H mirror of this slot into the shared pinned buffer (side stream) */
    void StartMirror() const;
    /*! \brief the pinned buffer holds this slot's current snapshot (or its copy is queued) */
    bool mirrored() const { return owner->pinned_owner_ == this; }
    void Load(Stream *) override;
    void Save(Stream *fo) const override;
  };
  struct LoaderImpl : public Serializable {
    DeviceCheckpoint *owner{nullptr};
    std::vector<void *> ptrs;
    std::vector<size_t> nbytes;
    void Load(Stream *fi) override;
    void Save(Stream *) const override;
  };
  DevicePlane *plane_;
  hipStream_t side_{nullptr};
  static constexpr int kSlots = 3;
  Half half_[kSlots];
  int nslots_{0};  // fixed at the first snapshot
  int slots_req_{0};
  size_t three_slot_max_{size_t(4) << 30};
  int cur_{-1};
  int mirror_mode_{kMirrorIdle};
  int mirror_engine_{kEngineHip};
  int mirror_ctas_{16};
  std::unique_ptr<DmaCopier> dma_;
  /*! \brief the mirror of h has finished (non-blocking) / wait for it */
  bool MirrorDone(const Half &h) const;
  void WaitMirror(const Half &h) const;
  char *pinned_{nullptr};  // the host mirror, shared by the slots
  size_t pinned_cap_{0};
  const Half *pinned_owner_{nullptr};
  const Half *last_mirror_{nullptr};  // slot of the most recently started mirror
  uint64_t mirrors_{0}, mirrors_deferred_{0};
  LoaderImpl loader_;
  std::string loaded_meta_;
  bool loader_active_{false};
  bool payload_delivered_{false};
};
}  // namespace device
}  // namespace rabit
#endif  // XRABIT_DEVICE_DEVICE_CHECKPOINT_H_
