/*!
 * \file local_replicas.h
 * \brief Storage of the replicated per-rank ("local") checkpoint state.
 *
 * Semantics kept from the reference (`src/allreduce_robust.h:645-656`):
 * every rank keeps its own local state plus those of its K = num_local_replica ring
 * predecessors — slot k of rank r holds the state of rank (r - k) mod n — in two versions
 * (the one being written and the last acknowledged one; the engine flips after
 * kLocalCheckAck).
 *
 * Design (not the reference's CSR string + ring passes): a slot is an independent buffer with
 * an explicit size or "absent", so any subset of slots can be valid and recovery is a plan of
 * one-hop holder -> requester copies (engine/local_recovery.cc).  The store is either host
 * memory (Serializable local models, TCP plane) or HBM (local tensors, device plane: slots are
 * hipMalloc'd once and reused, replication moves over xGMI), chosen at the first checkpoint.
 * An HBM store also mirrors the own slot into pinned host memory on a side stream.
 */
#ifndef XRABIT_ENGINE_LOCAL_REPLICAS_H_
#define XRABIT_ENGINE_LOCAL_REPLICAS_H_

#include <hip/hip_runtime_api.h>

#include <cstdint>
#include <memory>
#include <string>
#include <vector>

namespace rabit {
namespace device {
class DmaCopier;
}
namespace engine {

class LocalReplicas {
 public:
  static constexpr int64_t kAbsent = -1;
  LocalReplicas() = default;
  ~LocalReplicas();
  LocalReplicas(const LocalReplicas &) = delete;
  LocalReplicas &operator=(const LocalReplicas &) = delete;

  /*! \brief nslot = K + 1 slots per version; device: slots live in HBM of `device` */
  void Configure(int nslot, bool on_device, int device);
  bool configured() const { return nslot_ > 0; }
  int nslot() const { return nslot_; }
  bool on_device() const { return on_device_; }

  int64_t size(int v, int k) const { return slots_[v][k].size; }
  bool valid(int v, int k) const { return slots_[v][k].size != kAbsent; }
  /*! \brief number of valid slots of version v */
  int Count(int v) const;
  /*! \brief sizes of all slots of version v (kAbsent where missing) */
  std::vector<int64_t> Sizes(int v) const;
  /*! \brief mark every slot of version v absent (storage is kept for reuse) */
  void Clear(int v);
  /*! \brief mark slot k of version v absent (device storage is kept for reuse) */
  void Drop(int v, int k) {
    slots_[v][k].size = kAbsent;
    if (!on_device_) slots_[v][k].host.clear();
  }
  /*! \brief make slot k of version v a valid slot of `bytes` bytes; returns its storage */
  void *Alloc(int v, int k, size_t bytes);
  void *Data(int v, int k) { return slot_ptr(slots_[v][k]); }
  const void *Data(int v, int k) const { return slot_ptr(slots_[v][k]); }
  /*! \brief bytes held by valid slots of version v */
  size_t Bytes(int v) const;
  /*! \brief host bytes of slot k (host store only; for Serializable loads) */
  std::string *HostSlot(int v, int k) { return &slots_[v][k].host; }

  /*!
   * \brief device store: start an asynchronous copy of slot 0 of version v into pinned host
   *        memory on the side stream, ordered after `stream` (skipped while the previous
   *        mirror is still running: the next checkpoint catches up)
   */
  void Mirror(int v, hipStream_t stream);
  /*! \brief order `stream` after a pending mirror that still reads version v (call before
   *         rewriting its slots) */
  void BeforeWrite(int v, hipStream_t stream);
  uint64_t mirrors() const { return mirrors_; }
  uint64_t mirrors_skipped() const { return mirrors_skipped_; }
  /*! \brief workgroups of the narrow D2H copy kernel of the mirror; 0: hipMemcpyAsync */
  void set_mirror_ctas(int c) { mirror_ctas_ = c; }
  /*! \brief the checkpoint mirror settings of the engine (rabit_device_ckpt_mirror,
   *  rabit_device_mirror_engine) apply to the local state too: off = no host mirror; sdma = the
   *  copy runs on an SDMA engine (device/dma_copier.h) instead of a blit kernel */
  void set_mirror_off(bool off) { mirror_off_ = off; }
  void set_mirror_sdma(bool sdma);

 private:
  struct Slot {
    int64_t size{kAbsent};
    std::string host;
    void *dev{nullptr};
    size_t cap{0};
  };
  static void *slot_ptr(const Slot &s) {
    return s.dev != nullptr ? s.dev : const_cast<char *>(s.host.data());
  }
  int nslot_{0};
  bool on_device_{false};
  int device_{-1};
  std::vector<Slot> slots_[2];
  // pinned mirror of the own slot
  hipStream_t side_{nullptr};
  hipEvent_t ready_{nullptr}, done_{nullptr};
  void *pinned_{nullptr};
  size_t pinned_cap_{0};
  bool mirror_pending_{false};
  int mirror_ctas_{0};
  bool mirror_off_{false};
  std::unique_ptr<device::DmaCopier> dma_;  // SDMA mirror engine (nullptr: HIP stream copy)
  uint64_t dma_ticket_{0};
  int mirror_version_{-1};
  uint64_t mirrors_{0}, mirrors_skipped_{0};
};
}  // namespace engine
}  // namespace rabit
#endif  // XRABIT_ENGINE_LOCAL_REPLICAS_H_
