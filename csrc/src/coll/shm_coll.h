/*!
 * \file shm_coll.h
 * \brief Shared-memory transport for host buffers of ranks that share a host (the 8 ranks of
 *        an MI355X node): the CPU counterpart of the device direct transport (peer_coll.h).
 *
 * Every rank creates one POSIX shared-memory segment [flag header | stage 0 | stage 1] and
 * maps its peers' segments.  Collectives stage their input in the local stage buffer, meet at a
 * flag barrier, and then read the peers' stage buffers directly:
 *
 *  - Allreduce (two-shot): stage; barrier; rank r reduces segment r of all n stages into its
 *    own stage (and its output); barrier; everyone copies the other n-1 reduced segments.
 *    Each byte is copied once into shared memory and read where it is needed — over loopback
 *    TCP the reference moves every byte through two kernel copies per hop.
 *  - Broadcast: the root stages; barrier; everyone copies.
 *  - AllgatherV (rabit's variable, wrapping slices): stage own slice; barrier; copy the rest.
 *
 * Stage buffers alternate between ops (parity), which lets two barriers per allreduce chunk
 * and one per broadcast chunk suffice.  The TCP links stay the control plane: a barrier gives
 * up when the failure probe sees a peer link hang up or the deadline passes, and the owner
 * drops the group (a new one is built after recovery, like a device-transport epoch).
 * Segments are unlinked as soon as every peer has mapped them, so a crash leaks nothing.
 */
#ifndef XRABIT_COLL_SHM_COLL_H_
#define XRABIT_COLL_SHM_COLL_H_

#include <cstddef>
#include <cstdint>
#include <functional>
#include <string>
#include <vector>

#include "coll/host_coll.h"

namespace rabit {
namespace coll {

constexpr int kMaxShmRanks = 64;

/*! \brief fixed-size record every rank contributes when a group is built */
struct ShmRecord {
  char host[64];
  char name[64];  // shm_open name of the rank's segment ("" if it has none)
  uint64_t stage_bytes;
  int32_t pid;
  int32_t ok;
};

class ShmGroup {
 public:
  typedef std::function<bool()> Probe;
  /*! \brief create and map this rank's segment (ok() false when shared memory is unusable) */
  ShmGroup(size_t stage_bytes, double deadline_sec);
  ~ShmGroup();
  ShmGroup(const ShmGroup &) = delete;
  ShmGroup &operator=(const ShmGroup &) = delete;

  bool ok() const { return own_ != nullptr; }
  const ShmRecord &local() const { return local_; }
  /*! \brief map every peer's segment (all on this host, equal stage sizes) */
  bool Open(const std::vector<ShmRecord> &all, int rank, std::string *why);
  /*! \brief first barrier of a new group: after it every peer has mapped every segment, and
   *  the names are unlinked (collective) */
  Status Seal(const Probe &probe);

  /*! \brief dst = reduce over ranks of src (count items of tn bytes); src may equal dst */
  Status Allreduce(const void *src, void *dst, size_t tn, size_t count, ReduceFn red,
                   const Probe &probe);
  Status Broadcast(void *buf, size_t bytes, int root, const Probe &probe);
  /*!
   * \brief rabit's allgather with variable, wrapping slices: rank r owns bytes
   *        [begin[r], begin[r] + size[r]) mod total of buf (every rank passes all slices)
   */
  Status AllgatherV(void *buf, size_t total, const std::vector<size_t> &begin,
                    const std::vector<size_t> &size, const Probe &probe);
  uint64_t ops() const { return ops_; }

 private:
  Status Barrier(const Probe &probe);
  char *stage(int r, int which) const;

  size_t stage_bytes_;
  size_t seg_bytes_;
  double deadline_sec_;
  int fd_{-1};
  char *own_{nullptr};
  std::vector<char *> peer_;  // mapped segments (own = own_)
  ShmRecord local_{};
  int n_{0}, rank_{0};
  uint64_t epoch_{0};
  int parity_{0};
  bool sealed_{false};
  uint64_t ops_{0};
};

}  // namespace coll
}  // namespace rabit
#endif  // XRABIT_COLL_SHM_COLL_H_
