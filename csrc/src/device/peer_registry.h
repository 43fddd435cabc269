/*!
 * \file peer_registry.h
 * \brief Zero-copy inputs for the direct transport: ordinary HBM allocations (a torch tensor, a
 *        hipMalloc buffer) that peers read in place over xGMI instead of this rank staging them.
 *
 * The symmetric heap (SymAlloc) only covers buffers the caller allocates from it.  Everything
 * else used to pay a full stage copy before the first barrier of the pull two-shot (28-32 % of
 * the op at N = 2..8 in the round-3 rehearsals).  The registry exports the allocation behind an
 * input once and lets every peer map it, so later ops on the same allocation go zero copy:
 *
 *  - exporter (the rank whose input it is): the allocation behind the pointer is found with
 *    hipDrvPointerGetAttributes (base, size, buffer id), exported with hipIpcGetMemHandle and
 *    written into one of kMaxRegs slots of this rank's registry page, a small POSIX shared-memory
 *    segment (the direct transport only runs between ranks of one host).  A slot carries a
 *    generation (seqlock: odd while it is rewritten); the buffer id tells a freed and re-made
 *    allocation at the same address from the old one, which then gets a new generation.
 *  - importer (every other rank), at the start of each allreduce: a changed registry version of
 *    a peer makes it open the new handles (hipIpcOpenMemHandle), put the mapped bases into a
 *    device table the barrier kernel resolves mailboxes with (an async copy on the group's
 *    stream), and acknowledge (generation, first op it is valid for) in ITS OWN page.  A mapping
 *    that is replaced is closed only after the stream drained, so no enqueued op still uses it.
 *  - handles are compared byte for byte before a mapping is opened: an allocation freed by its
 *    exporter releases its export, so a later allocation can come back with identical handle
 *    bytes (the same descriptor number of the same process), and the runtime would hand out the
 *    old mapping again -- stale memory.  The importer closes such a mapping first.  An exporter
 *    whose allocation was re-made at the same address rewrites that allocation's slot.
 *  - an op is zero copy on the exporter when every peer acknowledged the slot's current
 *    generation for an op index at or below this one: every rank numbers its allreduces alike
 *    (collectives in one order), and the importer enqueued the table update before the kernels
 *    of that op.  Otherwise the op stages as before; the first op on a new allocation always does.
 *
 * Everything a rank writes lives in its own page; it only reads its peers'.  Ranks decide zero
 * copy for their own input independently (the mailbox tells the readers where it is), exactly as
 * for the symmetric heap.
 */
#ifndef XRABIT_DEVICE_PEER_REGISTRY_H_
#define XRABIT_DEVICE_PEER_REGISTRY_H_

#include <hip/hip_runtime_api.h>

#include <atomic>
#include <cstddef>
#include <cstdint>
#include <string>
#include <vector>

namespace rabit {
namespace device {

constexpr int kMaxRegPeers = 8;   // = kMaxPeers (peer_coll.h)
constexpr int kMaxRegs = 32;      // exported allocations per rank
/*! \brief mailbox flag: the input lives in registered allocation (bits 56..61) at an offset */
constexpr unsigned long long kMailboxReg = 1ull << 62;
constexpr int kMailboxRegShift = 56;
constexpr unsigned long long kMailboxOffsetMask = (1ull << kMailboxRegShift) - 1;

/*! \brief one rank's page in shared memory (written by that rank only) */
struct RegistryPage {
  uint64_t magic;
  std::atomic<uint64_t> version;  // bumped after every slot change
  struct Slot {
    std::atomic<uint64_t> gen;  // 0: empty; odd: being written; even: valid
    uint64_t bytes;
    char ipc[64];
  } slot[kMaxRegs];
  // what this rank has mapped of peer p's slot k: generation, and the first op index of this
  // rank's group for which its device table holds the mapping
  struct Ack {
    std::atomic<uint64_t> from_op;
    std::atomic<uint64_t> gen;
  } ack[kMaxRegPeers][kMaxRegs];
};

class PeerRegistry {
 public:
  PeerRegistry() = default;
  ~PeerRegistry();
  PeerRegistry(const PeerRegistry &) = delete;
  PeerRegistry &operator=(const PeerRegistry &) = delete;

  /*! \brief create this rank's page; false (why) if shared memory is unavailable */
  bool Create(std::string *why);
  /*! \brief shm name of this rank's page (travels in the PeerRecord) */
  const char *name() const { return name_; }
  /*! \brief map the pages of every rank (names in rank order) and the device table */
  bool Open(const std::vector<std::string> &names, int rank, std::string *why);
  /*! \brief every peer has mapped this rank's page: its name may go */
  void Seal();
  bool opened() const { return opened_; }

  /*!
   * \brief importer side, once per allreduce before its kernels are enqueued (op = this op's
   *        index): map peers' new registrations, update the device table on `stream`, acknowledge.
   *        A replaced mapping is closed once `stream` drained, waiting at most `drain_sec`
   *        (hipErrorLaunchTimeOut after that: the stream is wedged).  hipSuccess or the first
   *        error.
   */
  hipError_t Refresh(uint64_t op, hipStream_t stream, double drain_sec);
  /*!
   * \brief exporter side: true when [p, p + bytes) may be read in place by every peer in op
   *        `op`; *mailbox then holds the mailbox word of its start.  Registers an allocation
   *        seen for the first time (false for this op).
   */
  bool Resolve(const void *p, size_t bytes, uint64_t op, unsigned long long *mailbox);
  /*! \brief device table: kMaxRegPeers x kMaxRegs mapped bases (nullptr before Open) */
  const char *const *device_table() const { return dev_table_; }

  uint64_t exports() const { return exports_; }
  uint64_t imports() const { return imports_; }
  uint64_t unexportable() const { return unexportable_; }
  uint64_t pending() const { return pending_; }

 private:
  struct Local {
    uintptr_t base{0};
    size_t bytes{0};
    uint64_t buffer_id{0};
    uint64_t gen{0};
    uint64_t last_use{0};
  };
  int FindOrExport(uintptr_t p, size_t bytes, uint64_t op);

  char name_[48]{};
  int fd_{-1};
  RegistryPage *mine_{nullptr};
  std::vector<RegistryPage *> pages_;  // by rank (own = mine_)
  int n_{0}, rank_{0};
  bool opened_{false}, sealed_{false};
  Local local_[kMaxRegs];
  std::vector<uint64_t> bad_ids_;  // buffer ids hipIpcGetMemHandle refused
  // importer state
  std::vector<uint64_t> seen_version_;
  char *mapped_[kMaxRegPeers][kMaxRegs]{};
  char handle_[kMaxRegPeers][kMaxRegs][64]{};  // the IPC handle behind each mapping
  uint64_t mapped_gen_[kMaxRegPeers][kMaxRegs]{};
  const char **host_table_{nullptr};  // pinned mirror of the device table
  const char **dev_table_raw_{nullptr};
  const char *const *dev_table_{nullptr};
  uint64_t exports_{0}, imports_{0}, unexportable_{0}, pending_{0};
};

}  // namespace device
}  // namespace rabit
#endif  // XRABIT_DEVICE_PEER_REGISTRY_H_
