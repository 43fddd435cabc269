/*!
 * \file host_coll.h
 * \brief Collective algorithms over host TCP links (the CPU data plane and the control plane).
 *
 * Algorithm inventory: A1 pipelined tree allreduce, A2 ring reduce-scatter,
 * A3 ring allreduce, A4 ring allgather with variable wrapping slices, A5 tree broadcast,
 * A8 ring passing.  Parity with reference `src/allreduce_base.cc:454-977` and
 * `src/allreduce_robust.cc:1529-1587`.  Every primitive is a non-blocking poll() loop that
 * returns a Status instead of throwing, so the robust engine can repair links and retry.
 * Loops wake up at least every `poll_interval_ms` to honour an abort flag (set by the
 * watchdog when a peer dies or a deadline passes).
 */
#ifndef XRABIT_COLL_HOST_COLL_H_
#define XRABIT_COLL_HOST_COLL_H_

#include <atomic>
#include <cstddef>

#include "net/links.h"
#include "rabit/internal/engine.h"

namespace rabit {
namespace coll {

using net::PeerLink;
using net::Status;
using net::Topology;
typedef engine::IEngine::ReduceFunction *ReduceFn;

/*! \brief tunables of the host algorithms (reference allreduce_base.cc:18-46) */
struct HostCollConfig {
  size_t reduce_ring_mincount{32 << 10};  // > this many elements => ring, else tree
  size_t tree_reduce_minsize{1 << 20};    // tree pipelining chunk in bytes
  size_t reduce_buffer_bytes{256u << 20}; // per-link staging ring cap
  int poll_interval_ms{100};
};

class HostCollectives {
 public:
  HostCollectives(Topology *topo, const HostCollConfig *cfg, const int *rank,
                  const int *world_size)
      : topo_(topo), cfg_(cfg), rank_(rank), world_(world_size) {}

  /*! \brief abort flag polled by every loop (owned by the engine) */
  void SetAbortFlag(const std::atomic<bool> *flag) { abort_ = flag; }
  /*! \brief link that caused the last error (reference err_link) */
  PeerLink *err_link() const { return err_link_; }

  /*!
   * \brief tree for small counts, ring (RS+AG) for large ones.  src != nullptr: out of place,
   *        the inputs are read from src and buf only receives results (src is never written,
   *        so a failed attempt can be retried from it)
   */
  Status Allreduce(void *buf, size_t type_nbytes, size_t count, ReduceFn red,
                   const void *src = nullptr);
  Status TreeAllreduce(void *buf, size_t type_nbytes, size_t count, ReduceFn red);
  /*! \brief after it, this rank's segment of buf is reduced (src: see Allreduce) */
  Status RingReduceScatter(void *buf, size_t type_nbytes, size_t count, ReduceFn red,
                           const void *src = nullptr);
  Status RingAllreduce(void *buf, size_t type_nbytes, size_t count, ReduceFn red,
                       const void *src = nullptr);
  Status RingAllgather(void *buf, size_t total, size_t slice_begin, size_t slice_end,
                       size_t size_prev_slice);
  Status TreeBroadcast(void *buf, size_t size, int root);
  /*!
   * \brief stream along the ring: buf[0, read_ptr) is local, receive [read_ptr, read_end)
   *        from read_link, forward [write_ptr, write_end) to write_link once available
   */
  Status RingPass(void *buf, size_t read_ptr, size_t read_end, size_t write_ptr,
                  size_t write_end, PeerLink *read_link, PeerLink *write_link);
  /*! \brief record an error against a link and return it */
  Status Fail(PeerLink *link, Status s) {
    err_link_ = link;
    return s;
  }
  bool Aborted() const { return abort_ != nullptr && abort_->load(std::memory_order_relaxed); }
  int poll_ms() const { return cfg_->poll_interval_ms; }

 private:
  Topology *topo_;
  const HostCollConfig *cfg_;
  const int *rank_;
  const int *world_;
  const std::atomic<bool> *abort_{nullptr};
  PeerLink *err_link_{nullptr};
};

/*! \brief host reduce function for a built-in (dtype, op); nullptr if unsupported */
ReduceFn HostReducer(engine::mpi::DataType dtype, engine::mpi::OpType op);
/*! \brief element size of a dtype */
size_t DTypeSize(engine::mpi::DataType dtype);
}  // namespace coll
}  // namespace rabit
#endif  // XRABIT_COLL_HOST_COLL_H_
