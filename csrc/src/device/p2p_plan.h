/*!
 * \file p2p_plan.h
 * \brief Pure plans of the RCCL point-to-point paths of the device plane, and the
 *        classification of RCCL results.  Nothing here touches a GPU: device_plane.cc turns the
 *        plans into ncclSend / ncclRecv / ncclBroadcast calls, and tests/cpp/unit_tests.cc checks
 *        them offline for every rank of n = 2..8 (each send has a matching receive of equal bytes
 *        in the same per-peer order, every element is reduced exactly once, every byte lands at
 *        its offset).  These paths only run with two or more GPUs, which the test machine does
 *        not have, so the plans are what can be verified before the first multi-GPU run.
 *
 * Parity: the reference's ring reduce-scatter / allgather segment arithmetic
 * (`src/allreduce_base.cc:779-843,857-946`) is replaced by these all-to-all plans: on a fully
 * connected xGMI mesh every segment moves in one hop instead of n-1.
 */
#ifndef XRABIT_DEVICE_P2P_PLAN_H_
#define XRABIT_DEVICE_P2P_PLAN_H_

#include <algorithm>
#include <cstddef>
#include <vector>

namespace rabit {
namespace device {

// ---------------------------------------------------------------- RCCL results
/*! \brief what an RCCL return code means for the engine */
enum class RcclOutcome {
  kOk,           // done (enqueued)
  kPending,      // non-blocking communicator: poll ncclCommGetAsyncError until it settles
  kPeerFailure,  // a dead or aborted peer can cause it: abort the communicator, recover, retry
  kFatal         // a usage error of this library: retrying cannot help
};
/*!
 * \brief classify an ncclResult_t (values of rccl.h: 0 success, 1 unhandled device error,
 *        2 system error, 3 internal error, 4 invalid argument, 5 invalid usage, 6 remote error,
 *        7 in progress).  System, internal, remote and device errors are what a peer that died
 *        mid-operation (or a communicator aborted under it) produces, so they are recoverable.
 */
inline RcclOutcome ClassifyRccl(int r) {
  switch (r) {
    case 0: return RcclOutcome::kOk;
    case 7: return RcclOutcome::kPending;
    case 1:
    case 2:
    case 3:
    case 6: return RcclOutcome::kPeerFailure;
    default: return RcclOutcome::kFatal;
  }
}

// ---------------------------------------------------------------- point-to-point ops
/*! \brief which buffer an op's offset refers to */
enum P2PBuf { kBufIn = 0, kBufOut = 1, kBufInbox = 2 };
/*! \brief one ncclSend (send = true) or ncclRecv of a grouped call, as seen by one rank */
struct P2POp {
  bool send;
  int peer;
  int buf;        // P2PBuf
  size_t offset;  // bytes into buf
  size_t bytes;
};

/*!
 * \brief segments of the kernel-reduced allreduce (custom reductions, BitOR, fused prepare):
 *        rank k owns elements [lo(k), hi(k)).  Segments are whole 256-element blocks so every
 *        segment start is as aligned as the buffer; trailing ranks may own nothing.
 */
struct SegmentPlan {
  size_t count{0}, seg{0}, tn{1};
  int n{1};
  SegmentPlan(size_t count_, size_t tn_, int n_) : count(count_), tn(tn_), n(n_) {
    seg = ((count + n - 1) / n + 255) / 256 * 256;
  }
  size_t lo(int k) const { return std::min(count, seg * static_cast<size_t>(k)); }
  size_t hi(int k) const { return std::min(count, seg * static_cast<size_t>(k + 1)); }
  size_t elems(int k) const { return hi(k) - lo(k); }
  /*! \brief bytes between inbox slots (one slot per sender, 256-byte aligned) */
  size_t slot_bytes(int rank) const { return (elems(rank) * tn + 255) / 256 * 256; }
  size_t inbox_bytes(int rank) const { return std::max<size_t>(slot_bytes(rank) * n, 256); }

  /*!
   * \brief step 1 (reduce-scatter's exchange): segment k of every rank's input goes to rank k,
   *        which receives the copy of sender s into inbox slot s.  Per peer: the send first, then
   *        the receive (RCCL matches sends and receives per peer pair in issue order; within a
   *        group the two directions do not block each other).
   */
  std::vector<P2POp> ScatterOps(int rank) const {
    std::vector<P2POp> ops;
    const size_t mine = elems(rank);
    for (int k = 0; k < n; ++k) {
      if (k == rank) continue;
      if (elems(k) != 0) ops.push_back({true, k, kBufIn, lo(k) * tn, elems(k) * tn});
      if (mine != 0) {
        ops.push_back({false, k, kBufInbox, static_cast<size_t>(k) * slot_bytes(rank), mine * tn});
      }
    }
    return ops;
  }
  /*!
   * \brief step 3 (allgather): every rank's reduced segment to every other rank, straight into
   *        its place in the output buffer
   */
  std::vector<P2POp> GatherOps(int rank) const {
    std::vector<P2POp> ops;
    const size_t mine = elems(rank);
    for (int k = 0; k < n; ++k) {
      if (k == rank) continue;
      if (mine != 0) ops.push_back({true, k, kBufOut, lo(rank) * tn, mine * tn});
      if (elems(k) != 0) ops.push_back({false, k, kBufOut, lo(k) * tn, elems(k) * tn});
    }
    return ops;
  }
  /*!
   * \brief step 2: the reduce passes of this rank's segment, in rank order, at most `max_src`
   *        sources per pass.  Source -1 is the running result (the output segment itself),
   *        source == rank is this rank's own input, any other s is inbox slot s.
   */
  std::vector<std::vector<int>> ReducePasses(int rank, int max_src) const {
    std::vector<std::vector<int>> passes;
    if (elems(rank) == 0) return passes;
    int done = 0;
    while (done < n) {
      std::vector<int> p;
      if (done > 0) p.push_back(-1);
      while (done < n && static_cast<int>(p.size()) < max_src) p.push_back(done++);
      passes.push_back(p);
    }
    return passes;
  }
};

/*! \brief one ncclBroadcast of a variable allgather: `bytes` at `offset`, from `root` */
struct BcastPiece {
  int root;
  size_t offset, bytes;
};
/*!
 * \brief rabit's variable, wrapping allgather slices (slice r = [begin[r], begin[r] + size[r])
 *        mod total) as broadcasts in place: a slice that wraps past the end becomes two pieces.
 *        Every rank computes the same list from the same (begin, size) vectors.
 */
inline std::vector<BcastPiece> AllgatherPieces(size_t total, const std::vector<size_t> &begin,
                                               const std::vector<size_t> &size) {
  std::vector<BcastPiece> out;
  if (total == 0) return out;
  for (size_t r = 0; r < begin.size(); ++r) {
    const size_t b = begin[r] % total, s = std::min(size[r], total);
    const size_t first = std::min(s, total - b);
    if (first != 0) out.push_back({static_cast<int>(r), b, first});
    if (s > first) out.push_back({static_cast<int>(r), 0, s - first});
  }
  return out;
}
/*! \brief true if the slices are the uniform, rank-ordered layout ncclAllGather expects */
inline bool AllgatherUniform(size_t total, const std::vector<size_t> &begin,
                             const std::vector<size_t> &size) {
  const size_t n = begin.size();
  if (n == 0 || total != size[0] * n) return false;
  for (size_t r = 0; r < n; ++r) {
    if (begin[r] != r * size[0] || size[r] != size[0]) return false;
  }
  return true;
}

/*!
 * \brief this rank's share of a device exchange plan (ExchangeItem list in global order):
 *        index i of the result is the plan item each op serves.  Items with src == dst are
 *        local copies (returned in *local), zero-byte items move nothing.  Because every rank
 *        walks the same list in the same order, the k-th send from s to d and the k-th receive
 *        at d from s are the same item.
 */
template <typename Item>
inline std::vector<P2POp> ExchangeOps(const std::vector<Item> &plan, int rank,
                                      std::vector<size_t> *item_of,
                                      std::vector<size_t> *local = nullptr) {
  std::vector<P2POp> ops;
  item_of->clear();
  for (size_t i = 0; i < plan.size(); ++i) {
    const Item &x = plan[i];
    if (x.bytes == 0) continue;
    if (x.src == x.dst) {
      if (x.src == rank && local != nullptr) local->push_back(i);
      continue;
    }
    if (x.src == rank) {
      ops.push_back({true, x.dst, kBufIn, 0, x.bytes});
      item_of->push_back(i);
    } else if (x.dst == rank) {
      ops.push_back({false, x.src, kBufOut, 0, x.bytes});
      item_of->push_back(i);
    }
  }
  return ops;
}
}  // namespace device
}  // namespace rabit
#endif  // XRABIT_DEVICE_P2P_PLAN_H_
