/*!
 * \file bcast_plan.h
 * \brief The direct transport's pipelined broadcast as a pure plan (no GPU): which copies each
 *        rank makes in each round between two barriers.  PeerGroup::Broadcast walks it and
 *        tests/cpp/unit_tests.cc checks it offline for n = 1..8, every root and odd sizes: every
 *        byte reaches every rank's user buffer and log slot exactly once, nothing reads a stage
 *        region before the barrier after its write, and no region is rewritten while a peer may
 *        still read it.
 *
 * Why pipelined.  A broadcast by scatter + allgather moves each chunk twice over xGMI: the root
 * hands segment j of the chunk to non-root j (the root's 7 outgoing links), then every non-root
 * pulls the other segments from the other non-roots (the links among non-roots).  The two phases
 * use DISJOINT link directions, so the allgather of chunk k can run in the same round as the
 * scatter of chunk k+1: a chunk then costs one round of S/(n-1) bytes per link instead of two.
 * The root keeps no segment of its own (segments go to the n-1 non-roots only), so the root's
 * stage buffer is only read in the round right after it was written.
 *
 * Rounds t = 0 .. nchunks+1, a barrier before every round t >= 1 (n = 2: not before the last
 * round, which is a local copy):
 *   root      : t < nchunks          stage chunk t (one read of the user buffer: stage + log)
 *   non-root j: 1 <= t <= nchunks    segment j of chunk t-1, root's stage -> own stage + user
 *               2 <= t               chunk t-2: every other non-root's segment from its stage
 *                                    -> user + log; the own segment own stage -> log
 * Chunk k lives in stage parity (base ^ k) & 1.  A region written in round t is read in round
 * t+1 at the latest and rewritten in round t+2 at the earliest, after the barrier that follows
 * every read of it.  The op's last remote reads (round nchunks+1) are of parity
 * base ^ ((nchunks-1) & 1), so the next op starts on the other parity, base ^ (nchunks & 1).
 *
 * Parity: the reference's tree broadcast (`src/allreduce_base.cc:641-720`) forwards the whole
 * buffer down a tree over TCP; on a fully connected xGMI mesh every byte crosses one link.
 */
#ifndef XRABIT_DEVICE_BCAST_PLAN_H_
#define XRABIT_DEVICE_BCAST_PLAN_H_

#include <algorithm>
#include <cmath>
#include <cstddef>
#include <vector>

namespace rabit {
namespace device {

/*! \brief one copy of a pipelined broadcast round, as seen by the rank making it */
struct BcastCopy {
  size_t chunk;   // chunk index k
  int from;       // rank whose stage (parity of chunk k) is read; -1: this rank's user buffer
  size_t off;     // byte offset within the chunk (same offset in stage, user and log)
  size_t bytes;
  bool to_stage;  // into this rank's own stage (parity of chunk k)
  bool to_user;   // into the user buffer
  bool to_log;    // into the result-log slot (when the op has one)
};

struct BcastPipeline {
  size_t bytes{0}, chunk{1};
  int n{1}, root{0};
  size_t nchunks{0};

  /*!
   * \brief chunk size of a broadcast of `bytes` on n ranks: sqrt(bytes * 4 MiB) rounded up to
   *        64 KiB, within [1 MiB, stage].  A round costs a barrier (~7-10 us) plus S/(n-1) bytes
   *        per link; the total (S/c + 1) (barrier + c / link rate of 7 links, ~0.5 TB/s) is least
   *        near c = sqrt(S x barrier x rate) = sqrt(S x ~5 MB): 64 MiB chunks for 1 GiB.
   */
  static size_t AutoChunk(size_t bytes, size_t stage) {
    const double c = std::sqrt(static_cast<double>(bytes) * (4.0 * (1 << 20)));
    size_t ch = (static_cast<size_t>(c) + (64u << 10) - 1) / (64u << 10) * (64u << 10);
    ch = std::max<size_t>(ch, 1u << 20);
    return std::max<size_t>(1, std::min(ch, stage));
  }
  BcastPipeline(size_t bytes_, size_t chunk_, int n_, int root_)
      : bytes(bytes_), chunk(std::max<size_t>(chunk_, 1)), n(n_), root(root_) {
    nchunks = (bytes + chunk - 1) / chunk;
  }
  size_t len(size_t k) const { return std::min(chunk, bytes - k * chunk); }
  /*! \brief segment of chunk k per non-root: whole 256-byte blocks */
  size_t seg(size_t k) const {
    const size_t parts = static_cast<size_t>(std::max(n - 1, 1));
    return ((len(k) + parts - 1) / parts + 255) / 256 * 256;
  }
  /*! \brief non-root slot of a rank: 0 .. n-2 (the root has none: -1) */
  int slot(int rank) const { return rank == root ? -1 : (rank - root - 1 + n) % n; }
  int rank_of_slot(int j) const { return (root + 1 + j) % n; }
  void seg_range(size_t k, int j, size_t *lo, size_t *hi) const {
    *lo = std::min(len(k), seg(k) * static_cast<size_t>(j));
    *hi = std::min(len(k), *lo + seg(k));
  }
  size_t rounds() const { return nchunks == 0 || n < 2 ? 0 : nchunks + 2; }
  /*! \brief a barrier precedes round t (the same answer on every rank) */
  bool barrier_before(size_t t) const {
    if (t == 0 || t >= rounds()) return false;
    return t <= nchunks || n > 2;
  }
  /*! \brief stage parity of chunk k when the op started on parity `base` */
  static int parity(int base, size_t k) { return base ^ static_cast<int>(k & 1); }
  /*! \brief parity the next op starts on */
  int next_parity(int base) const { return base ^ static_cast<int>(nchunks & 1); }

  /*! \brief the copies `rank` makes in round t */
  std::vector<BcastCopy> Round(int rank, size_t t) const {
    std::vector<BcastCopy> out;
    if (t >= rounds()) return out;
    if (rank == root) {
      if (t < nchunks) out.push_back({t, -1, 0, len(t), true, false, true});
      return out;
    }
    const int j = slot(rank);
    size_t lo, hi;
    if (t >= 2 && t - 2 < nchunks) {
      const size_t k = t - 2;
      for (int i = 0; i < n - 1; ++i) {
        seg_range(k, i, &lo, &hi);
        if (hi <= lo) continue;
        if (i == j) {
          out.push_back({k, rank, lo, hi - lo, false, false, true});
        } else {
          out.push_back({k, rank_of_slot(i), lo, hi - lo, false, true, true});
        }
      }
    }
    if (t >= 1 && t - 1 < nchunks) {
      const size_t k = t - 1;
      seg_range(k, j, &lo, &hi);
      if (hi > lo) out.push_back({k, root, lo, hi - lo, true, true, false});
    }
    return out;
  }
};

}  // namespace device
}  // namespace rabit
#endif  // XRABIT_DEVICE_BCAST_PLAN_H_
