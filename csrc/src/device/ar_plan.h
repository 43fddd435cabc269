/*!
 * \file ar_plan.h
 * \brief The direct transport's pipelined two-shot allreduce as a pure plan (no GPU): which
 *        copies and which reduce each rank makes in each round between two barriers.
 *        PeerGroup::AllreduceImpl walks it and tests/cpp/unit_tests.cc checks it offline for
 *        n = 2..8 and odd sizes: every element is reduced once from every rank's input, every
 *        result byte reaches the output (and the second destination) exactly once, nothing reads
 *        a stage region before the barrier after its write, and no region is rewritten in the
 *        barrier interval of a read or write of it by another rank (also across two ops).
 *
 * Why pipelined.  The two-shot allreduce moves each chunk over xGMI twice: a reduce-scatter (here
 * by PUSH: rank r writes segment q of its input into an inbox slot of rank q, outgoing links) and
 * an allgather (PULL: rank r reads every owner's reduced segment, incoming links).  The two use
 * opposite link directions, so the allgather of chunk k-2 runs in the same round as the push of
 * chunk k, and the local reduce of chunk k-1 between them: one barrier per round, a round costs
 * max(push, gather) instead of their sum.  The classic push form takes two barriers per chunk
 * and runs the phases one after the other.
 *
 * Stage layout per parity (elements of the op's type): n inbox slots of `segmax` elements
 * (slot s: written by rank s), then one result slot of `segmax` (the owner's reduced segment,
 * read by the gathers).  Chunk k lives in parity (base ^ k) & 1.
 *
 * Rounds t = 0 .. nchunks+1, a barrier after every round but the last:
 *   push   (t < nchunks)        segment q of chunk t: own input -> inbox slot `rank` of rank q
 *   reduce (1 <= t <= nchunks)  chunk t-1: own n inbox slots -> own result slot
 *   gather (2 <= t)             chunk t-2: result slot of every owner q -> output (+ second)
 * Within a round the copy batch (pushes and gathers together: opposite link directions) is
 * launched before the reduce; they touch disjoint regions.
 *
 * The robust engine passes a second destination (the user buffer) that may only change once
 * the op succeeded on this rank: gathers before the last barrier store the output alone, and a
 * copy guarded by the group's failure word moves those chunks to the second destination in the
 * last round (second_tail), in the same launch as the last chunk's gather, which follows the
 * last barrier and stores both.
 *
 * The op's last reads (the final gather, no barrier after it) are of parity
 * base ^ ((nchunks-1) & 1), so the next op starts on the other one, base ^ (nchunks & 1).
 *
 * Parity: the reference's ring allreduce (`src/allreduce_base.cc:857-977`, reduce-scatter then
 * allgather over one ring link per direction) is the algorithm being replaced; on a fully
 * connected xGMI mesh every byte crosses one link per phase, on all 7 links at once.
 */
#ifndef XRABIT_DEVICE_AR_PLAN_H_
#define XRABIT_DEVICE_AR_PLAN_H_

#include <algorithm>
#include <cmath>
#include <cstddef>
#include <vector>

namespace rabit {
namespace device {

/*! \brief one copy of a pipelined allreduce round, as seen by the rank making it (elements) */
struct ArCopy {
  bool push;      // true: own input -> a peer's inbox (remote write); false: a gather
  size_t chunk;   // chunk index k
  int peer;       // push: the owner q written to; gather: the owner q read from
  size_t lo, hi;  // element range within the chunk
};

/*! \brief the reduce of one round: chunk k, this rank's segment [lo, hi) of it */
struct ArReduce {
  bool any{false};
  size_t chunk{0}, lo{0}, hi{0};
};

struct ArPipeline {
  size_t count{0}, chunk{1};  // elements of the op, elements per chunk (a multiple of 256 n)
  int n{1};
  size_t nchunks{0};
  size_t segmax{0};           // elements per inbox / result slot

  /*!
   * \brief elements per chunk for an op of `count` elements of `tn` bytes on n ranks with stage
   *        buffers of `stage` bytes: sqrt(bytes x 4 MiB) (as the pipelined broadcast: a round
   *        costs a barrier plus the chunk's bytes over 7 links), at least 1 MiB, and at most
   *        what (n + 1) slots of a stage hold; a multiple of 256 n elements
   */
  static size_t AutoChunk(size_t count, size_t tn, int n, size_t stage) {
    const size_t q = 256 * static_cast<size_t>(n);
    const size_t cap = stage / tn / static_cast<size_t>(n + 1) / 256 * 256 * static_cast<size_t>(n);
    const double want_b = std::sqrt(static_cast<double>(count * tn) * (4.0 * (1 << 20)));
    size_t c = static_cast<size_t>(std::max(want_b, static_cast<double>(1 << 20)) /
                                   static_cast<double>(tn));
    c = (c + q - 1) / q * q;
    return std::max(q, std::min(c, cap));
  }
  ArPipeline(size_t count_, size_t chunk_, int n_)
      : count(count_), chunk(std::max<size_t>(chunk_, 1)), n(n_) {
    nchunks = (count + chunk - 1) / chunk;
    segmax = ((chunk + static_cast<size_t>(n) - 1) / static_cast<size_t>(n) + 255) / 256 * 256;
  }
  /*! \brief stage bytes one parity needs */
  size_t stage_bytes(size_t tn) const { return static_cast<size_t>(n + 1) * segmax * tn; }
  size_t len(size_t k) const { return std::min(chunk, count - k * chunk); }
  /*! \brief segment q of chunk k: [lo, hi) within the chunk (whole 256-element blocks) */
  void seg_range(size_t k, int q, size_t *lo, size_t *hi) const {
    const size_t nn = static_cast<size_t>(n);
    const size_t s = ((len(k) + nn - 1) / nn + 255) / 256 * 256;
    *lo = std::min(len(k), s * static_cast<size_t>(q));
    *hi = std::min(len(k), *lo + s);
  }
  size_t rounds() const { return nchunks == 0 ? 0 : nchunks + 2; }
  /*! \brief a barrier follows round t */
  bool barrier_after(size_t t) const { return t + 1 < rounds(); }
  static int parity(int base, size_t k) { return base ^ static_cast<int>(k & 1); }
  int next_parity(int base) const { return base ^ static_cast<int>(nchunks & 1); }
  /*! \brief element offset of inbox slot s / of the result slot in a parity's stage */
  size_t inbox(int s) const { return static_cast<size_t>(s) * segmax; }
  size_t result() const { return static_cast<size_t>(n) * segmax; }
  /*! \brief the gather of chunk k may store the second destination (it follows the last
   *  barrier); earlier chunks reach it through the guarded tail copy */
  bool second_in_gather(size_t k) const { return k + 1 == nchunks; }
  /*! \brief elements [0, second_tail()) are copied output -> second destination in the last
   *  round, after the last barrier (guarded: only when every barrier held) */
  size_t second_tail() const { return nchunks == 0 ? 0 : (nchunks - 1) * chunk; }

  /*! \brief the copies `rank` makes in round t (pushes first, then gathers) */
  std::vector<ArCopy> Copies(int rank, size_t t) const {
    std::vector<ArCopy> out;
    if (t >= rounds()) return out;
    size_t lo, hi;
    if (t < nchunks) {
      for (int q = 0; q < n; ++q) {
        seg_range(t, q, &lo, &hi);
        if (hi > lo) out.push_back({true, t, q, lo, hi});
      }
    }
    if (t >= 2) {
      const size_t k = t - 2;
      for (int q = 0; q < n; ++q) {
        seg_range(k, q, &lo, &hi);
        if (hi > lo) out.push_back({false, k, q, lo, hi});
      }
    }
    (void)rank;
    return out;
  }
  /*! \brief the reduce `rank` runs in round t */
  ArReduce Reduce(int rank, size_t t) const {
    ArReduce r;
    if (t == 0 || t > nchunks) return r;
    r.chunk = t - 1;
    seg_range(r.chunk, rank, &r.lo, &r.hi);
    r.any = r.hi > r.lo;
    return r;
  }
};

}  // namespace device
}  // namespace rabit
#endif  // XRABIT_DEVICE_AR_PLAN_H_
