/*!
 * \file host_stager.h
 * \brief Pipelined staging of a HOST-buffer collective through HBM (rabit_host_via_device: the
 *        reference's own benchmark shape, test/speed_test.cc, on a GPU node).
 *
 * The unpipelined form is three serial steps: hipMemcpy of the whole pageable host buffer into
 * HBM, the device collective, and hipMemcpy back.  A pageable copy runs through the HIP
 * runtime's own pinned bounce buffer, filled by one CPU thread, so each direction moves at the
 * speed of one memcpy thread (~16 GB/s measured with 2 ranks on one box), and nothing overlaps.
 *
 * Here the buffer moves in chunks through two pinned slots per direction:
 *
 *     CPU (T threads)   copy-in k+1 ........ copy-out k-1 ........
 *     h2d stream          H2D k+1 ................................
 *     plane stream             collective k .....................
 *     d2h stream                    D2H k-1 ......................
 *
 * - a pool of T threads splits every memcpy between pageable memory and a pinned slot, so the
 *   host side is not held to one memcpy thread;
 * - the H2D of one chunk, the collective of the chunk before, and the D2H of the chunk before
 *   that run together on separate streams, ordered by events;
 * - every wait on the collective goes through the caller's `wait` (the device plane's waits
 *   watch the failure probe and the op deadline), so a dead peer still ends in a recoverable
 *   status, not a hang.
 *
 * Reference: src/allreduce_base.cc:476-668 (the host allreduce the reference runs instead).
 */
#ifndef XRABIT_DEVICE_HOST_STAGER_H_
#define XRABIT_DEVICE_HOST_STAGER_H_

#include <hip/hip_runtime_api.h>

#include <condition_variable>
#include <cstddef>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

#include "net/socket.h"

namespace rabit {
namespace device {

/*! \brief a persistent pool of threads that split one memcpy between them */
class CopyPool {
 public:
  explicit CopyPool(int threads);
  ~CopyPool();
  CopyPool(const CopyPool &) = delete;
  CopyPool &operator=(const CopyPool &) = delete;
  int threads() const { return static_cast<int>(workers_.size()) + 1; }
  /*! \brief dst[0, n) = src[0, n), in 64 KiB-aligned pieces over all threads (the caller's
   *  included); returns when every piece is done */
  void Copy(void *dst, const void *src, size_t n);
  /*! \brief the CPUs this process may use: OMP_NUM_THREADS, else its CPU affinity */
  static int HostShare();
  /*! \brief threads for one rank: HostShare() divided among `local` ranks (0: the
   *  LOCAL_WORLD_SIZE environment variable, else 1), between 1 and 8 */
  static int AutoThreads(int local = 0);

 private:
  /*! \brief the job of generation `gen`: copy its next piece; false when that job has no
   *  piece left or a newer job replaced it (a helper waking late never touches a newer job
   *  with an older job's pointers, and never counts a piece twice) */
  bool TakePiece(uint64_t gen);
  void Work();
  std::vector<std::thread> workers_;
  std::mutex mu_;
  std::condition_variable cv_;       // workers: a new job (or stop)
  std::condition_variable done_cv_;  // the caller: the last piece of its job is done
  bool stop_{false};
  uint64_t gen_{0};
  // the current job (all under mu_)
  char *dst_{nullptr};
  const char *src_{nullptr};
  size_t n_{0}, piece_{0};
  int pieces_{0}, next_{0}, done_{0};
};

class HostStager {
 public:
  /*! \brief chunk: bytes per pipeline stage (two pinned slots per direction); threads: memcpy
   *  threads (0: CopyPool::AutoThreads) */
  HostStager(int device, size_t chunk, int threads);
  ~HostStager();
  HostStager(const HostStager &) = delete;
  HostStager &operator=(const HostStager &) = delete;
  size_t chunk() const { return chunk_; }
  int threads() const { return pool_.threads(); }
  /*! \brief seconds spent, over all Runs so far: copying in / out on the host, waiting for a
   *  pinned input slot to be free, waiting for a chunk's result to arrive; and in Run overall */
  struct Times {
    double copy_in{0}, copy_out{0}, wait_in{0}, wait_out{0}, enqueue{0}, total{0};
    uint64_t runs{0};
  };
  /*! \brief one stream: the copies go on the plane stream too (GPU-side copies and collective
   *  serialise; the host copies still overlap them).  Fewer hardware queues per process. */
  void set_single_stream(bool v) { single_stream_ = v; }
  bool single_stream() const { return single_stream_; }
  const Times &times() const { return times_; }

  /*! \brief enqueue the collective on chunk [off, off + len) of the HBM copy (on the plane
   *  stream, no host wait) */
  typedef std::function<net::Status(size_t off, size_t len)> ChunkOp;
  /*! \brief wait for an event recorded on the plane stream, watching for peer failures */
  typedef std::function<net::Status(hipEvent_t ev)> EventWait;
  /*!
   * \brief host_out[0, bytes) = collective(host_in[0, bytes)) through the HBM buffer dev, chunk
   *        by chunk as described above.  chunk boundaries are multiples of `align` bytes (the
   *        element size).  On a failed chunk the pipeline drains and that status is returned
   *        (host_out is then partly written, as for any failed collective).
   */
  net::Status Run(void *host_out, const void *host_in, size_t bytes, size_t align, char *dev,
                  hipStream_t plane, const ChunkOp &op, const EventWait &wait);

 private:
  int device_;
  size_t chunk_;
  CopyPool pool_;
  hipStream_t h2d_{nullptr}, d2h_{nullptr};
  char *pin_in_[2]{}, *pin_out_[2]{};
  hipEvent_t ev_in_[2]{}, ev_op_[2]{}, ev_out_[2]{};
  Times times_;
  bool single_stream_{false};
};

}  // namespace device
}  // namespace rabit
#endif  // XRABIT_DEVICE_HOST_STAGER_H_
