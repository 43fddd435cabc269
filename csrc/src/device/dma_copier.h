/*!
 * \file dma_copier.h
 * \brief Device-to-host copies on an SDMA engine, issued through ROCr
 *        (hsa_amd_memory_async_copy_on_engine), for the checkpoint host mirrors.
 *
 * Why not hipMemcpyAsync: inside a PyTorch process the HIP runtime in use is the one PyTorch
 * ships, and it runs D2H copies as a blit kernel with one 512-lane workgroup on every CU
 * (measured: profiles/r2_s15_mirror).  A 256 MiB mirror then holds the whole chip for ~5 ms,
 * and a training step that overlaps it loses about half of that.  The SDMA engines move the
 * same bytes at the same PCIe rate (~57 GB/s) without touching a CU.
 *
 * Ordering: a job waits on a hipEvent (the snapshot it copies) in the copier's own thread, then
 * submits the DMA and waits for its completion signal; jobs run in submission order, so copies
 * into one host buffer never overlap.  Completion is a ticket number the caller polls or waits
 * on (the role the mirror's hipEvent plays on the hipMemcpyAsync path).
 */
#ifndef XRABIT_DEVICE_DMA_COPIER_H_
#define XRABIT_DEVICE_DMA_COPIER_H_

#include <hip/hip_runtime_api.h>

#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <deque>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

namespace rabit {
namespace device {

class DmaCopier {
 public:
  /*! \brief find the ROCr agents of HIP device `device` and of the host; ok() tells */
  explicit DmaCopier(int device);
  ~DmaCopier();
  bool ok() const { return ok_; }
  const std::string &why() const { return why_; }
  /*!
   * \brief queue dst (pinned host) <- src (HBM) once `ready` has completed; returns the job's
   *        ticket (tickets grow by one per job, 0 is "nothing")
   */
  uint64_t Submit(void *dst, const void *src, size_t bytes, hipEvent_t ready);
  /*! \brief the job with this ticket (and every earlier one) has finished (copied or failed) */
  bool Done(uint64_t ticket) const;
  /*!
   * \brief block until the job with this ticket has finished; false if its bytes did not land
   *        (the SDMA copy and the worker's hipMemcpyAsync fallback both failed), in which case
   *        the caller redoes the copy another way.  Any unreported failure of a job up to this
   *        ticket counts, and is reported once.
   */
  bool Wait(uint64_t ticket);
  /*! \brief block until every queued job has finished; false if any of them failed (never
   *  throws: also called from destructors) */
  bool WaitAll();
  uint64_t fallbacks() const { return fallbacks_.load(); }

 private:
  struct Job {
    void *dst;
    const void *src;
    size_t bytes;
    hipEvent_t ready;
    uint64_t ticket;
  };
  void Run();
  bool ok_{false};
  std::string why_;
  uint64_t gpu_agent_{0}, cpu_agent_{0};  // hsa_agent_t handles
  mutable std::mutex mu_;
  std::condition_variable cv_;       // jobs queued / stop
  std::condition_variable done_cv_;  // a job finished
  std::deque<Job> jobs_;
  uint64_t submitted_{0};
  uint64_t completed_{0};
  std::vector<uint64_t> failed_;   // tickets whose copy failed, not yet reported by Wait
  std::atomic<uint64_t> fallbacks_{0};
  bool stop_{false};
  std::thread worker_;
};

}  // namespace device
}  // namespace rabit
#endif  // XRABIT_DEVICE_DMA_COPIER_H_
