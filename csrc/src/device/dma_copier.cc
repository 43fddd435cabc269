/*!
 * \file dma_copier.cc
 * \brief SDMA device-to-host copies through ROCr (see dma_copier.h).
 */
#include "device/dma_copier.h"

#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>

#include <algorithm>
#include <cstdio>

#include "device/device_plane.h"
#include "rabit/internal/utils.h"

namespace rabit {
namespace device {
namespace {

struct AgentSearch {
  uint32_t domain, bdf;
  hsa_agent_t gpu{0}, cpu{0};
  bool have_gpu{false}, have_cpu{false};
};

hsa_status_t VisitAgent(hsa_agent_t agent, void *arg) {
  AgentSearch *s = static_cast<AgentSearch *>(arg);
  hsa_device_type_t type;
  if (hsa_agent_get_info(agent, HSA_AGENT_INFO_DEVICE, &type) != HSA_STATUS_SUCCESS) {
    return HSA_STATUS_SUCCESS;
  }
  if (type == HSA_DEVICE_TYPE_CPU && !s->have_cpu) {
    s->cpu = agent;
    s->have_cpu = true;
  } else if (type == HSA_DEVICE_TYPE_GPU && !s->have_gpu) {
    uint32_t bdf = 0, domain = 0;
    if (hsa_agent_get_info(agent, static_cast<hsa_agent_info_t>(HSA_AMD_AGENT_INFO_BDFID), &bdf) ==
            HSA_STATUS_SUCCESS &&
        hsa_agent_get_info(agent, static_cast<hsa_agent_info_t>(HSA_AMD_AGENT_INFO_DOMAIN),
                           &domain) == HSA_STATUS_SUCCESS &&
        bdf == s->bdf && domain == s->domain) {
      s->gpu = agent;
      s->have_gpu = true;
    }
  }
  return HSA_STATUS_SUCCESS;
}

}  // namespace

DmaCopier::DmaCopier(int device) {
  char pci[32] = {0};
  unsigned dom = 0, bus = 0, dev = 0, fn = 0;
  if (hipDeviceGetPCIBusId(pci, sizeof(pci), device) != hipSuccess ||
      std::sscanf(pci, "%x:%x:%x.%x", &dom, &bus, &dev, &fn) != 4) {
    (void)hipGetLastError();
    why_ = "no PCI id for HIP device " + std::to_string(device);
    return;
  }
  // HIP has initialised ROCr already; this only takes a reference (dropped in the destructor)
  if (hsa_init() != HSA_STATUS_SUCCESS) {
    why_ = "hsa_init failed";
    return;
  }
  AgentSearch s;
  s.domain = dom;
  s.bdf = (bus << 8) | (dev << 3) | fn;
  hsa_iterate_agents(VisitAgent, &s);
  if (!s.have_gpu || !s.have_cpu) {
    why_ = std::string("no ROCr ") + (s.have_gpu ? "CPU" : "GPU") + " agent for " + pci;
    hsa_shut_down();
    return;
  }
  gpu_agent_ = s.gpu.handle;
  cpu_agent_ = s.cpu.handle;
  ok_ = true;
  worker_ = std::thread([this]() { Run(); });
}

DmaCopier::~DmaCopier() {
  if (!ok_) return;
  {
    std::lock_guard<std::mutex> lk(mu_);
    stop_ = true;
  }
  cv_.notify_all();
  worker_.join();  // finishes the queued jobs first
  hsa_shut_down();
}

uint64_t DmaCopier::Submit(void *dst, const void *src, size_t bytes, hipEvent_t ready) {
  utils::Check(ok_, "SDMA copier unavailable: %s", why_.c_str());
  std::lock_guard<std::mutex> lk(mu_);
  const uint64_t t = ++submitted_;
  jobs_.push_back(Job{dst, src, bytes, ready, t});
  cv_.notify_one();
  return t;
}

bool DmaCopier::Done(uint64_t ticket) const {
  std::lock_guard<std::mutex> lk(mu_);
  return completed_ >= ticket;
}

bool DmaCopier::Wait(uint64_t ticket) {
  std::unique_lock<std::mutex> lk(mu_);
  done_cv_.wait(lk, [&]() { return completed_ >= ticket; });
  // a mirror is several jobs (one per buffer) and is waited for by its last ticket: any
  // unreported failure up to it counts (an older one only costs a redundant redo)
  const size_t before = failed_.size();
  failed_.erase(std::remove_if(failed_.begin(), failed_.end(),
                               [ticket](uint64_t t) { return t <= ticket; }),
                failed_.end());
  return failed_.size() == before;
}

bool DmaCopier::WaitAll() {
  std::unique_lock<std::mutex> lk(mu_);
  const uint64_t last = submitted_;
  done_cv_.wait(lk, [&]() { return completed_ >= last; });
  const bool ok = failed_.empty();
  failed_.clear();
  return ok;
}

void DmaCopier::Run() {
  hsa_signal_t sig;
  const bool have_sig = hsa_signal_create(1, 0, nullptr, &sig) == HSA_STATUS_SUCCESS;
  // fallback for a copy the SDMA path refused or failed: the same bytes by hipMemcpyAsync on a
  // stream of this thread (a blit kernel; slower for the caller's kernels, but the mirror lands)
  hipStream_t fallback = nullptr;
  if (hipStreamCreateWithFlags(&fallback, hipStreamNonBlocking) != hipSuccess) {
    (void)hipGetLastError();
    fallback = nullptr;
  }
  hsa_agent_t gpu{gpu_agent_}, cpu{cpu_agent_};
  // the first engine ROCr reports free for this direction (engine 0 if it cannot say)
  uint32_t mask = 0;
  hsa_amd_sdma_engine_id_t engine = HSA_AMD_SDMA_ENGINE_0;
  if (hsa_amd_memory_copy_engine_status(cpu, gpu, &mask) == HSA_STATUS_SUCCESS && mask != 0) {
    engine = static_cast<hsa_amd_sdma_engine_id_t>(mask & (~mask + 1));
  }
  for (;;) {
    Job job;
    {
      std::unique_lock<std::mutex> lk(mu_);
      cv_.wait(lk, [&]() { return stop_ || !jobs_.empty(); });
      if (jobs_.empty()) break;  // stop requested and drained
      job = jobs_.front();
      jobs_.pop_front();
    }
    const bool ready = hipEventSynchronize(job.ready) == hipSuccess;
    bool ok = have_sig && ready;
    if (ok && job.bytes != 0) {
      hsa_signal_store_relaxed(sig, 1);
      hsa_status_t st = hsa_amd_memory_async_copy_on_engine(job.dst, cpu, job.src, gpu, job.bytes,
                                                            0, nullptr, sig, engine, true);
      if (st != HSA_STATUS_SUCCESS) {
        // the chosen engine may be busy or absent for this pair: let ROCr pick
        st = hsa_amd_memory_async_copy(job.dst, cpu, job.src, gpu, job.bytes, 0, nullptr, sig);
      }
      ok = st == HSA_STATUS_SUCCESS &&
           hsa_signal_wait_scacquire(sig, HSA_SIGNAL_CONDITION_LT, 1, UINT64_MAX,
                                     HSA_WAIT_STATE_BLOCKED) == 0;
    }
    if (!ok && ready && job.bytes != 0 && fallback != nullptr) {
      if (fallbacks_.fetch_add(1) == 0) {
        utils::HandleLogInfo("[xrabit] SDMA mirror copy failed: copying with hipMemcpyAsync\n");
      }
      ok = hipMemcpyAsync(job.dst, job.src, job.bytes, hipMemcpyDeviceToHost, fallback) ==
               hipSuccess &&
           hipStreamSynchronize(fallback) == hipSuccess;
      if (!ok) (void)hipGetLastError();
    }
    {
      std::lock_guard<std::mutex> lk(mu_);
      if (!ok) failed_.push_back(job.ticket);
      completed_ = job.ticket;
    }
    done_cv_.notify_all();
  }
  if (fallback != nullptr) (void)hipStreamDestroy(fallback);
  if (have_sig) hsa_signal_destroy(sig);
}

}  // namespace device
}  // namespace rabit
