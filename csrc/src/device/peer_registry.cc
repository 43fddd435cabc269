/*!
 * \file peer_registry.cc
 * \brief Registered zero-copy inputs of the direct transport; see peer_registry.h.
 */
#include "device/peer_registry.h"

#include <fcntl.h>
#include <sys/mman.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <thread>

namespace rabit {
namespace device {
namespace {
constexpr uint64_t kRegistryMagic = 0x7872656731ull;  // "xreg1"
constexpr size_t kPageBytes = (sizeof(RegistryPage) + 4095) / 4096 * 4096;
constexpr size_t kTableBytes = sizeof(char *) * kMaxRegPeers * kMaxRegs;

/*! \brief wait for `stream` to drain, at most `sec` seconds (a wedged stream must not hang the
 *  rank here: the op then fails and the engine recovers or restarts the worker) */
hipError_t Drain(hipStream_t stream, double sec) {
  using clock = std::chrono::steady_clock;
  const auto t0 = clock::now();
  for (;;) {
    const hipError_t e = hipStreamQuery(stream);
    if (e != hipErrorNotReady) return e;
    if (std::chrono::duration<double>(clock::now() - t0).count() > sec) {
      return hipErrorLaunchTimeOut;
    }
    std::this_thread::sleep_for(std::chrono::microseconds(50));
  }
}
}  // namespace

PeerRegistry::~PeerRegistry() {
  for (int q = 0; q < kMaxRegPeers; ++q) {
    for (int k = 0; k < kMaxRegs; ++k) {
      if (mapped_[q][k] != nullptr) (void)hipIpcCloseMemHandle(mapped_[q][k]);
    }
  }
  for (size_t r = 0; r < pages_.size(); ++r) {
    if (pages_[r] != nullptr && pages_[r] != mine_) munmap(pages_[r], kPageBytes);
  }
  if (mine_ != nullptr) munmap(mine_, kPageBytes);
  if (fd_ >= 0) close(fd_);
  if (!sealed_ && name_[0] != '\0') shm_unlink(name_);
  if (dev_table_raw_ != nullptr) (void)hipFree(dev_table_raw_);
  if (host_table_ != nullptr) (void)hipHostFree(host_table_);
}

bool PeerRegistry::Create(std::string *why) {
  static std::atomic<int> counter{0};
  std::snprintf(name_, sizeof(name_), "/xrabit_reg_%d_%d", static_cast<int>(getpid()),
                counter.fetch_add(1));
  fd_ = shm_open(name_, O_CREAT | O_EXCL | O_RDWR, 0600);
  if (fd_ < 0) {
    *why = std::string("shm_open(") + name_ + ") failed";
    name_[0] = '\0';
    return false;
  }
  if (ftruncate(fd_, static_cast<off_t>(kPageBytes)) != 0) {
    *why = "ftruncate of the registry page failed";
    return false;
  }
  void *p = mmap(nullptr, kPageBytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd_, 0);
  if (p == MAP_FAILED) {
    *why = "mmap of the registry page failed";
    return false;
  }
  std::memset(p, 0, kPageBytes);  // fresh segment: zeroed anyway; atomics start at 0
  mine_ = static_cast<RegistryPage *>(p);
  mine_->magic = kRegistryMagic;
  return true;
}

bool PeerRegistry::Open(const std::vector<std::string> &names, int rank, std::string *why) {
  n_ = static_cast<int>(names.size());
  rank_ = rank;
  if (mine_ == nullptr || n_ > kMaxRegPeers) {
    *why = "registry not created";
    return false;
  }
  pages_.assign(n_, nullptr);
  for (int r = 0; r < n_; ++r) {
    if (r == rank) {
      pages_[r] = mine_;
      continue;
    }
    const int fd = shm_open(names[r].c_str(), O_RDONLY, 0600);
    if (fd < 0) {
      *why = "shm_open(" + names[r] + ") failed";
      return false;
    }
    void *p = mmap(nullptr, kPageBytes, PROT_READ, MAP_SHARED, fd, 0);
    close(fd);
    if (p == MAP_FAILED) {
      *why = "mmap of a peer registry page failed";
      return false;
    }
    pages_[r] = static_cast<RegistryPage *>(p);
    if (pages_[r]->magic != kRegistryMagic) {
      *why = "peer registry page has a wrong magic";
      return false;
    }
  }
  void *h = nullptr;
  if (hipHostMalloc(&h, kTableBytes, hipHostMallocDefault) != hipSuccess) {
    (void)hipGetLastError();
    *why = "hipHostMalloc(registry table) failed";
    return false;
  }
  host_table_ = static_cast<const char **>(h);
  std::memset(host_table_, 0, kTableBytes);
  void *d = nullptr;
  if (hipMalloc(&d, kTableBytes) != hipSuccess || hipMemset(d, 0, kTableBytes) != hipSuccess) {
    (void)hipGetLastError();
    *why = "hipMalloc(registry table) failed";
    return false;
  }
  dev_table_raw_ = static_cast<const char **>(d);
  dev_table_ = dev_table_raw_;
  seen_version_.assign(n_, 0);
  opened_ = true;
  return true;
}

void PeerRegistry::Seal() {
  if (!sealed_ && name_[0] != '\0') shm_unlink(name_);
  sealed_ = true;
}

hipError_t PeerRegistry::Refresh(uint64_t op, hipStream_t stream, double drain_sec) {
  if (!opened_) return hipSuccess;
  bool dirty = false, drained = false;
  struct PendingAck {
    int q, k;
    uint64_t gen;
  };
  PendingAck acks[kMaxRegPeers * kMaxRegs];
  int nacks = 0;
  for (int q = 0; q < n_; ++q) {
    if (q == rank_) continue;
    RegistryPage *pg = pages_[q];
    const uint64_t v = pg->version.load(std::memory_order_acquire);
    if (v == seen_version_[q]) continue;
    bool complete = true;
    for (int k = 0; k < kMaxRegs; ++k) {
      RegistryPage::Slot &s = pg->slot[k];
      const uint64_t g = s.gen.load(std::memory_order_acquire);
      if ((g & 1u) != 0) {  // being rewritten: look again at the next op
        complete = false;
        continue;
      }
      if (g == mapped_gen_[q][k]) continue;
      hipIpcMemHandle_t handle;
      std::memcpy(&handle, s.ipc, sizeof(handle));
      std::atomic_thread_fence(std::memory_order_acquire);
      if (s.gen.load(std::memory_order_relaxed) != g) {
        complete = false;
        continue;
      }
      if (mapped_[q][k] != nullptr) {
        // an op already enqueued may still read through the old mapping: drain first
        if (!drained) {
          hipError_t e = Drain(stream, drain_sec);
          if (e != hipSuccess) return e;
          drained = true;
        }
        (void)hipIpcCloseMemHandle(mapped_[q][k]);
        mapped_[q][k] = nullptr;
        host_table_[q * kMaxRegs + k] = nullptr;
        dirty = true;
      }
      mapped_gen_[q][k] = g;
      if (g == 0) continue;
      // a mapping opened from the same handle bytes is an earlier allocation whose export was
      // released (see the header): close it, or the runtime returns it for this handle
      for (int k2 = 0; k2 < kMaxRegs; ++k2) {
        if (k2 == k || mapped_[q][k2] == nullptr ||
            std::memcmp(handle_[q][k2], &handle, sizeof(handle)) != 0) {
          continue;
        }
        if (!drained) {
          hipError_t e = Drain(stream, drain_sec);
          if (e != hipSuccess) return e;
          drained = true;
        }
        (void)hipIpcCloseMemHandle(mapped_[q][k2]);
        mapped_[q][k2] = nullptr;
        host_table_[q * kMaxRegs + k2] = nullptr;
        dirty = true;
      }
      void *m = nullptr;
      if (hipIpcOpenMemHandle(&m, handle, hipIpcMemLazyEnablePeerAccess) != hipSuccess) {
        (void)hipGetLastError();
        continue;  // never acknowledged: the exporter keeps staging this allocation
      }
      mapped_[q][k] = static_cast<char *>(m);
      std::memcpy(handle_[q][k], &handle, sizeof(handle));
      host_table_[q * kMaxRegs + k] = mapped_[q][k];
      dirty = true;
      ++imports_;
      acks[nacks++] = PendingAck{q, k, g};
    }
    if (complete) seen_version_[q] = v;
  }
  if (dirty) {
    hipError_t e = hipMemcpyAsync(dev_table_raw_, host_table_, kTableBytes, hipMemcpyHostToDevice,
                                  stream);
    if (e != hipSuccess) return e;
  }
  // the table update is enqueued ahead of op `op`'s kernels: valid from that op on
  for (int i = 0; i < nacks; ++i) {
    RegistryPage::Ack &a = mine_->ack[acks[i].q][acks[i].k];
    a.from_op.store(op, std::memory_order_release);
    a.gen.store(acks[i].gen, std::memory_order_release);
  }
  return hipSuccess;
}

int PeerRegistry::FindOrExport(uintptr_t p, size_t bytes, uint64_t op) {
  hipPointer_attribute attrs[3] = {HIP_POINTER_ATTRIBUTE_RANGE_START_ADDR,
                                   HIP_POINTER_ATTRIBUTE_RANGE_SIZE,
                                   HIP_POINTER_ATTRIBUTE_BUFFER_ID};
  hipDeviceptr_t start = nullptr;
  size_t size = 0;
  unsigned long long id = 0;
  void *data[3] = {&start, &size, &id};
  if (hipDrvPointerGetAttributes(3, attrs, data, reinterpret_cast<hipDeviceptr_t>(p)) !=
      hipSuccess) {
    (void)hipGetLastError();
    return -1;
  }
  const uintptr_t base = reinterpret_cast<uintptr_t>(start);
  if (base == 0 || id == 0 || p < base || p + bytes > base + size) return -1;
  for (int k = 0; k < kMaxRegs; ++k) {
    if (local_[k].gen != 0 && local_[k].base == base && local_[k].buffer_id == id) {
      local_[k].last_use = op;
      return k;
    }
  }
  if (std::find(bad_ids_.begin(), bad_ids_.end(), id) != bad_ids_.end()) return -1;
  hipIpcMemHandle_t h;
  if (hipIpcGetMemHandle(&h, start) != hipSuccess) {
    (void)hipGetLastError();
    ++unexportable_;
    if (bad_ids_.size() >= 256) bad_ids_.erase(bad_ids_.begin());
    bad_ids_.push_back(id);
    return -1;
  }
  // the slot of an earlier allocation at this address (freed and re-made: the peers drop the old
  // mapping when they see the slot rewritten), else a free slot, else the least recently used
  int k = -1;
  for (int j = 0; j < kMaxRegs && k < 0; ++j) {
    if (local_[j].gen != 0 && local_[j].base == base) k = j;
  }
  for (int j = 0; j < kMaxRegs && k < 0; ++j) {
    if (local_[j].gen == 0) k = j;
  }
  if (k < 0) {
    k = 0;
    for (int j = 1; j < kMaxRegs; ++j) {
      if (local_[j].last_use < local_[k].last_use) k = j;
    }
  }
  RegistryPage::Slot &s = mine_->slot[k];
  const uint64_t g = s.gen.load(std::memory_order_relaxed);
  s.gen.store(g + 1, std::memory_order_relaxed);  // odd: being rewritten
  std::atomic_thread_fence(std::memory_order_release);
  s.bytes = size;
  static_assert(sizeof(h) <= sizeof(s.ipc), "ipc handle size");
  std::memcpy(s.ipc, &h, sizeof(h));
  s.gen.store(g + 2, std::memory_order_release);
  mine_->version.fetch_add(1, std::memory_order_release);
  local_[k] = Local{base, size, id, g + 2, op};
  ++exports_;
  return -2;  // just exported: nobody has mapped it yet
}

bool PeerRegistry::Resolve(const void *p, size_t bytes, uint64_t op,
                           unsigned long long *mailbox) {
  if (!opened_ || n_ < 2) return false;
  const uintptr_t at = reinterpret_cast<uintptr_t>(p);
  const int k = FindOrExport(at, bytes, op);
  if (k < 0) return false;
  for (int q = 0; q < n_; ++q) {
    if (q == rank_) continue;
    RegistryPage::Ack &a = pages_[q]->ack[rank_][k];
    const uint64_t g = a.gen.load(std::memory_order_acquire);
    const uint64_t from = a.from_op.load(std::memory_order_relaxed);
    if (g != local_[k].gen || from > op) {
      ++pending_;
      return false;
    }
  }
  const unsigned long long off = at - local_[k].base;
  if (off > kMailboxOffsetMask) return false;
  *mailbox = kMailboxReg | (static_cast<unsigned long long>(k) << kMailboxRegShift) | off;
  return true;
}

}  // namespace device
}  // namespace rabit
