/*!
 * \file shm_coll.cc
 * \brief Shared-memory host transport (see shm_coll.h).
 */
#include "coll/shm_coll.h"

#include <fcntl.h>
#include <sched.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstring>

#include "core/wait_state.h"
#include "rabit/internal/utils.h"

namespace rabit {
namespace coll {
namespace {
constexpr size_t kHeaderBytes = 64u << 10;  // flag lines; keeps the stages 64 KiB aligned
constexpr size_t kFlagStride = 64;          // one cache line per arrival flag
constexpr size_t kPiece = 256u << 10;       // reduce in cache-sized pieces
static_assert(kMaxShmRanks * kFlagStride <= kHeaderBytes, "flag header too small");

inline uint64_t *Flag(char *seg, int slot) {
  return reinterpret_cast<uint64_t *>(seg + static_cast<size_t>(slot) * kFlagStride);
}

inline void CpuRelax() {
#if defined(__x86_64__) || defined(__i386__)
  __builtin_ia32_pause();
#endif
}

std::atomic<uint64_t> g_segment_counter{0};
}  // namespace

ShmGroup::ShmGroup(size_t stage_bytes, double deadline_sec)
    : stage_bytes_((std::max<size_t>(stage_bytes, 1u << 20) + 4095) & ~static_cast<size_t>(4095)),
      deadline_sec_(deadline_sec) {
  seg_bytes_ = kHeaderBytes + 2 * stage_bytes_;
  gethostname(local_.host, sizeof(local_.host) - 1);
  local_.pid = static_cast<int32_t>(getpid());
  local_.stage_bytes = stage_bytes_;
  snprintf(local_.name, sizeof(local_.name), "/xrabit-%d-%llu", static_cast<int>(getpid()),
           static_cast<unsigned long long>(g_segment_counter.fetch_add(1)));
  fd_ = shm_open(local_.name, O_CREAT | O_EXCL | O_RDWR, 0600);
  if (fd_ < 0) {
    local_.name[0] = '\0';
    return;
  }
  // reserve the pages now: a tmpfs that runs out later would SIGBUS a writer
  if (ftruncate(fd_, static_cast<off_t>(seg_bytes_)) != 0 ||
      posix_fallocate(fd_, 0, static_cast<off_t>(seg_bytes_)) != 0) {
    close(fd_);
    fd_ = -1;
    shm_unlink(local_.name);
    local_.name[0] = '\0';
    return;
  }
  void *p = mmap(nullptr, seg_bytes_, PROT_READ | PROT_WRITE, MAP_SHARED, fd_, 0);
  if (p == MAP_FAILED) {
    close(fd_);
    fd_ = -1;
    shm_unlink(local_.name);
    local_.name[0] = '\0';
    return;
  }
  own_ = static_cast<char *>(p);
  std::memset(own_, 0, kHeaderBytes);
  local_.ok = 1;
}

ShmGroup::~ShmGroup() {
  for (char *p : peer_) {
    if (p != nullptr && p != own_) munmap(p, seg_bytes_);
  }
  if (own_ != nullptr) munmap(own_, seg_bytes_);
  if (fd_ >= 0) close(fd_);
  if (!sealed_ && local_.name[0] != '\0') shm_unlink(local_.name);
}

bool ShmGroup::Open(const std::vector<ShmRecord> &all, int rank, std::string *why) {
  const int n = static_cast<int>(all.size());
  if (n < 1 || n > kMaxShmRanks) {
    *why = "group size out of range";
    return false;
  }
  peer_.assign(n, nullptr);
  for (int r = 0; r < n; ++r) {
    if (!all[r].ok || std::strncmp(all[r].host, local_.host, sizeof(local_.host)) != 0 ||
        all[r].stage_bytes != stage_bytes_) {
      *why = "rank " + std::to_string(r) + " has no compatible segment on this host";
      return false;
    }
    if (r == rank) {
      peer_[r] = own_;
      continue;
    }
    const int fd = shm_open(all[r].name, O_RDWR, 0600);
    if (fd < 0) {
      *why = std::string("shm_open(") + all[r].name + ") failed";
      return false;
    }
    void *p = mmap(nullptr, seg_bytes_, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
    close(fd);
    if (p == MAP_FAILED) {
      *why = "mmap of a peer segment failed";
      return false;
    }
    peer_[r] = static_cast<char *>(p);
  }
  n_ = n;
  rank_ = rank;
  return true;
}

Status ShmGroup::Seal(const Probe &probe) {
  Status s = Barrier(probe);
  if (s != Status::kSuccess) return s;
  // every peer mapped every segment before arriving: the names are no longer needed
  shm_unlink(local_.name);
  sealed_ = true;
  return Status::kSuccess;
}

char *ShmGroup::stage(int r, int which) const {
  return peer_[r] + kHeaderBytes + static_cast<size_t>(which) * stage_bytes_;
}

Status ShmGroup::Barrier(const Probe &probe) {
  core::WaitScope waiting;
  const uint64_t e = ++epoch_;
  // release: this rank's stage writes before the arrival flag, in every peer's header
  for (int p = 0; p < n_; ++p) __atomic_store_n(Flag(peer_[p], rank_), e, __ATOMIC_RELEASE);
  using clock = std::chrono::steady_clock;
  const auto t0 = clock::now();
  auto last_probe = t0;
  for (int q = 0; q < n_; ++q) {
    uint64_t spins = 0;
    while (__atomic_load_n(Flag(own_, q), __ATOMIC_ACQUIRE) < e) {
      CpuRelax();
      if ((++spins & 255) != 0) continue;
      // ranks may outnumber cores: let the others run
      sched_yield();
      const auto now = clock::now();
      if (std::chrono::duration<double>(now - last_probe).count() > 1e-3) {
        last_probe = now;
        if (probe && probe()) return Status::kConnReset;
        if (std::chrono::duration<double>(now - t0).count() > deadline_sec_) {
          return Status::kTimeout;
        }
      }
    }
  }
  return Status::kSuccess;
}

Status ShmGroup::Allreduce(const void *src_, void *dst_, size_t tn, size_t count, ReduceFn red,
                           const Probe &probe) {
  const char *src = static_cast<const char *>(src_);
  char *dst = static_cast<char *>(dst_);
  const size_t chunk = std::max<size_t>(stage_bytes_ / tn, 1);
  const MPI::Datatype dt(tn);
  for (size_t off = 0; off < count; off += chunk) {
    const size_t c = std::min(chunk, count - off);
    const int which = parity_;
    parity_ ^= 1;
    char *mine = stage(rank_, which);
    std::memcpy(mine, src + off * tn, c * tn);
    Status s = Barrier(probe);
    if (s != Status::kSuccess) return s;
    const size_t seg = (c + n_ - 1) / n_;
    const size_t lo = std::min(c, seg * rank_), hi = std::min(c, lo + seg);
    const size_t piece = std::max<size_t>(kPiece / tn, 1);
    for (size_t a = lo; a < hi; a += piece) {
      const size_t len = std::min(piece, hi - a);
      for (int p = 0; p < n_; ++p) {
        if (p != rank_) red(stage(p, which) + a * tn, mine + a * tn, static_cast<int>(len), dt);
      }
      std::memcpy(dst + (off + a) * tn, mine + a * tn, len * tn);
    }
    s = Barrier(probe);
    if (s != Status::kSuccess) return s;
    for (int q = 0; q < n_; ++q) {
      if (q == rank_) continue;
      const size_t qlo = std::min(c, seg * q), qhi = std::min(c, qlo + seg);
      if (qhi > qlo) {
        std::memcpy(dst + (off + qlo) * tn, stage(q, which) + qlo * tn, (qhi - qlo) * tn);
      }
    }
  }
  ++ops_;
  return Status::kSuccess;
}

Status ShmGroup::Broadcast(void *buf_, size_t bytes, int root, const Probe &probe) {
  char *buf = static_cast<char *>(buf_);
  for (size_t off = 0; off < bytes; off += stage_bytes_) {
    const size_t c = std::min(stage_bytes_, bytes - off);
    const int which = parity_;
    parity_ ^= 1;
    if (rank_ == root) std::memcpy(stage(root, which), buf + off, c);
    Status s = Barrier(probe);
    if (s != Status::kSuccess) return s;
    if (rank_ != root) std::memcpy(buf + off, stage(root, which), c);
  }
  ++ops_;
  return Status::kSuccess;
}

Status ShmGroup::AllgatherV(void *buf_, size_t total, const std::vector<size_t> &begin,
                            const std::vector<size_t> &size, const Probe &probe) {
  char *buf = static_cast<char *>(buf_);
  // the (at most two) byte ranges of slice r in [0, total)
  auto ranges = [&](int r, size_t lo[2], size_t hi[2]) {
    if (size[r] == 0) return 0;
    const size_t b = begin[r] % total;
    lo[0] = b;
    hi[0] = std::min(total, b + size[r]);
    if (b + size[r] <= total) return 1;
    lo[1] = 0;
    hi[1] = b + size[r] - total;
    return 2;
  };
  // windows of one stage buffer each; a window holds the bytes [wlo, whi) of buf
  for (size_t wlo = 0; wlo < total; wlo += stage_bytes_) {
    const size_t whi = std::min(total, wlo + stage_bytes_);
    const int which = parity_;
    parity_ ^= 1;
    size_t lo[2], hi[2];
    int k = ranges(rank_, lo, hi);
    for (int j = 0; j < k; ++j) {
      const size_t a = std::max(lo[j], wlo), z = std::min(hi[j], whi);
      if (z > a) std::memcpy(stage(rank_, which) + (a - wlo), buf + a, z - a);
    }
    Status s = Barrier(probe);
    if (s != Status::kSuccess) return s;
    for (int p = 0; p < n_; ++p) {
      if (p == rank_) continue;
      k = ranges(p, lo, hi);
      for (int j = 0; j < k; ++j) {
        const size_t a = std::max(lo[j], wlo), z = std::min(hi[j], whi);
        if (z > a) std::memcpy(buf + a, stage(p, which) + (a - wlo), z - a);
      }
    }
  }
  ++ops_;
  return Status::kSuccess;
}
}  // namespace coll
}  // namespace rabit
