/*!
 * \file host_coll.cc
 * \brief Host TCP collective algorithms (see host_coll.h).
 */
#include "coll/host_coll.h"

#include <algorithm>
#include <cstring>
#include <type_traits>

#include "rabit/internal/half.h"
#include "rabit/internal/utils.h"

namespace rabit {
namespace coll {

using engine::mpi::DataType;
using engine::mpi::OpType;

namespace {
template <typename T, OpType kOp>
void ReduceLoop(const void *src_, void *dst_, int n, const MPI::Datatype &) {
  const T *__restrict__ src = static_cast<const T *>(src_);
  T *__restrict__ dst = static_cast<T *>(dst_);
  if (kOp == engine::mpi::kSum) {
    for (int i = 0; i < n; ++i) dst[i] += src[i];
  } else if (kOp == engine::mpi::kMax) {
    for (int i = 0; i < n; ++i) dst[i] = src[i] > dst[i] ? src[i] : dst[i];
  } else if (kOp == engine::mpi::kMin) {
    for (int i = 0; i < n; ++i) dst[i] = src[i] < dst[i] ? src[i] : dst[i];
  }
}
template <typename T>
void OrLoop(const void *src_, void *dst_, int n, const MPI::Datatype &) {
  const T *__restrict__ src = static_cast<const T *>(src_);
  T *__restrict__ dst = static_cast<T *>(dst_);
  for (int i = 0; i < n; ++i) dst[i] |= src[i];
}
template <typename T>
ReduceFn PickOp(OpType op) {
  switch (op) {
    case engine::mpi::kSum: return ReduceLoop<T, engine::mpi::kSum>;
    case engine::mpi::kMax: return ReduceLoop<T, engine::mpi::kMax>;
    case engine::mpi::kMin: return ReduceLoop<T, engine::mpi::kMin>;
    case engine::mpi::kBitwiseOR:
      if (std::is_integral<T>::value) return OrLoop<typename std::conditional<
          std::is_integral<T>::value, T, int>::type>;
      return nullptr;
  }
  return nullptr;
}
}  // namespace

ReduceFn HostReducer(DataType dtype, OpType op) {
  switch (dtype) {
    case engine::mpi::kChar: return PickOp<signed char>(op);
    case engine::mpi::kUChar: return PickOp<unsigned char>(op);
    case engine::mpi::kInt: return PickOp<int32_t>(op);
    case engine::mpi::kUInt: return PickOp<uint32_t>(op);
    case engine::mpi::kLong: return PickOp<int64_t>(op);
    case engine::mpi::kULong: return PickOp<uint64_t>(op);
    case engine::mpi::kFloat: return PickOp<float>(op);
    case engine::mpi::kDouble: return PickOp<double>(op);
    case engine::mpi::kLongLong: return PickOp<int64_t>(op);
    case engine::mpi::kULongLong: return PickOp<uint64_t>(op);
    case engine::mpi::kHalf: return PickOp<half_t>(op);
    case engine::mpi::kBFloat16: return PickOp<bf16_t>(op);
  }
  return nullptr;
}

size_t DTypeSize(DataType dtype) {
  switch (dtype) {
    case engine::mpi::kChar:
    case engine::mpi::kUChar: return 1;
    case engine::mpi::kHalf:
    case engine::mpi::kBFloat16: return 2;
    case engine::mpi::kInt:
    case engine::mpi::kUInt:
    case engine::mpi::kFloat: return 4;
    default: return 8;
  }
}

Status HostCollectives::Allreduce(void *buf, size_t tn, size_t count, ReduceFn red,
                                  const void *src) {
  if (count > cfg_->reduce_ring_mincount && *world_ > 1) {
    return RingAllreduce(buf, tn, count, red, src);
  }
  // the tree path is latency-bound (small counts): stage the input
  if (src != nullptr && src != buf) std::memcpy(buf, src, tn * count);
  return TreeAllreduce(buf, tn, count, red);
}

Status HostCollectives::TreeAllreduce(void *buf_, size_t tn, size_t count, ReduceFn red) {
  auto &links = topo_->tree;
  if (links.empty() || count == 0) return Status::kSuccess;
  char *buf = static_cast<char *>(buf_);
  const size_t total = tn * count;
  const int pidx = topo_->parent_index;
  PeerLink *parent = pidx >= 0 ? links[pidx] : nullptr;
  const size_t nchild = links.size() - (parent ? 1 : 0);
  const size_t chunk = std::max(cfg_->tree_reduce_minsize / tn, static_cast<size_t>(1)) * tn;
  const MPI::Datatype dt(tn);
  for (size_t i = 0; i < links.size(); ++i) {
    links[i]->ResetProgress();
    if (static_cast<int>(i) != pidx) links[i]->InitRing(tn, count, cfg_->reduce_buffer_bytes);
  }
  // reduced: prefix of buf already combined with every child (ready for the parent)
  size_t reduced = nchild == 0 ? total : 0;
  net::Poller poller;
  for (;;) {
    if (Aborted()) return Fail(nullptr, Status::kAborted);
    const size_t down = parent ? parent->size_read : reduced;  // final bytes for children
    bool done = true;
    poller.Clear();
    for (size_t i = 0; i < links.size(); ++i) {
      PeerLink *l = links[i];
      const int fd = l->sock.fd();
      if (static_cast<int>(i) == pidx) {
        if (l->size_write < total) {
          done = false;
          if (l->size_write < reduced) poller.WatchWrite(fd);
        }
        if (l->size_read < total) {
          done = false;
          poller.WatchRead(fd);
        }
      } else {
        if (l->size_read < total) {
          done = false;
          poller.WatchRead(fd);
        }
        if (l->size_write < total) {
          done = false;
          if (l->size_write < down) poller.WatchWrite(fd);
        }
      }
    }
    if (done) break;
    if (poller.Poll(cfg_->poll_interval_ms) == 0) continue;
    // children -> staging rings, then reduce the common prefix
    if (nchild != 0) {
      size_t avail = total;
      for (size_t i = 0; i < links.size(); ++i) {
        if (static_cast<int>(i) == pidx) continue;
        PeerLink *l = links[i];
        if (l->size_read < total && poller.CanRead(l->sock.fd())) {
          Status s = l->FillRing(reduced, total);
          if (s != Status::kSuccess) return Fail(l, s);
        }
        avail = std::min(avail, l->size_read);
      }
      avail = avail / tn * tn;
      if (avail > reduced && (avail - reduced >= chunk || avail == total)) {
        while (reduced < avail) {
          size_t cap = 0;
          for (size_t i = 0; i < links.size(); ++i) {
            if (static_cast<int>(i) != pidx) cap = links[i]->ring_bytes();
          }
          const size_t off = reduced % cap;
          const size_t n = std::min(avail - reduced, cap - off);
          for (size_t i = 0; i < links.size(); ++i) {
            if (static_cast<int>(i) == pidx) continue;
            red(links[i]->ring() + off, buf + reduced, static_cast<int>(n / tn), dt);
          }
          reduced += n;
        }
      }
    }
    if (parent != nullptr) {
      const int fd = parent->sock.fd();
      if (parent->size_write < reduced && poller.CanWrite(fd)) {
        Status s = parent->SendFrom(buf, reduced);
        if (s != Status::kSuccess) return Fail(parent, s);
      }
      if (parent->size_read < total && poller.CanRead(fd)) {
        Status s = parent->RecvTo(buf, total);
        if (s != Status::kSuccess) return Fail(parent, s);
      }
    }
    const size_t down2 = parent ? parent->size_read : reduced;
    for (size_t i = 0; i < links.size(); ++i) {
      if (static_cast<int>(i) == pidx) continue;
      PeerLink *l = links[i];
      if (l->size_write < down2 && poller.CanWrite(l->sock.fd())) {
        Status s = l->SendFrom(buf, down2);
        if (s != Status::kSuccess) return Fail(l, s);
      }
    }
  }
  return Status::kSuccess;
}

namespace {
constexpr size_t kOutOfPlacePiece = 256u << 10;
inline size_t SegBegin(size_t k, size_t step, size_t count, size_t tn) {
  return std::min(k * step, count) * tn;
}
}  // namespace

Status HostCollectives::RingReduceScatter(void *buf_, size_t tn, size_t count, ReduceFn red,
                                          const void *src_) {
  const int n = *world_;
  if (n <= 1 || count == 0) return Status::kSuccess;
  PeerLink *next = topo_->ring_next, *prev = topo_->ring_prev;
  utils::Assert(next != nullptr && prev != nullptr, "ring links missing");
  const int rank = *rank_;
  utils::Assert(next->rank == (rank + 1) % n && prev->rank == (rank + n - 1) % n,
                "ring must be relabelled so that next == rank + 1");
  char *buf = static_cast<char *>(buf_);
  const char *src = src_ == buf_ ? nullptr : static_cast<const char *>(src_);
  const size_t total = tn * count;
  const size_t step = (count + n - 1) / n;
  const MPI::Datatype dt(tn);
  // Data flows rank -> rank-1.  This rank streams out every segment except its own,
  // starting with its successor's segment (raw) and continuing with the segments it has
  // reduced; it receives the stream of its successor, which starts one segment later.
  // Positions are unwrapped stream offsets (mod total gives the buffer offset).
  size_t write_ptr = SegBegin(next->rank, step, count, tn);
  size_t read_ptr = SegBegin(next->rank + 1, step, count, tn);
  if (next->rank + 1 == n) read_ptr = total;  // successor is the last rank: wrap
  size_t reduce_ptr = read_ptr;
  const size_t stop_read = total + write_ptr;
  size_t stop_write = total + SegBegin(rank, step, count, tn);
  if (stop_write > stop_read) stop_write -= total;
  // the first segment streamed out (the successor's) is raw input: out of place it is sent
  // straight from src; everything after it is sent from buf once reduced
  const size_t raw_end = read_ptr;
  next->InitRing(tn, step, cfg_->reduce_buffer_bytes);
  next->size_read = read_ptr;
  const size_t cap = next->ring_bytes();
  net::Poller poller;
  for (;;) {
    if (Aborted()) return Fail(nullptr, Status::kAborted);
    bool done = true;
    poller.Clear();
    if (read_ptr < stop_read) {
      done = false;
      poller.WatchRead(next->sock.fd());
    }
    if (write_ptr < stop_write) {
      done = false;
      if (write_ptr < reduce_ptr) poller.WatchWrite(prev->sock.fd());
    }
    if (done) break;
    if (poller.Poll(cfg_->poll_interval_ms) == 0) continue;
    if (read_ptr < stop_read && poller.CanRead(next->sock.fd())) {
      Status s = next->FillRing(reduce_ptr, stop_read);
      if (s != Status::kSuccess) return Fail(next, s);
      read_ptr = next->size_read;
      const size_t max_reduce = read_ptr / tn * tn;
      while (reduce_ptr < max_reduce) {
        const size_t roff = reduce_ptr % cap;
        const size_t boff = reduce_ptr % total;
        size_t len = std::min({max_reduce - reduce_ptr, cap - roff, total - boff});
        if (src != nullptr) {
          // buf = src op received, in cache-sized pieces (the copy's lines are still in cache
          // when the reduction rewrites them)
          len = std::min(len, std::max<size_t>(kOutOfPlacePiece / tn, 1) * tn);
          std::memcpy(buf + boff, src + boff, len);
        }
        red(next->ring() + roff, buf + boff, static_cast<int>(len / tn), dt);
        reduce_ptr += len;
      }
    }
    if (write_ptr < stop_write && write_ptr < reduce_ptr && poller.CanWrite(prev->sock.fd())) {
      size_t lim = std::min(reduce_ptr, stop_write);
      const char *from = buf;
      if (src != nullptr && write_ptr < raw_end) {
        lim = std::min(lim, raw_end);
        from = src;
      }
      const size_t start = write_ptr % total;
      const size_t len = std::min(lim - write_ptr, total - start);
      ssize_t k = prev->sock.Send(from + start, len);
      if (k >= 0) {
        write_ptr += static_cast<size_t>(k);
      } else {
        Status s = net::StatusFromErrno();
        if (s != Status::kSuccess) return Fail(prev, s);
      }
    }
  }
  return Status::kSuccess;
}

Status HostCollectives::RingAllreduce(void *buf, size_t tn, size_t count, ReduceFn red,
                                      const void *src) {
  Status s = RingReduceScatter(buf, tn, count, red, src);
  if (s != Status::kSuccess) return s;
  const int n = *world_;
  if (n <= 1) return Status::kSuccess;
  const size_t step = (count + n - 1) / n;
  const int rank = *rank_;
  const int prank = topo_->ring_prev->rank;
  const size_t begin = SegBegin(rank, step, count, tn);
  const size_t end = SegBegin(rank + 1, step, count, tn);
  const size_t prev_size = SegBegin(prank + 1, step, count, tn) - SegBegin(prank, step, count, tn);
  return RingAllgather(buf, tn * count, begin, end, prev_size);
}

Status HostCollectives::RingAllgather(void *buf_, size_t total, size_t slice_begin,
                                      size_t slice_end, size_t size_prev_slice) {
  const int n = *world_;
  if (n <= 1 || total == 0) return Status::kSuccess;
  PeerLink *next = topo_->ring_next, *prev = topo_->ring_prev;
  utils::Assert(next != nullptr && prev != nullptr, "ring links missing");
  const int rank = *rank_;
  utils::Assert(next->rank == (rank + 1) % n && prev->rank == (rank + n - 1) % n,
                "ring must be relabelled so that next == rank + 1");
  utils::Check(slice_begin <= slice_end && slice_end <= total + slice_begin,
               "Allgather: invalid slice");
  char *buf = static_cast<char *>(buf_);
  size_t read_ptr = slice_end;
  const size_t stop_read = total + slice_begin;
  size_t write_ptr = slice_begin;
  const size_t stop_write = total + slice_begin - size_prev_slice;
  net::Poller poller;
  for (;;) {
    if (Aborted()) return Fail(nullptr, Status::kAborted);
    bool done = true;
    poller.Clear();
    if (read_ptr < stop_read) {
      done = false;
      poller.WatchRead(next->sock.fd());
    }
    if (write_ptr < stop_write) {
      done = false;
      if (write_ptr < read_ptr) poller.WatchWrite(prev->sock.fd());
    }
    if (done) break;
    if (poller.Poll(cfg_->poll_interval_ms) == 0) continue;
    if (read_ptr < stop_read && poller.CanRead(next->sock.fd())) {
      const size_t start = read_ptr % total;
      const size_t len = std::min(stop_read - read_ptr, total - start);
      ssize_t k = next->sock.Recv(buf + start, len);
      if (k > 0) {
        read_ptr += static_cast<size_t>(k);
      } else {
        Status s = k == 0 ? Status::kRecvZeroLen : net::StatusFromErrno();
        if (s != Status::kSuccess) return Fail(next, s);
      }
    }
    if (write_ptr < stop_write && write_ptr < read_ptr && poller.CanWrite(prev->sock.fd())) {
      const size_t lim = std::min(read_ptr, stop_write);
      const size_t start = write_ptr % total;
      const size_t len = std::min(lim - write_ptr, total - start);
      ssize_t k = prev->sock.Send(buf + start, len);
      if (k >= 0) {
        write_ptr += static_cast<size_t>(k);
      } else {
        Status s = net::StatusFromErrno();
        if (s != Status::kSuccess) return Fail(prev, s);
      }
    }
  }
  return Status::kSuccess;
}

Status HostCollectives::TreeBroadcast(void *buf, size_t size, int root) {
  auto &links = topo_->tree;
  if (links.empty() || size == 0) return Status::kSuccess;
  // in_link: -1 = this node is the root, -2 = not known yet (first readable link)
  int in_link = (*rank_ == root) ? -1 : -2;
  for (auto *l : links) l->ResetProgress();
  net::Poller poller;
  for (;;) {
    if (Aborted()) return Fail(nullptr, Status::kAborted);
    const size_t avail = in_link == -1 ? size : (in_link >= 0 ? links[in_link]->size_read : 0);
    bool done = true;
    poller.Clear();
    for (size_t i = 0; i < links.size(); ++i) {
      PeerLink *l = links[i];
      if (in_link == -2) {
        done = false;
        poller.WatchRead(l->sock.fd());
      } else if (static_cast<int>(i) == in_link) {
        if (l->size_read < size) {
          done = false;
          poller.WatchRead(l->sock.fd());
        }
      } else if (l->size_write < size) {
        done = false;
        if (l->size_write < avail) poller.WatchWrite(l->sock.fd());
      }
    }
    if (done) break;
    if (poller.Poll(cfg_->poll_interval_ms) == 0) continue;
    if (in_link == -2) {
      for (size_t i = 0; i < links.size(); ++i) {
        if (poller.CanRead(links[i]->sock.fd())) {
          in_link = static_cast<int>(i);
          break;
        }
      }
      if (in_link == -2) continue;
    }
    if (in_link >= 0) {
      PeerLink *l = links[in_link];
      if (l->size_read < size && poller.CanRead(l->sock.fd())) {
        Status s = l->RecvTo(buf, size);
        if (s != Status::kSuccess) return Fail(l, s);
      }
    }
    const size_t avail2 = in_link == -1 ? size : links[in_link]->size_read;
    for (size_t i = 0; i < links.size(); ++i) {
      if (static_cast<int>(i) == in_link) continue;
      PeerLink *l = links[i];
      if (l->size_write < avail2 && poller.CanWrite(l->sock.fd())) {
        Status s = l->SendFrom(buf, avail2);
        if (s != Status::kSuccess) return Fail(l, s);
      }
    }
  }
  return Status::kSuccess;
}

Status HostCollectives::RingPass(void *buf_, size_t read_ptr, size_t read_end, size_t write_ptr,
                                 size_t write_end, PeerLink *read_link, PeerLink *write_link) {
  if (read_link == nullptr || write_link == nullptr || read_end == 0) return Status::kSuccess;
  utils::Assert(write_end <= read_end && read_ptr <= read_end && write_ptr <= write_end,
                "RingPass: boundary check");
  char *buf = static_cast<char *>(buf_);
  net::Poller poller;
  for (;;) {
    if (Aborted()) return Fail(nullptr, Status::kAborted);
    bool done = true;
    poller.Clear();
    if (read_ptr != read_end) {
      done = false;
      poller.WatchRead(read_link->sock.fd());
    }
    if (write_ptr != write_end) {
      done = false;
      if (write_ptr < read_ptr) poller.WatchWrite(write_link->sock.fd());
    }
    if (done) break;
    if (poller.Poll(cfg_->poll_interval_ms) == 0) continue;
    if (read_ptr != read_end && poller.CanRead(read_link->sock.fd())) {
      ssize_t k = read_link->sock.Recv(buf + read_ptr, read_end - read_ptr);
      if (k > 0) {
        read_ptr += static_cast<size_t>(k);
      } else {
        Status s = k == 0 ? Status::kRecvZeroLen : net::StatusFromErrno();
        if (s != Status::kSuccess) return Fail(read_link, s);
      }
    }
    if (write_ptr != write_end && write_ptr < read_ptr &&
        poller.CanWrite(write_link->sock.fd())) {
      const size_t len = std::min(write_end, read_ptr) - write_ptr;
      ssize_t k = write_link->sock.Send(buf + write_ptr, len);
      if (k >= 0) {
        write_ptr += static_cast<size_t>(k);
      } else {
        Status s = net::StatusFromErrno();
        if (s != Status::kSuccess) return Fail(write_link, s);
      }
    }
  }
  return Status::kSuccess;
}
}  // namespace coll
}  // namespace rabit
