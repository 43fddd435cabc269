/*!
 * \file links.h
 * \brief Peer links and the tree/ring topology handed out by the tracker.
 *
 * Parity: reference LinkRecord / RefLinkVector (`src/allreduce_base.h:298-411`).
 * A PeerLink tracks per-operation byte progress and owns an optional staging ring
 * (8-byte aligned storage) used when incoming data must be reduced before it can be
 * consumed: the ring never overwrites bytes that have not been consumed yet.
 */
#ifndef XRABIT_NET_LINKS_H_
#define XRABIT_NET_LINKS_H_

#include <algorithm>
#include <cstdint>
#include <memory>
#include <vector>

#include "net/socket.h"

namespace rabit {
namespace net {

class PeerLink {
 public:
  TcpSocket sock;
  int rank{-1};
  /*! \brief bytes received / sent in the current operation */
  size_t size_read{0}, size_write{0};

  void ResetProgress() { size_read = size_write = 0; }
  /*!
   * \brief size the staging ring for a transfer of count elements of type_nbytes,
   *        capped at cap_bytes and rounded down to whole elements
   */
  void InitRing(size_t type_nbytes, size_t count, size_t cap_bytes) {
    size_t want = std::min(type_nbytes * count, cap_bytes);
    want = std::max(want / type_nbytes, static_cast<size_t>(1)) * type_nbytes;
    storage_.resize((want + 7) / 8);
    ring_ = reinterpret_cast<char *>(storage_.data());
    ring_bytes_ = want;
  }
  char *ring() const { return ring_; }
  size_t ring_bytes() const { return ring_bytes_; }

  /*!
   * \brief receive into the ring; bytes at stream positions < protect_start may be
   *        overwritten, later ones are kept; never read past stream position limit
   */
  Status FillRing(size_t protect_start, size_t limit) {
    size_t upto = std::min(limit, protect_start + ring_bytes_);
    if (size_read >= upto) return Status::kSuccess;
    size_t off = size_read % ring_bytes_;
    size_t n = std::min(upto - size_read, ring_bytes_ - off);
    return Account(sock.Recv(ring_ + off, n));
  }
  /*! \brief receive straight into base[size_read, limit) */
  Status RecvTo(void *base, size_t limit) {
    if (size_read >= limit) return Status::kSuccess;
    return Account(sock.Recv(static_cast<char *>(base) + size_read, limit - size_read));
  }
  /*! \brief send base[size_write, limit) */
  Status SendFrom(const void *base, size_t limit) {
    if (size_write >= limit) return Status::kSuccess;
    ssize_t n = sock.Send(static_cast<const char *>(base) + size_write, limit - size_write);
    if (n >= 0) {
      size_write += static_cast<size_t>(n);
      return Status::kSuccess;
    }
    return StatusFromErrno();
  }

 private:
  Status Account(ssize_t n) {
    if (n > 0) {
      size_read += static_cast<size_t>(n);
      return Status::kSuccess;
    }
    if (n == 0) return Status::kRecvZeroLen;
    return StatusFromErrno();
  }
  std::vector<uint64_t> storage_;
  char *ring_{nullptr};
  size_t ring_bytes_{0};
};

/*! \brief all peer links plus the tree and ring views */
struct Topology {
  std::vector<std::unique_ptr<PeerLink>> links;
  std::vector<PeerLink *> tree;
  int parent_index{-1};
  int parent_rank{-1};
  PeerLink *ring_prev{nullptr};
  PeerLink *ring_next{nullptr};

  PeerLink *Find(int rank) {
    for (auto &l : links) {
      if (l->rank == rank) return l.get();
    }
    return nullptr;
  }
  void CloseAll() {
    for (auto &l : links) l->sock.Close();
  }
};
}  // namespace net
}  // namespace rabit
#endif  // XRABIT_NET_LINKS_H_
