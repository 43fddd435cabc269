/*!
 * \file link_reset.cc
 * \brief see link_reset.h
 */
#include "net/link_reset.h"

#include <errno.h>

#include <algorithm>
#include <chrono>

namespace rabit {
namespace net {
namespace {
enum Step : int { kSendUrgent, kSendMark, kDrain, kReadMark, kSendAck, kReadAck, kDone, kFailed };

bool WouldBlock(ssize_t n) {
  return n < 0 && (errno == EAGAIN || errno == EWOULDBLOCK || errno == EINTR);
}
}  // namespace

Status ResetLinks(const std::vector<TcpSocket *> &socks, int timeout_ms) {
  const size_t n = socks.size();
  std::vector<int> wstep(n, kSendUrgent), rstep(n, kDrain);
  for (size_t i = 0; i < n; ++i) {
    if (socks[i]->IsClosed()) {
      wstep[i] = rstep[i] = kFailed;
    } else {
      socks[i]->SetNonBlock(true);
    }
  }
  auto fail = [&](size_t i) {
    socks[i]->Close();
    wstep[i] = rstep[i] = kFailed;
  };
  const auto deadline = std::chrono::steady_clock::now() + std::chrono::milliseconds(timeout_ms);
  char junk[4096];
  // advance link i as far as it goes without blocking; false if it failed
  auto advance = [&](size_t i) {
    TcpSocket *s = socks[i];
    for (bool progressed = true; progressed;) {
      progressed = false;
      ssize_t k;
      switch (wstep[i]) {
        case kSendUrgent:
          k = s->SendUrgent(kResetOOB);
          if (k == 1) { wstep[i] = kSendMark; progressed = true; }
          else if (!WouldBlock(k)) return false;
          break;
        case kSendMark: {
          const char m = kResetMark;
          k = s->Send(&m, 1);
          if (k == 1) { wstep[i] = kSendAck; progressed = true; }
          else if (!WouldBlock(k)) return false;
          break;
        }
        case kSendAck:
          // the ack goes out only after the peer's mark was read (it has finished its drain)
          if (rstep[i] == kReadAck || rstep[i] == kDone) {
            const char a = kResetAck;
            k = s->Send(&a, 1);
            if (k == 1) { wstep[i] = kDone; progressed = true; }
            else if (!WouldBlock(k)) return false;
          }
          break;
        default:
          break;
      }
      switch (rstep[i]) {
        case kDrain: {
          const int at = s->AtMark();
          if (at < 0) return false;
          if (at == 1) {
            char oob;
            (void)s->RecvUrgent(&oob);  // the urgent byte itself is not in the stream
            rstep[i] = kReadMark;
            progressed = true;
            break;
          }
          k = s->Recv(junk, sizeof(junk));  // a read never crosses the mark
          if (k > 0) progressed = true;
          else if (k == 0 || !WouldBlock(k)) return false;
          break;
        }
        case kReadMark:
        case kReadAck: {
          char c;
          k = s->Recv(&c, 1);
          if (k == 1) {
            if (c != (rstep[i] == kReadMark ? kResetMark : kResetAck)) return false;
            rstep[i] = rstep[i] == kReadMark ? kReadAck : kDone;
            progressed = true;
          } else if (k == 0 || !WouldBlock(k)) {
            return false;
          }
          break;
        }
        default:
          break;
      }
    }
    return true;
  };
  for (;;) {
    bool pending = false;
    Poller poll;
    for (size_t i = 0; i < n; ++i) {
      if (wstep[i] == kFailed) continue;
      if (!advance(i)) {
        fail(i);
        continue;
      }
      if (wstep[i] != kDone || rstep[i] != kDone) {
        pending = true;
        if (rstep[i] != kDone) poll.WatchRead(socks[i]->fd());
        if (wstep[i] == kSendUrgent || wstep[i] == kSendMark) poll.WatchWrite(socks[i]->fd());
      }
    }
    if (!pending) break;
    const auto now = std::chrono::steady_clock::now();
    if (now >= deadline) {
      for (size_t i = 0; i < n; ++i) {
        if (wstep[i] != kDone || rstep[i] != kDone) fail(i);
      }
      break;
    }
    const int left = static_cast<int>(
        std::chrono::duration_cast<std::chrono::milliseconds>(deadline - now).count());
    poll.Poll(std::min(left, 50));
  }
  for (size_t i = 0; i < n; ++i) {
    if (wstep[i] != kDone || rstep[i] != kDone) return Status::kSockError;
  }
  return Status::kSuccess;
}
}  // namespace net
}  // namespace rabit
