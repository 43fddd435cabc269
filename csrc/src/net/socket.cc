/*!
 * \file socket.cc
 * \brief TCP socket implementation (Linux).
 */
#include "net/socket.h"

#include <arpa/inet.h>
#include <errno.h>
#include <fcntl.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <sys/ioctl.h>
#include <sys/socket.h>
#include <unistd.h>

#include <cstring>

#include "core/wait_state.h"
#include "rabit/internal/utils.h"

namespace rabit {
namespace net {

const char *StatusName(Status s) {
  switch (s) {
    case Status::kSuccess: return "success";
    case Status::kConnReset: return "connection-reset";
    case Status::kRecvZeroLen: return "peer-closed";
    case Status::kSockError: return "socket-error";
    case Status::kGetExcept: return "exception";
    case Status::kTimeout: return "timeout";
    case Status::kAborted: return "aborted";
  }
  return "unknown";
}

Status StatusFromErrno() {
  int e = errno;
  if (e == EAGAIN || e == EWOULDBLOCK || e == EINTR) return Status::kSuccess;
  if (e == ECONNRESET || e == EPIPE) return Status::kConnReset;
  return Status::kSockError;
}

std::string ResolveIPv4(const std::string &host) {
  addrinfo hints;
  std::memset(&hints, 0, sizeof(hints));
  hints.ai_family = AF_INET;
  hints.ai_socktype = SOCK_STREAM;
  addrinfo *res = nullptr;
  int rc = getaddrinfo(host.c_str(), nullptr, &hints, &res);
  utils::Check(rc == 0 && res != nullptr, "cannot resolve host %s: %s", host.c_str(),
               gai_strerror(rc));
  char buf[INET_ADDRSTRLEN];
  const sockaddr_in *sa = reinterpret_cast<const sockaddr_in *>(res->ai_addr);
  inet_ntop(AF_INET, &sa->sin_addr, buf, sizeof(buf));
  freeaddrinfo(res);
  return std::string(buf);
}

std::string HostName() {
  char buf[256];
  if (gethostname(buf, sizeof(buf)) != 0) return "localhost";
  buf[sizeof(buf) - 1] = '\0';
  return std::string(buf);
}

void TcpSocket::Create() {
  Close();
  fd_ = socket(AF_INET, SOCK_STREAM | SOCK_CLOEXEC, 0);
  utils::Check(fd_ >= 0, "socket(): %s", strerror(errno));
}

bool TcpSocket::Connect(const std::string &host, int port) {
  sockaddr_in addr;
  std::memset(&addr, 0, sizeof(addr));
  addr.sin_family = AF_INET;
  addr.sin_port = htons(static_cast<uint16_t>(port));
  std::string ip = ResolveIPv4(host);
  if (inet_pton(AF_INET, ip.c_str(), &addr.sin_addr) != 1) return false;
  return connect(fd_, reinterpret_cast<sockaddr *>(&addr), sizeof(addr)) == 0;
}

int TcpSocket::BindListenRange(int start, int end, int backlog) {
  // SO_REUSEADDR: a port whose earlier connections linger in TIME_WAIT (a restarted worker's, or
  // another job's on this host) may be listened on again; without it, many restarts on one host
  // use the range up 60 s at a time.  Two processes may then both bind a free port, and only
  // the first listen() succeeds: the other gets EADDRINUSE there and moves on with a new socket
  // (a bound socket cannot be bound again).
  for (int port = start; port < end; ++port) {
    if (fd_ < 0) Create();
    const int one = 1;
    (void)setsockopt(fd_, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
    sockaddr_in addr;
    std::memset(&addr, 0, sizeof(addr));
    addr.sin_family = AF_INET;
    addr.sin_addr.s_addr = htonl(INADDR_ANY);
    addr.sin_port = htons(static_cast<uint16_t>(port));
    if (bind(fd_, reinterpret_cast<sockaddr *>(&addr), sizeof(addr)) != 0) {
      if (errno != EADDRINUSE && errno != EACCES) return -1;
      continue;  // still unbound: the next port with the same socket
    }
    if (listen(fd_, backlog) == 0) return port;
    if (errno != EADDRINUSE) return -1;
    Close();
  }
  return -1;
}

TcpSocket TcpSocket::Accept() {
  int fd;
  do {
    fd = accept4(fd_, nullptr, nullptr, SOCK_CLOEXEC);
  } while (fd < 0 && errno == EINTR);
  utils::Check(fd >= 0, "accept(): %s", strerror(errno));
  return TcpSocket(fd);
}

void TcpSocket::Close() {
  if (fd_ >= 0) {
    ::close(fd_);
    fd_ = -1;
  }
}

void TcpSocket::SetNonBlock(bool nonblock) {
  int flags = fcntl(fd_, F_GETFL, 0);
  utils::Check(flags != -1, "fcntl(F_GETFL): %s", strerror(errno));
  flags = nonblock ? (flags | O_NONBLOCK) : (flags & ~O_NONBLOCK);
  utils::Check(fcntl(fd_, F_SETFL, flags) != -1, "fcntl(F_SETFL): %s", strerror(errno));
}

void TcpSocket::SetKeepAlive(bool keepalive) {
  int v = keepalive ? 1 : 0;
  setsockopt(fd_, SOL_SOCKET, SO_KEEPALIVE, &v, sizeof(v));
}

void TcpSocket::SetNoDelay(bool nodelay) {
  int v = nodelay ? 1 : 0;
  setsockopt(fd_, IPPROTO_TCP, TCP_NODELAY, &v, sizeof(v));
}

bool TcpSocket::BadSocket() const {
  if (fd_ < 0) return true;
  int err = 0;
  socklen_t len = sizeof(err);
  if (getsockopt(fd_, SOL_SOCKET, SO_ERROR, &err, &len) != 0) return true;
  return err == EBADF || err == EINTR || err == ECONNRESET || err == EPIPE;
}

bool TcpSocket::PeerHungUp() const {
  if (fd_ < 0) return true;
  pollfd p;
  p.fd = fd_;
  p.events = POLLRDHUP;
  p.revents = 0;
  if (poll(&p, 1, 0) < 0) return false;
  return (p.revents & (POLLRDHUP | POLLHUP | POLLERR | POLLNVAL)) != 0;
}

ssize_t TcpSocket::Send(const void *buf, size_t len) {
  return ::send(fd_, buf, len, MSG_NOSIGNAL);
}

ssize_t TcpSocket::Recv(void *buf, size_t len) { return ::recv(fd_, buf, len, 0); }

ssize_t TcpSocket::SendUrgent(char c) { return ::send(fd_, &c, 1, MSG_OOB | MSG_NOSIGNAL); }

ssize_t TcpSocket::RecvUrgent(char *c) { return ::recv(fd_, c, 1, MSG_OOB); }

int TcpSocket::AtMark() const {
  int atmark = 0;
  if (ioctl(fd_, SIOCATMARK, &atmark) < 0) return -1;
  return atmark != 0 ? 1 : 0;
}

size_t TcpSocket::SendAll(const void *buf, size_t len) {
  core::WaitScope waiting;
  const char *p = static_cast<const char *>(buf);
  size_t done = 0;
  while (done < len) {
    ssize_t n = ::send(fd_, p + done, len - done, MSG_NOSIGNAL);
    if (n < 0) {
      if (errno == EINTR) continue;
      if (errno == EAGAIN || errno == EWOULDBLOCK) {
        pollfd pf{fd_, POLLOUT, 0};
        poll(&pf, 1, 1000);
        continue;
      }
      return done;
    }
    done += static_cast<size_t>(n);
  }
  return done;
}

size_t TcpSocket::RecvAll(void *buf, size_t len) {
  core::WaitScope waiting;
  char *p = static_cast<char *>(buf);
  size_t done = 0;
  while (done < len) {
    ssize_t n = ::recv(fd_, p + done, len - done, MSG_WAITALL);
    if (n == 0) return done;
    if (n < 0) {
      if (errno == EINTR) continue;
      if (errno == EAGAIN || errno == EWOULDBLOCK) {
        pollfd pf{fd_, POLLIN, 0};
        poll(&pf, 1, 1000);
        continue;
      }
      return done;
    }
    done += static_cast<size_t>(n);
  }
  return done;
}

void TcpSocket::SendInt(int32_t v) {
  utils::Check(SendAll(&v, sizeof(v)) == sizeof(v), "socket send failed: %s", strerror(errno));
}

int32_t TcpSocket::RecvInt() {
  int32_t v = 0;
  utils::Check(RecvAll(&v, sizeof(v)) == sizeof(v), "socket recv failed (peer closed?)");
  return v;
}

void TcpSocket::SendStr(const std::string &s) {
  SendInt(static_cast<int32_t>(s.length()));
  if (!s.empty()) {
    utils::Check(SendAll(s.data(), s.length()) == s.length(), "socket send failed");
  }
}

std::string TcpSocket::RecvStr() {
  int32_t len = RecvInt();
  utils::Check(len >= 0, "invalid string length %d", len);
  std::string s(static_cast<size_t>(len), '\0');
  if (len != 0) {
    utils::Check(RecvAll(&s[0], s.length()) == s.length(), "socket recv failed");
  }
  return s;
}

pollfd &Poller::Entry(int fd) {
  for (auto &p : fds_) {
    if (p.fd == fd) return p;
  }
  fds_.push_back(pollfd{fd, 0, 0});
  return fds_.back();
}

short Poller::Revents(int fd) const {
  for (const auto &p : fds_) {
    if (p.fd == fd) return p.revents;
  }
  return 0;
}

int Poller::Poll(int timeout_ms) {
  core::WaitScope waiting;
  for (auto &p : fds_) p.revents = 0;
  int rc;
  do {
    rc = poll(fds_.data(), fds_.size(), timeout_ms);
  } while (rc < 0 && errno == EINTR);
  utils::Check(rc >= 0, "poll(): %s", strerror(errno));
  return rc;
}
}  // namespace net
}  // namespace rabit
