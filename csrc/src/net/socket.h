/*!
 * \file socket.h
 * \brief Host TCP transport of the control plane (and of the CPU data plane).
 *
 * Parity: reference `include/rabit/internal/socket.h:50-533` (SockAddr, TCPSocket with
 * SendAll/RecvAll/SendStr/RecvStr, PollHelper).  This is a fresh, Linux-only design:
 * a move-only RAII socket, int32 length-prefixed strings on the wire, and a poll() set that
 * also reports hang-ups (POLLRDHUP) so the device-plane watchdog can observe peer death
 * without consuming bytes.
 */
#ifndef XRABIT_NET_SOCKET_H_
#define XRABIT_NET_SOCKET_H_

#include <poll.h>
#include <sys/types.h>

#include <cstdint>
#include <string>
#include <vector>

namespace rabit {
namespace net {

/*! \brief outcome of a non-blocking transfer step (reference ReturnType,
 *  allreduce_base.h:257-296) */
enum class Status : int {
  kSuccess = 0,
  kConnReset = 1,   // peer reset the connection
  kRecvZeroLen = 2, // orderly shutdown of the peer (EOF)
  kSockError = 3,   // other socket error
  kGetExcept = 4,   // exceptional condition reported by poll
  kTimeout = 5,     // xrabit: operation deadline exceeded
  kAborted = 6      // xrabit: device plane aborted (peer failure seen by the watchdog)
};
const char *StatusName(Status s);

/*! \brief map the current errno of a failed send/recv to a Status (EAGAIN => success) */
Status StatusFromErrno();

/*! \brief resolve host name to a dotted IPv4 string */
std::string ResolveIPv4(const std::string &host);
/*! \brief this machine's host name */
std::string HostName();

/*! \brief move-only TCP socket */
class TcpSocket {
 public:
  TcpSocket() = default;
  explicit TcpSocket(int fd) : fd_(fd) {}
  ~TcpSocket() { Close(); }
  TcpSocket(const TcpSocket &) = delete;
  TcpSocket &operator=(const TcpSocket &) = delete;
  TcpSocket(TcpSocket &&o) noexcept : fd_(o.fd_) { o.fd_ = -1; }
  TcpSocket &operator=(TcpSocket &&o) noexcept {
    if (this != &o) {
      Close();
      fd_ = o.fd_;
      o.fd_ = -1;
    }
    return *this;
  }

  /*! \brief create an IPv4 stream socket */
  void Create();
  /*! \brief blocking connect; false on failure (errno kept) */
  bool Connect(const std::string &host, int port);
  /*! \brief bind to the first free port in [start, end); returns the port or -1 */
  /*! \brief listen on the first free port of [start, end): the port, or -1 */
  int BindListenRange(int start, int end, int backlog = 256);
  TcpSocket Accept();
  void Close();
  bool IsClosed() const { return fd_ < 0; }
  int fd() const { return fd_; }

  void SetNonBlock(bool nonblock);
  void SetKeepAlive(bool keepalive);
  void SetNoDelay(bool nodelay);
  /*! \brief true if the socket has a pending error or is closed */
  bool BadSocket() const;
  /*! \brief true if the peer has closed / reset, without consuming data */
  bool PeerHungUp() const;

  /*! \brief single non-blocking send/recv; -1 with errno on failure */
  ssize_t Send(const void *buf, size_t len);
  ssize_t Recv(void *buf, size_t len);
  /*! \brief send one urgent (MSG_OOB) byte: marks a position in the byte stream */
  ssize_t SendUrgent(char c);
  /*! \brief read the pending urgent byte (clears POLLPRI); <0 if none */
  ssize_t RecvUrgent(char *c);
  /*! \brief 1 if the read position is at the urgent mark, 0 if not, -1 on error (SIOCATMARK) */
  int AtMark() const;
  /*! \brief blocking loops; return bytes moved (short count means error / EOF) */
  size_t SendAll(const void *buf, size_t len);
  size_t RecvAll(void *buf, size_t len);
  /*! \brief checked helpers used by the tracker protocol; throw rabit::Error on failure */
  void SendInt(int32_t v);
  int32_t RecvInt();
  void SendStr(const std::string &s);
  std::string RecvStr();

 private:
  int fd_{-1};
};

/*! \brief poll() set over a handful of sockets */
class Poller {
 public:
  void Clear() { fds_.clear(); }
  void WatchRead(int fd) { Entry(fd).events |= POLLIN; }
  void WatchWrite(int fd) { Entry(fd).events |= POLLOUT; }
  void WatchHangup(int fd) { Entry(fd).events |= POLLRDHUP; }
  /*! \brief urgent (out-of-band) data, e.g. a link-reset mark
   *  (reference PollHelper::WatchException) */
  void WatchExcept(int fd) { Entry(fd).events |= POLLPRI; }
  /*! \brief poll with a timeout in ms (-1 = infinite); returns poll()'s result */
  int Poll(int timeout_ms);
  bool CanRead(int fd) const { return Revents(fd) & (POLLIN | POLLHUP | POLLERR); }
  bool CanWrite(int fd) const { return Revents(fd) & (POLLOUT | POLLHUP | POLLERR); }
  bool CanExcept(int fd) const { return Revents(fd) & POLLPRI; }
  bool HungUp(int fd) const { return Revents(fd) & (POLLRDHUP | POLLHUP | POLLERR | POLLNVAL); }
  bool Empty() const { return fds_.empty(); }

 private:
  pollfd &Entry(int fd);
  short Revents(int fd) const;
  std::vector<pollfd> fds_;
};
}  // namespace net
}  // namespace rabit
#endif  // XRABIT_NET_SOCKET_H_
