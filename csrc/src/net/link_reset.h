/*!
 * \file link_reset.h
 * \brief In-place reset of live peer links: discard every byte in flight and resynchronise both
 *        ends without going through the tracker.
 *
 * Parity: reference AllreduceRobust::TryResetLinks (`src/allreduce_robust.cc:567-679`, documented
 * there as unused — its engine reconnects instead, as xrabit's does by default).  Here it is a
 * standalone primitive with a non-blocking design: one poll loop drives a small state machine per
 * link under a deadline (the reference ends with blocking recv calls that can hang on a silent
 * peer).  Per link, both ends run the same steps:
 *   1. send one urgent (MSG_OOB) byte — its position splits stale bytes from fresh ones — and
 *      then an in-band kResetMark byte;
 *   2. read and discard in-band bytes until the socket is at the urgent mark (SIOCATMARK), then
 *      read the kResetMark byte;
 *   3. send kResetAck and read the peer's kResetAck.
 * A link that errors, closes or misses the deadline is closed; the result is kSuccess only when
 * every link finished (otherwise the caller falls back to reconnecting through the tracker).
 */
#ifndef XRABIT_NET_LINK_RESET_H_
#define XRABIT_NET_LINK_RESET_H_

#include <vector>

#include "net/socket.h"

namespace rabit {
namespace net {

constexpr char kResetOOB = 95;
constexpr char kResetMark = 97;
constexpr char kResetAck = 97;

/*! \brief reset the given sockets (all must be connected, non-blocking is set here) */
Status ResetLinks(const std::vector<TcpSocket *> &socks, int timeout_ms);
}  // namespace net
}  // namespace rabit
#endif  // XRABIT_NET_LINK_RESET_H_
