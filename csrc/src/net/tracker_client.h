/*!
 * \file tracker_client.h
 * \brief Worker side of the tracker protocol (wire-compatible with the dmlc tracker that
 *        the reference talks to; see SURVEY.md Appendix A and reference
 *        `src/allreduce_base.cc:221-438`).
 */
#ifndef XRABIT_NET_TRACKER_CLIENT_H_
#define XRABIT_NET_TRACKER_CLIENT_H_

#include <string>

#include "net/links.h"
#include "net/socket.h"

namespace rabit {
namespace net {

/*! \brief magic number of the handshake */
constexpr int32_t kTrackerMagic = 0xff99;

struct TrackerConfig {
  std::string uri{"NULL"};
  int port{9091};
  std::string task_id{"NULL"};
  int connect_retry{5};
  int worker_port{9010};
  int nport_trial{1000};
  bool tcp_nodelay{false};
};

class TrackerClient {
 public:
  explicit TrackerClient(const TrackerConfig *cfg) : cfg_(cfg) {}
  /*! \brief open a connection and run the handshake */
  TcpSocket Connect(int rank, int world_size) const;
  /*! \brief send a message to be printed by the tracker */
  void Print(int rank, int world_size, const std::string &msg) const;
  /*! \brief tell the tracker this rank finished */
  void Shutdown(int rank, int world_size) const;
  /*!
   * \brief (re)build peer links: "start" at init, "recover" after a failure.
   *        Healthy links in topo are kept, broken ones are re-established.
   * \param rank in/out; -1 on first start
   * \param world_size in/out
   */
  void Relink(const char *cmd, int *rank, int *world_size, Topology *topo) const;

 private:
  const TrackerConfig *cfg_;
};
}  // namespace net
}  // namespace rabit
#endif  // XRABIT_NET_TRACKER_CLIENT_H_
