/*!
 * \file tracker_client.cc
 * \brief Worker side of the tracker protocol.
 */
#include "net/tracker_client.h"

#include <unistd.h>

#include <cstdio>
#include <set>
#include <vector>

#include "core/wait_state.h"
#include "rabit/internal/utils.h"

namespace rabit {
namespace net {

TcpSocket TrackerClient::Connect(int rank, int world_size) const {
  TcpSocket s;
  for (int attempt = 1;; ++attempt) {
    s.Create();
    if (s.Connect(cfg_->uri, cfg_->port)) break;
    if (attempt >= cfg_->connect_retry) {
      utils::Error("cannot connect to the tracker at %s:%d after %d attempts",
                   cfg_->uri.c_str(), cfg_->port, attempt);
    }
    fprintf(stderr, "xrabit: retry connecting to tracker %s:%d (attempt %d)\n",
            cfg_->uri.c_str(), cfg_->port, attempt);
    // linear-exponential backoff as in the reference (sleep(retry << 1))
    core::WaitScope waiting;
    sleep(static_cast<unsigned>(attempt << 1));
  }
  s.SendInt(kTrackerMagic);
  utils::Check(s.RecvInt() == kTrackerMagic, "tracker handshake: bad magic");
  s.SendInt(rank);
  s.SendInt(world_size);
  s.SendStr(cfg_->task_id);
  return s;
}

void TrackerClient::Print(int rank, int world_size, const std::string &msg) const {
  TcpSocket s = Connect(rank, world_size);
  s.SendStr("print");
  s.SendStr(msg);
}

void TrackerClient::Shutdown(int rank, int world_size) const {
  TcpSocket s = Connect(rank, world_size);
  s.SendStr("shutdown");
}

void TrackerClient::Relink(const char *cmd, int *rank, int *world_size, Topology *topo) const {
  TcpSocket tracker = Connect(*rank, *world_size);
  tracker.SendStr(cmd);
  const int new_rank = tracker.RecvInt();
  const int parent_rank = tracker.RecvInt();
  const int new_world = tracker.RecvInt();
  utils::Check(*rank == -1 || *rank == new_rank,
               "tracker changed the rank of a running worker (%d -> %d)", *rank, new_rank);
  if (new_rank == -1) {
    // the tracker refuses this worker (e.g. job already finished)
    fprintf(stderr, "xrabit: tracker assigned no rank, exiting\n");
    std::_Exit(255);
  }
  *rank = new_rank;
  *world_size = new_world;
  std::set<int> tree_nbrs;
  const int num_nbrs = tracker.RecvInt();
  for (int i = 0; i < num_nbrs; ++i) tree_nbrs.insert(tracker.RecvInt());
  const int prev_rank = tracker.RecvInt();
  const int next_rank = tracker.RecvInt();

  TcpSocket listener;
  listener.Create();
  int port = listener.BindListenRange(cfg_->worker_port, cfg_->worker_port + cfg_->nport_trial);
  utils::Check(port != -1, "cannot listen on a worker port in [%d, %d)", cfg_->worker_port,
               cfg_->worker_port + cfg_->nport_trial);

  auto adopt = [topo](TcpSocket &&sock, int peer) {
    PeerLink *l = topo->Find(peer);
    if (l == nullptr) {
      topo->links.emplace_back(new PeerLink());
      l = topo->links.back().get();
      l->rank = peer;
    }
    utils::Check(l->sock.IsClosed(), "link to rank %d is still active", peer);
    l->sock = std::move(sock);
  };

  int num_accept = 0;
  for (;;) {
    std::vector<int> good;
    for (auto &l : topo->links) {
      if (!l->sock.IsClosed() && !l->sock.BadSocket()) {
        good.push_back(l->rank);
      } else {
        l->sock.Close();
      }
    }
    tracker.SendInt(static_cast<int32_t>(good.size()));
    for (int r : good) tracker.SendInt(r);
    const int num_conn = tracker.RecvInt();
    num_accept = tracker.RecvInt();
    int num_error = 0;
    for (int i = 0; i < num_conn; ++i) {
      std::string host = tracker.RecvStr();
      const int peer_port = tracker.RecvInt();
      const int peer_rank = tracker.RecvInt();
      TcpSocket s;
      s.Create();
      if (!s.Connect(host, peer_port)) {
        ++num_error;
        continue;
      }
      s.SendInt(new_rank);
      utils::Check(s.RecvInt() == peer_rank, "peer rank mismatch when connecting to %d",
                   peer_rank);
      adopt(std::move(s), peer_rank);
    }
    tracker.SendInt(num_error);
    if (num_error == 0) break;
  }
  tracker.SendInt(port);
  tracker.Close();
  for (int i = 0; i < num_accept; ++i) {
    TcpSocket s = listener.Accept();
    s.SendInt(new_rank);
    int peer_rank = s.RecvInt();
    adopt(std::move(s), peer_rank);
  }
  listener.Close();

  // rebuild the views
  topo->tree.clear();
  topo->parent_index = -1;
  topo->parent_rank = parent_rank;
  topo->ring_prev = topo->ring_next = nullptr;
  for (auto &l : topo->links) {
    if (l->sock.IsClosed()) continue;
    l->sock.SetNonBlock(true);
    l->sock.SetKeepAlive(true);
    if (cfg_->tcp_nodelay) l->sock.SetNoDelay(true);
    if (tree_nbrs.count(l->rank) != 0) {
      if (l->rank == parent_rank) topo->parent_index = static_cast<int>(topo->tree.size());
      topo->tree.push_back(l.get());
    }
    if (l->rank == prev_rank) topo->ring_prev = l.get();
    if (l->rank == next_rank) topo->ring_next = l.get();
  }
  utils::Check(parent_rank == -1 || topo->parent_index != -1, "parent link missing");
  utils::Check(prev_rank == -1 || topo->ring_prev != nullptr, "ring prev link missing");
  utils::Check(next_rank == -1 || topo->ring_next != nullptr, "ring next link missing");
}
}  // namespace net
}  // namespace rabit
