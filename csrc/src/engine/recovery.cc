/*!
 * \file recovery.cc
 * \brief Recovery protocol of the robust engine.
 *
 * Parity: reference `src/allreduce_robust.cc:687-1587` and `src/allreduce_robust-inl.h`.
 *  - RecoverExec: consensus loop deciding, from the reduced ActionSummary, whether to serve a
 *    checkpoint load, replay a result to a lagging peer, restore bootstrap-cache entries, or
 *    execute the requested action;
 *  - TryDecideRouting: two tree message-passing rounds (nearest holder by hop count, then the
 *    set of edges that must carry data) -> TryRecoverData streams the bytes along that route,
 *    relaying through bounded staging rings on pass-through nodes;
 *  - local (per-rank) checkpoints: engine/local_recovery.cc.
 * HBM-resident results and device checkpoints reach each requester by a device copy from one
 * holder (one xGMI hop; ranks that neither hold nor request move nothing) when every rank has a
 * device plane, otherwise they are staged through host memory on the ranks of the route.
 */
#include <algorithm>
#include <chrono>
#include <cstring>
#include <limits>
#include <thread>
#include <utility>

#include "core/trace.h"
#include "core/wait_state.h"
#include "engine/engine_robust.h"
#include "rabit/internal/io.h"
#include "rabit/internal/timer.h"
#include "rabit/internal/utils.h"

namespace rabit {
namespace engine {

// ------------------------------------------------------------------ failure handling
bool EngineRobust::CheckAndRecover(Status s) {
  if (s == Status::kSuccess) {
    recovering_since_.store(0.0);
    return true;
  }
  const double t0 = utils::GetTime();
  trace::Scope ts("recover", rank_, version_number_, seq_counter_, 0, 0);
  // detection: from the start of the attempt that failed to the failure seen here (the first
  // failure of a recovery only: later ones are part of the recovery itself)
  if (recovering_since_.load() == 0.0 && attempt_start_ > 0.0) {
    stats_.phases.detect += t0 - attempt_start_;
  }
  fast_mode_ = false;
  recover_counter_ += 1;
  stats_.n_recover_events += 1;
  wd_rank_.store(rank_);
  if (recovering_since_.load() == 0.0) recovering_since_.store(t0);
  if (debug_) {
    utils::HandleLogInfo("[%d] failure detected (%s, link %d), recovering\n", rank_,
                         net::StatusName(s),
                         host_->err_link() != nullptr ? host_->err_link()->rank : -1);
  }
  // the communicator contains the failed peer: abort it, a new epoch is built on demand
  if (dev_) dev_->AbortComm();
  // the shared-memory group contains the failed peer too: rebuilt on first use after rejoin
  ResetShm();
  // simplest consistent repair: drop every link so the failure propagates, then rejoin
  for (auto &l : topo_.links) l->sock.Close();
  // spread the reconnect load on the tracker (reference: 10 ms x rank; rabit_recover_stagger_ms)
  {
    core::WaitScope waiting;
    std::this_thread::sleep_for(
        std::chrono::microseconds(static_cast<int64_t>(recover_stagger_ms_ * 1000.0) *
                                  std::max(rank_, 0)));
  }
  const double t1 = utils::GetTime();
  stats_.phases.drop_links += t1 - t0;
  ReconnectLinks("recover");
  wd_rank_.store(rank_);
  const double t2 = utils::GetTime();
  stats_.phases.relink += t2 - t1;
  attempt_start_ = t2;  // the next attempt (a failure of it is detected relative to this)
  stats_.t_recover += t2 - t0;
  return false;
}

// ------------------------------------------------------------------ message passing
template <typename NodeT, typename EdgeT>
Status EngineRobust::MsgPassing(const NodeT &node, std::vector<EdgeT> *p_in,
                                std::vector<EdgeT> *p_out,
                                EdgeT (*func)(const NodeT &, const std::vector<EdgeT> &, size_t)) {
  auto &links = topo_.tree;
  const int nlink = static_cast<int>(links.size());
  const int pidx = topo_.parent_index;
  std::vector<EdgeT> &in = *p_in;
  std::vector<EdgeT> &out = *p_out;
  in.assign(nlink, EdgeT());
  out.assign(nlink, EdgeT());
  if (nlink == 0) return Status::kSuccess;
  constexpr size_t kSz = sizeof(EdgeT);
  std::vector<size_t> nrecv(nlink, 0), nsent(nlink, 0);
  std::vector<char> ready(nlink, 0);
  bool up_done = false, down_done = false;
  net::Poller poller;
  for (;;) {
    if (host_->Aborted()) return host_->Fail(nullptr, Status::kAborted);
    bool children_in = true;
    for (int i = 0; i < nlink; ++i) {
      if (i != pidx && nrecv[i] != kSz) children_in = false;
    }
    // upward: once every child reported, send the aggregate to the parent
    if (children_in && !up_done) {
      if (pidx >= 0) {
        out[pidx] = func(node, in, static_cast<size_t>(pidx));
        ready[pidx] = 1;
      }
      up_done = true;
    }
    // downward: once the parent answered, every child gets its message
    const bool parent_in = pidx < 0 || nrecv[pidx] == kSz;
    if (up_done && parent_in && !down_done) {
      for (int i = 0; i < nlink; ++i) {
        if (i == pidx) continue;
        out[i] = func(node, in, static_cast<size_t>(i));
        ready[i] = 1;
      }
      down_done = true;
    }
    bool done = down_done;
    poller.Clear();
    for (int i = 0; i < nlink; ++i) {
      if (nrecv[i] != kSz) {
        done = false;
        poller.WatchRead(links[i]->sock.fd());
      }
      if (nsent[i] != kSz) {
        done = false;
        if (ready[i]) poller.WatchWrite(links[i]->sock.fd());
      }
    }
    if (done) break;
    if (poller.Poll(host_->poll_ms()) == 0) continue;
    for (int i = 0; i < nlink; ++i) {
      const int fd = links[i]->sock.fd();
      if (nrecv[i] != kSz && poller.CanRead(fd)) {
        ssize_t k = links[i]->sock.Recv(reinterpret_cast<char *>(&in[i]) + nrecv[i],
                                        kSz - nrecv[i]);
        if (k > 0) {
          nrecv[i] += static_cast<size_t>(k);
        } else {
          Status st = k == 0 ? Status::kRecvZeroLen : net::StatusFromErrno();
          if (st != Status::kSuccess) return host_->Fail(links[i], st);
        }
      }
      if (ready[i] && nsent[i] != kSz && poller.CanWrite(fd)) {
        ssize_t k = links[i]->sock.Send(reinterpret_cast<const char *>(&out[i]) + nsent[i],
                                        kSz - nsent[i]);
        if (k >= 0) {
          nsent[i] += static_cast<size_t>(k);
        } else {
          Status st = net::StatusFromErrno();
          if (st != Status::kSuccess) return host_->Fail(links[i], st);
        }
      }
    }
  }
  return Status::kSuccess;
}

namespace {
/*! \brief (hops to the nearest data holder, data size) seen through an edge */
typedef std::pair<int, size_t> DistMsg;
constexpr int kUnreachable = std::numeric_limits<int>::max();

DistMsg ShortestDist(const std::pair<bool, size_t> &node, const std::vector<DistMsg> &in,
                     size_t out_index) {
  if (node.first) return DistMsg(1, node.second);
  DistMsg best(kUnreachable, 0);
  for (size_t i = 0; i < in.size(); ++i) {
    if (i == out_index || in[i].first == kUnreachable) continue;
    if (in[i].first + 1 < best.first) best = DistMsg(in[i].first + 1, in[i].second);
  }
  return best;
}

/*! \brief 1 if data must flow to us over out_index (we or someone behind us requests it) */
char DataRequest(const std::pair<bool, int> &node, const std::vector<char> &in,
                 size_t out_index) {
  if (static_cast<int>(out_index) != node.second) return 0;
  if (node.first) return 1;
  for (size_t i = 0; i < in.size(); ++i) {
    if (i != out_index && in[i] != 0) return 1;
  }
  return 0;
}
}  // namespace

Status EngineRobust::TryDecideRouting(RecoverType role, size_t *p_size, int *p_recvlink,
                                      std::vector<bool> *p_req_in) {
  int best_link = -2;
  {
    std::vector<DistMsg> dist_in, dist_out;
    Status s = MsgPassing(std::make_pair(role == kHaveData, *p_size), &dist_in, &dist_out,
                          ShortestDist);
    if (s != Status::kSuccess) return s;
    if (role != kHaveData) {
      for (size_t i = 0; i < dist_in.size(); ++i) {
        if (dist_in[i].first == kUnreachable) continue;
        utils::Check(best_link == -2 || *p_size == dist_in[i].second,
                     "[%d] recovery: inconsistent data size (%zu vs %zu)", rank_, *p_size,
                     dist_in[i].second);
        if (best_link == -2 || dist_in[i].first < dist_in[best_link].first) {
          best_link = static_cast<int>(i);
          *p_size = dist_in[i].second;
        }
      }
      utils::Check(best_link != -2, "Too many nodes went down and we cannot recover..");
    } else {
      best_link = -1;
    }
  }
  std::vector<char> req_in, req_out;
  Status s = MsgPassing(std::make_pair(role == kRequestData, best_link), &req_in, &req_out,
                        DataRequest);
  if (s != Status::kSuccess) return s;
  if (role != kRequestData) ServeHook(kServeRouting);
  p_req_in->assign(req_in.size(), false);
  for (size_t i = 0; i < req_in.size(); ++i) {
    (*p_req_in)[i] = req_in[i] != 0;
    if (req_out[i] != 0) {
      utils::Assert(req_in[i] == 0, "cannot both request and serve on one link");
      utils::Assert(static_cast<int>(i) == best_link, "request routed off the best link");
    }
  }
  *p_recvlink = best_link;
  return Status::kSuccess;
}

Status EngineRobust::TryRecoverData(RecoverType role, void *buf_, size_t size, int recv_link,
                                    const std::vector<bool> &req_in) {
  auto &links = topo_.tree;
  const int nlink = static_cast<int>(links.size());
  if (nlink == 0 || size == 0) return Status::kSuccess;
  utils::Assert(static_cast<int>(req_in.size()) == nlink, "TryRecoverData: request vector");
  bool involved = role == kRequestData;
  for (int i = 0; i < nlink; ++i) {
    if (req_in[i]) {
      utils::Assert(i != recv_link, "TryRecoverData: serving the link we receive from");
      involved = true;
    }
  }
  if (!involved) return Status::kSuccess;
  utils::Assert(recv_link >= 0 || role == kHaveData, "TryRecoverData: no receive link");
  char *buf = static_cast<char *>(buf_);
  net::PeerLink *src = recv_link >= 0 ? links[recv_link] : nullptr;
  if (role == kPassData) src->InitRing(1, size, hcfg_.reduce_buffer_bytes);
  for (auto *l : links) l->ResetProgress();
  net::Poller poller;
  bool sent_any = false;  // (fault injection: a server dies once its first bytes left)
  for (;;) {
    if (host_->Aborted()) return host_->Fail(nullptr, Status::kAborted);
    if (!sent_any && role != kRequestData) {
      for (int i = 0; i < nlink && !sent_any; ++i) sent_any = req_in[i] && links[i]->size_write > 0;
      if (sent_any) ServeHook(kServeData);
    }
    // bytes this node can forward so far
    const size_t avail = role == kHaveData ? size : src->size_read;
    bool done = true;
    poller.Clear();
    if (src != nullptr && src->size_read != size) {
      done = false;
      poller.WatchRead(src->sock.fd());
    }
    for (int i = 0; i < nlink; ++i) {
      if (!req_in[i] || links[i]->size_write == size) continue;
      done = false;
      if (links[i]->size_write < avail) poller.WatchWrite(links[i]->sock.fd());
    }
    if (done) break;
    if (poller.Poll(host_->poll_ms()) == 0) continue;
    if (src != nullptr && src->size_read != size && poller.CanRead(src->sock.fd())) {
      Status s;
      if (role == kRequestData) {
        s = src->RecvTo(buf, size);
      } else {
        // relay: never overwrite bytes some requester has not received yet
        size_t min_write = size;
        for (int i = 0; i < nlink; ++i) {
          if (req_in[i]) min_write = std::min(min_write, links[i]->size_write);
        }
        s = src->FillRing(min_write, size);
      }
      if (s != Status::kSuccess) return host_->Fail(src, s);
    }
    const size_t avail2 = role == kHaveData ? size : src->size_read;
    for (int i = 0; i < nlink; ++i) {
      net::PeerLink *l = links[i];
      if (!req_in[i] || l->size_write >= avail2 || !poller.CanWrite(l->sock.fd())) continue;
      if (role == kPassData) {
        const size_t cap = src->ring_bytes();
        const size_t off = l->size_write % cap;
        const size_t len = std::min(cap - off, avail2 - l->size_write);
        ssize_t k = l->sock.Send(src->ring() + off, len);
        if (k >= 0) {
          l->size_write += static_cast<size_t>(k);
        } else {
          Status st = net::StatusFromErrno();
          if (st != Status::kSuccess) return host_->Fail(l, st);
        }
      } else {
        Status st = l->SendFrom(buf, avail2);
        if (st != Status::kSuccess) return host_->Fail(l, st);
      }
    }
  }
  return Status::kSuccess;
}

// ------------------------------------------------------------------ results & checkpoints
Status EngineRobust::TryGetResult(void *sendrecvbuf, size_t size, int seqno, bool requester) {
  if (static_cast<uint32_t>(seqno) == ActionSummary::kLocalCheckAck) return Status::kSuccess;
  if (static_cast<uint32_t>(seqno) == ActionSummary::kLocalCheckPoint) {
    // some ranks finished the local checkin of the new version, others did not: fill the
    // missing replicas of the new version from the ranks that hold them
    return TryRecoverLocalState(!local_chkpt_version_);
  }
  trace::Scope ts("replay", rank_, version_number_, seqno, size, 0);
  // time of this catch-up step: the requester's replay or a holder's / relay's serving
  struct PhaseTimer {
    double *acc;
    double t0;
    ~PhaseTimer() { *acc += utils::GetTime() - t0; }
  } phase_timer{requester ? &stats_.phases.replay : &stats_.phases.serve_replay, utils::GetTime()};
  if (requester) {
    stats_.phases.replays += 1;
  } else {
    stats_.phases.serves += 1;
  }
  RecoverType role;
  void *data = nullptr;
  bool data_dev = false;
  if (!requester) {
    const ResultLog::Entry *e = resbuf_.Query(seqno);
    if (e != nullptr) {
      role = kHaveData;
      size = e->size;
      data = resbuf_.Data(*e);
      data_dev = e->on_device;
      if (e->spilled) {
        stats_.n_spilled_replays += 1;
        if (device_replay_) {
          // served over xGMI like an HBM entry: back into the HBM stage first
          void *stage = dev_->Scratch(size, device::DevicePlane::kSpillScratch);
          dev_->EnterFromUser();
          dev_->CopyAsync(stage, data, size);
          data = stage;
          data_dev = true;
        } else {
          // the TCP route reads the slot on the host: its D2H copy must have landed
          dev_->Synchronize();
        }
      }
    } else {
      role = kPassData;
    }
  } else {
    role = kRequestData;
    data = sendrecvbuf;
    data_dev = OnDevice(sendrecvbuf);
  }
  int recv_link;
  std::vector<bool> req_in;
  size_t data_size = size;
  Status s = TryDecideRouting(role, &data_size, &recv_link, &req_in);
  if (s != Status::kSuccess) return s;
  utils::Check(data_size != 0, "zero size check point is not allowed");
  if (role == kRequestData || role == kHaveData) {
    utils::Check(data_size == size,
                 "Allreduce recovered data size does not match the call (%zu vs %zu). Check "
                 "that the recovered program issues the same calls in this version",
                 data_size, size);
  }
  if (device_replay_) {
    // one hop on the xGMI mesh: when every rank has a device plane and the result sits in HBM
    // on a holder and is wanted in HBM by the requesters, each requester gets it by a device
    // copy from one holder (holders taken in turn), instead of streaming it through host
    // memory along the TCP tree.  Ranks that neither hold nor request move no bytes.
    std::vector<int> code;
    const int mine = (dev_ != nullptr && (role == kPassData || data_dev) ? kReplayCapable : 0) |
                     (role == kHaveData ? kReplayHolder : 0) |
                     (role == kRequestData ? kReplayRequester : 0);
    s = GatherCodes(mine, &code);
    if (s != Status::kSuccess) return s;
    std::vector<int> holders, requesters;
    bool capable = true;
    for (int r = 0; r < static_cast<int>(code.size()); ++r) {
      capable = capable && (code[r] & kReplayCapable) != 0;
      if (code[r] & kReplayHolder) holders.push_back(r);
      if (code[r] & kReplayRequester) requesters.push_back(r);
    }
    if (capable && !holders.empty()) {
      std::vector<device::ExchangeItem> plan;
      for (size_t i = 0; i < requesters.size(); ++i) {
        device::ExchangeItem x;
        x.src = holders[i % holders.size()];
        x.dst = requesters[i];
        x.key = 0;
        x.bytes = data_size;
        x.src_ptr = x.src == rank_ ? data : nullptr;
        x.dst_ptr = x.dst == rank_ ? data : nullptr;
        plan.push_back(x);
      }
      device::DeviceGuard dg(dev_->device());
      s = EnsureDeviceComm();
      if (s != Status::kSuccess) return s;
      if (role == kHaveData) ServeHook(kServeDevice);
      size_t got = 0;
      dev_->EnterFromUser();
      s = dev_->Exchange(plan, &got, MakeProbe());
      if (s == Status::kSuccess) s = dev_->Finish(MakeProbe());
      if (s == Status::kSuccess) {
        stats_.bytes_replay_in += static_cast<double>(got);
        if (role == kRequestData) stats_.n_device_replays += 1;
      }
      return s;
    }
  }
  if (data_dev) {
    // HBM-resident: stage through host memory, only if this rank is on the route
    const bool on_route = role == kRequestData ||
                          std::find(req_in.begin(), req_in.end(), true) != req_in.end();
    if (!on_route) return Status::kSuccess;
    std::vector<uint64_t> tmp((data_size + 7) / 8);
    if (role == kHaveData) dev_->StageToHost(tmp.data(), data, data_size);
    s = TryRecoverData(role, tmp.data(), data_size, recv_link, req_in);
    if (s == Status::kSuccess && role == kRequestData) {
      dev_->EnterFromUser();
      dev_->StageToDevice(data, tmp.data(), data_size);
      dev_->Finish(MakeProbe(), false);
    }
    return s;
  }
  return TryRecoverData(role, data, data_size, recv_link, req_in);
}

Status EngineRobust::TryLoadCheckPoint(bool requester) {
  const RecoverType role = requester ? kRequestData : kHaveData;
  Status s;
  struct PhaseTimer {
    double *acc;
    double t0;
    ~PhaseTimer() { *acc += utils::GetTime() - t0; }
  } phase_timer{requester ? &stats_.phases.load_checkpoint : &stats_.phases.serve_load,
                utils::GetTime()};
  if (num_local_replica_ != 0) {
    if (requester) local_.Clear(local_chkpt_version_);
    s = TryRecoverLocalState(local_chkpt_version_);
    if (s != Status::kSuccess) return s;
    const int nlocal = local_.Count(local_chkpt_version_);
    // 1: complete, 2: nothing, 4: partial; any partial node fails the load
    unsigned state = nlocal == num_local_replica_ + 1 ? 1u : (nlocal == 0 ? 2u : 4u);
    s = host_->TreeAllreduce(&state, sizeof(state), 1,
                             coll::HostReducer(mpi::kUInt, mpi::kBitwiseOR));
    if (s != Status::kSuccess) return s;
    utils::Check(state == 1 || state == 2,
                 "LoadCheckPoint: too many nodes failed, cannot recover local state");
  }
  if (device_replay_) {
    // a failure of the device route (a peer died while it ran) is returned like any other;
    // only a route that does not apply falls through to TCP -- falling through on a failure
    // would materialise the holders' HBM snapshots for a route the dead peer breaks anyway,
    // leaving the retry without device holders
    bool used = false;
    s = TryLoadDeviceCheckPoint(role, &used);
    if (s != Status::kSuccess || used) return s;
  }
  // A rank that loaded this version over the device route keeps only its header: the payload
  // went into the caller's tensors, which the caller has changed since.  On the TCP route it
  // relays; offering the header as the checkpoint would hand requesters a truncated model (or,
  // next to a real holder, fail the routing on two sizes).
  const RecoverType tcp_role =
      role == kHaveData && global_lazycheck_ == nullptr && ckpt_header_only_ ? kPassData : role;
  if (role == kHaveData && global_lazycheck_ != nullptr) {
    // materialise a lazy checkpoint now that a peer needs the bytes
    global_checkpoint_.clear();
    utils::MemoryBufferStream fs(&global_checkpoint_);
    fs.Write(&version_number_, sizeof(version_number_));
    global_lazycheck_->Save(&fs);
    global_lazycheck_ = nullptr;
  }
  size_t size = global_checkpoint_.length();
  int recv_link;
  std::vector<bool> req_in;
  s = TryDecideRouting(tcp_role, &size, &recv_link, &req_in);
  if (s != Status::kSuccess) return s;
  if (role == kRequestData) {
    global_checkpoint_.resize(size);
    ckpt_header_only_ = false;
  }
  if (size == 0) return Status::kSuccess;
  return TryRecoverData(tcp_role, BeginPtr(global_checkpoint_), size, recv_link, req_in);
}

Status EngineRobust::TryLoadDeviceCheckPoint(RecoverType role, bool *used) {
  // A device checkpoint (HBM snapshot) on the holders and an HBM loader on the requesters: the
  // lowest holder broadcasts the small header over the TCP tree, and every requester copies
  // the buffers from one holder's snapshot (one xGMI hop, holders taken in turn) instead of
  // serialising the model through host memory; the other ranks move no payload.  Every rank
  // runs the agreement round; *used = false (with no side effect) means "take the TCP route",
  // any other outcome is the route's own status.
  const bool holder_dev = role == kHaveData && global_lazycheck_ != nullptr && dev_ckpt_ &&
                          dev_ckpt_->IsSnapshot(global_lazycheck_);
  const bool req_dev = role == kRequestData && dev_ckpt_ && dev_ckpt_->loader_active();
  std::vector<int> code;
  const int mine =
      (dev_ != nullptr && (role == kRequestData ? req_dev : true) ? kReplayCapable : 0) |
      (holder_dev ? kReplayHolder : 0) | (role == kRequestData ? kReplayRequester : 0);
  Status s = GatherCodes(mine, &code);
  if (s != Status::kSuccess) return s;
  std::vector<int> holders, requesters;
  bool capable = true;
  for (int r = 0; r < static_cast<int>(code.size()); ++r) {
    capable = capable && (code[r] & kReplayCapable) != 0;
    if (code[r] & kReplayHolder) holders.push_back(r);
    if (code[r] & kReplayRequester) requesters.push_back(r);
  }
  *used = capable && !holders.empty();
  if (!*used) return Status::kSuccess;
  device::DeviceGuard dg(dev_->device());
  const int root = holders[0];
  std::string hdr;
  if (rank_ == root) {
    utils::MemoryBufferStream fs(&hdr);
    fs.Write(&version_number_, sizeof(version_number_));
    dev_ckpt_->SaveHeader(global_lazycheck_, &fs);
  }
  uint64_t len = hdr.size();
  s = host_->TreeBroadcast(&len, sizeof(len), root);
  if (s != Status::kSuccess) return s;
  hdr.resize(len);
  s = host_->TreeBroadcast(&hdr[0], len, root);
  if (s != Status::kSuccess) return s;
  // parse: int version, u64 meta_len, meta, u64 n, n x u64 size
  utils::MemoryFixSizeBuffer fs(&hdr[0], hdr.size());
  int version = 0;
  uint64_t ml = 0, n = 0;
  utils::Check(fs.Read(&version, sizeof(version)) == sizeof(version) &&
                   fs.Read(&ml, sizeof(ml)) == sizeof(ml),
               "device checkpoint header");
  fs.Seek(sizeof(version) + sizeof(ml) + ml);
  utils::Check(fs.Read(&n, sizeof(n)) == sizeof(n), "device checkpoint header count");
  std::vector<uint64_t> sizes(n);
  for (auto &z : sizes) utils::Check(fs.Read(&z, sizeof(z)) == sizeof(z), "header sizes");
  if (role == kRequestData) {
    utils::Check(dev_ckpt_->loader_targets().size() == n,
                 "device checkpoint holds %llu buffers, %zu given",
                 static_cast<unsigned long long>(n), dev_ckpt_->loader_targets().size());
  }
  // every requester reads every buffer from one holder's snapshot (holders taken in turn)
  std::vector<device::ExchangeItem> plan;
  for (size_t q = 0; q < requesters.size(); ++q) {
    const int src = holders[q % holders.size()];
    for (size_t i = 0; i < n; ++i) {
      if (sizes[i] == 0) continue;
      device::ExchangeItem x;
      x.src = src;
      x.dst = requesters[q];
      x.key = static_cast<int>(i);
      x.bytes = sizes[i];
      x.src_ptr = src == rank_ ? dev_ckpt_->SnapshotBuffer(global_lazycheck_, i) : nullptr;
      x.dst_ptr = nullptr;
      if (x.dst == rank_) {
        utils::Check(dev_ckpt_->loader_sizes()[i] == sizes[i],
                     "device checkpoint buffer %zu: %llu bytes stored, %zu given", i,
                     static_cast<unsigned long long>(sizes[i]), dev_ckpt_->loader_sizes()[i]);
        x.dst_ptr = dev_ckpt_->loader_targets()[i];
      }
      plan.push_back(x);
    }
  }
  s = EnsureDeviceComm();
  if (s != Status::kSuccess) return s;
  if (holder_dev) ServeHook(kServeDevice);
  size_t got = 0;
  dev_->EnterFromUser();
  s = dev_->Exchange(plan, &got, MakeProbe());
  if (s == Status::kSuccess) s = dev_->Finish(MakeProbe());
  if (s != Status::kSuccess) return s;
  stats_.bytes_ckpt_in += static_cast<double>(got);
  if (role == kRequestData) {
    global_checkpoint_ = hdr;  // version + header; the payload is already in the targets
    ckpt_header_only_ = true;
    dev_ckpt_->MarkPayloadDelivered();
  }
  stats_.n_device_ckpt_loads += 1;
  return Status::kSuccess;
}

Status EngineRobust::GatherCodes(int mine, std::vector<int> *all) {
  const int n = GetWorldSize();
  all->assign(n, 0);
  (*all)[rank_] = mine;
  if (n == 1) return Status::kSuccess;
  return host_->RingAllgather(all->data(), sizeof(int) * n, sizeof(int) * rank_,
                              sizeof(int) * (rank_ + 1), sizeof(int));
}

Status EngineRobust::TryRestoreCache(bool requester, int min_seq, int max_seq) {
  (void)min_seq;
  if (requester) {
    utils::Assert(cur_cache_seq_ <= max_seq, "requester should hold fewer cache entries");
    cachebuf_.Clear();
    lookupbuf_.Clear();
    cur_cache_seq_ = 0;
  }
  const RecoverType role = requester ? kRequestData : kHaveData;
  size_t size = 1;
  int recv_link;
  std::vector<bool> req_in;
  Status s = TryDecideRouting(role, &size, &recv_link, &req_in);
  if (s != Status::kSuccess) return s;
  for (int i = 0; i < max_seq; ++i) {
    for (ResultLog *log : {&lookupbuf_, &cachebuf_}) {
      uint64_t nbytes = 0;
      if (!requester) {
        const ResultLog::Entry *e = log->Query(i);
        utils::Assert(e != nullptr, "bootstrap cache entry %d missing on a holder", i);
        nbytes = e->size;
      }
      s = TryRecoverData(role, &nbytes, sizeof(nbytes), recv_link, req_in);
      if (s != Status::kSuccess) return s;
      void *data;
      if (requester) {
        log->AllocTemp(nbytes, false);
        log->PushTemp(i, nbytes);
        data = log->Data(*log->Query(i));
      } else {
        data = log->Data(*log->Query(i));
      }
      s = TryRecoverData(role, data, nbytes, recv_link, req_in);
      if (s != Status::kSuccess) return s;
    }
    if (requester) cur_cache_seq_ += 1;
  }
  return Status::kSuccess;
}

// ------------------------------------------------------------------ consensus state machine
bool EngineRobust::RecoverExec(void *buf, size_t size, int flag, int seqno, int cache_seqno,
                               const char *caller) {
  if (flag != 0 && flag != ActionSummary::kLoadBootstrapCache) {
    utils::Assert(static_cast<uint32_t>(seqno) == ActionSummary::kSpecialOp,
                  "%s: only normal operations carry a sequence number", caller);
  }
  utils::Assert(seqno >= 0, "%s: negative seqno %d (flag %d, version %d)", caller, seqno, flag,
                version_number_);
  if (recovering_since_.load() == 0.0) attempt_start_ = utils::GetTime();
  // steady state: everybody agreed to execute the previous op and nobody saw a failure
  // since, so the only possible outcome of this round is "execute"
  if (fast_mode_ && flag == 0 && static_cast<uint32_t>(seqno) < ActionSummary::kLocalCheckPoint) {
    stats_.n_consensus_elided += 1;
    return false;
  }
  const ActionSummary req(flag, flag, static_cast<uint32_t>(seqno),
                          static_cast<uint32_t>(cache_seqno));
  for (;;) {
    ReportStatus();
    ActionSummary act = req;
    const double t0 = utils::GetTime();
    Status s;
    {
      trace::Scope ts("consensus", rank_, version_number_, seqno, sizeof(act), 0);
      s = host_->TreeAllreduce(&act, sizeof(act), 1, ActionSummary::Reducer);
    }
    stats_.n_consensus += 1;
    stats_.t_consensus += utils::GetTime() - t0;
    if (!CheckAndRecover(s)) continue;

    if (act.check_ack()) {
      if (act.check_point()) {
        utils::Assert(!act.diff_seq(), "check ack & check pt cannot mix with normal ops");
        if (req.check_point()) return true;
      } else if (act.load_check()) {
        if (!CheckAndRecover(TryLoadCheckPoint(req.load_check()))) continue;
        if (req.load_check()) return true;
      } else if (req.check_ack()) {
        return true;
      }
      continue;  // the requested action is not done yet
    }
    if (act.check_point()) {
      if (act.diff_seq()) {
        // some nodes reached the checkpoint, others lag behind: the laggards (min seqno)
        // replay from the result log
        utils::Assert(act.seqno() != ActionSummary::kSpecialOp, "min seq bug");
        if (debug_) {
          utils::HandleLogInfo("[%d] %s: checkpoint with lagging peers (min seq %u)\n", rank_,
                               caller, act.seqno());
        }
        const bool requester = req.seqno() == act.seqno();
        if (!act.load_cache()) {
          if (act.seqno() > 0) {
            // A non-requester serves the laggard's op from its result log, or relays it.  The
            // reference asserts that every non-requester is at the checkpoint
            // (allreduce_robust.cc:1227), which holds for two levels only: with a second
            // restarted rank part-way through its replay (between the laggard and the
            // checkpoint) it fired on every retry, and the job ran out of attempts (found by the
            // device chaos fuzz at 8 ranks, seed 307).  That rank ran the op, so it holds the
            // result like a rank at the checkpoint does.
            if (!CheckAndRecover(TryGetResult(buf, size, static_cast<int>(act.seqno()),
                                              requester))) {
              continue;
            }
          }
        } else {
          utils::Assert(act.seqno(kCache) != ActionSummary::kSpecialOp, "checkpoint cache seq");
          int max_cache_seq = cur_cache_seq_;
          if (host_->TreeAllreduce(&max_cache_seq, sizeof(max_cache_seq), 1,
                                   coll::HostReducer(mpi::kInt, mpi::kMax)) != Status::kSuccess) {
            continue;
          }
          if (TryRestoreCache(req.load_cache(), static_cast<int>(act.seqno()), max_cache_seq) !=
              Status::kSuccess) {
            continue;
          }
        }
        if (requester) return true;
      } else if (req.check_point()) {
        return true;
      }
      continue;
    }
    if (act.load_check()) {
      // every node asked to load: fresh start, nothing to recover
      if (!act.diff_seq()) return false;
      if (!CheckAndRecover(TryLoadCheckPoint(req.load_check()))) continue;
      if (req.load_check()) return true;
      continue;
    }
    if (act.load_cache()) {
      utils::Assert(!act.check_point() && !act.check_ack(),
                    "bootstrap cache restore cannot overlap a checkpoint");
      if (act.load_cache(kCache)) return false;  // everybody is a requester: nothing cached
      // Requesters and holders are mixed: restore.  The reference restores only when the
      // seqnos differ (allreduce_robust.cc:1281-1285), assuming a requester (seqno = its op
      // count before LoadCheckPoint, 0) always lags the holders; survivors blocked in op 0 of a
      // version carry seqno 0 too, and the requester then took "restored" for an empty cache
      // and ran its bootstrap op against the survivors' op 0 (a hang; found by the chaos test,
      // tests/test_chaos.py seed 129).
      if (TryRestoreCache(req.load_cache(), static_cast<int>(act.seqno()),
                          static_cast<int>(act.seqno(kCache))) != Status::kSuccess) {
        continue;
      }
      if (req.load_cache()) return true;
      continue;
    }
    utils::Assert(!req.load_cache(), "load cache request reached sequence catch-up");
    utils::Assert(act.seqno() != ActionSummary::kSpecialOp, "min seq bug");
    if (act.diff_seq()) {
      const bool requester = req.seqno() == act.seqno();
      if (!CheckAndRecover(TryGetResult(buf, size, static_cast<int>(act.seqno()), requester))) {
        continue;
      }
      if (requester) return true;
      continue;
    }
    // every node proposes the same newest action: execute it
    if (elide_consensus_ && !bootstrap_cache_ && flag == 0) fast_mode_ = true;
    return false;
  }
}
}  // namespace engine
}  // namespace rabit
