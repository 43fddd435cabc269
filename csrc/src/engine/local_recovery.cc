/*!
 * \file local_recovery.cc
 * \brief Replication and recovery of the local (per-rank) checkpoint state.
 *
 * Parity target: the reference's local-model replication (`src/allreduce_robust.cc:484-557`
 * for the checkpoint flow, `:1329-1511` for check-in and recovery), i.e. every rank's local
 * state survives as long as one of the num_local_replica ring successors that hold a copy
 * survives, and a restarted rank gets its own state and its predecessors' states back.
 *
 * How it is done here (re-derived for an 8-GPU node whose GPUs are all one xGMI hop apart):
 *  1. every rank publishes the sizes of its slots over the TCP control plane (a ring allgather
 *     of n x (K+1) integers), so every rank knows which rank holds which state;
 *  2. from that table every rank derives the same plan of one-hop copies: slot k of rank r
 *     must hold the state of s = r - k; it is copied from a rank that holds s (the owner
 *     first, then the nearest successor), or from another slot of r itself;
 *  3. the plan runs on the data plane that holds the state:
 *     - HBM store: one DevicePlane::Exchange (grouped ncclSend/ncclRecv over xGMI, or the
 *       direct transport's stage exchange); check-in is the same with the plan "slot k of r
 *       <- slot 0 of r - k".  No byte goes through host memory;
 *     - host store: check-in is K one-hop shifts along the ring; recovery routes each missing
 *       state from its nearest holder over the tree (TryDecideRouting / TryRecoverData).
 *  A slot that no surviving rank holds stays absent; LoadCheckPoint then fails the job as the
 *  reference does ("too many nodes failed").
 */
#include <algorithm>
#include <cstring>
#include <string>
#include <vector>

#include "core/trace.h"
#include "engine/engine_robust.h"
#include "rabit/internal/utils.h"

namespace rabit {
namespace engine {
namespace {
inline int Mod(int a, int n) { return ((a % n) + n) % n; }

/*! \brief a copy of the plan: requester slot (r, k) from holder slot (h, kh) */
struct SlotCopy {
  int r, k, h, kh;
  int64_t bytes;
};

/*!
 * \brief which slot (h, kh) should serve the state of rank s to requester r.  table[h * stride +
 *        kh] is the size of slot kh of rank h (kAbsent if missing).  Prefers a copy r already
 *        holds, then the owner's own slot, then the closest successor.  false: nobody holds s.
 */
bool PickHolder(const std::vector<int64_t> &table, int stride, int n, int nslot, int s, int r,
                int *h_out, int *kh_out) {
  for (int kh = 0; kh < nslot; ++kh) {
    if (Mod(r - kh, n) == s && table[r * stride + kh] != LocalReplicas::kAbsent) {
      *h_out = r;
      *kh_out = kh;
      return true;
    }
  }
  // slot kh of rank s + kh holds s: walk kh = 0 (the owner), 1 (its successor), ...
  for (int kh = 0; kh < nslot; ++kh) {
    const int h = Mod(s + kh, n);
    if (table[h * stride + kh] != LocalReplicas::kAbsent) {
      *h_out = h;
      *kh_out = kh;
      return true;
    }
  }
  return false;
}
}  // namespace

Status EngineRobust::GatherLocalSizes(int v, std::vector<int64_t> *table) {
  const int n = GetWorldSize(), nslot = local_.nslot(), stride = nslot + 1;
  table->assign(static_cast<size_t>(n) * stride, 0);
  std::vector<int64_t> mine = local_.Sizes(v);
  std::copy(mine.begin(), mine.end(), table->begin() + static_cast<size_t>(rank_) * stride);
  (*table)[static_cast<size_t>(rank_) * stride + nslot] = local_.on_device() ? 1 : 0;
  if (n == 1) return Status::kSuccess;
  const size_t row = sizeof(int64_t) * stride;
  Status s = host_->RingAllgather(table->data(), row * n, row * rank_, row * (rank_ + 1), row);
  if (s != Status::kSuccess) return s;
  for (int r = 0; r < n; ++r) {
    utils::Check((*table)[static_cast<size_t>(r) * stride + nslot] == (local_.on_device() ? 1 : 0),
                 "local checkpoints: rank %d keeps its local model in %s memory, rank %d in %s",
                 r, (*table)[static_cast<size_t>(r) * stride + nslot] ? "device" : "host", rank_,
                 local_.on_device() ? "device" : "host");
  }
  return Status::kSuccess;
}

Status EngineRobust::TryCheckinLocalState(int v) {
  if (num_local_replica_ == 0) return Status::kSuccess;
  const int n = GetWorldSize(), nslot = local_.nslot(), stride = nslot + 1;
  utils::Assert(local_.valid(v, 0), "local check-in without an own state");
  trace::Scope ts("local_checkin", rank_, version_number_, seq_counter_, local_.size(v, 0),
                  local_.on_device());
  std::vector<int64_t> table;
  Status s = GatherLocalSizes(v, &table);
  if (s != Status::kSuccess) return s;
  auto own_size = [&](int r) { return table[static_cast<size_t>(r) * stride]; };
  // a failed attempt keeps the own state and drops the replicas it started to write
  auto rollback = [&]() {
    for (int k = 1; k < nslot; ++k) local_.Drop(v, k);
  };
  if (local_.on_device()) {
    // slot k of rank r <- slot 0 of rank r - k: one exchange, every copy one xGMI hop
    std::vector<device::ExchangeItem> plan;
    for (int r = 0; r < n; ++r) {
      for (int k = 1; k < nslot; ++k) {
        const int src = Mod(r - k, n);
        device::ExchangeItem x;
        x.src = src;
        x.dst = r;
        x.key = 0;
        x.bytes = static_cast<size_t>(own_size(src));
        x.src_ptr = src == rank_ ? local_.Data(v, 0) : nullptr;
        x.dst_ptr = r == rank_ ? local_.Alloc(v, k, x.bytes) : nullptr;
        plan.push_back(x);
      }
    }
    device::DeviceGuard dg(dev_->device());
    s = EnsureDeviceComm();
    if (s == Status::kSuccess) {
      size_t got = 0;
      dev_->EnterFromUser();
      s = dev_->Exchange(plan, &got, MakeProbe());
      if (s == Status::kSuccess) s = dev_->Finish(MakeProbe());
      if (s == Status::kSuccess) stats_.bytes_local_in += static_cast<double>(got);
    }
    if (s != Status::kSuccess) rollback();
    return s;
  }
  // host store: K shifts by one hop along the ring; shift j moves slot j-1 to the successor's
  // slot j (the state of rank r - j reaches rank r after j shifts)
  for (int j = 1; j < nslot; ++j) {
    const size_t out = static_cast<size_t>(local_.size(v, j - 1));
    const size_t in = static_cast<size_t>(own_size(Mod(rank_ - j, n)));
    if (n == 1) {
      std::string tmp(static_cast<const char *>(local_.Data(v, j - 1)), out);
      std::memcpy(local_.Alloc(v, j, out), tmp.data(), out);
      continue;
    }
    std::string buf(out + in, '\0');
    if (out != 0) std::memcpy(&buf[0], local_.Data(v, j - 1), out);
    s = host_->RingPass(&buf[0], out, out + in, 0, out, topo_.ring_prev, topo_.ring_next);
    if (s != Status::kSuccess) {
      rollback();
      return s;
    }
    void *dst = local_.Alloc(v, j, in);
    if (in != 0) std::memcpy(dst, buf.data() + out, in);
  }
  return Status::kSuccess;
}

Status EngineRobust::TryRecoverLocalState(int v) {
  if (num_local_replica_ == 0) return Status::kSuccess;
  const int n = GetWorldSize(), nslot = local_.nslot(), stride = nslot + 1;
  trace::Scope ts("local_recover", rank_, version_number_, seq_counter_, 0, local_.on_device());
  std::vector<int64_t> table;
  Status s = GatherLocalSizes(v, &table);
  if (s != Status::kSuccess) return s;
  auto at = [&](int r, int k) -> int64_t & { return table[static_cast<size_t>(r) * stride + k]; };
  // every copy of one state must have the same size
  for (int src = 0; src < n; ++src) {
    int64_t seen = LocalReplicas::kAbsent;
    for (int k = 0; k < nslot; ++k) {
      const int64_t z = at(Mod(src + k, n), k);
      if (z == LocalReplicas::kAbsent) continue;
      utils::Check(seen == LocalReplicas::kAbsent || seen == z,
                   "local checkpoint of rank %d has copies of different sizes (%lld, %lld)", src,
                   static_cast<long long>(seen), static_cast<long long>(z));
      seen = z;
    }
  }
  // the plan (identical on every rank): each missing slot from one holder
  std::vector<SlotCopy> plan;
  for (int r = 0; r < n; ++r) {
    for (int k = 0; k < nslot; ++k) {
      if (at(r, k) != LocalReplicas::kAbsent) continue;
      int h, kh;
      if (PickHolder(table, stride, n, nslot, Mod(r - k, n), r, &h, &kh)) {
        plan.push_back(SlotCopy{r, k, h, kh, at(h, kh)});
      }
    }
  }
  if (plan.empty()) return Status::kSuccess;
  const std::vector<int64_t> before = local_.Sizes(v);
  // a failed attempt drops the slots it started to fill; the ones held before stay
  auto rollback = [&]() {
    for (int k = 0; k < nslot; ++k) {
      if (before[k] == LocalReplicas::kAbsent) local_.Drop(v, k);
    }
  };
  if (local_.on_device()) {
    std::vector<device::ExchangeItem> xs;
    for (const SlotCopy &c : plan) {
      device::ExchangeItem x;
      x.src = c.h;
      x.dst = c.r;
      x.key = c.kh;  // one payload per holder slot, however many requesters read it
      x.bytes = static_cast<size_t>(c.bytes);
      x.src_ptr = c.h == rank_ ? local_.Data(v, c.kh) : nullptr;
      x.dst_ptr = c.r == rank_ ? local_.Alloc(v, c.k, x.bytes) : nullptr;
      xs.push_back(x);
    }
    device::DeviceGuard dg(dev_->device());
    s = EnsureDeviceComm();
    if (s == Status::kSuccess) {
      bool serving = false;
      for (const SlotCopy &c : plan) serving = serving || (c.h == rank_ && c.r != rank_);
      if (serving) ServeHook(kServeDevice);
      size_t got = 0;
      dev_->EnterFromUser();
      s = dev_->Exchange(xs, &got, MakeProbe());
      if (s == Status::kSuccess) s = dev_->Finish(MakeProbe());
      if (s == Status::kSuccess) stats_.bytes_local_in += static_cast<double>(got);
    }
    if (s != Status::kSuccess) rollback();
    return s;
  }
  // host store: one routed transfer per state that some rank is missing from a remote holder
  for (int src = 0; src < n; ++src) {
    bool remote = false;
    for (const SlotCopy &c : plan) remote = remote || (Mod(c.r - c.k, n) == src && c.h != c.r);
    if (!remote) continue;
    RecoverType role = kPassData;
    size_t size = 0;
    const void *have = nullptr;
    for (int k = 0; k < nslot && have == nullptr; ++k) {
      if (Mod(rank_ - k, n) == src && before[k] != LocalReplicas::kAbsent) {
        have = local_.Data(v, k);
        size = static_cast<size_t>(before[k]);
        role = kHaveData;
      }
    }
    bool want = false;
    for (const SlotCopy &c : plan) {
      want = want || (c.r == rank_ && c.h != rank_ && Mod(c.r - c.k, n) == src);
    }
    if (role != kHaveData && want) role = kRequestData;
    int recv_link;
    std::vector<bool> req_in;
    s = TryDecideRouting(role, &size, &recv_link, &req_in);
    if (s != Status::kSuccess) {
      rollback();
      return s;
    }
    std::string buf;
    if (role == kRequestData) buf.resize(size);
    void *data = role == kHaveData ? const_cast<void *>(have) : (buf.empty() ? nullptr : &buf[0]);
    s = TryRecoverData(role, data, size, recv_link, req_in);
    if (s != Status::kSuccess) {
      rollback();
      return s;
    }
    if (role == kRequestData) {
      for (const SlotCopy &c : plan) {
        if (c.r == rank_ && c.h != rank_ && Mod(c.r - c.k, n) == src) {
          void *dst = local_.Alloc(v, c.k, size);
          if (size != 0) std::memcpy(dst, buf.data(), size);
        }
      }
    }
  }
  // copies between slots of the same rank
  for (const SlotCopy &c : plan) {
    if (c.r != rank_ || c.h != rank_) continue;
    std::string tmp(static_cast<const char *>(local_.Data(v, c.kh)), static_cast<size_t>(c.bytes));
    void *dst = local_.Alloc(v, c.k, tmp.size());
    if (!tmp.empty()) std::memcpy(dst, tmp.data(), tmp.size());
  }
  return Status::kSuccess;
}
}  // namespace engine
}  // namespace rabit
