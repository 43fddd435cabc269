/*!
 * \file device_setup.cc
 * \brief EngineBase: bringing up the device transports of an epoch — the GPU records and peer
 *        preflight, the direct (IPC) transport, the RCCL communicator (agreed on by every rank,
 *        optionally channel-tuned) and the start-up calibration that routes ops between them.
 *        The host engine itself is engine_base.cc.
 */
#include <algorithm>
#include <cstring>
#include <sstream>
#include <string>
#include <vector>

#include "device/kernels.h"
#include "engine/engine_base.h"
#include "engine/routing.h"
#include "rabit/internal/io.h"
#include "rabit/internal/timer.h"
#include "rabit/internal/utils.h"

namespace rabit {
namespace engine {

Status EngineBase::EnsureDeviceComm() {
  utils::Check(dev_ != nullptr, "device buffer given but the device plane is disabled");
  device::DeviceGuard dg(dev_->device());
  if (dev_->ready()) return Status::kSuccess;
  const int n = GetWorldSize();
  // Every rank brings the transports up at the same op (this is a collective), a restarted rank
  // and the survivors of a failure alike: per-epoch decisions that must match across ranks start
  // over here.  The host-staging trial counts ops on each rank, and a rank restarted after the
  // survivors decided would otherwise run the trial's forms against their decided one.
  host_stage_trial_ = 0;
  host_stage_pipe_ = false;
  EngineStats::Phases &ph = stats_.phases;
  ph.bringups += 1;
  double tp = utils::GetTime();
  auto lap = [&tp](double *acc) {
    const double now = utils::GetTime();
    *acc += now - tp;
    tp = now;
  };
  // 1. every rank describes its GPU (and exports its peer buffers when the direct transport
  //    may be used); the records travel around the host ring
  device::PeerRecord rec;
  std::memset(&rec, 0, sizeof(rec));
  std::string why;
  bool have_peers = false;
  if (dcfg_.algo != 1 && n <= device::kMaxPeers) {
    have_peers = dev_->PreparePeers(&rec, &why);
    if (!have_peers && debug_) {
      utils::HandleLogInfo("[%d] direct transport unavailable: %s\n", rank_, why.c_str());
    }
  }
  if (!have_peers) dev_->DescribeDevice(&rec);
  const size_t rb = sizeof(rec);
  std::vector<device::PeerRecord> all(n);
  std::memcpy(&all[rank_], &rec, rb);
  Status s = host_->RingAllgather(all.data(), rb * n, rb * rank_, rb * (rank_ + 1), rb);
  if (s != Status::kSuccess) return s;
  bool same_host = true, dup_gpu = false, all_peers = true;
  int on_my_host = 0;
  for (int r = 0; r < n; ++r) {
    on_my_host += std::strncmp(all[r].host, all[rank_].host, sizeof(rec.host)) == 0 ? 1 : 0;
    same_host = same_host && std::strncmp(all[r].host, all[0].host, sizeof(rec.host)) == 0;
    all_peers = all_peers && all[r].stage_bytes != 0;
    for (int q = 0; q < r; ++q) {
      dup_gpu = dup_gpu || (std::strncmp(all[r].host, all[q].host, sizeof(rec.host)) == 0 &&
                            std::strncmp(all[r].pci, all[q].pci, sizeof(rec.pci)) == 0);
    }
  }
  dev_->set_local_ranks(on_my_host);  // the host-staging thread pool's share of this host
  lap(&ph.records);
  // 2. direct transport: check that every visible peer GPU is reachable (peer access, link
  //    type), then map the peers' buffers; every rank must succeed (min-allreduce), otherwise
  //    the job runs on RCCL alone
  int ok = 0;
  const bool reachable = dev_->Preflight(all, rank_, &why);
  if (!reachable) utils::HandleLogInfo("[%d] direct transport off: %s\n", rank_, why.c_str());
  if (have_peers && all_peers && same_host && reachable) {
    ok = dev_->OpenPeers(all, rank_, &why) ? 1 : 0;
    if (!ok) utils::HandleLogInfo("[%d] direct transport: %s\n", rank_, why.c_str());
  }
  s = host_->Allreduce(&ok, sizeof(int), 1, coll::HostReducer(mpi::kInt, mpi::kMin));
  if (s != Status::kSuccess) return s;
  if (!ok) dev_->DropPeers();
  if (ok) dev_->SealPeers();  // every rank mapped every registry page
  lap(&ph.peer_open);
  // 3. RCCL: RCCL refuses several ranks on one GPU, which the direct transport handles alone
  // (test hook rabit_mock_rccl_init_fail: every rank's communicator "fails" to come up)
  const bool want_rccl = dcfg_.algo != 2 && (!dup_gpu || mock_rccl_fail_);
  if (want_rccl) {
    bool up = false;
    s = BuildRccl(&up);
    if (s != Status::kSuccess) return s;
    if (!up) {
      rccl_failed_ += 1;
      utils::HandleLogInfo("[%d] RCCL communicator did not come up on every rank: %s\n", rank_,
                           dev_->has_peers() ? "running on the direct transport alone"
                                             : "no device transport left");
    }
  }
  utils::Check(dev_->ready(), "no device transport: %s and the direct IPC transport is %s",
               dup_gpu ? "ranks share a GPU (RCCL refuses)"
                       : (dcfg_.algo == 2 ? "RCCL is disabled (rabit_device_algo=direct)"
                                          : "the RCCL communicator did not come up"),
               dcfg_.algo == 1 ? "disabled (rabit_device_algo=rccl)" : "unavailable");
  lap(&ph.rccl);
  dev_->BeginEpoch(n, rank_);
  if (want_rccl) {
    // every rank takes part in a tuning or none does (a restarted rank adopts the survivors'
    // choice through BuildRccl's agreement on the CTA bounds)
    int tune = rccl_tune_ && !rccl_tuned_ && dev_->has_comm() ? 1 : 0;
    s = host_->Allreduce(&tune, sizeof(int), 1, coll::HostReducer(mpi::kInt, mpi::kMin));
    if (s != Status::kSuccess) return s;
    rccl_tuned_ = true;
    if (tune) {
      s = TuneRcclChannels();
      if (s != Status::kSuccess) return s;
    }
  }
  lap(&ph.tune);
  if ((dev_->has_comm() || calibrate_test_) && dev_->has_peers() && dcfg_.algo == 0 &&
      calibrate_) {
    // a recovery epoch: the survivors hold the job's calibration, measured on this same set of
    // GPUs and links -- adopt it (one verified op per transport) instead of re-measuring
    bool adopted = false;
    if (adopt_calibration_) {
      s = AdoptCalibration(&adopted);
      if (s != Status::kSuccess) return s;
      lap(&ph.adopt);
    }
    if (adopted) {
      ph.adoptions += 1;
    } else {
      s = CalibrateDevice();
      if (s != Status::kSuccess) return s;
      if (dev_->has_peers()) {
        s = CalibrateBroadcast();
        if (s != Status::kSuccess) return s;
      }
      calib_valid_ = dev_->has_peers();
      ph.calibrations += 1;
      lap(&ph.calibration);
    }
  }
  if (debug_) {
    utils::HandleLogInfo("[%d] device transport epoch %d: rccl=%d direct=%d "
                         "(direct for >= %zu B)\n",
                         rank_, dev_->epoch(), dev_->has_comm() ? 1 : 0,
                         dev_->has_peers() ? 1 : 0, dcfg_.direct_min_bytes);
  }
  return Status::kSuccess;
}

Status EngineBase::AdoptCalibration(bool *adopted) {
  *adopted = false;
  const int n = GetWorldSize();
  // the lowest rank holding a calibration of this job (every survivor holds the same one: the
  // calibration's decisions were agreed over all ranks)
  int holder = calib_valid_ ? rank_ : n;
  Status s = host_->Allreduce(&holder, sizeof(int), 1, coll::HostReducer(mpi::kInt, mpi::kMin));
  if (s != Status::kSuccess) return s;
  if (holder >= n) return Status::kSuccess;  // the job's first bring-up: nothing to adopt
  std::string blob;
  if (rank_ == holder) blob = SerializeCalibration();
  uint64_t len = blob.size();
  s = host_->TreeBroadcast(&len, sizeof(len), holder);
  if (s != Status::kSuccess) return s;
  blob.resize(len);
  s = host_->TreeBroadcast(&blob[0], len, holder);
  if (s != Status::kSuccess) return s;
  ApplyCalibration(blob);
  bool good = false;
  s = VerifyTransports(&good);
  if (s != Status::kSuccess) return s;
  int ok = good ? 1 : 0;
  s = host_->Allreduce(&ok, sizeof(int), 1, coll::HostReducer(mpi::kInt, mpi::kMin));
  if (s != Status::kSuccess) return s;
  if (ok) {
    *adopted = true;
    calib_valid_ = true;
  }
  if (debug_ || rank_ == 0) {
    utils::HandleLogInfo("[xrabit] device epoch %d: %s rank %d's calibration\n", dev_->epoch(),
                         ok ? "adopted" : "verification failed, re-measuring instead of", holder);
  }
  return Status::kSuccess;
}

namespace {
template <typename T>
void Put(utils::MemoryBufferStream *fs, const T &v) {
  fs->Write(&v, sizeof(v));
}
template <typename T>
void Get(utils::MemoryFixSizeBuffer *fs, T *v) {
  utils::Check(fs->Read(v, sizeof(*v)) == sizeof(*v), "calibration record truncated");
}
}  // namespace

std::string EngineBase::SerializeCalibration() const {
  std::string blob;
  utils::MemoryBufferStream fs(&blob);
  typedef device::DevicePlane::RouteChoice RC;
  for (const std::vector<RC> *v : {&dev_->transport_bands(), &dev_->form_bands()}) {
    Put(&fs, static_cast<uint64_t>(v->size()));
    for (const RC &c : *v) Put(&fs, c);
  }
  Put(&fs, dev_->default_form());
  Put(&fs, static_cast<uint64_t>(dev_->direct_min_bytes()));
  Put(&fs, static_cast<uint64_t>(dev_->direct_below_bytes()));
  Put(&fs, static_cast<int32_t>(dev_->bcast_routed() ? 1 : 0));
  Put(&fs, static_cast<uint64_t>(dev_->bcast_min_bytes()));
  Put(&fs, static_cast<uint64_t>(dev_->bcast_below_bytes()));
  Put(&fs, calib_);
  Put(&fs, calib_form_us_);
  Put(&fs, calib_bcast_);
  Put(&fs, static_cast<int32_t>(calib_heap_src_ ? 1 : 0));
  Put(&fs, static_cast<uint64_t>(calib_matrix_json_.size()));
  fs.Write(calib_matrix_json_.data(), calib_matrix_json_.size());
  return blob;
}

void EngineBase::ApplyCalibration(const std::string &blob) {
  utils::MemoryFixSizeBuffer fs(const_cast<char *>(blob.data()), blob.size());
  typedef device::DevicePlane::RouteChoice RC;
  std::vector<RC> bands[2];
  for (auto &v : bands) {
    uint64_t k = 0;
    Get(&fs, &k);
    utils::Check(k <= 64, "calibration record: %llu bands", static_cast<unsigned long long>(k));
    v.resize(k);
    for (RC &c : v) Get(&fs, &c);
  }
  RC def;
  Get(&fs, &def);
  uint64_t dmin = 0, dbelow = 0, bmin = 0, bbelow = 0;
  int32_t brouted = 0, heap_src = 0;
  Get(&fs, &dmin);
  Get(&fs, &dbelow);
  Get(&fs, &brouted);
  Get(&fs, &bmin);
  Get(&fs, &bbelow);
  Get(&fs, &calib_);
  Get(&fs, &calib_form_us_);
  Get(&fs, &calib_bcast_);
  Get(&fs, &heap_src);
  uint64_t jl = 0;
  Get(&fs, &jl);
  calib_matrix_json_.resize(jl);
  if (jl != 0) utils::Check(fs.Read(&calib_matrix_json_[0], jl) == jl, "calibration record");
  calib_heap_src_ = heap_src != 0;
  dev_->SetRoutes(bands[0], bands[1]);
  dev_->SetDefaultForm(def.push != 0, def.pipeline != 0, def.fused != 0);
  dev_->RestoreCalibrated();
  dev_->set_direct_min_bytes(static_cast<size_t>(dmin));
  dev_->set_direct_below_bytes(static_cast<size_t>(dbelow));
  if (brouted) dev_->set_bcast_routing(static_cast<size_t>(bmin), static_cast<size_t>(bbelow));
}

Status EngineBase::VerifyTransports(bool *good) {
  *good = true;
  const int n = GetWorldSize();
  const size_t maxn = (1u << 20) / 4;
  float *src = static_cast<float *>(dev_->Scratch(maxn * 4, 0));
  float *dst = static_cast<float *>(dev_->Scratch(maxn * 4, 1));
  std::vector<float> host;
  const float want = 0.5f * n * (n + 1);
  // the direct transport at 1 MiB (the two-shot path in its calibrated form) and RCCL at 64 KiB
  for (int which : {1, 0}) {
    if ((which == 1 && !dev_->has_peers()) || (which == 0 && !dev_->has_comm())) continue;
    const size_t count = which == 1 ? maxn : (64u << 10) / 4;
    dev_->ForceTransport(which);
    device::CheckHip(device::LaunchFill(src, count, mpi::kFloat, rank_ + 1.0, dev_->stream()),
                     "LaunchFill");
    Status st = dev_->Allreduce(src, dst, nullptr, count, mpi::kFloat, mpi::kSum,
                                device::kPrepCopy, 1.0, MakeProbe());
    if (st == Status::kSuccess) st = dev_->Finish(MakeProbe());
    dev_->ForceTransport(-1);
    if (st != Status::kSuccess) return st;
    host.resize(count);
    dev_->StageToHost(host.data(), dst, count * 4);
    for (size_t i = 0; i < count && *good; ++i) *good = host[i] == want;
  }
  dev_->RestoreCalibrated();
  return Status::kSuccess;
}

Status EngineBase::BuildRccl(bool *up) {
  *up = false;
  // the CTA bounds of the communicator: the largest any rank holds (a restarted rank has none
  // yet and adopts the survivors' tuned value), so every rank asks RCCL for the same
  int ctas[2] = {dev_->rccl_min_ctas(), dev_->config().rccl_max_ctas};
  Status s = host_->Allreduce(ctas, sizeof(int), 2, coll::HostReducer(mpi::kInt, mpi::kMax));
  if (s != Status::kSuccess) return s;
  dev_->set_rccl_ctas(ctas[0], ctas[1]);
  // the id travels with a validity byte: a rank 0 that cannot create one tells everyone
  std::string id(sizeof(ncclUniqueId) + 1, '\0');
  if (rank_ == 0) {
    try {
      id = device::DevicePlane::NewUniqueId() + '\1';
    } catch (const std::exception &e) {
      utils::HandleLogInfo("[xrabit] RCCL unavailable: %s\n", e.what());
    }
  }
  s = host_->TreeBroadcast(&id[0], id.size(), 0);
  if (s != Status::kSuccess) return s;
  int ok = 0;
  if (id.back() == '\1' && !mock_rccl_fail_) {
    id.pop_back();
    ok = dev_->InitComm(id, GetWorldSize(), rank_, MakeProbe()) == Status::kSuccess ? 1 : 0;
  }
  // a communicator that did not come up on every rank is an environment problem, not a peer
  // failure (retrying would fail the same way): every rank drops it
  s = host_->Allreduce(&ok, sizeof(int), 1, coll::HostReducer(mpi::kInt, mpi::kMin));
  if (s != Status::kSuccess) return s;
  if (!ok) dev_->DropComm();
  *up = ok != 0;
  return Status::kSuccess;
}

Status EngineBase::TuneRcclChannels() {
  // one 128 MiB float32 sum per repetition, both destinations (as the robust engine runs it),
  // best of 3 after a warm-up, max over ranks; the candidates are RCCL's own channel choice and
  // fixed CTA counts (one CTA drives one channel: more channels, more of the 7 links busy)
  const size_t count = std::max<size_t>(dcfg_.calib_big / 4, 1u << 20);
  float *src = static_cast<float *>(dev_->Scratch(count * 4, 0));
  float *dst = static_cast<float *>(dev_->Scratch(count * 4, 1));
  float *dst2 = static_cast<float *>(dev_->Scratch(count * 4, device::DevicePlane::kCalibScratch));
  device::CheckHip(device::LaunchFill(src, count, mpi::kFloat, 1.0, dev_->stream()), "LaunchFill");
  std::vector<int> cands = {0};
  {
    std::istringstream in(rccl_tune_ctas_);
    std::string c;
    while (std::getline(in, c, ',')) {
      if (atoi(c.c_str()) > 0) cands.push_back(atoi(c.c_str()));
    }
  }
  const int base_min = dev_->rccl_min_ctas(), base_max = dev_->config().rccl_max_ctas;
  std::vector<double> times(cands.size(), 1e30);
  for (size_t i = 0; i < cands.size(); ++i) {
    if (i > 0) {
      dev_->DropComm();
      dev_->set_rccl_ctas(cands[i], cands[i]);
      bool up = false;
      Status s = BuildRccl(&up);
      if (s != Status::kSuccess) return s;
      if (!up) continue;  // this bound refused on some rank: skip it
    }
    dev_->ForceTransport(0);
    double best = 1e30;
    for (int rep = 0; rep < 4; ++rep) {
      const double t0 = utils::GetTime();
      Status s = dev_->Allreduce(src, dst, dst2, count, mpi::kFloat, mpi::kSum, device::kPrepCopy,
                                 1.0, MakeProbe());
      if (s == Status::kSuccess) s = dev_->Finish(MakeProbe());
      if (s != Status::kSuccess) {
        dev_->ForceTransport(-1);
        return s;  // a failed RCCL op: a real failure, the caller recovers
      }
      dev_->Synchronize();
      if (rep > 0) best = std::min(best, utils::GetTime() - t0);
    }
    dev_->ForceTransport(-1);
    times[i] = best;
  }
  Status s = host_->Allreduce(times.data(), sizeof(double), times.size(),
                              coll::HostReducer(mpi::kDouble, mpi::kMax));
  if (s != Status::kSuccess) return s;
  size_t best = 0;
  for (size_t i = 1; i < cands.size(); ++i) {
    if (times[i] < times[best]) best = i;
  }
  std::ostringstream js;
  js << "{\"bytes\":" << count * 4 << ",\"us\":{";
  for (size_t i = 0; i < cands.size(); ++i) {
    js << (i ? "," : "") << "\"" << (cands[i] ? std::to_string(cands[i]) : "rccl") << "\":"
       << (times[i] < 1e29 ? times[i] * 1e6 : -1.0);
  }
  js << "},\"chosen\":\"" << (cands[best] ? std::to_string(cands[best]) : "rccl") << "\"}";
  rccl_tune_json_ = js.str();
  if (rank_ == 0 || debug_) {
    utils::HandleLogInfo("[xrabit] RCCL channel tuning: %s\n", rccl_tune_json_.c_str());
  }
  // the communicator in place is the last candidate's; rebuild with the winner if it differs
  const int want_min = cands[best] ? cands[best] : base_min;
  const int want_max = cands[best] ? cands[best] : base_max;
  if (best != cands.size() - 1 || times[best] >= 1e29) {
    dev_->DropComm();
    dev_->set_rccl_ctas(want_min, want_max);
    bool up = false;
    s = BuildRccl(&up);
    if (s != Status::kSuccess) return s;
    if (!up) rccl_failed_ += 1;
  }
  // later epochs (after a recovery) build with the same bounds
  dcfg_.rccl_min_ctas = want_min;
  dcfg_.rccl_max_ctas = want_max;
  return Status::kSuccess;
}

namespace {
/*! \brief a form of the direct two-shot path the calibration times */
struct DirectForm {
  bool push, pipe, fused;
  const char *name;
};
const char *FormName(bool push, bool pipe, bool fused) {
  if (pipe) return "push-pipelined";
  if (push) return fused ? "push-fused" : "push-classic";
  return fused ? "pull-fused" : "pull-classic";
}
}  // namespace

Status EngineBase::CalibrateDevice() {
  // The routing is measured where training sizes live, at several points (bytes): a latency
  // point, gradient-bucket sizes and the large point (at most one stage chunk).  Each candidate
  // -- RCCL and every direct form the configuration allows -- is timed at every point (median of
  // kReps after a warm-up), the times are agreed (max over ranks), and routing.h turns them into
  // size bands: per band the faster transport, and per band the fastest direct form (used
  // whenever an op goes direct).  Every rank runs the same sequence: this is a collective.
  const size_t stage_cap = dev_->has_peers() ? dcfg_.peer_stage : 0;
  const size_t big_bytes =
      std::max<size_t>(std::min<size_t>(dcfg_.calib_big, stage_cap) / 1024 * 1024, 1u << 20);
  std::vector<size_t> pts;  // float32 element counts
  for (size_t b : {size_t(64) << 10, size_t(1) << 20, size_t(4) << 20, size_t(32) << 20}) {
    if (b < big_bytes) pts.push_back(b / 4);
  }
  pts.push_back(big_bytes / 4);
  const int np = static_cast<int>(pts.size());
  const size_t maxn = pts.back();
  // Inputs come from the free tail of the symmetric heap when the job has one: its buffers
  // live there, and the calibration then times the paths they take (the direct transport reads
  // heap inputs in place; RCCL reads the same uncached memory).  Otherwise from scratch HBM,
  // which the zero-copy registry exports after the first ops (so the median is steady state).
  const device::SymHeapInfo &heap = dev_->sym_heap();
  const bool heap_src = heap.base != nullptr && heap.bytes - dev_->sym_heap_used() >= maxn * 4;
  float *src = heap_src ? reinterpret_cast<float *>(heap.base + dev_->sym_heap_used())
                        : static_cast<float *>(dev_->Scratch(maxn * 4, 0));
  float *dst = static_cast<float *>(dev_->Scratch(maxn * 4, 1));
  // the robust engine stores every device result twice (result log + user buffer): the direct
  // kernels do it in the same pass, RCCL needs a copy after the collective.  Time what the
  // engine runs, both destinations and the copy included.
  float *dst2 = static_cast<float *>(dev_->Scratch(maxn * 4, device::DevicePlane::kCalibScratch));
  const int n = GetWorldSize();
  // the direct forms the configuration allows (auto modes try every alternative)
  std::vector<DirectForm> forms;
  for (int push = 0; push < 2; ++push) {
    if ((dcfg_.direct_mode == 1 && push) || (dcfg_.direct_mode == 2 && !push)) continue;
    for (int pipe = 0; pipe < 2; ++pipe) {
      if (pipe && !push) continue;
      if ((dcfg_.pipeline_mode == 0 && pipe) || (dcfg_.pipeline_mode == 1 && push && !pipe)) {
        continue;
      }
      for (int fused = 0; fused < 2; ++fused) {
        if (fused && pipe) continue;  // the pipelined form has no fused variant
        if ((dcfg_.fused_mode == 0 && fused) || (dcfg_.fused_mode == 1 && !fused)) continue;
        forms.push_back(DirectForm{push != 0, pipe != 0, fused != 0, FormName(push, pipe, fused)});
      }
    }
  }
  const int nf = static_cast<int>(forms.size());
  const int nc = 1 + nf;  // candidate 0: RCCL
  std::vector<double> t(static_cast<size_t>(nc) * np, -1.0);
  auto T = [&](int c, int i) -> double & { return t[static_cast<size_t>(c) * np + i]; };
  dev_->SetRoutes({}, {});  // measure with the forms set below, not a previous epoch's bands
  dev_->SetPeerDeadline(5.0);
  std::vector<float> host;
  constexpr int kReps = 6;  // a warm-up + 5 timed
  // Timed allreduce of pts[i] on the forced transport, median of the timed reps; false on
  // failure.  Every repetition reduces different values (rank + 1 + 16 rep), so the check of the
  // last one also catches a peer mapping that serves stale bytes of an earlier op.
  const float want = 0.5f * n * (n + 1) + 16.0f * (kReps - 1) * n;
  auto measure = [&](int which, size_t count, double *out, Status *st) {
    dev_->ForceTransport(which == 0 && !dev_->has_comm() ? 1 : which);
    std::vector<double> reps;
    for (int rep = 0; rep < kReps; ++rep) {
      device::CheckHip(device::LaunchFill(src, count, mpi::kFloat, rank_ + 1.0 + 16.0 * rep,
                                          dev_->stream()),
                       "LaunchFill");
      *st = dev_->Finish(MakeProbe());
      if (*st != Status::kSuccess) return false;
      const double t0 = utils::GetTime();
      *st = dev_->Allreduce(src, dst, dst2, count, mpi::kFloat, mpi::kSum, device::kPrepCopy, 1.0,
                            MakeProbe());
      if (*st == Status::kSuccess) *st = dev_->Finish(MakeProbe());
      if (*st != Status::kSuccess) return false;
      dev_->Synchronize();  // the second destination's copy (RCCL) is part of the op
      if (rep > 0) reps.push_back(utils::GetTime() - t0);
    }
    std::sort(reps.begin(), reps.end());
    *out = reps[reps.size() / 2];
    return true;
  };
  auto verified = [&](size_t count) {
    host.resize(count);
    dev_->StageToHost(host.data(), dst, count * 4);
    for (size_t i = 0; i < count; ++i) {
      if (host[i] != want) return false;
    }
    return true;
  };
  // 1. the direct forms.  A rank stops at its first failure; its peers' next barrier then
  //    times out (5 s deadline), so every rank leaves this phase in bounded time.  A failed
  //    barrier disables the direct transport; a wrong result only rules that form out.
  int ok = 1;
  std::vector<int> form_ok(nf, 1);
  for (int f = 0; f < nf && ok; ++f) {
    dev_->SetDirectPush(forms[f].push);
    dev_->SetPipeline(forms[f].pipe);
    dev_->SetFused(forms[f].fused);
    for (int i = 0; i < np && ok && form_ok[f]; ++i) {
      Status st;
      if (!measure(1, pts[i], &T(1 + f, i), &st)) {
        ok = 0;
        break;
      }
      if (debug_) {
        utils::HandleLogInfo("[%d] calibration %s %zu B: %.1f us\n", rank_, forms[f].name,
                             pts[i] * 4, T(1 + f, i) * 1e6);
      }
      // the latency point and the large point take different code paths: verify both
      if ((i == 0 || i == np - 1) && !verified(pts[i])) {
        form_ok[f] = 0;
        utils::HandleLogInfo("[%d] direct %s verification failed (%zu B)\n", rank_, forms[f].name,
                             pts[i] * 4);
      }
    }
  }
  dev_->SetPeerDeadline(dcfg_.peer_deadline_sec);
  std::vector<int> flags(1 + nf);
  flags[0] = ok;
  for (int f = 0; f < nf; ++f) flags[1 + f] = form_ok[f];
  Status s = host_->Allreduce(flags.data(), sizeof(int), flags.size(),
                              coll::HostReducer(mpi::kInt, mpi::kMin));
  if (s != Status::kSuccess) return s;
  ok = flags[0];
  for (int f = 0; f < nf; ++f) form_ok[f] = ok && flags[1 + f];
  // 2. RCCL (only worth timing when the direct transport is usable: the choice is uniform)
  if (ok) {
    dev_->SetDirectPush(forms[0].push);  // (the test hook's "RCCL" leg runs this direct form)
    dev_->SetPipeline(forms[0].pipe);
    dev_->SetFused(forms[0].fused);
    for (int i = 0; i < np; ++i) {
      Status st;
      if (!measure(0, pts[i], &T(0, i), &st)) {
        dev_->ForceTransport(-1);
        return st;  // RCCL failed: a real failure, the caller recovers
      }
    }
  }
  dev_->ForceTransport(-1);
  // identical decision everywhere: max time over ranks
  s = host_->Allreduce(t.data(), sizeof(double), t.size(),
                       coll::HostReducer(mpi::kDouble, mpi::kMax));
  if (s != Status::kSuccess) return s;
  for (int f = 0; f < nf; ++f) {
    if (!form_ok[f]) {
      for (int i = 0; i < np; ++i) T(1 + f, i) = -1.0;
    }
  }
  // A fused form hands tiles between the ranks' workgroups, so it needs every rank's grid
  // resident at once.  Ranks on separate GPUs have that; ranks sharing one GPU (rehearsals,
  // tests) do not -- the hardware time-slices separate processes' queues and other kernels hold
  // slots -- and a fused op there can wait out the peer deadline.  Its times are reported, but
  // nothing is routed to it.
  const bool shared_gpu = dev_->peers_share_gpu();
  std::vector<int> routable(nf, 1);
  for (int f = 0; f < nf; ++f) routable[f] = form_ok[f] && !(shared_gpu && forms[f].fused);
  std::ostringstream js;
  js << "{\"bytes\":[";
  for (int i = 0; i < np; ++i) js << (i ? "," : "") << pts[i] * 4;
  js << "],\"us\":{\"rccl\":[";
  for (int i = 0; i < np; ++i) js << (i ? "," : "") << (T(0, i) >= 0 ? T(0, i) * 1e6 : -1.0);
  js << "]";
  for (int f = 0; f < nf; ++f) {
    js << ",\"" << forms[f].name << "\":[";
    for (int i = 0; i < np; ++i) {
      js << (i ? "," : "") << (T(1 + f, i) >= 0 ? T(1 + f, i) * 1e6 : -1.0);
    }
    js << "]";
  }
  js << "},\"unrouted_forms\":[";
  for (int f = 0, k = 0; f < nf; ++f) {
    if (form_ok[f] && !routable[f]) js << (k++ ? "," : "") << "\"" << forms[f].name << "\"";
  }
  js << "]";
  size_t threshold = static_cast<size_t>(-1);
  int best_big = -1;  // direct form fastest at the large point
  if (!ok) {
    dev_->DropPeers();
    js << ",\"transport_bands\":[],\"form_bands\":[]}";
  } else {
    std::vector<double> xs(np);
    for (int i = 0; i < np; ++i) xs[i] = static_cast<double>(pts[i] * 4);
    std::vector<std::vector<double>> all(nc, std::vector<double>(np));
    std::vector<std::vector<double>> direct(nf, std::vector<double>(np));
    for (int c = 0; c < nc; ++c) {
      for (int i = 0; i < np; ++i) all[c][i] = c == 0 || routable[c - 1] ? T(c, i) : -1.0;
    }
    for (int f = 0; f < nf; ++f) direct[f] = all[1 + f];
    const std::vector<RouteBand> tb = ChooseRoutes(xs, all);
    const std::vector<RouteBand> fb = ChooseRoutes(xs, direct);
    std::vector<device::DevicePlane::RouteChoice> tbands, fbands;
    for (const RouteBand &b : tb) {
      tbands.push_back(device::DevicePlane::RouteChoice{
          static_cast<size_t>(b.lo), b.choice > 0 ? int8_t(1) : int8_t(0), 0, 0, 0});
    }
    for (const RouteBand &b : fb) {
      const DirectForm &f = forms[b.choice];
      fbands.push_back(
          device::DevicePlane::RouteChoice{static_cast<size_t>(b.lo), 1, f.push, f.pipe, f.fused});
    }
    for (int f = 0; f < nf; ++f) {
      if (routable[f] && (best_big < 0 || T(1 + f, np - 1) < T(1 + best_big, np - 1))) best_big = f;
    }
    if (best_big < 0) best_big = 0;
    dev_->SetRoutes(tbands, fbands);  // (clears the forced form)
    dev_->SetDefaultForm(forms[best_big].push, forms[best_big].pipe, forms[best_big].fused);
    dev_->RestoreCalibrated();
    js << ",\"transport_bands\":[";
    for (size_t k = 0; k < tb.size(); ++k) {
      js << (k ? "," : "") << "{\"from\":" << static_cast<size_t>(tb[k].lo) << ",\"use\":\""
         << (tb[k].choice == 0 ? "rccl" : "direct") << "\"}";
    }
    js << "],\"form_bands\":[";
    for (size_t k = 0; k < fb.size(); ++k) {
      js << (k ? "," : "") << "{\"from\":" << static_cast<size_t>(fb[k].lo) << ",\"form\":\""
         << forms[fb[k].choice].name << "\"}";
    }
    js << "]}";
    // the two-threshold summary of the bands (stats; used when no bands exist)
    const double d0 = all[1 + best_big][0], d1 = all[1 + best_big][np - 1];
    if (all[0][0] >= 0 && all[0][np - 1] >= 0) {
      const DirectRouting route = ChooseDirectRouting(xs[0], xs[np - 1], all[0][0],
                                                      all[0][np - 1], d0, d1);
      threshold = route.min_bytes;
      dev_->set_direct_min_bytes(threshold);
      dev_->set_direct_below_bytes(route.below_bytes);
    }
  }
  calib_matrix_json_ = js.str();
  // legacy summary fields: RCCL and the best direct form at the latency and large points
  auto best_direct = [&](int i) {
    double b = -1;
    for (int f = 0; f < nf; ++f) {
      if (T(1 + f, i) >= 0 && (b < 0 || T(1 + f, i) < b)) b = T(1 + f, i);
    }
    return b < 0 ? 0.0 : b;
  };
  double push_big = 0;
  for (int k = 0; k < kCalibForms; ++k) calib_form_us_[k] = -1.0;
  for (int f = 0; f < nf; ++f) {
    // legacy slots: pull-classic, pull-fused, push-classic, push-fused, pipelined
    const int slot = forms[f].pipe ? 4 : (forms[f].push ? 2 : 0) + (forms[f].fused ? 1 : 0);
    calib_form_us_[slot] = T(1 + f, np - 1) >= 0 ? T(1 + f, np - 1) * 1e6 : -1.0;
    if (forms[f].push && !forms[f].pipe && !forms[f].fused && T(1 + f, np - 1) >= 0) {
      push_big = T(1 + f, np - 1);
    }
  }
  calib_ = {std::max(T(0, 0), 0.0), std::max(T(0, np - 1), 0.0), best_direct(0),
            best_direct(np - 1), static_cast<double>(pts[0] * 4),
            static_cast<double>(pts[np - 1] * 4), push_big};
  calib_heap_src_ = heap_src;
  if (debug_ || rank_ == 0) {
    utils::HandleLogInfo("[xrabit] device calibration (%d ranks, %d sizes, %d direct forms): %s\n",
                         n, np, nf, !ok ? "direct transport disabled (failed barrier)"
                                        : calib_matrix_json_.c_str());
  }
  return Status::kSuccess;
}

Status EngineBase::CalibrateBroadcast() {
  // byte sizes: a latency point and the allreduce calibration's large point (one stage)
  const size_t big = std::min<size_t>(dcfg_.calib_big, dcfg_.peer_stage);
  const size_t sizes[2] = {64u << 10, std::max<size_t>(big, 1u << 20) / 256 * 256};
  char *buf = static_cast<char *>(dev_->Scratch(sizes[1], 1));
  char *log = static_cast<char *>(dev_->Scratch(sizes[1], device::DevicePlane::kCalibScratch));
  constexpr int kReps = 4;
  const float want = 3.0f + (kReps - 1);  // root 0's value in the last repetition
  double t[2][2] = {{0, 0}, {0, 0}};     // [transport: 0 rccl, 1 direct][size]
  int ok = 1;
  dev_->SetPeerDeadline(5.0);
  // timed broadcast from root 0 into buf and the log slot (as the robust engine runs it: the
  // direct kernels store both, RCCL copies into the log after the collective); every other
  // rank's buffer holds -1 before each repetition, so stale bytes cannot pass the check
  auto measure = [&](int which, int k, Status *st) {
    const size_t count = sizes[k] / 4;
    dev_->ForceTransport(which == 0 && !dev_->has_comm() ? 1 : which);
    double best = 1e30;
    for (int rep = 0; rep < kReps; ++rep) {
      device::CheckHip(device::LaunchFill(buf, count, mpi::kFloat, rank_ == 0 ? 3.0 + rep : -1.0,
                                          dev_->stream()),
                       "LaunchFill");
      *st = dev_->Finish(MakeProbe());
      if (*st != Status::kSuccess) return false;
      const double t0 = utils::GetTime();
      *st = dev_->Broadcast(buf, sizes[k], 0, MakeProbe(), log);
      if (*st == Status::kSuccess) *st = dev_->Finish(MakeProbe());
      if (*st != Status::kSuccess) return false;
      dev_->Synchronize();
      if (rep > 0) best = std::min(best, utils::GetTime() - t0);
    }
    t[which][k] = best;
    return true;
  };
  std::vector<float> host;
  auto verified = [&](size_t bytes) {
    for (char *p : {buf, log}) {
      host.resize(bytes / 4);
      dev_->StageToHost(host.data(), p, bytes);
      for (float v : host) {
        if (v != want) return false;
      }
    }
    return true;
  };
  // 1. direct (a failed barrier leaves this phase within the 5 s deadline on every rank)
  int correct = 1;
  for (int k = 0; k < 2 && ok; ++k) {
    Status st;
    if (!measure(1, k, &st)) {
      ok = 0;
      break;
    }
    if (correct && !verified(sizes[k])) {
      correct = 0;
      utils::HandleLogInfo("[%d] direct broadcast verification failed (%zu B)\n", rank_, sizes[k]);
    }
  }
  dev_->ForceTransport(-1);
  dev_->SetPeerDeadline(dcfg_.peer_deadline_sec);
  int flags[2] = {ok, correct};
  Status s = host_->Allreduce(flags, sizeof(int), 2, coll::HostReducer(mpi::kInt, mpi::kMin));
  if (s != Status::kSuccess) return s;
  if (!flags[0]) {
    // the group failed a barrier: no direct transport for anything (as CalibrateDevice does)
    dev_->DropPeers();
    return Status::kSuccess;
  }
  // 2. RCCL
  for (int k = 0; k < 2; ++k) {
    Status st;
    if (!measure(0, k, &st)) {
      dev_->ForceTransport(-1);
      return st;  // RCCL failed: a real failure, the caller recovers
    }
  }
  dev_->ForceTransport(-1);
  double agg[4] = {t[0][0], t[0][1], t[1][0], t[1][1]};
  s = host_->Allreduce(agg, sizeof(double), 4, coll::HostReducer(mpi::kDouble, mpi::kMax));
  if (s != Status::kSuccess) return s;
  for (int i = 0; i < 4; ++i) calib_bcast_[i] = agg[i];
  if (!flags[1]) {
    dev_->set_bcast_routing(static_cast<size_t>(-1), 0);  // a wrong direct result: RCCL only
  } else {
    const DirectRouting route = ChooseDirectRouting(static_cast<double>(sizes[0]),
                                                    static_cast<double>(sizes[1]), agg[0], agg[1],
                                                    agg[2], agg[3]);
    dev_->set_bcast_routing(route.min_bytes, route.below_bytes);
  }
  if (debug_ || rank_ == 0) {
    utils::HandleLogInfo(
        "[xrabit] broadcast calibration (%d ranks): %zu B rccl %.1f us direct %.1f us; %zu B "
        "rccl %.1f us direct %.1f us -> direct %s%zu B%s\n",
        GetWorldSize(), sizes[0], agg[0] * 1e6, agg[2] * 1e6, sizes[1], agg[1] * 1e6, agg[3] * 1e6,
        !flags[1] ? "off (failed verification) "
                  : (dev_->bcast_below_bytes() > 0 ? "below " : "from "),
        dev_->bcast_below_bytes() > 0 ? dev_->bcast_below_bytes() : dev_->bcast_min_bytes(),
        dev_->bcast_min_bytes() == static_cast<size_t>(-1) && dev_->bcast_below_bytes() == 0
            ? " (never)" : "");
  }
  return Status::kSuccess;
}

}  // namespace engine
}  // namespace rabit
