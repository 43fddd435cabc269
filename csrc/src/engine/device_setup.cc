/*!
 * \file device_setup.cc
 * \brief EngineBase: bringing up the device transports of an epoch — the GPU records and peer
 *        preflight, the direct (IPC) transport, the RCCL communicator (agreed on by every rank,
 *        optionally channel-tuned) and the start-up calibration that routes ops between them.
 *        The host engine itself is engine_base.cc.
 */
#include <cstring>
#include <sstream>
#include <string>
#include <vector>

#include "device/kernels.h"
#include "engine/engine_base.h"
#include "engine/routing.h"
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
  if ((dev_->has_comm() || calibrate_test_) && dev_->has_peers() && dcfg_.algo == 0 &&
      calibrate_) {
    s = CalibrateDevice();
    if (s != Status::kSuccess) return s;
    if (dev_->has_peers()) {
      s = CalibrateBroadcast();
      if (s != Status::kSuccess) return s;
    }
  }
  if (debug_) {
    utils::HandleLogInfo("[%d] device transport epoch %d: rccl=%d direct=%d (direct for >= %zu B)\n",
                         rank_, dev_->epoch(), dev_->has_comm() ? 1 : 0,
                         dev_->has_peers() ? 1 : 0, dcfg_.direct_min_bytes);
  }
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

Status EngineBase::CalibrateDevice() {
  // sizes in float32 elements; every rank runs the same sequence (this is a collective)
  // the large point sits where gradient buckets and the headline op live: 128 MiB (one stage
  // chunk at most); on 8 ranks sharing a GPU the fastest form at 32 MiB was not the fastest
  // at 128 MiB (profiles/r2_s5_rehearsal_n8)
  const size_t big =
      std::min<size_t>(dcfg_.calib_big, dev_->has_peers() ? dcfg_.peer_stage : 0) / 4;
  const size_t sizes[2] = {64u << 10, std::max<size_t>(big, 1u << 20)};
  // Inputs come from the free tail of the symmetric heap when the job has one: its buffers
  // live there, and the calibration then times the paths they take (the direct transport reads
  // heap inputs in place; RCCL reads the same uncached memory).  Otherwise from scratch HBM.
  const device::SymHeapInfo &heap = dev_->sym_heap();
  const bool heap_src =
      heap.base != nullptr && heap.bytes - dev_->sym_heap_used() >= sizes[1] * 4;
  float *src = heap_src ? reinterpret_cast<float *>(heap.base + dev_->sym_heap_used())
                        : static_cast<float *>(dev_->Scratch(sizes[1] * 4, 0));
  float *dst = static_cast<float *>(dev_->Scratch(sizes[1] * 4, 1));
  // the robust engine stores every device result twice (result log + user buffer): the direct
  // kernels do it in the same pass, RCCL needs a copy after the collective.  Time what the
  // engine runs, both destinations and the copy included.
  float *dst2 = static_cast<float *>(dev_->Scratch(sizes[1] * 4, device::DevicePlane::kCalibScratch));
  const int n = GetWorldSize();
  double t[2][2] = {{0, 0}, {0, 0}};  // [transport: 0 rccl, 1 direct][size]
  int ok = 1;
  dev_->SetPeerDeadline(5.0);
  std::vector<float> host;
  constexpr int kCalibReps = 4;
  // the value every rank must hold after the last repetition
  const float want = 0.5f * n * (n + 1) + 16.0f * (kCalibReps - 1) * n;
  // Timed allreduce of sizes[k] on the forced transport; false on failure.  Every repetition
  // reduces different values (rank + 1 + 16 rep), so the check of the last one also catches a
  // peer mapping that serves stale bytes of the previous op on the same stage buffer (the
  // buffers alternate, so rep 3 reuses rep 1's), not only a broken one.
  auto measure = [&](int which, int k, Status *st) {
    const size_t count = sizes[k];
    // test hook: without RCCL (ranks sharing a GPU) the "RCCL" leg runs direct as well
    dev_->ForceTransport(which == 0 && !dev_->has_comm() ? 1 : which);
    double best = 1e30;
    for (int rep = 0; rep < kCalibReps; ++rep) {
      device::CheckHip(device::LaunchFill(src, count, mpi::kFloat, rank_ + 1.0 + 16.0 * rep,
                                          dev_->stream()),
                       "LaunchFill");
      *st = dev_->Finish(MakeProbe());
      if (*st != Status::kSuccess) return false;
      const double t0 = utils::GetTime();
      *st = dev_->Allreduce(src, dst, dst2, count, mpi::kFloat, mpi::kSum, device::kPrepCopy,
                            1.0, MakeProbe());
      if (*st == Status::kSuccess) *st = dev_->Finish(MakeProbe());
      if (*st != Status::kSuccess) return false;
      dev_->Synchronize();  // the second destination's copy (RCCL) is part of the op
      if (rep > 0) best = std::min(best, utils::GetTime() - t0);
    }
    t[which][k] = best;
    return true;
  };
  // 1. direct transport.  A rank stops at its first failure; its peers' next barrier then
  //    times out (5 s deadline), so every rank leaves this phase in bounded time.
  for (int k = 0; k < 2 && ok; ++k) {
    Status st;
    if (!measure(1, k, &st)) {
      ok = 0;
      break;
    }
    // verify the direct result on the host: a broken peer mapping must not go unnoticed
    host.resize(sizes[k]);
    dev_->StageToHost(host.data(), dst, sizes[k] * 4);
    for (size_t i = 0; i < sizes[k] && ok; ++i) ok = host[i] == want ? 1 : 0;
    if (!ok) utils::HandleLogInfo("[%d] direct transport verification failed\n", rank_);
  }
  // 1b. the other forms of the direct two-shot path at the large size, each verified like the
  //     first: push (remote writes) instead of pull, and the fused single-kernel form instead
  //     of the 5-launch one (or the reverse).  A failed run disables the direct transport
  //     altogether (a failed barrier drops the group); a wrong result only rules that form out.
  //     Variant 0 is the form step 1 measured.
  //     Form 4 is the pipelined push form (ar_plan.h: the push of one chunk and the gather of
  //     an older one share a round, over opposite link directions), timed when
  //     rabit_device_pipeline=auto; with rabit_device_pipeline=1 every push form is pipelined.
  const bool fused_auto = dcfg_.fused_mode == 2;
  const bool cfg_fused = dcfg_.fused_mode == 1;  // auto starts from the classic form
  const bool pipe_on = dcfg_.pipeline_mode == 1;
  struct Form {
    bool push, fused, pipe;
  };
  Form forms[kCalibForms] = {{dcfg_.direct_mode == 2, cfg_fused, dcfg_.direct_mode == 2 && pipe_on},
                             {dcfg_.direct_mode == 2, !cfg_fused, dcfg_.direct_mode == 2 && pipe_on},
                             {true, cfg_fused, pipe_on},
                             {true, !cfg_fused, pipe_on},
                             {true, false, true}};
  int form_ok[kCalibForms] = {ok, 0, 0, 0, 0};
  double t_form[kCalibForms] = {t[1][1], 0, 0, 0, 0};
  const bool try_push = dcfg_.direct_mode == 0;
  for (int f = 1; f < kCalibForms && ok; ++f) {
    if ((f == 1 || f == 3) && !fused_auto) continue;
    if (f >= 2 && !try_push) continue;
    if (f == 4 && dcfg_.pipeline_mode != 2) continue;
    dev_->SetDirectPush(forms[f].push);
    dev_->SetFused(forms[f].fused);
    dev_->SetPipeline(forms[f].pipe);
    Status st;
    if (!measure(1, 1, &st)) {
      ok = 0;
      break;
    }
    t_form[f] = t[1][1];
    host.resize(sizes[1]);
    dev_->StageToHost(host.data(), dst, sizes[1] * 4);
    form_ok[f] = 1;
    for (size_t i = 0; i < sizes[1] && form_ok[f]; ++i) form_ok[f] = host[i] == want ? 1 : 0;
    if (!form_ok[f]) {
      utils::HandleLogInfo("[%d] direct %s %s verification failed\n", rank_,
                           forms[f].push ? "push" : "pull",
                           forms[f].pipe ? "pipelined" : (forms[f].fused ? "fused" : "classic"));
    }
  }
  t[1][1] = t_form[0];
  if (dev_->has_peers()) {
    dev_->SetDirectPush(forms[0].push);
    dev_->SetFused(forms[0].fused);
    dev_->SetPipeline(forms[0].pipe);
  }
  dev_->ForceTransport(-1);
  dev_->SetPeerDeadline(dcfg_.peer_deadline_sec);
  int flags[1 + kCalibForms] = {ok};
  for (int f = 0; f < kCalibForms; ++f) flags[1 + f] = form_ok[f];
  Status s = host_->Allreduce(flags, sizeof(int), 1 + kCalibForms,
                              coll::HostReducer(mpi::kInt, mpi::kMin));
  if (s != Status::kSuccess) return s;
  ok = flags[0];
  for (int f = 0; f < kCalibForms; ++f) form_ok[f] = ok && flags[1 + f];
  // 2. RCCL (only worth timing when the direct transport is usable: the choice is uniform)
  if (ok) {
    for (int k = 0; k < 2; ++k) {
      Status st;
      if (!measure(0, k, &st)) {
        dev_->ForceTransport(-1);
        return st;  // RCCL failed: a real failure, the caller recovers
      }
    }
    dev_->ForceTransport(-1);
  }
  // identical decision everywhere: max time over ranks
  double agg[4 + kCalibForms] = {t[0][0], t[0][1], t[1][0], t[1][1]};
  for (int f = 0; f < kCalibForms; ++f) agg[4 + f] = t_form[f];
  s = host_->Allreduce(agg, sizeof(double), 4 + kCalibForms,
                       coll::HostReducer(mpi::kDouble, mpi::kMax));
  if (s != Status::kSuccess) return s;
  size_t threshold = static_cast<size_t>(-1);
  int best = 0;
  if (!ok) {
    dev_->DropPeers();
  } else {
    // the form of the two-shot path: the fastest verified one at the large size (same
    // everywhere: times and verdicts were agreed on above)
    for (int f = 1; f < kCalibForms; ++f) {
      if (form_ok[f] && agg[4 + f] < agg[4 + best]) best = f;
    }
    dev_->SetDirectPush(forms[best].push);
    dev_->SetFused(forms[best].fused);
    dev_->SetPipeline(forms[best].pipe);
    agg[3] = agg[4 + best];
    // linear model t = a + b * bytes per transport through the two points (routing.h)
    const DirectRouting route =
        ChooseDirectRouting(sizes[0] * 4.0, sizes[1] * 4.0, agg[0], agg[1], agg[2], agg[3]);
    threshold = route.min_bytes;
    dev_->set_direct_min_bytes(threshold);
    dev_->set_direct_below_bytes(route.below_bytes);
  }
  calib_ = {agg[0], agg[1], agg[2], agg[3], static_cast<double>(sizes[0] * 4),
            static_cast<double>(sizes[1] * 4), agg[4 + 2] > 0 ? agg[4 + 2] : 0.0};
  for (int f = 0; f < kCalibForms; ++f) calib_form_us_[f] = form_ok[f] ? agg[4 + f] * 1e6 : -1.0;
  calib_heap_src_ = heap_src;
  if (debug_ || rank_ == 0) {
    utils::HandleLogInfo(
        "[xrabit] device calibration (%d ranks): %zu B rccl %.1f us direct %.1f us; %zu B rccl "
        "%.1f us direct %.1f us (%s %s; forms %.1f %.1f %.1f %.1f %.1f us) -> direct %s\n",
        n, sizes[0] * 4, agg[0] * 1e6, agg[2] * 1e6, sizes[1] * 4, agg[1] * 1e6, agg[3] * 1e6,
        dev_->direct_push() ? "push" : "pull",
        forms[best].pipe ? "pipelined" : (forms[best].fused ? "fused" : "classic"),
        calib_form_us_[0], calib_form_us_[1], calib_form_us_[2], calib_form_us_[3],
        calib_form_us_[4],
        !ok ? "disabled (failed verification)"
            : (threshold != static_cast<size_t>(-1)
                   ? ("from " + std::to_string(threshold) + " B").c_str()
                   : (dev_->direct_below_bytes() > 0
                          ? ("below " + std::to_string(dev_->direct_below_bytes()) + " B").c_str()
                          : "off (RCCL faster)")));
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
        !flags[1] ? "off (failed verification) " : (dev_->bcast_below_bytes() > 0 ? "below " : "from "),
        dev_->bcast_below_bytes() > 0 ? dev_->bcast_below_bytes() : dev_->bcast_min_bytes(),
        dev_->bcast_min_bytes() == static_cast<size_t>(-1) && dev_->bcast_below_bytes() == 0
            ? " (never)" : "");
  }
  return Status::kSuccess;
}

}  // namespace engine
}  // namespace rabit
