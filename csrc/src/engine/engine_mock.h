/*!
 * \file engine_mock.h
 * \brief Fault-injection engine (parity: reference `src/allreduce_mock.h:20-206`).
 *
 * `mock=rank,version,seqno,ntrial` (repeatable) kills the process when this rank reaches
 * collective `seqno` of checkpoint `version` on restart attempt `ntrial`
 * (attempt = rabit_num_trial / DMLC_NUM_ATTEMPT, set by the launcher).  The hit raises
 * rabit::Error (as the reference); the C API turns an uncaught error into process exit,
 * which is what the launcher's restart logic observes.
 * Extensions: `mock_hang=rank,version,seqno,ntrial` makes the rank stop responding (sleeps
 * forever) instead of dying, to exercise the timeout watchdog; `mock_dev_hang=...` keeps the
 * process alive but wedges its GPU stream right before the device collective (a hung kernel:
 * the peers' barriers / RCCL time out, the rank finds its own stream stuck after the abort and
 * exits for a restart); `mock_die_mid=...` lets the rank start the device allreduce and exit
 * in its middle, once every peer has delivered the op's first chunk to its output (survivors
 * then fail the op part-way, which must leave their input intact for the retry);
 * `mock_die_serving=rank,version,seqno,ntrial[,where]` kills the rank while it serves another
 * rank's recovery (holder or relay of a replayed result, of a checkpoint load or of the
 * bootstrap cache) during op `seqno` of `version`: where = 1 after the routing decision, 2 once
 * the first bytes of a host transfer left, 3 right before a device exchange, 0 (default) at the
 * first of them reached.  The reference reaches this path only when a second failure happens
 * to coincide with a replay (`src/allreduce_robust.cc:861-973, 1037-1088, 1103-1140`);
 * `force_local` and `report_stats` behave as in the reference.
 */
#ifndef XRABIT_ENGINE_ENGINE_MOCK_H_
#define XRABIT_ENGINE_ENGINE_MOCK_H_

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <map>
#include <sstream>
#include <string>
#include <thread>
#include <tuple>

#include "core/exit.h"
#include "core/wait_state.h"
#include "engine/engine_robust.h"
#include "rabit/internal/timer.h"

namespace rabit {
namespace engine {

class EngineMock : public EngineRobust {
 public:
  void SetParam(const char *name, const char *val) override {
    EngineRobust::SetParam(name, val);
    if (!strcmp(name, "rabit_num_trial") || !strcmp(name, "DMLC_NUM_ATTEMPT")) {
      num_trial_ = atoi(val);
    }
    if (!strcmp(name, "report_stats")) report_stats_ = atoi(val);
    if (!strcmp(name, "force_local")) force_local_ = atoi(val);
    if (!strcmp(name, "mock_die_serving")) {
      Key k;
      int where = 0;
      const int got = sscanf(val, "%d,%d,%d,%d,%d", &std::get<0>(k), &std::get<1>(k),
                             &std::get<2>(k), &std::get<3>(k), &where);
      utils::Check(got == 4 || (got == 5 && where >= 0 && where <= 3),
                   "invalid mock_die_serving \"%s\" (expected rank,version,seqno,ntrial[,where])",
                   val);
      serve_map_[k] = where;
    }
    if (!strcmp(name, "mock") || !strcmp(name, "mock_hang") || !strcmp(name, "mock_dev_hang") ||
        !strcmp(name, "mock_die_mid")) {
      Key k;
      utils::Check(sscanf(val, "%d,%d,%d,%d", &std::get<0>(k), &std::get<1>(k), &std::get<2>(k),
                          &std::get<3>(k)) == 4,
                   "invalid mock parameter \"%s\" (expected rank,version,seqno,ntrial)", val);
      mock_map_[k] = !strcmp(name, "mock_hang")       ? 2
                     : !strcmp(name, "mock_dev_hang") ? 3
                     : !strcmp(name, "mock_die_mid")  ? 4
                                                      : 1;
    }
  }
  const char *EngineName() const override { return "mock"; }

  void Allreduce(void *buf, size_t type_nbytes, size_t count, ReduceFunction reducer,
                 PreprocFunction prepare_fun, void *prepare_arg, const char *_file,
                 const int _line, const char *_caller) override {
    Verify("AllReduce");
    const double t0 = utils::GetTime();
    EngineRobust::Allreduce(buf, type_nbytes, count, reducer, prepare_fun, prepare_arg, _file,
                            _line, _caller);
    tsum_allreduce_ += utils::GetTime() - t0;
  }
  void AllreduceTyped(void *buf, size_t count, mpi::DataType dtype, mpi::OpType op,
                      ReduceFunction reducer, PreprocFunction prepare_fun, void *prepare_arg,
                      const char *_file, const int _line, const char *_caller) override {
    Verify("AllReduce");
    const double t0 = utils::GetTime();
    EngineRobust::AllreduceTyped(buf, count, dtype, op, reducer, prepare_fun, prepare_arg, _file,
                                 _line, _caller);
    tsum_allreduce_ += utils::GetTime() - t0;
  }
  void AllreduceDevice(void *buf, size_t type_nbytes, size_t count,
                       DeviceReduceLauncher *dev_reducer, ReduceFunction host_reducer,
                       PreprocFunction prepare_fun, void *prepare_arg, const char *_file,
                       const int _line, const char *_caller) override {
    Verify("AllReduce");
    const double t0 = utils::GetTime();
    EngineRobust::AllreduceDevice(buf, type_nbytes, count, dev_reducer, host_reducer,
                                  prepare_fun, prepare_arg, _file, _line, _caller);
    tsum_allreduce_ += utils::GetTime() - t0;
  }
  void DevAllreducePrepared(void *dst, const void *src, size_t count, int dtype, int op,
                            int prep, double alpha, const char *_file, const int _line,
                            const char *_caller) override {
    Verify("AllReduce");
    EngineRobust::DevAllreducePrepared(dst, src, count, dtype, op, prep, alpha, _file, _line,
                                       _caller);
  }
  void Allgather(void *buf, size_t total, size_t begin, size_t end, size_t prev_size,
                 const char *_file, const int _line, const char *_caller) override {
    Verify("Allgather");
    const double t0 = utils::GetTime();
    EngineRobust::Allgather(buf, total, begin, end, prev_size, _file, _line, _caller);
    tsum_allgather_ += utils::GetTime() - t0;
  }
  void Broadcast(void *buf, size_t size, int root, const char *_file, const int _line,
                 const char *_caller) override {
    Verify("Broadcast");
    EngineRobust::Broadcast(buf, size, root, _file, _line, _caller);
  }
  int LoadCheckPoint(Serializable *global_model, Serializable *local_model) override {
    tsum_allreduce_ = tsum_allgather_ = 0.0;
    time_checkpoint_ = utils::GetTime();
    // device checkpoints fold force_local in DevLoadCheckPoint (the local tensors stay in HBM)
    if (force_local_ == 0 || local_model == &dev_local_) {
      return EngineRobust::LoadCheckPoint(global_model, local_model);
    }
    Dummy dum;
    Combo com(global_model, local_model);
    return EngineRobust::LoadCheckPoint(&dum, &com);
  }
  void CheckPoint(const Serializable *global_model, const Serializable *local_model) override {
    Verify("CheckPoint");
    const double t0 = utils::GetTime();
    const double between = t0 - time_checkpoint_;
    if (force_local_ == 0) {
      EngineRobust::CheckPoint(global_model, local_model);
    } else {
      Dummy dum;
      Combo com(global_model, local_model);
      EngineRobust::CheckPoint(&dum, &com);
    }
    time_checkpoint_ = utils::GetTime();
    const double cost = time_checkpoint_ - t0;
    if (report_stats_ != 0 && rank_ == 0) {
      std::ostringstream ss;
      ss << "[v" << version_number_ << "] global_size=" << global_checkpoint_.length()
         << ",local_size=" << (local_.configured() ? local_.Bytes(0) + local_.Bytes(1) : 0)
         << ",check_tcost=" << cost << " sec,allreduce_tcost=" << tsum_allreduce_
         << " sec,allgather_tcost=" << tsum_allgather_ << " sec,between_chpt=" << between
         << "sec\n";
      this->TrackerPrint(ss.str());
    }
    tsum_allreduce_ = tsum_allgather_ = 0.0;
  }
  void CheckPointDevice(const Serializable *global_model,
                        const Serializable *local_model) override {
    Verify("CheckPoint");
    EngineRobust::CheckPointDevice(global_model, local_model);
  }
  bool ForceLocal() const override { return force_local_ != 0; }
  void LazyCheckPoint(const Serializable *global_model) override {
    Verify("LazyCheckPoint");
    EngineRobust::LazyCheckPoint(global_model);
  }

  void ServeHook(ServePoint where) override {
    auto it = serve_map_.find(Key(rank_, version_number_, seq_counter_, num_trial_));
    if (it == serve_map_.end() || (it->second != 0 && it->second != static_cast<int>(where))) {
      return;
    }
    static const char *names[] = {"", "routing", "data", "device exchange"};
    fprintf(stderr, "[%d]@@@Hit Mock Die Serving (%s) at version %d seq %d\n", rank_,
            names[static_cast<int>(where)], version_number_, seq_counter_);
    fflush(stderr);
    // as a crash: no unwinding through the recovery code, no Finalize
    utils::ExitProcess(kMockDieServingExitCode);
  }
  static constexpr int kMockDieServingExitCode = 249;

  // white-box setters for unit tests
  void TestSetState(int rank, int version, int seq) {
    rank_ = rank;
    version_number_ = version;
    seq_counter_ = seq;
  }

 private:
  typedef std::tuple<int, int, int, int> Key;
  struct Dummy : public Serializable {
    void Load(Stream *) override {}
    void Save(Stream *) const override {}
  };
  struct Combo : public Serializable {
    Serializable *lhs, *rhs;
    const Serializable *clhs, *crhs;
    Combo(Serializable *l, Serializable *r) : lhs(l), rhs(r), clhs(l), crhs(r) {}
    Combo(const Serializable *l, const Serializable *r)
        : lhs(nullptr), rhs(nullptr), clhs(l), crhs(r) {}
    void Load(Stream *fi) override {
      if (lhs != nullptr) lhs->Load(fi);
      if (rhs != nullptr) rhs->Load(fi);
    }
    void Save(Stream *fo) const override {
      if (clhs != nullptr) clhs->Save(fo);
      if (crhs != nullptr) crhs->Save(fo);
    }
  };
  void Verify(const char *what) {
    auto it = mock_map_.find(Key(rank_, version_number_, seq_counter_, num_trial_));
    if (it == mock_map_.end()) return;
    num_trial_ += 1;
    if (it->second == 4) {
      fprintf(stderr, "[%d]@@@Hit Mock Die Mid (armed):%s\n", rank_, what);
      fflush(stderr);
      die_mid_armed_ = true;
      return;
    }
    if (it->second == 3) {
      // the process stays alive and responsive on the host; its GPU stream wedges right before
      // this collective, so its peers wait at the device barrier / in RCCL for it
      fprintf(stderr, "[%d]@@@Hit Mock Device Hang:%s\n", rank_, what);
      fflush(stderr);
      dev_hang_armed_ = true;
      return;
    }
    if (it->second == 2) {
      core::OpScope in_op;  // the hang is inside the collective (rabit_hang_timeout_sec)
      fprintf(stderr, "[%d]@@@Hit Mock Hang:%s\n", rank_, what);
      fflush(stderr);
      for (;;) std::this_thread::sleep_for(std::chrono::seconds(1));
    }
    if (MockKillsExit()) {
      fprintf(stderr,
              "[xrabit] [%d]@@@Hit Mock Error:%s\nxrabit: fatal: [%d]@@@Hit Mock Error:%s\n",
              rank_, what, rank_, what);
      utils::ExitProcess(254);
    }
    utils::Error("[%d]@@@Hit Mock Error:%s", rank_, what);
  }
  int num_trial_{0};
  int force_local_{0};
  int report_stats_{0};
  double tsum_allreduce_{0}, tsum_allgather_{0}, time_checkpoint_{0};
  std::map<Key, int> mock_map_;
  std::map<Key, int> serve_map_;  // mock_die_serving: where (0 any)
};
}  // namespace engine
}  // namespace rabit
#endif  // XRABIT_ENGINE_ENGINE_MOCK_H_
