/*!
 * \file wait_state.h
 * \brief Where this process is while inside a collective: waiting on peers / the device / the
 *        tracker, or working.  The hang watchdog (rabit_hang_timeout_sec) uses it to tell a
 *        rank that is stuck in its own code inside an op (its peers then wait for it forever:
 *        the reference cannot recover from that) from the ranks that merely wait for it.
 *
 * A rank that has been *working* — inside an op and not in any wait — for longer than the hang
 * timeout exits with a restartable status; its peers see the connection reset and run the
 * normal recovery, replaying what the restarted rank missed.  Ranks that wait never fire.
 * Process-wide state: an engine is driven by one thread at a time.
 */
#ifndef XRABIT_CORE_WAIT_STATE_H_
#define XRABIT_CORE_WAIT_STATE_H_

#include <atomic>
#include <chrono>

namespace rabit {
namespace core {

inline double MonotonicSec() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

struct WaitState {
  std::atomic<int> op_depth{0};        // > 0: inside a public collective / checkpoint
  std::atomic<int> wait_depth{0};      // > 0: blocked on peers, the device or the tracker
  std::atomic<double> working_since{0};  // start of the current working stretch (0: none)
  std::atomic<double> device_wait_since{0};  // start of the current wait on the GPU (0: none)
  std::atomic<double> device_op_deadline{0};  // deadline (s) of the device op being waited
                                              // for, which aborts it on its own (0: none)
};

inline WaitState &GlobalWaitState() {
  static WaitState s;
  return s;
}

/*! \brief marks a public operation; the working stretch starts when it is entered */
class OpScope {
 public:
  OpScope() {
    WaitState &w = GlobalWaitState();
    if (w.op_depth.fetch_add(1) == 0 && w.wait_depth.load() == 0) {
      w.working_since.store(MonotonicSec());
    }
  }
  ~OpScope() {
    WaitState &w = GlobalWaitState();
    if (w.op_depth.fetch_sub(1) == 1) w.working_since.store(0.0);
  }
  OpScope(const OpScope &) = delete;
  OpScope &operator=(const OpScope &) = delete;
};

/*! \brief marks a blocking wait on something outside this rank */
class WaitScope {
 public:
  WaitScope() {
    WaitState &w = GlobalWaitState();
    w.wait_depth.fetch_add(1);
    w.working_since.store(0.0);
  }
  ~WaitScope() {
    WaitState &w = GlobalWaitState();
    if (w.wait_depth.fetch_sub(1) == 1 && w.op_depth.load() > 0) {
      w.working_since.store(MonotonicSec());
    }
  }
  WaitScope(const WaitScope &) = delete;
  WaitScope &operator=(const WaitScope &) = delete;
};

/*!
 * \brief marks a host wait on this rank's GPU work (stream drain, blocking copies, collective
 *        completion); the watchdog terminates a rank whose wait exceeds the device wait limit,
 *        which covers HIP calls that block without any deadline of their own
 */
class DeviceWaitScope {
 public:
  DeviceWaitScope() {
    double zero = 0.0;
    outer_ = GlobalWaitState().device_wait_since.compare_exchange_strong(zero, MonotonicSec());
  }
  ~DeviceWaitScope() {
    if (outer_) GlobalWaitState().device_wait_since.store(0.0);
  }
  DeviceWaitScope(const DeviceWaitScope &) = delete;
  DeviceWaitScope &operator=(const DeviceWaitScope &) = delete;

 private:
  bool outer_{false};
};

/*! \brief seconds this rank has been waiting on its GPU (0: not waiting) */
inline double DeviceWaitingFor() {
  const double since = GlobalWaitState().device_wait_since.load();
  return since > 0 ? MonotonicSec() - since : 0.0;
}

/*!
 * \brief the limit the watchdog applies to a wait on this rank's GPU: the configured device
 *        wait limit, but never below the deadline of the device op being waited for plus the
 *        drain time its abort may take (that wait includes peers' barriers and RCCL, so a healthy
 *        rank waiting on a slow peer must reach its own op deadline first).  0: no limit.
 */
inline double EffectiveDeviceWaitLimit(double wait_limit, double op_deadline, double drain_sec) {
  if (wait_limit <= 0) return 0.0;
  if (op_deadline <= 0) return wait_limit;
  const double own = op_deadline + drain_sec + 5.0;
  return own > wait_limit ? own : wait_limit;
}

/*! \brief marks the deadline of the device op a wait is for (see EffectiveDeviceWaitLimit) */
class DeviceDeadlineScope {
 public:
  explicit DeviceDeadlineScope(double sec) { GlobalWaitState().device_op_deadline.store(sec); }
  ~DeviceDeadlineScope() { GlobalWaitState().device_op_deadline.store(0.0); }
  DeviceDeadlineScope(const DeviceDeadlineScope &) = delete;
  DeviceDeadlineScope &operator=(const DeviceDeadlineScope &) = delete;
};

/*! \brief seconds this rank has been working inside an op without waiting (0: not) */
inline double WorkingFor() {
  const double since = GlobalWaitState().working_since.load();
  return since > 0 ? MonotonicSec() - since : 0.0;
}
}  // namespace core
}  // namespace rabit
#endif  // XRABIT_CORE_WAIT_STATE_H_
