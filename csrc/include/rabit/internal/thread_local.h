/*!
 * \file thread_local.h
 * \brief Per-thread singleton holder (parity: reference `include/rabit/internal/thread_local.h:38-85`).
 *        C++11 `thread_local` gives destruction at thread exit, so no registry is needed.
 */
#ifndef RABIT_INTERNAL_THREAD_LOCAL_H_
#define RABIT_INTERNAL_THREAD_LOCAL_H_

namespace rabit {
/*! \brief one lazily constructed T per thread */
template <typename T>
class ThreadLocalStore {
 public:
  static T *Get() {
    static thread_local T inst;
    return &inst;
  }
};
}  // namespace rabit
#endif  // RABIT_INTERNAL_THREAD_LOCAL_H_
