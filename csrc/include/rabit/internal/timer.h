/*!
 * \file timer.h
 * \brief Wall-clock helper (parity: reference `include/rabit/internal/timer.h:21-38`).
 *        Uses the monotonic clock: durations must not jump with NTP adjustments.
 */
#ifndef RABIT_INTERNAL_TIMER_H_
#define RABIT_INTERNAL_TIMER_H_
#include <chrono>

namespace rabit {
namespace utils {
/*! \brief seconds since an arbitrary fixed point */
inline double GetTime() {
  using clock = std::chrono::steady_clock;
  return std::chrono::duration<double>(clock::now().time_since_epoch()).count();
}
}  // namespace utils
}  // namespace rabit
#endif  // RABIT_INTERNAL_TIMER_H_
