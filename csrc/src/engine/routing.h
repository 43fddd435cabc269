/*!
 * \file routing.h
 * \brief The calibration's size routing between RCCL and the direct transport, as a pure
 *        function of the measured times (unit-tested in tests/cpp/unit_tests.cc).
 */
#ifndef XRABIT_ENGINE_ROUTING_H_
#define XRABIT_ENGINE_ROUTING_H_

#include <algorithm>
#include <cstddef>

namespace rabit {
namespace engine {

/*! \brief ops of at least min_bytes, or below below_bytes, take the direct transport */
struct DirectRouting {
  size_t min_bytes;    // SIZE_MAX: no large-op range
  size_t below_bytes;  // 0: no small-op range
};

/*!
 * \brief fit t = a + b * bytes per transport through the two calibration points (x0 < x1 bytes;
 *        r0, r1 RCCL times, d0, d1 direct times) and route every size to the faster line:
 *  - direct faster at x1: direct from the crossover on (from 0 if it is faster everywhere);
 *  - else direct faster at x0: direct below the crossover (the latency path), at least up to x0;
 *  - else RCCL everywhere.  The ranges are clamped to [0, x1] (a measured point is never
 *    routed against its own measurement).
 */
inline DirectRouting ChooseDirectRouting(double x0, double x1, double r0, double r1, double d0,
                                         double d1) {
  DirectRouting out{static_cast<size_t>(-1), 0};
  const double br = (r1 - r0) / (x1 - x0), bd = (d1 - d0) / (x1 - x0);
  const double ar = r0 - br * x0, ad = d0 - bd * x0;
  if (d1 < r1) {
    const double cross = bd < br ? (ad - ar) / (br - bd) : 0.0;
    out.min_bytes = static_cast<size_t>(std::max(0.0, std::min(cross, x1)));
  } else if (d0 < r0) {
    const double cross = bd > br ? (ar - ad) / (bd - br) : x1;
    out.below_bytes = static_cast<size_t>(std::max(x0, std::min(cross, x1)));
  }
  return out;
}

}  // namespace engine
}  // namespace rabit
#endif  // XRABIT_ENGINE_ROUTING_H_
