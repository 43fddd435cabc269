/*!
 * \file routing.h
 * \brief The calibration's size routing between RCCL and the direct transport, as a pure
 *        function of the measured times (unit-tested in tests/cpp/unit_tests.cc).
 */
#ifndef XRABIT_ENGINE_ROUTING_H_
#define XRABIT_ENGINE_ROUTING_H_

#include <algorithm>
#include <cstddef>
#include <vector>

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

/*! \brief ops of at least lo bytes (up to the next band's lo) take candidate `choice` */
struct RouteBand {
  double lo;
  int choice;
};

/*!
 * \brief piecewise routing over several calibration points (reference: the size-based
 *        algorithm choice of `src/allreduce_base.cc:454-464`, here measured instead of fixed).
 *        x: the measured sizes, ascending (bytes); t[c][i]: time of candidate c at x[i], < 0 when
 *        c was not measured or failed there.  Between two neighbouring points every candidate
 *        measured at both is a straight line, and each size takes the lowest line (crossovers
 *        inside the interval split it); beyond the last point the last interval's lines are
 *        extended (bandwidth-bound sizes keep their slopes); below the first point the choice at
 *        the first point holds.  Ties go to the lower candidate index.  Returns bands in
 *        ascending lo with lo[0] = 0, neighbours merged when they choose the same candidate;
 *        empty when no candidate was measured anywhere.
 */
inline std::vector<RouteBand> ChooseRoutes(const std::vector<double> &x,
                                           const std::vector<std::vector<double>> &t) {
  std::vector<RouteBand> out;
  const int n = static_cast<int>(x.size());
  const int nc = static_cast<int>(t.size());
  auto push = [&](double lo, int c) {
    if (c < 0) return;
    if (!out.empty() && out.back().choice == c) return;
    if (!out.empty() && lo <= out.back().lo) {
      out.back().choice = c;  // an empty band: the later choice wins at this size
      if (out.size() >= 2 && out[out.size() - 2].choice == c) out.pop_back();
      return;
    }
    out.push_back(RouteBand{lo, c});
  };
  auto best_at = [&](int i) {
    int b = -1;
    for (int c = 0; c < nc; ++c) {
      if (t[c][i] >= 0 && (b < 0 || t[c][i] < t[b][i])) b = c;
    }
    return b;
  };
  if (n == 0) return out;
  // below (and at) the first point
  push(0.0, best_at(0));
  // one interval [x[k], x[k+1]] at a time (k = n - 1: the extension past the last point, with
  // the lines of the last interval)
  for (int k = 0; k < n; ++k) {
    const bool tail = k == n - 1;
    if (tail && n < 2) break;
    const int a = tail ? n - 2 : k, b = a + 1;
    const double x0 = x[a], x1 = x[b];
    std::vector<int> live;
    for (int c = 0; c < nc; ++c) {
      if (t[c][a] >= 0 && t[c][b] >= 0) live.push_back(c);
    }
    auto line = [&](int c, double s) {
      return t[c][a] + (t[c][b] - t[c][a]) * (s - x0) / (x1 - x0);
    };
    const double lo = tail ? x1 : x0, hi = tail ? 1e300 : x1;
    // every crossover of two live lines inside (lo, hi) splits the interval
    std::vector<double> cuts = {lo};
    for (size_t i = 0; i < live.size(); ++i) {
      for (size_t j = i + 1; j < live.size(); ++j) {
        const int p = live[i], q = live[j];
        const double sp = (t[p][b] - t[p][a]) / (x1 - x0), sq = (t[q][b] - t[q][a]) / (x1 - x0);
        if (sp == sq) continue;
        const double s = x0 + (t[q][a] - t[p][a]) / (sp - sq);
        if (s > lo && s < hi) cuts.push_back(s);
      }
    }
    std::sort(cuts.begin(), cuts.end());
    cuts.push_back(hi);
    for (size_t i = 0; i + 1 < cuts.size(); ++i) {
      if (cuts[i + 1] <= cuts[i]) continue;
      // the lowest line over (cuts[i], cuts[i+1]): evaluate inside the piece
      const double mid = cuts[i + 1] >= 1e299 ? cuts[i] * 2.0 + 1.0 : 0.5 * (cuts[i] + cuts[i + 1]);
      int bestc = -1;
      double bt = 0;
      for (int c : live) {
        const double v = line(c, mid);
        if (bestc < 0 || v < bt) {
          bestc = c;
          bt = v;
        }
      }
      if (bestc < 0) bestc = best_at(tail ? b : a);
      push(cuts[i], bestc);
    }
  }
  return out;
}

/*! \brief the candidate of the band holding `bytes` (-1: no bands) */
inline int RouteFor(const std::vector<RouteBand> &bands, double bytes) {
  int c = -1;
  for (const RouteBand &b : bands) {
    if (bytes >= b.lo) c = b.choice;
  }
  return c;
}

}  // namespace engine
}  // namespace rabit
#endif  // XRABIT_ENGINE_ROUTING_H_
