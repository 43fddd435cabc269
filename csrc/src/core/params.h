/*!
 * \file params.h
 * \brief Parameter collection: environment variables first, then argv `name=value`
 *        entries (argv wins).  Parity: reference `src/allreduce_base.cc:49-64,150-216`.
 */
#ifndef XRABIT_CORE_PARAMS_H_
#define XRABIT_CORE_PARAMS_H_

#include <cstdlib>
#include <cstring>
#include <string>
#include <utility>
#include <vector>

#include "rabit/internal/utils.h"

namespace rabit {
namespace core {

/*! \brief parse "<int>[B|K|M|G]" (suffix = binary multiple), as the reference ParseUnit */
inline size_t ParseUnit(const char *name, const char *val) {
  char *end = nullptr;
  unsigned long long amount = strtoull(val, &end, 10);  // NOLINT(*)
  utils::Check(end != val, "invalid value \"%s\" for %s: expected {integer}{B,K,M,G}", val,
               name);
  switch (*end) {
    case '\0':
    case 'B': return static_cast<size_t>(amount);
    case 'K': return static_cast<size_t>(amount) << 10;
    case 'M': return static_cast<size_t>(amount) << 20;
    case 'G': return static_cast<size_t>(amount) << 30;
    default: utils::Error("invalid unit in \"%s\" for %s", val, name);
  }
}

/*!
 * \brief ordered list of (name, value) from env vars in `env_names` followed by argv
 *        entries matching name=value
 */
inline std::vector<std::pair<std::string, std::string>> CollectParams(
    int argc, char *argv[], const std::vector<std::string> &env_names) {
  std::vector<std::pair<std::string, std::string>> out;
  for (const auto &n : env_names) {
    const char *v = getenv(n.c_str());
    if (v != nullptr) out.emplace_back(n, v);
  }
  for (int i = 0; i < argc; ++i) {
    if (argv[i] == nullptr) continue;
    const char *eq = strchr(argv[i], '=');
    if (eq == nullptr || eq == argv[i] || eq[1] == '\0') continue;
    out.emplace_back(std::string(argv[i], eq - argv[i]), std::string(eq + 1));
  }
  return out;
}
}  // namespace core
}  // namespace rabit
#endif  // XRABIT_CORE_PARAMS_H_
