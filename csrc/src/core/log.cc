/*!
 * \file log.cc
 * \brief Message sinks of utils.h.
 */
#include <atomic>
#include <cstdio>

#include "rabit/internal/utils.h"

namespace rabit {
namespace utils {
namespace {
std::atomic<ErrorHandler> g_error_handler{nullptr};
std::atomic<LogHandler> g_log_handler{nullptr};
}  // namespace

ErrorHandler SetErrorHandler(ErrorHandler h) { return g_error_handler.exchange(h); }
LogHandler SetLogHandler(LogHandler h) { return g_log_handler.exchange(h); }

void RaiseError(const std::string &msg) {
  ErrorHandler h = g_error_handler.load();
  if (h != nullptr) {
    h(msg.c_str());
  } else {
    fprintf(stderr, "[xrabit] %s\n", msg.c_str());
    fflush(stderr);
  }
  throw rabit::Error(msg);
}

void EmitLog(const std::string &msg) {
  LogHandler h = g_log_handler.load();
  if (h != nullptr) {
    h(msg.c_str());
  } else {
    fputs(msg.c_str(), stdout);
    fflush(stdout);
  }
}
}  // namespace utils
}  // namespace rabit
