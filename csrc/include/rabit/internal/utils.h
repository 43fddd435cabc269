/*!
 * \file utils.h
 * \brief Error handling and logging helpers of the xrabit runtime.
 *
 * API parity with the reference's `include/rabit/internal/utils.h:78-217`
 * (StringToBool, Assert/Check/Error, Printf, HandleLogInfo, FopenCheck, BeginPtr).
 * Differences by design:
 *  - errors throw `rabit::Error` (a std::runtime_error), there is no dmlc-core;
 *  - the message hooks are plain function pointers that can be swapped at run
 *    time (`utils::SetErrorHandler`, `utils::SetLogHandler`) instead of the
 *    compile-time RABIT_CUSTOMIZE_MSG_ switch.
 */
#ifndef RABIT_INTERNAL_UTILS_H_
#define RABIT_INTERNAL_UTILS_H_

#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

namespace rabit {

/*! \brief exception type thrown by every rabit failure (replaces dmlc::Error) */
class Error : public std::runtime_error {
 public:
  explicit Error(const std::string &msg) : std::runtime_error(msg) {}
};

namespace utils {

/*! \brief maximum length of one formatted message */
constexpr size_t kPrintBuffer = 1 << 12;

/*! \brief hook types: users may reroute messages (e.g. into a host program's log) */
typedef void (*ErrorHandler)(const char *msg);
typedef void (*LogHandler)(const char *msg);

/*! \brief replace the handler called before an error is thrown; returns the old one */
ErrorHandler SetErrorHandler(ErrorHandler h);
/*! \brief replace the log sink (default: stdout); returns the old one */
LogHandler SetLogHandler(LogHandler h);

/*! \brief format into a std::string */
inline std::string VFormat(const char *fmt, va_list args) {
  char buf[kPrintBuffer];
  vsnprintf(buf, sizeof(buf), fmt, args);
  return std::string(buf);
}
inline std::string Format(const char *fmt, ...) {
  va_list args;
  va_start(args, fmt);
  std::string s = VFormat(fmt, args);
  va_end(args);
  return s;
}

/*! \brief route a message through the installed error handler then throw */
[[noreturn]] void RaiseError(const std::string &msg);
/*! \brief route a message through the installed log handler */
void EmitLog(const std::string &msg);

/*! \brief "true"/"True"/nonzero integer => true */
inline bool StringToBool(const char *s) {
  if (s == nullptr) return false;
  if (!strcasecmp(s, "true")) return true;
  if (!strcasecmp(s, "false")) return false;
  return atoi(s) != 0;
}

/*! \brief internal invariant violation */
inline void Assert(bool exp, const char *fmt, ...) {
  if (exp) return;
  va_list args;
  va_start(args, fmt);
  std::string msg = "AssertError:" + VFormat(fmt, args);
  va_end(args);
  RaiseError(msg);
}
/*! \brief user-facing precondition */
inline void Check(bool exp, const char *fmt, ...) {
  if (exp) return;
  va_list args;
  va_start(args, fmt);
  std::string msg = VFormat(fmt, args);
  va_end(args);
  RaiseError(msg);
}
/*! \brief unconditional error */
[[noreturn]] inline void Error(const char *fmt, ...) {
  va_list args;
  va_start(args, fmt);
  std::string msg = VFormat(fmt, args);
  va_end(args);
  RaiseError(msg);
}
/*! \brief printf to the log sink */
inline void Printf(const char *fmt, ...) {
  va_list args;
  va_start(args, fmt);
  std::string msg = VFormat(fmt, args);
  va_end(args);
  EmitLog(msg);
}
/*! \brief informational log line (same sink as Printf) */
inline void HandleLogInfo(const char *fmt, ...) {
  va_list args;
  va_start(args, fmt);
  std::string msg = VFormat(fmt, args);
  va_end(args);
  EmitLog(msg);
}
/*! \brief fopen that raises on failure */
inline FILE *FopenCheck(const char *fname, const char *flag) {
  FILE *fp = fopen(fname, flag);
  Check(fp != nullptr, "can not open file \"%s\"\n", fname);
  return fp;
}
}  // namespace utils

/*! \brief pointer to the first element, nullptr for an empty container */
template <typename T>
inline T *BeginPtr(std::vector<T> &vec) {  // NOLINT(*)
  return vec.empty() ? nullptr : vec.data();
}
template <typename T>
inline const T *BeginPtr(const std::vector<T> &vec) {
  return vec.empty() ? nullptr : vec.data();
}
inline char *BeginPtr(std::string &str) {  // NOLINT(*)
  return str.empty() ? nullptr : &str[0];
}
inline const char *BeginPtr(const std::string &str) {
  return str.empty() ? nullptr : str.data();
}
}  // namespace rabit
#endif  // RABIT_INTERNAL_UTILS_H_
