/*!
 * \file trace.h
 * \brief Tracing: the reference only has ad-hoc timing printouts under
 *        rabit_debug.  xrabit records a span per engine phase (collective, consensus,
 *        recovery, checkpoint, device wait) into a bounded in-memory log that can be dumped
 *        as a Chrome/Perfetto trace, and mirrors every span as a roctx range so
 *        `rocprofv3 --marker-trace` lines engine phases up with the GPU kernels.
 *        Enabled by rabit_trace=1 (spans) / rabit_trace_roctx=1 (roctx ranges).
 */
#ifndef XRABIT_CORE_TRACE_H_
#define XRABIT_CORE_TRACE_H_

#include <cstddef>
#include <cstdint>
#include <mutex>
#include <string>
#include <vector>

namespace rabit {
namespace trace {

struct Span {
  const char *name;   // static string
  double t0, t1;      // seconds (steady clock)
  int rank;
  int version, seqno;
  uint64_t bytes;
  int on_device;
};

class Tracer {
 public:
  static Tracer &Get();
  void Configure(bool spans, bool roctx, size_t capacity);
  bool spans() const { return spans_; }
  bool roctx() const { return roctx_; }
  void Record(const Span &s);
  /*! \brief Chrome trace-event JSON of the recorded spans */
  std::string ChromeJson() const;
  size_t size() const;
  void Clear();

 private:
  bool spans_{false}, roctx_{false};
  size_t capacity_{1 << 16};
  size_t next_{0};
  bool wrapped_{false};
  std::vector<Span> ring_;
  mutable std::mutex mu_;
};

void RoctxPush(const char *name);
void RoctxPop();

/*! \brief RAII span: roctx range + recorded span when tracing is on */
class Scope {
 public:
  Scope(const char *name, int rank, int version, int seqno, uint64_t bytes, int on_device);
  ~Scope();

 private:
  Span span_;
  bool active_;
  bool roctx_;
};
}  // namespace trace
}  // namespace rabit
#endif  // XRABIT_CORE_TRACE_H_
