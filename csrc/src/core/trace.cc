/*!
 * \file trace.cc
 * \brief Span log + roctx ranges (see trace.h).
 */
#include "core/trace.h"

#include <rocprofiler-sdk-roctx/roctx.h>

#include <cstdio>
#include <sstream>

#include "rabit/internal/timer.h"

namespace rabit {
namespace trace {

Tracer &Tracer::Get() {
  static Tracer t;
  return t;
}

void Tracer::Configure(bool spans, bool roctx, size_t capacity) {
  std::lock_guard<std::mutex> lk(mu_);
  spans_ = spans;
  roctx_ = roctx;
  capacity_ = capacity == 0 ? 1 : capacity;
  ring_.clear();
  ring_.reserve(spans ? capacity_ : 0);
  next_ = 0;
  wrapped_ = false;
}

void Tracer::Record(const Span &s) {
  std::lock_guard<std::mutex> lk(mu_);
  if (ring_.size() < capacity_) {
    ring_.push_back(s);
  } else {
    ring_[next_] = s;
    next_ = (next_ + 1) % capacity_;
    wrapped_ = true;
  }
}

size_t Tracer::size() const {
  std::lock_guard<std::mutex> lk(mu_);
  return ring_.size();
}

void Tracer::Clear() {
  std::lock_guard<std::mutex> lk(mu_);
  ring_.clear();
  next_ = 0;
  wrapped_ = false;
}

std::string Tracer::ChromeJson() const {
  std::lock_guard<std::mutex> lk(mu_);
  std::ostringstream os;
  os << "{\"traceEvents\":[";
  const size_t n = ring_.size();
  for (size_t k = 0; k < n; ++k) {
    const Span &s = ring_[wrapped_ ? (next_ + k) % n : k];
    if (k != 0) os << ",";
    char buf[512];
    snprintf(buf, sizeof(buf),
             "{\"name\":\"%s\",\"ph\":\"X\",\"pid\":%d,\"tid\":0,\"ts\":%.3f,\"dur\":%.3f,"
             "\"args\":{\"version\":%d,\"seqno\":%d,\"bytes\":%llu,\"device\":%d}}",
             s.name, s.rank, s.t0 * 1e6, (s.t1 - s.t0) * 1e6, s.version, s.seqno,
             static_cast<unsigned long long>(s.bytes), s.on_device);
    os << buf;
  }
  os << "],\"displayTimeUnit\":\"ms\"}";
  return os.str();
}

void RoctxPush(const char *name) { roctxRangePushA(name); }
void RoctxPop() { roctxRangePop(); }

Scope::Scope(const char *name, int rank, int version, int seqno, uint64_t bytes, int on_device) {
  Tracer &t = Tracer::Get();
  active_ = t.spans();
  roctx_ = t.roctx();
  if (roctx_) RoctxPush(name);
  if (active_) span_ = Span{name, utils::GetTime(), 0.0, rank, version, seqno, bytes, on_device};
}

Scope::~Scope() {
  if (roctx_) RoctxPop();
  if (active_) {
    span_.t1 = utils::GetTime();
    Tracer::Get().Record(span_);
  }
}
}  // namespace trace
}  // namespace rabit
