/*!
 * \file dmlc/io.h
 * \brief Minimal stand-in for dmlc-core's io.h: Stream / SeekStream / Serializable and the
 *        exception type the reference rabit sources use (u64 element count, then
 *        the raw POD bytes, for vectors and strings).  Only for compiling the reference for
 *        speed comparisons; xrabit has its own csrc/include/rabit/serializable.h.
 */
#ifndef DMLC_IO_H_
#define DMLC_IO_H_
#include <cstddef>
#include <cstdint>
#include <stdexcept>
#include <string>
#include <vector>

#include "./base.h"

namespace dmlc {
struct Error : public std::runtime_error {
  explicit Error(const std::string &s) : std::runtime_error(s) {}
};

class Stream {
 public:
  virtual size_t Read(void *ptr, size_t size) = 0;
  virtual void Write(const void *ptr, size_t size) = 0;
  virtual ~Stream() {}
  template <typename T>
  void Write(const std::vector<T> &v) {
    uint64_t n = v.size();
    Write(&n, sizeof(n));
    if (n != 0) Write(v.data(), sizeof(T) * n);
  }
  template <typename T>
  bool Read(std::vector<T> *v) {
    uint64_t n;
    if (Read(&n, sizeof(n)) != sizeof(n)) return false;
    v->resize(n);
    return n == 0 || Read(v->data(), sizeof(T) * n) == sizeof(T) * n;
  }
  void Write(const std::string &s) {
    uint64_t n = s.size();
    Write(&n, sizeof(n));
    if (n != 0) Write(s.data(), n);
  }
  bool Read(std::string *s) {
    uint64_t n;
    if (Read(&n, sizeof(n)) != sizeof(n)) return false;
    s->resize(n);
    return n == 0 || Read(&(*s)[0], n) == n;
  }
  template <typename T>
  void Write(const T &v) {
    Write(&v, sizeof(T));
  }
  template <typename T>
  bool Read(T *v) {
    return Read(static_cast<void *>(v), sizeof(T)) == sizeof(T);
  }
};

class SeekStream : public Stream {
 public:
  virtual void Seek(size_t pos) = 0;
  virtual size_t Tell() = 0;
};

class Serializable {
 public:
  virtual ~Serializable() {}
  virtual void Load(Stream *fi) = 0;
  virtual void Save(Stream *fo) const = 0;
};
}  // namespace dmlc
#endif  // DMLC_IO_H_
