/*!
 * \file serializable.h
 * \brief Stream / Serializable interfaces used by checkpoints.
 *
 * The reference aliases these to dmlc-core (`include/rabit/serializable.h:18-23`),
 * which is not available here, so xrabit defines them itself.  The on-wire byte
 * format is the dmlc one so checkpoints stay byte compatible:
 *   - trivially copyable T           -> raw bytes
 *   - std::vector<T>, std::string    -> uint64 element count, then the elements
 *   - std::pair<A, B>                -> A then B
 */
#ifndef RABIT_SERIALIZABLE_H_
#define RABIT_SERIALIZABLE_H_

#include <cstdint>
#include <map>
#include <string>
#include <type_traits>
#include <utility>
#include <vector>

#include "rabit/internal/utils.h"

namespace rabit {

class Stream;

namespace serializer {
/*! \brief Handler<T>::Write/Read define the byte format of T */
template <typename T, typename Enable = void>
struct Handler;
}  // namespace serializer

/*! \brief byte stream interface */
class Stream {
 public:
  virtual ~Stream() = default;
  /*! \brief read up to size bytes, return number of bytes read */
  virtual size_t Read(void *ptr, size_t size) = 0;
  /*! \brief write size bytes */
  virtual void Write(const void *ptr, size_t size) = 0;
  /*! \brief typed write (vector / string / POD / pair) */
  template <typename T>
  inline void Write(const T &data) {
    serializer::Handler<T>::Write(this, data);
  }
  /*! \brief typed read, returns false on short read */
  template <typename T>
  inline bool Read(T *out) {
    return serializer::Handler<T>::Read(this, out);
  }
};

/*! \brief stream that supports random access */
class SeekStream : public Stream {
 public:
  virtual void Seek(size_t pos) = 0;
  virtual size_t Tell() = 0;
  virtual bool AtEnd() const { return false; }
};

/*! \brief interface of a model that can be checkpointed */
class Serializable {
 public:
  virtual ~Serializable() = default;
  virtual void Load(Stream *fi) = 0;
  virtual void Save(Stream *fo) const = 0;
};

namespace serializer {
// trivially copyable values: raw bytes
template <typename T>
struct Handler<T, typename std::enable_if<std::is_trivially_copyable<T>::value>::type> {
  static void Write(Stream *s, const T &v) { s->Write(&v, sizeof(T)); }
  static bool Read(Stream *s, T *v) { return s->Read(v, sizeof(T)) == sizeof(T); }
};
// vector of trivially copyable: count + one bulk copy
template <typename T>
struct Handler<std::vector<T>,
               typename std::enable_if<std::is_trivially_copyable<T>::value>::type> {
  static void Write(Stream *s, const std::vector<T> &v) {
    uint64_t n = v.size();
    s->Write(&n, sizeof(n));
    if (n != 0) s->Write(v.data(), sizeof(T) * v.size());
  }
  static bool Read(Stream *s, std::vector<T> *v) {
    uint64_t n;
    if (s->Read(&n, sizeof(n)) != sizeof(n)) return false;
    v->resize(static_cast<size_t>(n));
    if (n == 0) return true;
    return s->Read(v->data(), sizeof(T) * n) == sizeof(T) * n;
  }
};
// vector of composite values: count + element-wise
template <typename T>
struct Handler<std::vector<T>,
               typename std::enable_if<!std::is_trivially_copyable<T>::value>::type> {
  static void Write(Stream *s, const std::vector<T> &v) {
    uint64_t n = v.size();
    s->Write(&n, sizeof(n));
    for (const T &e : v) Handler<T>::Write(s, e);
  }
  static bool Read(Stream *s, std::vector<T> *v) {
    uint64_t n;
    if (s->Read(&n, sizeof(n)) != sizeof(n)) return false;
    v->resize(static_cast<size_t>(n));
    for (auto &e : *v) {
      if (!Handler<T>::Read(s, &e)) return false;
    }
    return true;
  }
};
template <>
struct Handler<std::string> {
  static void Write(Stream *s, const std::string &v) {
    uint64_t n = v.size();
    s->Write(&n, sizeof(n));
    if (n != 0) s->Write(v.data(), v.size());
  }
  static bool Read(Stream *s, std::string *v) {
    uint64_t n;
    if (s->Read(&n, sizeof(n)) != sizeof(n)) return false;
    v->resize(static_cast<size_t>(n));
    if (n == 0) return true;
    return s->Read(&(*v)[0], n) == n;
  }
};
template <typename A, typename B>
struct Handler<std::pair<A, B>,
               typename std::enable_if<!std::is_trivially_copyable<std::pair<A, B>>::value>::type> {
  static void Write(Stream *s, const std::pair<A, B> &v) {
    Handler<A>::Write(s, v.first);
    Handler<B>::Write(s, v.second);
  }
  static bool Read(Stream *s, std::pair<A, B> *v) {
    return Handler<A>::Read(s, &v->first) && Handler<B>::Read(s, &v->second);
  }
};
template <typename K, typename V>
struct Handler<std::map<K, V>> {
  static void Write(Stream *s, const std::map<K, V> &m) {
    std::vector<std::pair<K, V>> v(m.begin(), m.end());
    Handler<std::vector<std::pair<K, V>>>::Write(s, v);
  }
  static bool Read(Stream *s, std::map<K, V> *m) {
    std::vector<std::pair<K, V>> v;
    if (!Handler<std::vector<std::pair<K, V>>>::Read(s, &v)) return false;
    m->clear();
    m->insert(v.begin(), v.end());
    return true;
  }
};
}  // namespace serializer
}  // namespace rabit
#endif  // RABIT_SERIALIZABLE_H_
