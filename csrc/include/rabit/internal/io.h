/*!
 * \file io.h
 * \brief In-memory streams used for checkpoints and serialize-reduce.
 *
 * Parity: reference `include/rabit/internal/io.h:24-111`
 * (MemoryFixSizeBuffer with SeekEnd sentinel and overflow check, growing
 * MemoryBufferStream).
 */
#ifndef RABIT_INTERNAL_IO_H_
#define RABIT_INTERNAL_IO_H_

#include <algorithm>
#include <cstring>
#include <limits>
#include <string>

#include "rabit/serializable.h"
#include "rabit/internal/utils.h"

namespace rabit {
namespace utils {

/*! \brief stream over a caller-owned buffer of fixed size */
class MemoryFixSizeBuffer : public SeekStream {
 public:
  /*! \brief seeking here moves to the end of the buffer */
  static constexpr size_t kSeekEnd = std::numeric_limits<size_t>::max();
  static constexpr size_t SeekEnd = kSeekEnd;  // reference spelling

  MemoryFixSizeBuffer(void *p_buffer, size_t buffer_size)
      : base_(static_cast<char *>(p_buffer)), size_(buffer_size), pos_(0) {}

  size_t Read(void *ptr, size_t size) override {
    size_t n = std::min(size, size_ - pos_);
    if (n != 0) std::memcpy(ptr, base_ + pos_, n);
    pos_ += n;
    return n;
  }
  void Write(const void *ptr, size_t size) override {
    if (size == 0) return;
    Assert(pos_ + size <= size_, "MemoryFixSizeBuffer: write exceeds buffer size");
    std::memcpy(base_ + pos_, ptr, size);
    pos_ += size;
  }
  using Stream::Read;
  using Stream::Write;
  void Seek(size_t pos) override { pos_ = (pos == kSeekEnd) ? size_ : std::min(pos, size_); }
  size_t Tell() override { return pos_; }
  bool AtEnd() const override { return pos_ == size_; }

 private:
  char *base_;
  size_t size_;
  size_t pos_;
};

/*! \brief stream that appends to / reads from a std::string it does not own */
class MemoryBufferStream : public SeekStream {
 public:
  explicit MemoryBufferStream(std::string *p_buffer) : buf_(p_buffer), pos_(0) {}

  size_t Read(void *ptr, size_t size) override {
    Assert(pos_ <= buf_->length(), "MemoryBufferStream: read position out of range");
    size_t n = std::min(size, buf_->length() - pos_);
    if (n != 0) std::memcpy(ptr, buf_->data() + pos_, n);
    pos_ += n;
    return n;
  }
  void Write(const void *ptr, size_t size) override {
    if (size == 0) return;
    if (pos_ + size > buf_->length()) buf_->resize(pos_ + size);
    std::memcpy(&(*buf_)[pos_], ptr, size);
    pos_ += size;
  }
  using Stream::Read;
  using Stream::Write;
  void Seek(size_t pos) override { pos_ = pos; }
  size_t Tell() override { return pos_; }
  bool AtEnd() const override { return pos_ >= buf_->length(); }

 private:
  std::string *buf_;
  size_t pos_;
};
}  // namespace utils
}  // namespace rabit
#endif  // RABIT_INTERNAL_IO_H_
