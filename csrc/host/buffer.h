// buffer.h — growable binary codec (reference: utils/Buffer.h BasicBuffer /
// BinaryBuffer, :15-234).
//
// A byte buffer with a write end and a read cursor; POD values are memcpy'd
// (`<<` appends, `>>` consumes).  Strings are length-prefixed (u32).
// Fixes vs the reference: move-assignment keeps the capacity (Buffer.h:39-48
// drops it), reads past the end throw instead of reading garbage.
#pragma once
#include <cstring>
#include <string>
#include <type_traits>
#include <vector>

#include "common.h"

namespace ss {

class BinaryBuffer {
 public:
  BinaryBuffer() { data_.reserve(1024); }
  explicit BinaryBuffer(std::string bytes) : data_(bytes.begin(), bytes.end()) {}
  BinaryBuffer(const char* p, size_t n) : data_(p, p + n) {}

  BinaryBuffer(BinaryBuffer&&) = default;
  BinaryBuffer& operator=(BinaryBuffer&&) = default;
  BinaryBuffer(const BinaryBuffer&) = default;
  BinaryBuffer& operator=(const BinaryBuffer&) = default;

  template <typename T>
  typename std::enable_if<std::is_trivially_copyable<T>::value, BinaryBuffer&>::type operator<<(
      const T& v) {
    put_raw(&v, sizeof(T));
    return *this;
  }
  template <typename T>
  typename std::enable_if<std::is_trivially_copyable<T>::value, BinaryBuffer&>::type operator>>(
      T& v) {
    get_raw(&v, sizeof(T));
    return *this;
  }
  BinaryBuffer& operator<<(const std::string& s) {
    const uint32_t n = (uint32_t)s.size();
    *this << n;
    put_raw(s.data(), n);
    return *this;
  }
  BinaryBuffer& operator>>(std::string& s) {
    uint32_t n = 0;
    *this >> n;
    SS_CHECK_MSG(cursor_ + n <= data_.size(), "BinaryBuffer: read past end");
    s.assign(data_.data() + cursor_, n);
    cursor_ += n;
    return *this;
  }

  void put_raw(const void* p, size_t n) {
    const size_t o = data_.size();
    data_.resize(o + n);
    if (n) std::memcpy(data_.data() + o, p, n);
  }
  void get_raw(void* p, size_t n) {
    SS_CHECK_MSG(cursor_ + n <= data_.size(), "BinaryBuffer: read past end");
    if (n) std::memcpy(p, data_.data() + cursor_, n);
    cursor_ += n;
  }

  bool read_finished() const { return cursor_ >= data_.size(); }
  size_t size() const { return data_.size(); }
  size_t capacity() const { return data_.capacity(); }
  size_t cursor() const { return cursor_; }
  size_t remaining() const { return data_.size() - cursor_; }
  void set_cursor(size_t c) {
    SS_CHECK(c <= data_.size());
    cursor_ = c;
  }
  void clear() {
    data_.clear();
    cursor_ = 0;
  }
  const char* data() const { return data_.data(); }
  char* data() { return data_.data(); }
  std::string str() const { return std::string(data_.data(), data_.size()); }
  std::vector<char>& bytes() { return data_; }

 private:
  std::vector<char> data_;
  size_t cursor_ = 0;
};

}  // namespace ss
