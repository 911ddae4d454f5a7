// vec.h — dense parameter value type for host-side apps (the reference's
// utils/vec1.h `Vec`, the value type its word2vec-style apps keep in the
// SparseTable: /root/reference/src/utils/vec1.h:6-252).
//
// Same capabilities — elementwise arithmetic with vectors and scalars, dot,
// outer, sqrt, random init in the word2vec convention (u - offset) / size —
// built on std::vector<double> (no manual new/delete, so copy/move are the
// defaults), plus what a PS value type needs here: the BinaryBuffer codec
// (length-prefixed), the text form of the checkpoint (`v v v`, no "Vec:"
// prefix, so dumps parse back with utils/checkpoint.py) and a reset() that
// zeroes in place (the Grad contract of global_push_access.h:78).
// Size mismatches throw instead of reading out of bounds.
#pragma once
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <ostream>
#include <random>
#include <sstream>
#include <string>
#include <vector>

#include "buffer.h"
#include "common.h"

namespace ss {

class Vec {
 public:
  using value_type = double;

  Vec() = default;
  explicit Vec(size_t n, value_type fill = 0.0) : v_(n, fill) {}
  Vec(std::initializer_list<value_type> xs) : v_(xs) {}

  size_t size() const { return v_.size(); }
  bool empty() const { return v_.empty(); }
  value_type* data() { return v_.data(); }
  const value_type* data() const { return v_.data(); }
  value_type& operator[](size_t i) { return v_[i]; }
  const value_type& operator[](size_t i) const { return v_[i]; }

  // init(size, random): zero or random (word2vec convention) values
  void init(size_t n, bool random = false) {
    v_.assign(n, 0.0);
    if (random) rand_init();
  }
  // (u - offset) / size with u ~ U[0,1); the reference's randInit default
  // offset is 0.5 (vec1.h:223-226), `random()` uses offset 0 (vec1.h:85)
  void rand_init(double offset = 0.5, uint64_t seed = 0) {
    std::mt19937_64 g(seed ? seed : std::random_device{}());
    std::uniform_real_distribution<double> u(0.0, 1.0);
    const double n = (double)(v_.empty() ? 1 : v_.size());
    for (auto& x : v_) x = (u(g) - offset) / n;
  }
  void reset() { std::fill(v_.begin(), v_.end(), 0.0); }  // zero, keep size
  void resize(size_t n) { v_.assign(n, 0.0); }           // reference reset(size)

  value_type dot(const Vec& o) const {
    same_size(o, "dot");
    value_type s = 0;
    for (size_t i = 0; i < v_.size(); ++i) s += v_[i] * o.v_[i];
    return s;
  }
  value_type norm2() const { return dot(*this); }

  // elementwise, in place
  Vec& operator+=(const Vec& o) { return zip(o, "+=", [](double& a, double b) { a += b; }); }
  Vec& operator-=(const Vec& o) { return zip(o, "-=", [](double& a, double b) { a -= b; }); }
  Vec& operator*=(const Vec& o) { return zip(o, "*=", [](double& a, double b) { a *= b; }); }
  Vec& operator/=(const Vec& o) { return zip(o, "/=", [](double& a, double b) { a /= b; }); }
  Vec& operator+=(value_type b) { for (auto& x : v_) x += b; return *this; }
  Vec& operator-=(value_type b) { for (auto& x : v_) x -= b; return *this; }
  Vec& operator*=(value_type b) { for (auto& x : v_) x *= b; return *this; }
  Vec& operator/=(value_type b) { for (auto& x : v_) x /= b; return *this; }

  // axpy: this += a * x (the SGD update shape)
  Vec& axpy(value_type a, const Vec& x) {
    same_size(x, "axpy");
    for (size_t i = 0; i < v_.size(); ++i) v_[i] += a * x.v_[i];
    return *this;
  }

  friend Vec operator+(Vec a, const Vec& b) { return a += b; }
  friend Vec operator-(Vec a, const Vec& b) { return a -= b; }
  friend Vec operator*(Vec a, const Vec& b) { return a *= b; }
  friend Vec operator/(Vec a, const Vec& b) { return a /= b; }
  friend Vec operator+(Vec a, value_type b) { return a += b; }
  friend Vec operator+(value_type b, Vec a) { return a += b; }
  friend Vec operator-(Vec a, value_type b) { return a -= b; }
  friend Vec operator-(value_type b, const Vec& a) {
    Vec r(a.size());
    for (size_t i = 0; i < a.size(); ++i) r.v_[i] = b - a.v_[i];
    return r;
  }
  friend Vec operator*(Vec a, value_type b) { return a *= b; }
  friend Vec operator*(value_type b, Vec a) { return a *= b; }
  friend Vec operator/(Vec a, value_type b) { return a /= b; }
  friend Vec operator/(value_type b, const Vec& a) {
    Vec r(a.size());
    for (size_t i = 0; i < a.size(); ++i) r.v_[i] = b / a.v_[i];
    return r;
  }
  friend bool operator==(const Vec& a, const Vec& b) { return a.v_ == b.v_; }

  // outer product a (x) b: a.size() rows of b.size() (vec1.h:55-71)
  friend std::vector<Vec> outer(const Vec& a, const Vec& b) {
    std::vector<Vec> rows(a.size(), Vec(b.size()));
    for (size_t i = 0; i < a.size(); ++i)
      for (size_t j = 0; j < b.size(); ++j) rows[i].v_[j] = a.v_[i] * b.v_[j];
    return rows;
  }
  friend Vec sqrt(const Vec& a) {
    Vec r(a);
    for (auto& x : r.v_) x = std::sqrt(x);
    return r;
  }

  // checkpoint text form: space-separated values
  friend std::ostream& operator<<(std::ostream& os, const Vec& a) {
    for (size_t i = 0; i < a.size(); ++i) os << (i ? " " : "") << a.v_[i];
    return os;
  }
  std::string to_string() const {
    std::ostringstream ss;
    ss.precision(17);
    ss << *this;
    return ss.str();
  }
  static Vec parse(const std::string& text) {
    std::istringstream ss(text);
    Vec r;
    double x;
    while (ss >> x) r.v_.push_back(x);
    return r;
  }

  // wire codec: u32 length + raw doubles
  friend BinaryBuffer& operator<<(BinaryBuffer& bb, const Vec& a) {
    bb << (uint32_t)a.size();
    if (!a.empty()) bb.put_raw(a.v_.data(), a.size() * sizeof(double));
    return bb;
  }
  friend BinaryBuffer& operator>>(BinaryBuffer& bb, Vec& a) {
    uint32_t n = 0;
    bb >> n;
    a.v_.resize(n);
    if (n) bb.get_raw(a.v_.data(), n * sizeof(double));
    return bb;
  }

 private:
  void same_size(const Vec& o, const char* op) const {
    SS_CHECK_MSG(o.size() == size(), std::string("Vec ") + op + ": size mismatch");
  }
  template <typename F>
  Vec& zip(const Vec& o, const char* op, F f) {
    same_size(o, op);
    for (size_t i = 0; i < v_.size(); ++i) f(v_[i], o.v_[i]);
    return *this;
  }
  std::vector<value_type> v_;
};

}  // namespace ss
