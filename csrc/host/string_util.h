// string_util.h — string helpers (reference: /root/reference/src/utils/string.h).
//
// Same semantics as the reference: `split` treats every char of `delim` as a
// delimiter and skips empty fields (string.h:32-46); `key_value_split` splits
// on the FIRST delimiter only (string.h:48-61).
#pragma once
#include <cstdio>
#include <string>
#include <utility>
#include <vector>

#include "common.h"

namespace ss {

inline std::string& trim_inplace(std::string& s) {
  if (s.empty()) return s;
  s.erase(0, s.find_first_not_of(" \t\n\r"));
  const size_t e = s.find_last_not_of(" \t\n\r");
  if (e == std::string::npos)
    s.clear();
  else
    s.erase(e + 1);
  return s;
}
inline std::string trim(std::string s) { return trim_inplace(s); }

inline std::vector<std::string> split(const std::string& s, const std::string& delim) {
  std::vector<std::string> cols;
  size_t start = s.find_first_not_of(delim, 0);
  while (start != std::string::npos) {
    const size_t last = s.find_first_of(delim, start);
    cols.push_back(last == std::string::npos ? s.substr(start) : s.substr(start, last - start));
    if (last == std::string::npos) break;
    start = s.find_first_not_of(delim, last);
  }
  return cols;
}

inline std::pair<std::string, std::string> key_value_split(const std::string& s,
                                                           const std::string& delim) {
  const size_t i = s.find_first_of(delim);
  SS_CHECK_MSG(i != std::string::npos, "no delimiter '" << delim << "' in: " << s);
  return {s.substr(0, i), s.substr(i + 1)};
}

inline bool startswith(const std::string& s, const std::string& head) {
  return s.compare(0, head.size(), head) == 0;
}
inline bool headswith(const std::string& s, const std::string& head) { return startswith(s, head); }
inline bool endswith(const std::string& s, const std::string& tail) {
  return s.size() >= tail.size() && s.compare(s.size() - tail.size(), tail.size(), tail) == 0;
}

template <typename... Args>
std::string format_string(const char* fmt, Args... args) {
  const int len = std::snprintf(nullptr, 0, fmt, args...);
  SS_CHECK(len >= 0);
  std::string s((size_t)len + 1, '\0');
  std::snprintf(&s[0], (size_t)len + 1, fmt, args...);
  s.resize((size_t)len);
  return s;
}

// getdelim-based line reader with a reusable buffer (string.h:89-114).
class LineFileReader : NonCopyable {
 public:
  ~LineFileReader() { std::free(buf_); }
  char* getline(FILE* f) { return getdelim(f, '\n'); }
  char* getdelim(FILE* f, char delim) {
    const ssize_t r = ::getdelim(&buf_, &cap_, delim, f);
    if (r < 0) {
      len_ = 0;
      return nullptr;
    }
    size_t n = (size_t)r;
    if (n >= 1 && buf_[n - 1] == delim) buf_[--n] = 0;
    len_ = n;
    return buf_;
  }
  char* get() { return buf_; }
  size_t length() const { return len_; }

 private:
  char* buf_ = nullptr;
  size_t cap_ = 0;
  size_t len_ = 0;
};

}  // namespace ss
