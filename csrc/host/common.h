// common.h — host runtime basics: error/check macros, logging, small utils.
//
// Reference: /root/reference/src/utils/common.h (glog CHECK/LOG, index_t,
// guarded popen) and utils/VirtualObject.h.  Differences: failed checks throw
// ss::Error (surfaced to Python as RuntimeError) instead of aborting the
// process, and keys are 64-bit (index_t = uint32_t cannot hold 10B keys).
#pragma once
#include <atomic>
#include <chrono>
#include <cstdarg>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <mutex>
#include <sstream>
#include <stdexcept>
#include <string>

namespace ss {

using key_t = uint64_t;
using index_t = uint32_t;

struct Error : std::runtime_error {
  using std::runtime_error::runtime_error;
};

namespace detail {
[[noreturn]] inline void fail(const char* file, int line, const std::string& msg) {
  std::ostringstream os;
  os << file << ":" << line << ": " << msg;
  throw Error(os.str());
}
}  // namespace detail

#define SS_CHECK(cond)                                                    \
  do {                                                                    \
    if (!(cond)) ::ss::detail::fail(__FILE__, __LINE__, "check failed: " #cond); \
  } while (0)

#define SS_CHECK_MSG(cond, msg)                                           \
  do {                                                                    \
    if (!(cond)) {                                                        \
      std::ostringstream _ss_os;                                          \
      _ss_os << "check failed: " #cond " — " << msg;                      \
      ::ss::detail::fail(__FILE__, __LINE__, _ss_os.str());               \
    }                                                                     \
  } while (0)

// ------------------------------------------------------------------ logging
enum class LogLevel : int { kDebug = 0, kInfo = 1, kWarning = 2, kError = 3 };

inline std::atomic<int>& log_level_ref() {
  static std::atomic<int> lvl{[] {
    const char* e = std::getenv("SS_LOG_LEVEL");
    return e ? std::atoi(e) : (int)LogLevel::kWarning;
  }()};
  return lvl;
}
inline std::mutex& log_mutex() {
  static std::mutex m;
  return m;
}

inline void logf(LogLevel lvl, const char* fmt, ...) {
  if ((int)lvl < log_level_ref().load()) return;
  static const char* tag = "DIWE";
  char buf[2048];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  const double t = std::chrono::duration<double>(
                       std::chrono::steady_clock::now().time_since_epoch())
                       .count();
  std::lock_guard<std::mutex> lk(log_mutex());
  std::fprintf(stderr, "%c %.6f ss] %s\n", tag[(int)lvl], t, buf);
}

#define SS_LOG_DEBUG(...) ::ss::logf(::ss::LogLevel::kDebug, __VA_ARGS__)
#define SS_LOG_INFO(...) ::ss::logf(::ss::LogLevel::kInfo, __VA_ARGS__)
#define SS_LOG_WARN(...) ::ss::logf(::ss::LogLevel::kWarning, __VA_ARGS__)
#define SS_LOG_ERROR(...) ::ss::logf(::ss::LogLevel::kError, __VA_ARGS__)

// Non-copyable base (reference VirtualObject, utils/VirtualObject.h:14-20).
struct NonCopyable {
  NonCopyable() = default;
  NonCopyable(const NonCopyable&) = delete;
  NonCopyable& operator=(const NonCopyable&) = delete;
};

// Wall timer (reference Timer, utils/Timer.h:14-44 truncates to whole
// seconds; this one keeps sub-microsecond resolution).
class Timer {
 public:
  Timer() { reset(); }
  void reset() { t0_ = std::chrono::steady_clock::now(); }
  double elapsed() const {
    return std::chrono::duration<double>(std::chrono::steady_clock::now() - t0_).count();
  }
  bool timeout(double span_s) const { return elapsed() > span_s; }

 private:
  std::chrono::steady_clock::time_point t0_;
};

}  // namespace ss
