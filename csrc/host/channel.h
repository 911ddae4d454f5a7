// channel.h — closeable MPMC channel, thread pool, barriers, spin lock.
//
// Reference: core/BasicChannel.h:37-112 (channel), core/AsynExec.h:38-148
// (thread pool fed by a channel, `async_exec(n, task)`), utils/Barrier.h:79-135
// (StateBarrier with a watchdog, CounterBarrier), utils/SpinLock.h:42-53,
// utils/queue.h (threadsafe_queue / queue_with_capacity).
//
// Fixes of known reference defects:
//   * Channel::pop drains queued items before reporting closed (the
//     reference drops them, BasicChannel.h:46-53);
//   * StateBarrier notifies under the mutex (no lost wake-ups, Barrier.h:103)
//     and its timeout is a bounded wait, not a detached watchdog thread that
//     captures `this` (Barrier.h:90-101).
#pragma once
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <deque>
#include <functional>
#include <memory>
#include <mutex>
#include <optional>
#include <thread>
#include <vector>

#include "common.h"

namespace ss {

template <typename T>
class Channel : NonCopyable {
 public:
  explicit Channel(size_t capacity = 0) : cap_(capacity) {}

  // false if the channel is closed
  bool push(T v) {
    std::unique_lock<std::mutex> lk(mu_);
    not_full_.wait(lk, [&] { return closed_ || cap_ == 0 || q_.size() < cap_; });
    if (closed_) return false;
    q_.push_back(std::move(v));
    not_empty_.notify_one();
    return true;
  }
  // blocks until an item is available; false once closed AND drained
  bool pop(T& out) {
    std::unique_lock<std::mutex> lk(mu_);
    not_empty_.wait(lk, [&] { return closed_ || !q_.empty(); });
    if (q_.empty()) return false;
    out = std::move(q_.front());
    q_.pop_front();
    not_full_.notify_one();
    return true;
  }
  bool try_pop(T& out) {
    std::lock_guard<std::mutex> lk(mu_);
    if (q_.empty()) return false;
    out = std::move(q_.front());
    q_.pop_front();
    not_full_.notify_one();
    return true;
  }
  template <class Rep, class Per>
  bool pop_for(T& out, std::chrono::duration<Rep, Per> d) {
    std::unique_lock<std::mutex> lk(mu_);
    if (!not_empty_.wait_for(lk, d, [&] { return closed_ || !q_.empty(); })) return false;
    if (q_.empty()) return false;
    out = std::move(q_.front());
    q_.pop_front();
    not_full_.notify_one();
    return true;
  }
  void close() {
    std::lock_guard<std::mutex> lk(mu_);
    closed_ = true;
    not_empty_.notify_all();
    not_full_.notify_all();
  }
  bool closed() const {
    std::lock_guard<std::mutex> lk(mu_);
    return closed_;
  }
  size_t size() const {
    std::lock_guard<std::mutex> lk(mu_);
    return q_.size();
  }
  bool empty() const { return size() == 0; }

 private:
  mutable std::mutex mu_;
  std::condition_variable not_empty_, not_full_;
  std::deque<T> q_;
  size_t cap_;
  bool closed_ = false;
};

// Fixed-size worker pool draining a task channel (reference AsynExec).
class ThreadPool : NonCopyable {
 public:
  using Task = std::function<void()>;
  explicit ThreadPool(int nthreads) {
    SS_CHECK(nthreads > 0);
    for (int i = 0; i < nthreads; ++i)
      threads_.emplace_back([this] {
        Task t;
        while (ch_.pop(t)) {
          try {
            t();
          } catch (const std::exception& e) {
            SS_LOG_ERROR("ThreadPool task threw: %s", e.what());
          }
          pending_.fetch_sub(1);
          {
            std::lock_guard<std::mutex> lk(idle_mu_);
          }
          idle_cv_.notify_all();
        }
      });
  }
  ~ThreadPool() { stop(); }
  bool submit(Task t) {
    pending_.fetch_add(1);
    if (!ch_.push(std::move(t))) {
      pending_.fetch_sub(1);
      return false;
    }
    return true;
  }
  // run `task(i)` for i in [0, n) on the pool and wait (AsynExec::async_exec)
  void parallel_for(int n, const std::function<void(int)>& task) {
    if (n <= 0) return;
    std::atomic<int> left{n};
    std::mutex mu;
    std::condition_variable cv;
    // the count drops under the mutex: the waiter can only see it reach 0
    // after the last task released the lock, so it never destroys `mu`/`cv`
    // (this frame) while a task still uses them
    for (int i = 0; i < n; ++i)
      submit([&, i] {
        task(i);
        std::lock_guard<std::mutex> lk(mu);
        if (left.fetch_sub(1) == 1) cv.notify_all();
      });
    std::unique_lock<std::mutex> lk(mu);
    cv.wait(lk, [&] { return left.load() == 0; });
  }
  void wait_idle() {
    std::unique_lock<std::mutex> lk(idle_mu_);
    idle_cv_.wait(lk, [&] { return pending_.load() == 0; });
  }
  void stop() {
    ch_.close();
    for (auto& t : threads_)
      if (t.joinable()) t.join();
    threads_.clear();
  }
  int size() const { return (int)threads_.size(); }

 private:
  Channel<Task> ch_;
  std::vector<std::thread> threads_;
  std::atomic<int> pending_{0};
  std::mutex idle_mu_;
  std::condition_variable idle_cv_;
};

// Barrier that opens when its state is set valid (reference StateBarrier).
class StateBarrier : NonCopyable {
 public:
  void set_state_valid() {
    std::lock_guard<std::mutex> lk(mu_);
    valid_ = true;
    cv_.notify_all();
  }
  void reset() {
    std::lock_guard<std::mutex> lk(mu_);
    valid_ = false;
  }
  void block() {
    std::unique_lock<std::mutex> lk(mu_);
    cv_.wait(lk, [&] { return valid_; });
  }
  // false on timeout (the reference aborts the process from a watchdog)
  bool block_for(double seconds) {
    std::unique_lock<std::mutex> lk(mu_);
    return cv_.wait_for(lk, std::chrono::duration<double>(seconds), [&] { return valid_; });
  }
  bool valid() const {
    std::lock_guard<std::mutex> lk(mu_);
    return valid_;
  }

 private:
  mutable std::mutex mu_;
  std::condition_variable cv_;
  bool valid_ = false;
};

// Count-down latch (reference CounterBarrier / the pull/push response countdown).
class CountDownLatch : NonCopyable {
 public:
  explicit CountDownLatch(long n = 0) : n_(n) {}
  void add(long k) {
    std::lock_guard<std::mutex> lk(mu_);
    n_ += k;
  }
  void count_down() {
    std::lock_guard<std::mutex> lk(mu_);
    if (n_ > 0 && --n_ == 0) cv_.notify_all();
  }
  void wait() {
    std::unique_lock<std::mutex> lk(mu_);
    cv_.wait(lk, [&] { return n_ <= 0; });
  }
  bool wait_for(double s) {
    std::unique_lock<std::mutex> lk(mu_);
    return cv_.wait_for(lk, std::chrono::duration<double>(s), [&] { return n_ <= 0; });
  }
  long count() const {
    std::lock_guard<std::mutex> lk(mu_);
    return n_;
  }

 private:
  mutable std::mutex mu_;
  std::condition_variable cv_;
  long n_;
};

class SpinLock : NonCopyable {
 public:
  void lock() {
    while (f_.test_and_set(std::memory_order_acquire)) std::this_thread::yield();
  }
  bool try_lock() { return !f_.test_and_set(std::memory_order_acquire); }
  void unlock() { f_.clear(std::memory_order_release); }

 private:
  std::atomic_flag f_ = ATOMIC_FLAG_INIT;
};

}  // namespace ss
