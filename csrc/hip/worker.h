// worker.h — native (C++) GPU worker API: pull(keys) / push(keys, grads) on
// one MI355X's HBM table, with asynchronous handles.
//
// The reference's worker talks to the servers through
// GlobalPullAccess::pull_with_barrier / GlobalPushAccess::push_with_barrier
// (/root/reference/src/core/parameter/global_pull_access.h:40-120,
// global_push_access.h:36-149): group keys per server, send, block on a
// StateBarrier until every response arrived, values land in the worker's
// GlobalParamCache.  Here a C++ program drives the same two calls against a
// device table without Python:
//
//   ss::GpuWorker w(table, size_ctr, err, init, opt, G, max_keys);
//   ss::Handle h = w.pull(keys_dev, n, vals_dev, stream);  // dedup -> lookup-or-init -> gather
//   ...compute grads on the stream...
//   w.push(keys_dev, n, grads_dev, stream).wait();         // dedup -> merge -> optimizer update
//
// Each call is enqueued on `stream` and returns at once; Handle::wait()
// blocks on a HIP event (the StateBarrier of the reference).  Duplicate keys
// in a call are merged first (one table probe and one update per unique key),
// so a push applies the SUM of a key's gradients once, like the reference's
// merge_push_value (sparse_access_method.h:39-40).  The multi-GPU round
// engine (RCCL all-to-all-v, pull-ahead) is swiftsnails_amd.parallel.PSEngine.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <memory>

#include "ss_device.h"
#include "ss_launch.h"

namespace ss {

// Completion of one enqueued pull / push (an event recorded behind its work).
class Handle {
 public:
  Handle() = default;
  explicit Handle(hipStream_t st);
  bool done() const;  // non-blocking query
  void wait() const;  // block the host until the call's kernels finished
 private:
  std::shared_ptr<void> ev_;  // hipEvent_t, destroyed with the last copy
};

class GpuWorker {
 public:
  // `t` views a table whose storage, size counter and error word live on the
  // device (HbmTable allocates them); `max_keys` bounds n per call.
  GpuWorker(const DevTable& t, unsigned long long* size_ctr, int* err, const InitParams& init,
            const OptParams& opt, int G, long long max_keys);
  ~GpuWorker();
  GpuWorker(const GpuWorker&) = delete;
  GpuWorker& operator=(const GpuWorker&) = delete;

  // vals[n][dim] <- rows of keys[n] (missing keys are inserted and
  // initialised), in occurrence order
  Handle pull(const uint64_t* keys, long long n, float* vals, hipStream_t st);
  // optimizer update with the per-key sum of grads[n][dim] (keys inserted if
  // missing)
  Handle push(const uint64_t* keys, long long n, const float* grads, hipStream_t st);
  // unique keys of the last call (device count, valid once its handle is done)
  const unsigned long long* unique_count() const { return ucount_; }
  long long max_keys() const { return max_keys_; }

 private:
  void dedup(const uint64_t* keys, long long n, hipStream_t st);

  DevTable t_;
  unsigned long long* size_ctr_;
  int* err_;
  InitParams init_;
  OptParams opt_;
  int G_;
  long long max_keys_;
  // dedup scratch (hash mode, one destination)
  unsigned long long scap_ = 0;
  uint64_t* skeys_ = nullptr;
  uint32_t* stag_ = nullptr;
  uint32_t* slot_of_ = nullptr;
  uint32_t* blk_cnt_ = nullptr;
  int* frag_map_ = nullptr;
  bool scratch_dirty_ = true;
  // per-call results
  uint32_t* inv_ = nullptr;             // occurrence -> unique id
  uint64_t* ukeys_ = nullptr;           // unique keys
  unsigned long long* ucount_ = nullptr;
  long long* slots_ = nullptr;          // table slot of each unique key
  float* urows_ = nullptr;              // [max_keys][dim] unique rows / merged grads
};

}  // namespace ss
