// host_table.h — CPU sparse parameter table (server shard for CPU clusters and
// the reference-semantics CPU baseline; the GPU shard is csrc/hip/table.hip).
//
// Reference: SparseTable / SparseTableShard (core/parameter/sparsetable.h:5-121):
// `shard_num` lock-striped shards selected by fmix64(key) % shard_num
// (sparsetable.h:115), lookup-or-init on pull (:142-149), apply on push
// (:181-192), text dump `key\tvalue\n` (:49-56).
//
// Each shard is an open-addressed table (same probe function and the same
// init/optimizer code — ss/optim.h — as the HBM table) guarded by its own
// mutex; batch pull/push partition the keys by shard and process shards in
// parallel on a thread pool.  Unlike the reference, push updates hold the
// shard lock (no unlocked Hogwild writes, SURVEY §5 known defects).
#pragma once
#include <algorithm>
#include <cstring>
#include <thread>
#include <unordered_map>
#include <cstdio>
#include <fstream>
#include <memory>
#include <functional>
#include <mutex>
#include <string>
#include <vector>

#include "channel.h"
#include "common.h"
#include "ss/hash.h"
#include "ss/optim.h"
#include "string_util.h"

namespace ss {

class HostShard : NonCopyable {
 public:
  HostShard(int dim, int width, size_t cap) : dim_(dim), width_(width) { alloc(cap < 16 ? 16 : cap); }

  // returns row pointer; *inserted set when created
  float* find_or_insert(uint64_t key, const InitParams& ip, bool* inserted) {
    if ((size_ + 1) * 10 > cap_ * 7) grow();
    size_t s = fastrange64(table_hash(key), cap_);
    for (;;) {
      if (keys_[s] == key) return &rows_[s * width_];
      if (keys_[s] == kEmptyKey) {
        keys_[s] = key;
        ++size_;
        float* r = &rows_[s * width_];
        for (int j = 0; j < width_; ++j)
          r[j] = j < dim_ ? init_value(ip, key, (uint32_t)j, (uint32_t)dim_) : ip.state_init;
        if (inserted) *inserted = true;
        return r;
      }
      s = (s + 1 == cap_) ? 0 : s + 1;
    }
  }
  float* find(uint64_t key) {
    size_t s = fastrange64(table_hash(key), cap_);
    for (size_t n = 0; n < cap_; ++n) {
      if (keys_[s] == key) return &rows_[s * width_];
      if (keys_[s] == kEmptyKey) return nullptr;
      s = (s + 1 == cap_) ? 0 : s + 1;
    }
    return nullptr;
  }
  void assign(uint64_t key, const float* row) {
    float* r = find_or_insert(key, InitParams{kInitZero, 0.f, 0.f, 0, -1}, nullptr);
    std::copy(row, row + width_, r);
  }
  template <class F>
  void for_each(F&& f) const {
    for (size_t s = 0; s < cap_; ++s)
      if (keys_[s] != kEmptyKey) f(keys_[s], &rows_[s * width_]);
  }
  size_t size() const { return size_; }
  size_t capacity() const { return cap_; }
  std::mutex& mutex() { return mu_; }

 private:
  void alloc(size_t cap) {
    cap_ = cap;
    keys_.assign(cap, kEmptyKey);
    rows_.assign(cap * (size_t)width_, 0.f);
    size_ = 0;
  }
  void grow() {
    std::vector<uint64_t> ok;
    std::vector<float> orows;
    ok.swap(keys_);
    orows.swap(rows_);
    const size_t ocap = cap_;
    alloc(ocap * 2);
    for (size_t s = 0; s < ocap; ++s)
      if (ok[s] != kEmptyKey) {
        size_t t = fastrange64(table_hash(ok[s]), cap_);
        while (keys_[t] != kEmptyKey) t = (t + 1 == cap_) ? 0 : t + 1;
        keys_[t] = ok[s];
        std::copy(&orows[s * width_], &orows[s * width_] + width_, &rows_[t * width_]);
        ++size_;
      }
  }
  int dim_, width_;
  size_t cap_ = 0, size_ = 0;
  std::vector<uint64_t> keys_;
  std::vector<float> rows_;
  std::mutex mu_;
};

// Text checkpoint codec shared by the CPU table and the HBM table dump path
// (K8 host half: device compaction -> pinned D2H -> these formatters).
// Line format: "key\tv0 v1 ... v{dim-1}[ | s0 s1 ...]\n" (sparsetable.h:49-56;
// the optional " | state" tail makes a dump resumable).
inline void format_rows_into(std::string& o, const uint64_t* keys, const float* rows, size_t n,
                             int dim, int width, bool with_state, int precision) {
  char buf[64];
  const int w = with_state ? width : dim;
  for (size_t i = 0; i < n; ++i) {
    o += std::to_string(keys[i]);
    o += '\t';
    const float* r = rows + i * (size_t)width;
    for (int j = 0; j < w; ++j) {
      if (j) o += (with_state && j == dim) ? " | " : " ";
      const int len = std::snprintf(buf, sizeof(buf), "%.*g", precision, (double)r[j]);
      o.append(buf, (size_t)len);
    }
    o += '\n';
  }
}

inline std::string format_rows(const uint64_t* keys, const float* rows, size_t n, int dim,
                               int width, bool with_state, int precision, int nthreads = 8) {
  nthreads = std::max(1, std::min(nthreads, (int)(n / 4096) + 1));
  std::vector<std::string> parts((size_t)nthreads);
  std::vector<std::thread> th;
  const size_t per = (n + nthreads - 1) / nthreads;
  for (int t = 0; t < nthreads; ++t)
    th.emplace_back([&, t] {
      const size_t a = std::min(n, per * t), b = std::min(n, per * (t + 1));
      parts[t].reserve((b - a) * (size_t)(12 + 12 * (with_state ? width : dim)));
      format_rows_into(parts[t], keys + a, rows + a * (size_t)width, b - a, dim, width,
                       with_state, precision);
    });
  for (auto& x : th) x.join();
  std::string out;
  size_t tot = 0;
  for (auto& p : parts) tot += p.size();
  out.reserve(tot);
  for (auto& p : parts) out += p;
  return out;
}

// Parses one checkpoint line into (key, row[width]); missing state floats
// are left as given in `row` (caller pre-fills state_init).
inline bool parse_row_line(const char* p, int dim, int width, uint64_t* key, float* row) {
  char* e = nullptr;
  *key = std::strtoull(p, &e, 10);
  if (e == p || *e != '\t') return false;
  p = e + 1;
  if (std::strncmp(p, "Vec:", 4) == 0) p += 4;
  int j = 0;
  bool in_state = false;
  while (*p) {
    while (*p == ' ' || *p == '\t') ++p;
    if (!*p || *p == '\n') break;
    if (*p == '|') {
      in_state = true;
      j = dim;
      ++p;
      continue;
    }
    const float v = std::strtof(p, &e);
    if (e == p) return false;
    if (j < width && (in_state || j < dim)) row[j] = v;
    ++j;
    p = e;
  }
  return true;
}

class HostTable : NonCopyable {
 public:
  HostTable(int dim, int shard_num, InitParams ip, OptParams op, int nthreads = 0,
            size_t cap_per_shard = 1024)
      : dim_(dim), width_(dim + opt_state_width(op.kind, dim)), ip_(ip), op_(op) {
    SS_CHECK(dim > 0 && shard_num > 0);
    for (int i = 0; i < shard_num; ++i)
      shards_.emplace_back(new HostShard(dim_, width_, cap_per_shard));
    if (nthreads <= 0) nthreads = std::max(1u, std::min(8u, std::thread::hardware_concurrency()));
    pool_.reset(new ThreadPool(nthreads));
  }

  int dim() const { return dim_; }
  int width() const { return width_; }
  int shard_num() const { return (int)shards_.size(); }
  int to_shard_id(uint64_t key) const { return (int)(fmix64(key) % (uint64_t)shards_.size()); }
  void set_opt(const OptParams& op) {
    SS_CHECK_MSG(dim_ + opt_state_width(op.kind, dim_) == width_, "optimizer state width differs");
    op_ = op;
  }
  const OptParams& opt() const { return op_; }

  // User-defined access methods, the reference's PullAccessMethod::init_param
  // and PushAccessMethod::apply_push_value (sparse_access_method.h:10-48):
  // `init(key, row, dim, width)` fills a new key's row (params, then
  // `width - dim` optimizer-state floats) after the built-in init rule,
  // `apply(key, row, grad, dim, width)` updates a row in place.  Both run per
  // key under the key's shard lock.  Empty functions restore the built-ins.
  using InitFn = std::function<void(uint64_t key, float* row, int dim, int width)>;
  using ApplyFn =
      std::function<void(uint64_t key, float* row, const float* grad, int dim, int width)>;
  // Batch form for interpreted callers (Python): the rows of a whole push,
  // gathered to rows[n][width], updated in place, written back.  Runs on the
  // pushing thread outside the shard locks, so concurrent pushes of the same
  // key may lose an update (the reference applies without a lock at all,
  // sparsetable.h:181-192).
  using BatchApplyFn =
      std::function<void(const uint64_t* keys, size_t n, float* rows, const float* grads)>;
  void set_access_methods(InitFn init, ApplyFn apply) {
    init_fn_ = std::move(init);
    apply_fn_ = std::move(apply);
  }
  void set_batch_apply(BatchApplyFn f) { batch_fn_ = std::move(f); }

  // lookup-or-init + gather (reference get_pull_value)
  void pull(const uint64_t* keys, size_t n, float* out) {
    run_sharded(keys, n, [&](HostShard& sh, size_t i) {
      const float* r = row_of(sh, keys[i]);
      std::copy(r, r + dim_, out + i * dim_);
    });
  }
  // apply (reference apply_push_value); missing keys are created first.
  // Duplicate keys in one call are applied sequentially under the shard lock.
  void push(const uint64_t* keys, size_t n, const float* grads) {
    if (batch_fn_) {
      // the rule sees each key once: duplicates are merged (gradients summed,
      // the reference's merge_push_value, sparse_access_method.h:39-40) —
      // each copy would otherwise start from the same row and the last
      // write-back would drop the others' updates
      std::unordered_map<uint64_t, size_t> first;
      first.reserve(n * 2);
      std::vector<uint64_t> ukeys;
      std::vector<float> ugrads;
      ukeys.reserve(n);
      ugrads.reserve(n * (size_t)dim_);
      for (size_t i = 0; i < n; ++i) {
        auto it = first.emplace(keys[i], ukeys.size());
        const float* g = grads + i * (size_t)dim_;
        if (it.second) {
          ukeys.push_back(keys[i]);
          ugrads.insert(ugrads.end(), g, g + dim_);
        } else {
          float* acc = ugrads.data() + it.first->second * (size_t)dim_;
          for (int j = 0; j < dim_; ++j) acc[j] += g[j];
        }
      }
      const size_t u = ukeys.size();
      std::vector<float> rows(u * (size_t)width_);
      run_sharded(ukeys.data(), u, [&](HostShard& sh, size_t i) {
        const float* r = row_of(sh, ukeys[i]);
        std::copy(r, r + width_, rows.data() + i * width_);
      });
      batch_fn_(ukeys.data(), u, rows.data(), ugrads.data());
      assign(ukeys.data(), u, rows.data());
      return;
    }
    run_sharded(keys, n, [&](HostShard& sh, size_t i) {
      float* r = row_of(sh, keys[i]);
      if (apply_fn_) {
        apply_fn_(keys[i], r, grads + i * dim_, dim_, width_);
        return;
      }
      for (int j = 0; j < dim_; ++j) opt_apply(op_, r, r + dim_, dim_, j, grads[i * dim_ + j]);
    });
  }
  void assign(const uint64_t* keys, size_t n, const float* rows) {
    run_sharded(keys, n, [&](HostShard& sh, size_t i) { sh.assign(keys[i], rows + i * width_); });
  }
  // full rows (params + state) of existing keys; missing -> false in found
  void get_rows(const uint64_t* keys, size_t n, float* rows, uint8_t* found) {
    run_sharded(keys, n, [&](HostShard& sh, size_t i) {
      const float* r = sh.find(keys[i]);
      found[i] = r != nullptr;
      if (r) std::copy(r, r + width_, rows + i * width_);
      else std::fill(rows + i * width_, rows + (i + 1) * width_, 0.f);
    });
  }
  size_t size() {
    size_t s = 0;
    for (auto& sh : shards_) {
      std::lock_guard<std::mutex> lk(sh->mutex());
      s += sh->size();
    }
    return s;
  }
  void export_all(std::vector<uint64_t>& keys, std::vector<float>& rows) {
    keys.clear();
    rows.clear();
    for (auto& sh : shards_) {
      std::lock_guard<std::mutex> lk(sh->mutex());
      sh->for_each([&](uint64_t k, const float* r) {
        keys.push_back(k);
        rows.insert(rows.end(), r, r + width_);
      });
    }
  }

  // Text checkpoint: "key\tv0 v1 ...\n" per key (sparsetable.h:49-56), shards
  // formatted in parallel.  with_state appends optimizer state after a '|'.
  size_t write_text(const std::string& path, int precision = 9, bool with_state = false) {
    std::vector<std::string> parts(shards_.size());
    pool_->parallel_for((int)shards_.size(), [&](int s) {
      auto& sh = *shards_[s];
      std::lock_guard<std::mutex> lk(sh.mutex());
      std::string& o = parts[s];
      char buf[64];
      sh.for_each([&](uint64_t k, const float* r) {
        o += std::to_string(k);
        o += '\t';
        const int w = with_state ? width_ : dim_;
        for (int j = 0; j < w; ++j) {
          if (j) o += (with_state && j == dim_) ? " | " : " ";
          const int len = std::snprintf(buf, sizeof(buf), "%.*g", precision, (double)r[j]);
          o.append(buf, (size_t)len);
        }
        o += '\n';
      });
    });
    FILE* f = path == "-" ? stdout : std::fopen(path.c_str(), "w");
    SS_CHECK_MSG(f, "cannot open " << path);
    size_t bytes = 0;
    for (auto& p : parts) bytes += std::fwrite(p.data(), 1, p.size(), f);
    if (f != stdout) std::fclose(f);
    else std::fflush(f);
    return bytes;
  }
  // Loads "key\tv..." (optionally "Vec:\t" prefixed values and " | state").
  size_t load_text(const std::string& path) {
    std::ifstream in(path);
    SS_CHECK_MSG((bool)in, "cannot open " << path);
    std::vector<uint64_t> keys;
    std::vector<float> rows;
    std::string line;
    std::vector<float> row((size_t)width_);
    while (std::getline(in, line)) {
      if (line.empty()) continue;
      const size_t tab = line.find('\t');
      SS_CHECK_MSG(tab != std::string::npos, "bad checkpoint line: " << line);
      keys.push_back(std::stoull(line.substr(0, tab)));
      std::fill(row.begin(), row.end(), 0.f);
      for (int j = dim_; j < width_; ++j) row[j] = ip_.state_init;
      const char* p = line.c_str() + tab + 1;
      if (std::strncmp(p, "Vec:", 4) == 0) p += 4;
      int j = 0;
      bool in_state = false;
      while (*p) {
        while (*p == ' ' || *p == '\t') ++p;
        if (!*p) break;
        if (*p == '|') {
          in_state = true;
          j = dim_;
          ++p;
          continue;
        }
        char* e = nullptr;
        const float v = std::strtof(p, &e);
        SS_CHECK_MSG(e != p, "bad number in: " << line);
        if (j < width_ && (in_state || j < dim_)) row[j] = v;
        ++j;
        p = e;
      }
      rows.insert(rows.end(), row.begin(), row.end());
    }
    assign(keys.data(), keys.size(), rows.data());
    return keys.size();
  }

 private:
  template <class F>
  void run_sharded(const uint64_t* keys, size_t n, F&& f) {
    const int S = (int)shards_.size();
    std::vector<std::vector<uint32_t>> buckets((size_t)S);
    for (size_t i = 0; i < n; ++i) buckets[to_shard_id(keys[i])].push_back((uint32_t)i);
    auto work = [&](int s) {
      if (buckets[s].empty()) return;
      auto& sh = *shards_[s];
      std::lock_guard<std::mutex> lk(sh.mutex());
      for (uint32_t i : buckets[s]) f(sh, i);
    };
    if (n < 4096 || S == 1) {
      for (int s = 0; s < S; ++s) work(s);
    } else {
      pool_->parallel_for(S, work);
    }
  }

  // lookup-or-init of one key (shard lock held), with the user init method
  float* row_of(HostShard& sh, uint64_t key) {
    bool inserted = false;
    float* r = sh.find_or_insert(key, ip_, &inserted);
    if (inserted && init_fn_) init_fn_(key, r, dim_, width_);
    return r;
  }

  int dim_, width_;
  InitParams ip_;
  OptParams op_;
  InitFn init_fn_;
  ApplyFn apply_fn_;
  BatchApplyFn batch_fn_;
  std::vector<std::unique_ptr<HostShard>> shards_;
  std::unique_ptr<ThreadPool> pool_;
};

}  // namespace ss
