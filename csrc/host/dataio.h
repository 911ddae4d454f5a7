// dataio.h — native training-data input: parallel line scanning, sparse CTR
// datasets (libsvm / categorical TSV) and a word2vec corpus + skip-gram batch
// sampler.
//
// Reference: the reference's apps read their data through
// `scan_file_by_line(FILE*, mutex, handler)` (utils/file.h:14-33: N threads
// pull lines from ONE FILE* under a mutex) and `LineFileReader`
// (utils/string.h:89-114), with `BaseAlgorithm::parse_record(line)` as the
// app hook (core/framework/SwiftWorker.h:19-30); the word2vec corpus format is
// the one written by src/tools/gen-word2vec-data.py (one sentence of
// integer word ids per line).
//
// Here the file is memory-mapped and cut into byte ranges aligned to line
// starts, so N threads parse disjoint ranges with no shared lock; a rank of a
// W-rank job keeps only its own contiguous share of the ranges (data
// parallelism).  Batches come out in exactly the layouts the GPU
// kernels consume (B x F padded key rows; the k_w2v_gen key layout) and are
// filled by native threads with the GIL released, so Python only schedules
// prefetch and the H2D copy.
#pragma once
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <string>
#include <thread>
#include <unordered_map>
#include <utility>
#include <vector>

#include "common.h"
#include "ss/hash.h"
#include "ss/w2v_window.h"

namespace ss {

static constexpr uint64_t kDataEmptyKey = ~0ull;

// Read-only memory map of a whole file.
class MappedFile : NonCopyable {
 public:
  explicit MappedFile(const std::string& path) {
    fd_ = ::open(path.c_str(), O_RDONLY);
    SS_CHECK_MSG(fd_ >= 0, "cannot open data file " << path);
    struct stat st;
    SS_CHECK(::fstat(fd_, &st) == 0);
    size_ = (size_t)st.st_size;
    if (size_ > 0) {
      void* p = ::mmap(nullptr, size_, PROT_READ, MAP_PRIVATE, fd_, 0);
      SS_CHECK_MSG(p != MAP_FAILED, "mmap failed for " << path);
      data_ = static_cast<const char*>(p);
      ::madvise(p, size_, MADV_SEQUENTIAL);
    }
  }
  ~MappedFile() {
    if (data_) ::munmap(const_cast<char*>(data_), size_);
    if (fd_ >= 0) ::close(fd_);
  }
  const char* data() const { return data_; }
  size_t size() const { return size_; }

 private:
  int fd_ = -1;
  const char* data_ = nullptr;
  size_t size_ = 0;
};

// Byte ranges [b, e) over `size` bytes, each starting at a line start.
inline std::vector<std::pair<size_t, size_t>> line_ranges(const char* d, size_t size, int nparts) {
  nparts = std::max(1, nparts);
  std::vector<size_t> cut(nparts + 1, size);
  cut[0] = 0;
  for (int i = 1; i < nparts; ++i) {
    size_t p = std::max(cut[i - 1], size * (size_t)i / (size_t)nparts);
    while (p < size && p > 0 && d[p - 1] != '\n') ++p;
    cut[i] = p;
  }
  std::vector<std::pair<size_t, size_t>> r;
  for (int i = 0; i < nparts; ++i) r.emplace_back(cut[i], cut[i + 1]);
  return r;
}

// Parallel line scan of this shard's part of the file: on_line(thread, ptr, len)
// (no trailing newline / carriage return).  Shard s of nshards gets the s-th
// contiguous 1/nshards of the bytes (line aligned).
inline void scan_lines_parallel(const MappedFile& f, int nthreads, int shard, int nshards,
                                const std::function<void(int, const char*, size_t)>& on_line) {
  SS_CHECK(nshards >= 1 && shard >= 0 && shard < nshards);
  const auto shards = line_ranges(f.data(), f.size(), nshards);
  const size_t b0 = shards[shard].first, e0 = shards[shard].second;
  nthreads = std::max(1, nthreads);
  const auto parts = line_ranges(f.data() + b0, e0 - b0, nthreads);
  std::vector<std::thread> th;
  for (int t = 0; t < nthreads; ++t) {
    th.emplace_back([&, t] {
      const char* d = f.data() + b0;
      size_t p = parts[t].first;
      const size_t e = parts[t].second;
      while (p < e) {
        const char* nl = static_cast<const char*>(std::memchr(d + p, '\n', e - p));
        size_t q = nl ? (size_t)(nl - d) : e;
        size_t len = q - p;
        if (len && d[p + len - 1] == '\r') --len;
        if (len) on_line(t, d + p, len);
        p = q + 1;
      }
    });
  }
  for (auto& x : th) x.join();
}

// ---- token helpers (no allocation)
inline bool next_token(const char*& p, const char* e, const char*& tb, const char*& te,
                       const char* delims) {
  while (p < e && std::strchr(delims, *p)) ++p;
  if (p >= e) return false;
  tb = p;
  while (p < e && !std::strchr(delims, *p)) ++p;
  te = p;
  return true;
}
inline uint64_t hash_bytes(const char* b, const char* e) {  // FNV-1a then fmix64
  uint64_t h = 1469598103934665603ull;
  for (const char* p = b; p < e; ++p) h = (h ^ (uint8_t)*p) * 1099511628211ull;
  return fmix64(h);
}
inline bool parse_u64(const char* b, const char* e, uint64_t& v) {
  if (b == e) return false;
  uint64_t x = 0;
  for (const char* p = b; p < e; ++p) {
    if (*p < '0' || *p > '9') return false;
    x = x * 10 + (uint64_t)(*p - '0');
  }
  v = x;
  return true;
}
inline float parse_f32(const char* b, const char* e) {
  char buf[64];
  const size_t n = std::min<size_t>((size_t)(e - b), sizeof(buf) - 1);
  std::memcpy(buf, b, n);
  buf[n] = 0;
  return std::strtof(buf, nullptr);
}

// ---------------------------------------------------------------- sparse CTR
// CSR rows of (key, value) with a label.  Formats:
//   "libsvm": label idx[:val] idx[:val] ...        (key = idx)
//   "ctr":    label<TAB>tok1<TAB>tok2 ...  categorical fields; key =
//             (field << 48) | (hash(token) & (2^48-1)), empty tokens skipped
//             (Criteo-style; numeric columns are treated as tokens too).
// Labels <= 0 map to 0, > 0 to 1.
class SparseDataset : NonCopyable {
 public:
  SparseDataset(const std::string& path, const std::string& format, int nthreads, int shard,
                int nshards) {
    SS_CHECK_MSG(format == "libsvm" || format == "ctr", "unknown sparse format " << format);
    const bool libsvm = format == "libsvm";
    MappedFile f(path);
    nthreads = std::max(1, nthreads);
    struct Part {
      std::vector<float> labels, vals;
      std::vector<uint64_t> keys;
      std::vector<uint32_t> lens;
    };
    std::vector<Part> parts(nthreads);
    scan_lines_parallel(f, nthreads, shard, nshards, [&](int t, const char* s, size_t n) {
      Part& P = parts[t];
      const char* p = s;
      const char* e = s + n;
      const char *tb, *te;
      uint32_t len = 0;
      if (libsvm) {
        if (!next_token(p, e, tb, te, " \t")) return;
        P.labels.push_back(parse_f32(tb, te) > 0.f ? 1.f : 0.f);
        while (next_token(p, e, tb, te, " \t")) {
          const char* colon = static_cast<const char*>(std::memchr(tb, ':', (size_t)(te - tb)));
          uint64_t idx;
          if (!parse_u64(tb, colon ? colon : te, idx)) continue;
          P.keys.push_back(idx);
          P.vals.push_back(colon ? parse_f32(colon + 1, te) : 1.f);
          ++len;
        }
      } else {
        // label<TAB>col1<TAB>col2...: column i is field i (empty = missing)
        const char* tab = static_cast<const char*>(std::memchr(p, '\t', n));
        P.labels.push_back(parse_f32(p, tab ? tab : e) > 0.f ? 1.f : 0.f);
        uint64_t field = 0;
        while (tab) {
          const char* q = tab + 1;
          tab = static_cast<const char*>(std::memchr(q, '\t', (size_t)(e - q)));
          const char* ce = tab ? tab : e;
          if (ce > q) {
            P.keys.push_back((field << 48) | (hash_bytes(q, ce) & ((1ull << 48) - 1)));
            P.vals.push_back(1.f);
            ++len;
          }
          ++field;
        }
      }
      P.lens.push_back(len);
    });
    size_t rows = 0, nnz = 0;
    for (auto& P : parts) {
      rows += P.labels.size();
      nnz += P.keys.size();
    }
    labels_.reserve(rows);
    keys_.reserve(nnz);
    vals_.reserve(nnz);
    offs_.reserve(rows + 1);
    offs_.push_back(0);
    for (auto& P : parts) {
      labels_.insert(labels_.end(), P.labels.begin(), P.labels.end());
      keys_.insert(keys_.end(), P.keys.begin(), P.keys.end());
      vals_.insert(vals_.end(), P.vals.begin(), P.vals.end());
      for (uint32_t l : P.lens) {
        offs_.push_back(offs_.back() + l);
        max_nnz_ = std::max<size_t>(max_nnz_, l);
      }
    }
    for (float v : vals_)
      if (v != 1.f) {
        has_values_ = true;
        break;
      }
  }

  size_t rows() const { return labels_.size(); }
  size_t nnz() const { return keys_.size(); }
  size_t max_nnz() const { return max_nnz_; }
  bool has_values() const { return has_values_; }

  // Fill B rows starting at `cursor` (wrapping around) into B x F key/value
  // rows (short rows padded with the EMPTY key and value 0, long rows
  // truncated) + labels.  Returns the next cursor.  Thread-parallel.
  uint64_t fill(uint64_t cursor, int B, int F, uint64_t* keys, float* vals, float* labels,
                int nthreads) const {
    const size_t R = rows();
    SS_CHECK_MSG(R > 0, "empty dataset shard");
    nthreads = std::max(1, std::min(nthreads, B / 1024 + 1));
    auto work = [&](int t) {
      const int b0 = (int)((long long)B * t / nthreads), b1 = (int)((long long)B * (t + 1) / nthreads);
      for (int b = b0; b < b1; ++b) {
        const size_t r = (size_t)((cursor + (uint64_t)b) % R);
        const uint64_t o = offs_[r];
        const int len = (int)std::min<uint64_t>(offs_[r + 1] - o, (uint64_t)F);
        uint64_t* kr = keys + (size_t)b * F;
        for (int i = 0; i < len; ++i) kr[i] = keys_[o + i];
        for (int i = len; i < F; ++i) kr[i] = kDataEmptyKey;
        if (vals) {
          float* vr = vals + (size_t)b * F;
          for (int i = 0; i < len; ++i) vr[i] = vals_[o + i];
          for (int i = len; i < F; ++i) vr[i] = 0.f;
        }
        labels[b] = labels_[r];
      }
    };
    if (nthreads == 1) {
      work(0);
    } else {
      std::vector<std::thread> th;
      for (int t = 0; t < nthreads; ++t) th.emplace_back(work, t);
      for (auto& x : th) x.join();
    }
    return (cursor + (uint64_t)B) % R;
  }

  const std::vector<float>& labels() const { return labels_; }
  const std::vector<uint64_t>& keys() const { return keys_; }
  const std::vector<float>& vals() const { return vals_; }
  const std::vector<uint64_t>& offsets() const { return offs_; }

 private:
  std::vector<float> labels_, vals_;
  std::vector<uint64_t> keys_, offs_;
  size_t max_nnz_ = 0;
  bool has_values_ = false;
};

// ---------------------------------------------------------------- word2vec
// One sentence per line.  Integer tokens are word ids used as keys directly
// (the gen-word2vec-data.py corpus and the W2VSynth id space); any other
// token is hashed to a 40-bit key.  Words below min_count are dropped.
// Negatives come from the unigram^0.75 distribution (a 2^22-entry table),
// and frequent centers are sub-sampled with threshold `sample`
// (keep prob (sqrt(f/(s*T)) + 1) * s*T/f; 0 disables).
class Corpus : NonCopyable {
 public:
  static constexpr uint64_t kOutBit = 1ull << 40;

  Corpus(const std::string& path, int nthreads, int shard, int nshards, int min_count,
         double sample) {
    MappedFile f(path);
    nthreads = std::max(1, nthreads);
    std::vector<std::vector<uint64_t>> toks(nthreads);
    std::vector<std::vector<uint32_t>> lens(nthreads);
    scan_lines_parallel(f, nthreads, shard, nshards, [&](int t, const char* s, size_t n) {
      const char* p = s;
      const char* e = s + n;
      const char *tb, *te;
      uint32_t len = 0;
      while (next_token(p, e, tb, te, " \t")) {
        uint64_t v;
        if (!parse_u64(tb, te, v) || v >= kOutBit) v = hash_bytes(tb, te) & (kOutBit - 1);
        toks[t].push_back(v);
        ++len;
      }
      if (len) lens[t].push_back(len);
    });
    // global counts (per-thread maps merged)
    std::unordered_map<uint64_t, uint64_t> cnt;
    for (auto& v : toks)
      for (uint64_t k : v) ++cnt[k];
    // drop rare words, flatten
    sent_offs_.push_back(0);
    for (int t = 0; t < nthreads; ++t) {
      size_t p = 0;
      for (uint32_t l : lens[t]) {
        uint64_t kept = 0;
        for (uint32_t i = 0; i < l; ++i) {
          const uint64_t k = toks[t][p + i];
          if (cnt[k] >= (uint64_t)std::max(1, min_count)) {
            tokens_.push_back(k);
            ++kept;
          }
        }
        p += l;
        if (kept) sent_offs_.push_back(tokens_.size());
      }
      std::vector<uint64_t>().swap(toks[t]);
    }
    SS_CHECK_MSG(!tokens_.empty(), "empty corpus shard: " << path);
    sent_of_.resize(tokens_.size());
    for (size_t s = 0; s + 1 < sent_offs_.size(); ++s)
      for (uint64_t i = sent_offs_[s]; i < sent_offs_[s + 1]; ++i) sent_of_[i] = (uint32_t)s;
    // vocab + unigram^0.75 table + keep probabilities
    for (auto& kv : cnt)
      if (kv.second >= (uint64_t)std::max(1, min_count)) vocab_.push_back(kv);
    std::sort(vocab_.begin(), vocab_.end(),
              [](auto& a, auto& b) { return a.second != b.second ? a.second > b.second : a.first < b.first; });
    double z = 0;
    for (auto& kv : vocab_) z += std::pow((double)kv.second, 0.75);
    table_.resize(1u << 22);
    size_t w = 0;
    double acc = vocab_.empty() ? 1.0 : std::pow((double)vocab_[0].second, 0.75) / z;
    for (size_t i = 0; i < table_.size(); ++i) {
      table_[i] = vocab_[w].first;
      if ((double)(i + 1) / (double)table_.size() > acc && w + 1 < vocab_.size()) {
        ++w;
        acc += std::pow((double)vocab_[w].second, 0.75) / z;
      }
    }
    if (sample > 0) {
      const double T = (double)tokens_.size();
      for (auto& kv : vocab_) {
        const double fr = (double)kv.second;
        const double keep = (std::sqrt(fr / (sample * T)) + 1.0) * (sample * T) / fr;
        if (keep < 1.0) keep_[kv.first] = (float)keep;
      }
    }
  }

  size_t size() const { return tokens_.size(); }
  size_t sentences() const { return sent_offs_.size() - 1; }
  // the sampler's state, for an HBM-resident copy (csrc/hip/data.hip)
  const std::vector<uint64_t>& tokens() const { return tokens_; }
  const std::vector<uint64_t>& sent_offsets() const { return sent_offs_; }
  const std::vector<uint32_t>& sent_of() const { return sent_of_; }
  const std::vector<uint64_t>& noise_table() const { return table_; }
  bool subsampled() const { return !keep_.empty(); }
  // per-token keep probability of the frequent-word sub-sampling (2 = always
  // kept, as for words without an entry); empty without sub-sampling
  std::vector<float> keep_per_token() const {
    std::vector<float> k;
    if (keep_.empty()) return k;
    k.resize(tokens_.size(), 2.f);
    for (size_t i = 0; i < tokens_.size(); ++i) {
      auto it = keep_.find(tokens_[i]);
      if (it != keep_.end()) k[i] = it->second;
    }
    return k;
  }
  size_t vocab_size() const { return vocab_.size(); }
  const std::vector<std::pair<uint64_t, uint64_t>>& vocab() const { return vocab_; }

  // Skip-gram batch in the k_w2v_gen layout: keys[0,B) centers,
  // keys[B, B+B*C) contexts (| out bit), then nneg shared negatives (| out
  // bit).  Contexts are drawn from the center's sentence within +-W (with
  // replacement; a one-word sentence draws a noise word).  Deterministic in
  // (seed, step).
  // Windowed skip-gram run of `step` (layout: ss/w2v_window.h): keys =
  // [centers B][run positions B + 2W | out bit][negatives], meta per run
  // position.  Bit-identical to the resident device batcher
  // (k_w2v_corpus_window, csrc/hip/data.hip).
  void fill_skipgram_window(uint64_t seed, uint64_t step, int B, int W, long long nneg,
                            uint64_t* keys, int32_t* meta) const {
    const long long n = (long long)tokens_.size(), R = (long long)B + 2 * W;
    const uint64_t nsent = sent_offs_.empty() ? 0 : sent_offs_.size() - 1;
    const long long start = (long long)((step * (uint64_t)B) % (uint64_t)n) - W;
    for (long long i = 0; i < R; ++i) {
      const long long x = start + i;
      const long long lap = x >= 0 ? x / n : -((-x + n - 1) / n);
      const long long idx = x - lap * n;
      const uint64_t tok = tokens_[idx];
      int32_t m = w2v_meta((uint64_t)sent_of_[idx] + (uint64_t)(lap + 1) * nsent,
                           w2v_reduced_window(seed, (uint64_t)x, W));
      if (!keep_.empty()) {
        auto it = keep_.find(tok);
        if (it != keep_.end() && !w2v_keep(seed, step, (uint64_t)x, it->second)) m = -1;
      }
      keys[B + i] = tok | kOutBit;
      meta[i] = m;
      if (i >= W && i < W + B) keys[i - W] = tok;
    }
    for (long long q = 0; q < nneg; ++q) {
      const uint64_t r = splitmix64(seed ^ 0xBADC0DEull ^ (step * 0xD1B54A32D192ED03ull) ^ (uint64_t)q * 0x9E37ull);
      keys[(size_t)B + (size_t)R + q] = table_[r & (table_.size() - 1)] | kOutBit;
    }
  }

  void fill_skipgram(uint64_t seed, uint64_t step, int B, int C, int W, long long nneg,
                     uint64_t* keys, int nthreads) const {
    nthreads = std::max(1, std::min(nthreads, B / 512 + 1));
    const uint64_t N = tokens_.size();
    auto work = [&](int t) {
      const int b0 = (int)((long long)B * t / nthreads), b1 = (int)((long long)B * (t + 1) / nthreads);
      for (int b = b0; b < b1; ++b) {
        uint64_t r = splitmix64(seed ^ (step * 0x9E3779B97F4A7C15ull) ^ ((uint64_t)b << 20));
        uint64_t pos = 0;
        for (int tries = 0; tries < 16; ++tries) {  // frequent-word sub-sampling
          r = splitmix64(r);
          pos = fastrange64(r, N);
          if (keep_.empty()) break;
          auto it = keep_.find(tokens_[pos]);
          if (it == keep_.end() || u01(splitmix64(r ^ 7)) < it->second) break;
        }
        keys[b] = tokens_[pos];
        const uint32_t s = sent_of_[pos];
        const long long sb = (long long)sent_offs_[s], se = (long long)sent_offs_[s + 1];
        const long long lo = std::max(sb, (long long)pos - W), hi = std::min(se - 1, (long long)pos + W);
        const long long span = hi - lo;  // candidates excluding the center
        for (int c = 0; c < C; ++c) {
          r = splitmix64(r + (uint64_t)c);
          uint64_t x;
          if (span <= 0) {
            x = table_[r & (table_.size() - 1)];
          } else {
            long long q = lo + (long long)fastrange64(r, (uint64_t)span);
            if (q >= (long long)pos) ++q;
            x = tokens_[q];
          }
          keys[(size_t)B + (size_t)b * C + c] = x | kOutBit;
        }
      }
    };
    std::vector<std::thread> th;
    for (int t = 1; t < nthreads; ++t) th.emplace_back(work, t);
    work(0);
    for (auto& x : th) x.join();
    for (long long q = 0; q < nneg; ++q) {
      const uint64_t r = splitmix64(seed ^ 0xBADC0DEull ^ (step * 0xD1B54A32D192ED03ull) ^ (uint64_t)q * 0x9E37ull);
      keys[(size_t)B + (size_t)B * C + q] = table_[r & (table_.size() - 1)] | kOutBit;
    }
  }

 private:
  std::vector<uint64_t> tokens_, sent_offs_;
  std::vector<uint32_t> sent_of_;
  std::vector<std::pair<uint64_t, uint64_t>> vocab_;
  std::vector<uint64_t> table_;
  std::unordered_map<uint64_t, float> keep_;
};

}  // namespace ss
