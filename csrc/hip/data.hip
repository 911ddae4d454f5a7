// data.hip — HBM-resident training data: batch assembly on the device.
//
// The reference's apps parse text on the worker's CPU for every pass
// (BaseAlgorithm::parse_record over scan_file_by_line, /root/reference/src/
// core/framework/SwiftWorker.h:19-30, utils/file.h:14-33).  Here a file is
// parsed ONCE by the native loader (csrc/host/dataio.h, CSR: row offsets,
// keys, values, labels) and the whole shard is uploaded to HBM3E (288 GB per
// GPU holds e.g. 45M rows x 39 fields of u64 keys in 14 GB); each step's
// padded B x F batch is then cut out of it by one streaming kernel instead of
// a host fill + 82 MB PCIe copy per step (batch 262144 x 39).
#include "ss_device.h"
#include "ss_launch.h"
#include "ss/w2v_window.h"

namespace ss {

// One lane per (sample, field) of the batch: sample b is dataset row
// (cursor + b) mod rows; its first min(len, F) keys are copied, the rest of
// the F slots get the EMPTY key (the dedup skips it) and value 0 — the same
// layout SparseDataset::fill produces on the host.  Keys of a row are
// contiguous, so consecutive lanes read consecutive words.  With step_dev
// (hipGraph replays) the cursor is ((*step_dev + step_add) * B) mod rows.
__global__ __launch_bounds__(256) void k_csr_batch(const uint64_t* __restrict__ offs,
                                                   const uint64_t* __restrict__ keys,
                                                   const float* __restrict__ vals,
                                                   const float* __restrict__ labels,
                                                   unsigned long long rows,
                                                   unsigned long long cursor, int B, int F,
                                                   const long long* __restrict__ step_dev,
                                                   long long step_add,
                                                   uint64_t* __restrict__ out_keys,
                                                   float* __restrict__ out_vals,
                                                   float* __restrict__ out_labels) {
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i >= (long long)B * F) return;
  const int b = (int)(i / F), f = (int)(i - (long long)b * F);
  unsigned long long c0 = cursor;
  if (step_dev)
    c0 = ((unsigned long long)(*step_dev + step_add) * (unsigned long long)B) % rows;
  const unsigned long long r = (c0 + (unsigned long long)b) % rows;
  const uint64_t o = offs[r];
  const uint64_t len = offs[r + 1] - o;
  const bool have = (uint64_t)f < len;
  out_keys[i] = have ? keys[o + f] : kEmptyKey;
  if (out_vals) out_vals[i] = have ? (vals ? vals[o + f] : 1.f) : 0.f;
  if (f == 0) out_labels[b] = labels[r];
}

// Skip-gram batch of an HBM-resident corpus, bit-identical to the host
// sampler Corpus::fill_skipgram (csrc/host/dataio.h): keys[0,B) centers drawn
// uniformly over the shard's tokens (frequent-word sub-sampling by each
// token's keep probability, up to 16 draws), keys[B, B+B*C) contexts drawn
// with replacement from the center's sentence within +-W (a one-word
// sentence draws from the unigram^0.75 noise table), then nneg shared
// negatives from the noise table; context / negative keys carry the out bit.
// One lane per center (its C contexts) and one per negative.
__global__ __launch_bounds__(256) void k_w2v_corpus_batch(
    const uint64_t* __restrict__ tokens, const uint64_t* __restrict__ sent_offs,
    const uint32_t* __restrict__ sent_of, const uint64_t* __restrict__ table,
    unsigned long long table_mask, const float* __restrict__ keep, unsigned long long N,
    uint64_t seed, unsigned long long step, const long long* __restrict__ step_dev,
    long long step_add, int B, int C, int W, long long nneg, uint64_t out_bit,
    uint64_t* __restrict__ keys) {
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  const uint64_t st = step_dev ? (uint64_t)(*step_dev + step_add) : (uint64_t)step;
  if (i < B) {
    const int b = (int)i;
    uint64_t r = splitmix64(seed ^ (st * 0x9E3779B97F4A7C15ull) ^ ((uint64_t)b << 20));
    uint64_t pos = 0;
    for (int tries = 0; tries < 16; ++tries) {
      r = splitmix64(r);
      pos = fastrange64(r, N);
      if (!keep || u01(splitmix64(r ^ 7)) < keep[pos]) break;
    }
    keys[b] = tokens[pos];
    const uint32_t s = sent_of[pos];
    const long long sb = (long long)sent_offs[s], se = (long long)sent_offs[s + 1];
    const long long lo = max(sb, (long long)pos - W), hi = min(se - 1, (long long)pos + W);
    const long long span = hi - lo;
    for (int c = 0; c < C; ++c) {
      r = splitmix64(r + (uint64_t)c);
      uint64_t x;
      if (span <= 0) {
        x = table[r & table_mask];
      } else {
        long long q = lo + (long long)fastrange64(r, (uint64_t)span);
        if (q >= (long long)pos) ++q;
        x = tokens[q];
      }
      keys[(long long)B + (long long)b * C + c] = x | out_bit;
    }
  } else if (i < (long long)B + nneg) {
    const long long q = i - B;
    const uint64_t r = splitmix64(seed ^ 0xBADC0DEull ^ (st * 0xD1B54A32D192ED03ull) ^
                                  (uint64_t)q * 0x9E37ull);
    keys[(long long)B + (long long)B * C + q] = table[r & table_mask] | out_bit;
  }
}

void launch_w2v_corpus_batch(const uint64_t* tokens, const uint64_t* sent_offs,
                             const uint32_t* sent_of, const uint64_t* table, long long table_size,
                             const float* keep, long long N, uint64_t seed, long long step,
                             const long long* step_dev, long long step_add, int B, int C, int W,
                             long long nneg, uint64_t out_bit, uint64_t* keys, hipStream_t st) {
  if (N <= 0) throw_error("w2v_corpus_batch: empty corpus");
  if (table_size <= 0 || (table_size & (table_size - 1)) != 0)
    throw_error("w2v_corpus_batch: noise table size must be a power of two");
  const long long n = (long long)B + nneg;
  if (n <= 0) return;
  hipLaunchKernelGGL(k_w2v_corpus_batch, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st,
                     tokens, sent_offs, sent_of, table, (unsigned long long)(table_size - 1), keep,
                     (unsigned long long)N, seed, (unsigned long long)step, step_dev, step_add, B,
                     C, W, nneg, out_bit, keys);
  check_launch("k_w2v_corpus_batch");
}

// Windowed skip-gram runs from the resident corpus (layout: ss/w2v_window.h).
// Step `st` of this rank reads the run of B + 2W stream positions starting at
// st * B - W (mod N: the rank's corpus shard is cycled epoch after epoch, so
// consecutive steps walk it in order and every token is a center once per
// epoch).  A position's sentence tag is its sentence index plus the lap's
// offset (positions of different laps never pair), its reduced window and
// sub-sampling decision are hashes of its stream position: the host batcher
// (Corpus::fill_skipgram_window) produces the same batch bit for bit.
__global__ __launch_bounds__(256) void k_w2v_corpus_window(
    const uint64_t* __restrict__ tokens, const uint32_t* __restrict__ sent_of,
    unsigned long long nsent, const uint64_t* __restrict__ table, unsigned long long table_mask,
    const float* __restrict__ keep, unsigned long long N, uint64_t seed, unsigned long long step,
    const long long* __restrict__ step_dev, long long step_add, int B, int W, long long nneg,
    uint64_t out_bit, uint64_t* __restrict__ keys, int32_t* __restrict__ meta) {
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  const uint64_t st = step_dev ? (uint64_t)(*step_dev + step_add) : (uint64_t)step;
  const long long R = (long long)B + 2 * W;
  if (i < R) {
    const long long x = (long long)((st * (uint64_t)B) % N) - W + i;  // stream position
    const long long n = (long long)N;
    const long long lap = x >= 0 ? x / n : -((-x + n - 1) / n);
    const long long idx = x - lap * n;
    const uint64_t tok = tokens[idx];
    int32_t m = w2v_meta((uint64_t)sent_of[idx] + (uint64_t)(lap + 1) * nsent,
                         w2v_reduced_window(seed, (uint64_t)x, W));
    if (keep && !w2v_keep(seed, st, (uint64_t)x, keep[idx])) m = -1;
    keys[B + i] = tok | out_bit;
    meta[i] = m;
    if (i >= W && i < W + B) keys[i - W] = tok;
  } else if (i < R + nneg) {
    const long long q = i - R;
    const uint64_t r = splitmix64(seed ^ 0xBADC0DEull ^ (st * 0xD1B54A32D192ED03ull) ^
                                  (uint64_t)q * 0x9E37ull);
    keys[B + R + q] = table[r & table_mask] | out_bit;
  }
}

void launch_w2v_corpus_window(const uint64_t* tokens, const uint32_t* sent_of, long long nsent,
                              const uint64_t* table, long long table_size, const float* keep,
                              long long N, uint64_t seed, long long step,
                              const long long* step_dev, long long step_add, int B, int W,
                              long long nneg, uint64_t out_bit, uint64_t* keys, int32_t* meta,
                              hipStream_t st) {
  if (N <= 0) throw_error("w2v_corpus_window: empty corpus");
  if (W < 1 || W > kW2vMaxWindow) throw_error("w2v_corpus_window: window must be in [1, 15]");
  if (table_size <= 0 || (table_size & (table_size - 1)) != 0)
    throw_error("w2v_corpus_window: noise table size must be a power of two");
  const long long n = (long long)B + 2 * W + nneg;
  if (B <= 0) return;
  hipLaunchKernelGGL(k_w2v_corpus_window, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st,
                     tokens, sent_of, (unsigned long long)nsent, table,
                     (unsigned long long)(table_size - 1), keep, (unsigned long long)N, seed,
                     (unsigned long long)step, step_dev, step_add, B, W, nneg, out_bit, keys, meta);
  check_launch("k_w2v_corpus_window");
}

void launch_csr_batch(const uint64_t* offs, const uint64_t* keys, const float* vals,
                      const float* labels, long long rows, long long cursor, int B, int F,
                      const long long* step_dev, long long step_add, uint64_t* out_keys,
                      float* out_vals, float* out_labels, hipStream_t st) {
  if (rows <= 0) throw_error("csr_batch: empty dataset");
  if (B <= 0 || F <= 0) return;
  const long long n = (long long)B * F;
  hipLaunchKernelGGL(k_csr_batch, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, offs, keys,
                     vals, labels, (unsigned long long)rows,
                     (unsigned long long)(((cursor % rows) + rows) % rows), B, F, step_dev,
                     step_add, out_keys, out_vals, out_labels);
  check_launch("k_csr_batch");
}

}  // namespace ss
