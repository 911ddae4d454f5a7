// bdedup.hip — bucketed, global-atomic-free batch dedup + routing (K1/K2/K7).
//
// Same contract as dedup.hip (replaces the caller-side unordered_set and the
// per-destination grouping of pull_with_barrier / push_with_barrier,
// /root/reference/src/core/parameter/global_pull_access.h:40-72,
// global_push_access.h:80-99), redesigned after profiling dedup.hip on MI355X:
// its scratch-table CAS per occurrence runs at the memory side (the 8 XCD L2s
// are not coherent, so device-scope atomics bypass them) and cost 160 us for
// 2.56M keys, plus 75 us for the finish pass and ~140 us for the separate
// segmented-reduction plan of the gradient merge.
//
// Here every occurrence is first PARTITIONED into buckets by hash, then each
// bucket is deduplicated by ONE workgroup in an LDS hash table (LDS atomics
// only).  The bucket id is a function of the destination rank, so a
// destination's unique keys are the concatenation of its buckets — exactly the
// alltoallv send layout — and the same partition doubles as the plan for the
// duplicate-merging gradient reduction (k_bd_reduce), which needs no atomics
// to global memory at all.
//
//   1 count    per <=8192-occurrence chunk: LDS histogram over buckets, stored
//              chunk-major ([nch][P], coalesced)
//   2 colscan  per-bucket exclusive scan down the chunks + bucket totals; the
//              last workgroup to finish scans those into bucket start offsets
//   4 scatter  bucket-ordered keys and the occurrence list pj[pos] = j (two
//              arrays); pos_of[j] and the bucket bkt[j] (both coalesced)
//   5 dedup    one workgroup per bucket: reads its keys coalesced; LDS hash
//              insert + compaction;
//              bucket-local ids luid[pos], the bucket's keys (staged in its own
//              occurrence range, and — N>1 — straight into the destination's
//              send segment, + zeroed gradient rows) and its unique count;
//              the bucket's unique-id base is reserved with ONE device-scope
//              add per bucket on ucount[d] (zeroed by the count kernel): no
//              scan over buckets, no placement kernel (an arrival-counter
//              scan + a placement launch before; the placement stretched to
//              ~150 us beside the main stream)
//   7 inverse  (optional) inv[j] = ubase[bkt[j]] + luid[pos_of[j]]; consumers
//              that only need uid(j) read it through BdIndex instead
//
// Measured (profiles/): random 4-12 B stores cost ~5x their bytes in write
// requests (partial 64 B lines from 8 L2s), so only pj is stored permuted;
// an earlier single-pass variant with a decoupled look-back for the unique-id
// bases spent ~40% of each dedup workgroup's life waiting on predecessors.
//
// Bucket b = d * Pd + fastrange32(dedup_hash(key) >> 32, Pd) with
// d = map[fmix64(key) % frag_num] (hashfrag.h:48-53).  Pd is chosen so a
// bucket holds ~2048 occurrences (at most 2800) GIVEN THE DESTINATIONS THAT
// RECEIVE KEYS: `ndest` is the effective number of servers (frag_num over the
// largest per-server fragment count), so split roles (1 server in 4 ranks)
// do not pile 4x the keys into each bucket.  Its unique count is then far
// below the 4096-slot LDS table; a bucket that still overflows sets the
// sticky error word (scratch[0]), which Deduper.check() / PSEngine.check()
// turn into an exception at the engine's check points.
#include <algorithm>
#include <cstdlib>
#include <cstdio>
#include <string>

#include "bdindex.h"
#include "scan.h"
#include "ss_device.h"
#include "ss_launch.h"

namespace ss {

static constexpr uint32_t kBdInvalid = 0xFFFFFFFFu;
static constexpr int kBdMaxChunk = 8192;  // occurrences per count/scatter workgroup
static constexpr int kBdChunkLanes = 1024;  // chunk granularity (any CT below divides it)
static constexpr int kBdDT = 512;         // dedup workgroup size
// target occurrences per bucket (one rank; SS_BD_TARGET): 3584 measured
// 0.774-0.785 ms per bench step against 0.790-0.791 (3072) and 0.801-0.806
// (2048) with claimed pulls — longer (chunk, bucket) runs in the scatter,
// fewer and fuller claimed-pull workgroups
static constexpr int kBdTarget = 3584;
// N>1: a server merges bucket k of every source (server.hip); it splits the
// union of the N sources' runs into sub-buckets that fit one workgroup's
// table (the senders group each run by sub-bucket)
// (3072: 4 / 8 bench ranks on one GPU 4.24 / 8.03 ms per step at 1024, 3.94 /
// 7.19 at 2048, 3.72 / 6.98 at 3072 — bigger source buckets: longer scatter
// runs, fuller dedup workgroups, a smaller count histogram; the servers split
// them into proportionally more sub-buckets, so a server table holds the same;
// profiles/raw/r5_bucket_target_dist.txt)
static constexpr int kBdTargetDist = 3072;
// SS_BD_TARGET_DIST: occurrences per source bucket of the N>1 unique-key
// layout, 512..4096 (the servers' sub-bucket count follows it,
// server.hip srv_sub_buckets)
int bd_target_dist() {
  static const int v = [] {
    const char* e = std::getenv("SS_BD_TARGET_DIST");
    const int x = e ? std::atoi(e) : kBdTargetDist;
    return x < 512 ? 512 : (x > 4096 ? 4096 : x);
  }();
  return v;
}
// SS_BD_TARGET (one rank): occurrences per bucket, 1024..3584 (A/B: larger
// buckets make each (chunk, bucket) run of the scatter longer — fewer partial
// lines — at the price of a fuller LDS table in the dedup)
// N>1 record exchange (the kBdRecLayout bit of the layout's ndest argument,
// Deduper(record_layout=True)): the sources ship every occurrence, not their
// unique keys, so server bucket k is the union of N runs of records and must
// hold about one one-rank bucket: 3584 / N records per source bucket (the
// bucket-count cap raises it at N = 8, ~620 at the bench shape: ~5000
// records, ~2000 distinct keys per server bucket).  A property of the layout
// (every call and helper of a deduper passes the same ndest), not of the
// process: engines of either kind can coexist.
static constexpr int kBdRecLayout = 1 << 16;
// ... with kBdRecGroup as well (N>1 grouped records, round 6): the record
// placement but the unique layout's fuller source buckets (~3072
// occurrences); a pass after the scatter (k_rec_group) groups each bucket's
// records by the servers' sub-bucket, as the unique dedup groups its keys,
// so a server reads exact ranges.  The small buckets above (3584 / N) made
// the scatter's tile runs shorter than a sector at N >= 4 (P = 11K-16K
// buckets, 8K- down to 2K-key tiles)
static constexpr int kBdRecGroup = 1 << 17;
static int bd_target(int nranks, bool rec) {
  static const int one = [] {
    const char* e = std::getenv("SS_BD_TARGET");
    const int v = e ? std::atoi(e) : kBdTarget;
    return v < 1024 ? 1024 : (v > 3584 ? 3584 : v);
  }();
  if (nranks > 1 && rec) return std::max(256, kBdTarget / nranks);
  return nranks > 1 ? bd_target_dist() : one;
}
int bd_record_layout_bit() { return kBdRecLayout; }
int bd_record_group_bit() { return kBdRecGroup; }
// the occurrences-per-bucket target a layout of `nranks` ranks uses
int bd_target_for(int nranks, bool records) { return bd_target(nranks, records); }
static constexpr int kBdTS = 4096;      // LDS hash slots per bucket
static constexpr int kBdRegs = 8;       // occurrences per dedup thread kept in registers
static constexpr int kBdMaxBuckets = 16384;
static constexpr int kBdMaxSub = 64;    // server sub-buckets per bucket (srv_sub_buckets)

// The scatter -> dedup hand-off: the bucket-ordered keys (`rk`, the record
// buffer) and the occurrence list pj[pos] = j as two arrays.  A call whose
// keys all fit 32 bits (ids of a <= 4G-feature space: the count kernel ORs
// the high words, the column scan publishes the verdict) stores 4-byte keys,
// else 8-byte ones (SS_BD_REC=12 / 16: always 8).  Until round 6 key and j
// travelled as one interleaved (key, j) record that the dedup read whole and
// copied j out of into pj: 41 MB read + 41 MB written more per bench step
// (8-byte records; 12 / 16 bytes for wide keys before that, round 4: 12-byte
// records 0.850-0.854 -> 0.836-0.841 ms).

__device__ __forceinline__ uint32_t bd_bucket(uint64_t key, const RouteSpec& rs, uint32_t Pd) {
  const uint32_t d = rs.dest_of(key);
  if (rs.rbits) {
    // region tables: bucket floor(region * Pd / R) — every region inside ONE
    // bucket (the bucket's pull owns its inserts, k_pull_claim_bk)
    const uint64_t region = table_hash(key) >> (64 - rs.rbits);
    return d * Pd + (uint32_t)((region * (uint64_t)Pd) >> rs.rbits);
  }
  const uint32_t h = (uint32_t)(dedup_hash(key) >> 32);
  return d * Pd + __umulhi(h, Pd);
}

// SS_BD_XCD=1: the scatter's chunks in XCD-aware order (measured neutral:
// bench 0.779-0.784 vs 0.784-0.786 ms, the same WRITE_SIZE)
static int bd_xcd() {
  static const int v = [] {
    const char* e = std::getenv("SS_BD_XCD");
    return e ? std::atoi(e) : 0;
  }();
  return v;
}

// upper bound on count/scatter chunks (SS_BD_NCH knob): 128 — a chunk of the
// bench batch (10.2M keys) is 80K keys, looped in 8192-key register tiles, so
// each (chunk, bucket) run of positions is ~16 long and the scatter's
// partial-line stores merge in L2, and the route stream holds fewer CUs beside
// the main stream.  Measured (bench, A/B pairs): 512 -> 0.928-0.932 ms/step,
// 256 -> 0.914, 128 -> 0.886-0.899, 96 -> 0.888-0.894, 64 -> 0.90-0.916.  The
// N>1 path used 256 while its rounds pulled ahead (the route stream was its
// critical chain); with synchronous rounds 128 measured as good or better: the
// 1-rank N>1 path 1.065-1.105 vs 1.094-1.131 ms, 8 ranks on one GPU 8.48 vs
// 8.41-8.84 ms per 8-rank step.
static long long bd_max_chunks(int nranks) {
  (void)nranks;
  static const long long env = [] {
    const char* e = std::getenv("SS_BD_NCH");
    return e ? std::atoll(e) : 0ll;
  }();
  const long long x = env ? env : 128;
  return x < 64 ? 64 : x;
}

// ---- layout of the int scratch (u32 words), a function of (n, nranks) only
struct BdLayout {
  int P, Pd, nch, chunk;
  long long hist, btot, bstart, ubase, unum, ctr, wacc, wfin, total;
};

static int bd_clamp_ndest(int nranks, int ndest) {
  ndest &= ~(kBdRecLayout | kBdRecGroup);
  return ndest < 1 || ndest > nranks ? nranks : ndest;
}

static BdLayout bd_layout(long long n, int nranks, int ndest) {
  BdLayout L{};
  const bool rec = (ndest & kBdRecLayout) != 0 && !(ndest & kBdRecGroup);
  ndest = bd_clamp_ndest(nranks, ndest);
  // ~2048 occurrences per bucket, but at least ~1024 buckets for small calls
  // (>= 4 workgroups per CU; a word2vec step of 196K keys got only 96 buckets)
  const int tg = bd_target(nranks, rec);
  long long target = std::min<long long>(tg, std::max<long long>(128, n / 1024));
  if (n > (long long)kBdMaxBuckets * tg) target = (n + kBdMaxBuckets - 1) / kBdMaxBuckets;
  // buckets per destination from the keys one destination receives (n /
  // ndest), not n / nranks: ranks that host no shard get empty buckets
  long long pd = (n + (long long)ndest * target - 1) / ((long long)ndest * target);
  if (pd < 1) pd = 1;
  L.Pd = (int)pd;
  L.P = (int)(pd * nranks);
  // chunk count a multiple of the 256 CUs (balanced waves), chunk <= 8192 ...
  const long long waves = (n + 256ll * kBdMaxChunk - 1) / (256ll * kBdMaxChunk);
  const long long per = (n + 256 * waves - 1) / (256 * waves);
  long long chunk = ((per + kBdChunkLanes - 1) / kBdChunkLanes) * kBdChunkLanes;
  // ... but at most bd_max_chunks() chunks: the [nch][P] histogram grows as
  // n^2 (P ~ n/2048 buckets per chunk row), 25 MB at n = 10M with 8192-key
  // chunks; bigger chunks loop over 8192-key register tiles instead
  const long long cmax = bd_max_chunks(nranks);
  if ((n + chunk - 1) / chunk > cmax)
    chunk = (((n + cmax - 1) / cmax + kBdChunkLanes - 1) / kBdChunkLanes) * kBdChunkLanes;
  L.chunk = (int)chunk;
  L.nch = (int)((n + L.chunk - 1) / L.chunk);
  if (L.nch < 1) L.nch = 1;
  // words 0, 1: sticky error flag and the colscan arrival counter, at fixed
  // positions for any n (the scratch is sized for the largest call and
  // zeroed once; every other word is rewritten by each call)
  long long o = 4;
  L.ctr = 1;
  L.wacc = 2;  // count: some key of this call has high bits (atomicOr)
  L.wfin = 3;  // colscan's last workgroup: the call's value (wacc reset to 0)
  L.hist = o; o += (long long)L.P * L.nch;
  L.btot = o; o += L.P;
  L.bstart = o; o += L.P + 1;
  L.ubase = o; o += L.P;
  L.unum = o; o += L.P;
  L.total = o;
  return L;
}

// largest call the bucketed dedup takes (~2800 occurrences per bucket at
// the bucket-count cap); Deduper falls back to the scratch-hash dedup above
long long bd_max_keys() { return (long long)kBdMaxBuckets * 2800; }

// words for ANY call of up to n keys: the layout is not monotonic in n (the
// bucket target grows with n below 2M keys, the chunk count jumps with the
// wave count), so bound P and nch over all m <= n instead of sizing for n
long long bd_scratch_words(long long n, int nranks, int ndest) {
  if (n < 1) n = 1;
  const int ndest_arg = ndest;
  const bool rec = (ndest & kBdRecLayout) != 0 && !(ndest & kBdRecGroup);
  ndest = bd_clamp_ndest(nranks, ndest);
  // active buckets (those of receiving destinations), then all P = Pd * nranks
  const int tg = bd_target(nranks, rec);
  long long pact = std::max<long long>(1056, (n + tg - 1) / tg);
  pact = std::min<long long>(pact, kBdMaxBuckets) + 2 * ndest;
  const long long pmax = ((pact + ndest - 1) / ndest + 1) * nranks;
  const long long waves = (n + 256ll * kBdMaxChunk - 1) / (256ll * kBdMaxChunk);
  long long nchmax = std::min<long long>(256 * waves, bd_max_chunks(nranks));
  nchmax = std::min<long long>(nchmax, (n + kBdChunkLanes - 1) / kBdChunkLanes);
  nchmax = std::max<long long>(nchmax, 1);
  const long long bound = 4 + pmax * nchmax + 4 * pmax + 1;
  return std::max(bound, bd_layout(n, nranks, ndest_arg).total);
}
int bd_buckets(long long n, int nranks, int ndest) {
  return bd_layout(n < 1 ? 1 : n, nranks, ndest).P;
}
// (P, bstart, unum, ubase) word offsets into the scratch for a call of n keys
std::vector<long long> bd_offsets(long long n, int nranks, int ndest) {
  const BdLayout L = bd_layout(n < 1 ? 1 : n, nranks, ndest);
  return {L.P, L.bstart, L.unum, L.ubase};
}
long long bd_ubase_offset(long long n, int nranks, int ndest) {
  return bd_layout(n < 1 ? 1 : n, nranks, ndest).ubase;
}

// 1. per-chunk bucket histogram (dynamic LDS: P words), chunk-major output
template <int CT>
__global__ __launch_bounds__(CT) void k_bd_count(const uint64_t* __restrict__ keys, long long n,
                                                    RouteSpec rs, int Pd, int P, int chunk,
                                                    uint32_t* __restrict__ hist,
                                                    unsigned long long* __restrict__ ucount,
                                                    uint32_t* __restrict__ wacc) {
  extern __shared__ unsigned int h[];
  __shared__ unsigned int hiw;
  if (threadIdx.x == 0) hiw = 0u;
  // the dedup's per-destination unique counters start from zero (stream order)
  if (blockIdx.x == 0 && threadIdx.x < (unsigned)rs.nranks) ucount[threadIdx.x] = 0ull;
  for (int b = threadIdx.x; b < P; b += CT) h[b] = 0u;
  __syncthreads();
  // the chunk in register tiles of <= kBdMaxChunk keys (all loads of a tile
  // in flight together)
  for (int t0 = 0; t0 < chunk; t0 += kBdMaxChunk) {
    const long long base = (long long)blockIdx.x * chunk + t0 + threadIdx.x;
    const int per = min(chunk - t0, kBdMaxChunk) / CT;
    uint64_t k[(kBdMaxChunk / CT)];
#pragma unroll
    for (int e = 0; e < (kBdMaxChunk / CT); ++e) {
      const long long j = base + e * CT;
      k[e] = (e < per && j < n) ? keys[j] : kEmptyKey;
    }
    uint32_t hi = 0u;
#pragma unroll
    for (int e = 0; e < (kBdMaxChunk / CT); ++e)
      if (k[e] != kEmptyKey) {
        atomicAdd(&h[bd_bucket(k[e], rs, (uint32_t)Pd)], 1u);
        hi |= (uint32_t)(k[e] >> 32);
      }
    if (__ballot(hi != 0u) && (threadIdx.x & 63) == 0) hiw = 1u;  // benign race: all store 1
  }
  __syncthreads();
  if (threadIdx.x == 0 && hiw && wacc) atomicOr(wacc, 1u);
  uint32_t* row = hist + (long long)blockIdx.x * P;
  for (int b = threadIdx.x; b < P; b += CT) row[b] = h[b];
}

// 2+3. column scan of the [nch][P] histogram (64 buckets x CS/64 chunk
//    segments per workgroup, two passes of independent loads, no serial
//    chain); the LAST workgroup to finish (arrival counter) also scans the
//    bucket totals into bucket start offsets — no separate single-workgroup
//    launch.  CS = workgroup size (small workgroups are not starved by the
//    other stream's kernels: 1024-thread ones waited ~200 us for a CU with 16
//    free wave slots beside the pull)
// Record exchange (`gap` > 0, RecLay): destination d's buckets are placed
// from d * gap (its send segment in the mailbox layout) instead of after
// destination d-1's, the last workgroup writes the per-destination record
// counts and the run tables the servers read (ubase = the gapped bucket
// starts, unum = the bucket sizes), and the scatter's positions are then
// send-segment positions: the rows come back to exactly those positions.
static constexpr int kRecMaxDest = 64;  // destinations of a record-exchange layout
struct RecLay {
  long long gap;                 // 0: contiguous buckets
  int Pd;                        // buckets per destination
  unsigned long long* ucount;    // [nranks] records per destination
  uint32_t* ubase;               // [P] run bases (gapped bucket starts)
  uint32_t* unum;                // [P] run lengths
  uint32_t* err;                 // sticky flag: a destination got more than gap
};

template <int CS>
__global__ __launch_bounds__(CS) void k_bd_colscan(uint32_t* __restrict__ hist, int nch, int P,
                                                   uint32_t* __restrict__ btot,
                                                   uint32_t* __restrict__ bstart,
                                                   unsigned int* __restrict__ ctr,
                                                   uint32_t* __restrict__ wacc,
                                                   uint32_t* __restrict__ wfin,
                                                   RecLay rl = RecLay{}) {
  constexpr int NS = CS / 64;  // chunk segments per column
  __shared__ unsigned int ss[NS][64];
  __shared__ unsigned int wsum[16];
  __shared__ unsigned int tot;
  __shared__ bool last;
  const int col = threadIdx.x & 63, seg = threadIdx.x >> 6;
  const int b = blockIdx.x * 64 + col;
  const int R = (nch + NS - 1) / NS;
  const int c0 = seg * R, c1 = min(nch, c0 + R);
  unsigned int s = 0;
  if (b < P) {
#pragma unroll 8
    for (int c = c0; c < c1; ++c) s += hist[(long long)c * P + b];
  }
  ss[seg][col] = s;
  __syncthreads();
  unsigned int off = 0;
  for (int q = 0; q < seg; ++q) off += ss[q][col];
  if (b < P) {
#pragma unroll 8
    for (int c = c0; c < c1; ++c) {
      const long long i = (long long)c * P + b;
      const unsigned int v = hist[i];
      hist[i] = off;
      off += v;
    }
    if (seg == NS - 1) __hip_atomic_store(&btot[b], off, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  // publish btot: write-through stores drained by every wave, barrier, then
  // one arrival add; the last arriver reads btot write-through (guide G16 R1)
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) last = atomicAdd(ctr, 1u) == gridDim.x - 1;
  __syncthreads();
  if (!last) return;  // workgroup-uniform
  const int per = (P + CS - 1) / CS;
  const int b0 = threadIdx.x * per;
  unsigned int sum = 0;
  for (int k = 0; k < per; ++k)
    if (b0 + k < P)
      sum += __hip_atomic_load(&btot[b0 + k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const unsigned int e0 = block_excl_scan<NS>(sum, wsum, &tot);
  unsigned int e = e0;
  if (!rl.gap) {
    for (int k = 0; k < per; ++k)
      if (b0 + k < P) {
        bstart[b0 + k] = e;
        e += __hip_atomic_load(&btot[b0 + k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
  } else {
    // record exchange: E_d (the contiguous start of destination d's first
    // bucket) in LDS, then every bucket rebased to d * gap
    __shared__ unsigned int ed[kRecMaxDest + 1];
    const int nd = P / rl.Pd;
    for (int k = 0; k < per; ++k)
      if (b0 + k < P) {
        if ((b0 + k) % rl.Pd == 0) ed[(b0 + k) / rl.Pd] = e;
        e += __hip_atomic_load(&btot[b0 + k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    if (threadIdx.x == 0) ed[nd] = tot;
    __syncthreads();
    e = e0;
    for (int k = 0; k < per; ++k)
      if (b0 + k < P) {
        const int b = b0 + k, d = b / rl.Pd;
        const uint32_t c = __hip_atomic_load(&btot[b], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const uint32_t s = (uint32_t)((long long)d * rl.gap + (e - ed[d]));
        bstart[b] = s;
        rl.ubase[b] = s;
        rl.unum[b] = c;
        e += c;
      }
    for (int d = threadIdx.x; d < nd; d += CS) {
      const unsigned int c = ed[d + 1] - ed[d];
      rl.ucount[d] = c;
      if ((long long)c > rl.gap) atomicOr(rl.err, 1u);
    }
  }
  if (threadIdx.x == 0) {
    bstart[P] = tot;
    *ctr = 0u;  // ready for the next call (stream-ordered)
    // the record width of this call (kernel-ordered after the count)
    *wfin = wacc ? *wacc : 1u;
    if (wacc) *wacc = 0u;
  }
}

// 4. bucket-ordered occurrence list (dynamic LDS: P words)
template <int CT, int RW>
__global__ __launch_bounds__(CT) void k_bd_scatter(const uint64_t* __restrict__ keys, long long n,
                                                     RouteSpec rs, int Pd, int P, int chunk,
                                                     const uint32_t* __restrict__ hist,
                                                     const uint32_t* __restrict__ bstart,
                                                     uint32_t* __restrict__ pj,
                                                     uint32_t* __restrict__ pos_of,
                                                     uint32_t* __restrict__ bkt,
                                                     void* __restrict__ rec,
                                                     const uint32_t* __restrict__ wfin,
                                                     int xcd, uint64_t* __restrict__ skeys = nullptr,
                                                     uint32_t* __restrict__ spj = nullptr) {
  extern __shared__ unsigned int cur[];
  // XCD-aware chunk order (xcd != 0): blocks b and b + 8 share an XCD, so
  // they get ADJACENT chunks — a bucket's runs are laid out chunk after chunk,
  // and the line two neighbouring runs share is then written by one L2 and
  // merged there instead of leaving two partial lines for the fabric
  int c = blockIdx.x;
  if (xcd) {
    const int g = (int)gridDim.x, x = c & 7;
    c = x * (g >> 3) + min(x, g & 7) + (c >> 3);
  }
  // keys of 32 bits: 4-byte keys (RW 3 only)
  const bool narrow = RW == 3 && wfin && *wfin == 0u;
  uint32_t* rk32 = reinterpret_cast<uint32_t*>(rec);
  uint64_t* rk64 = reinterpret_cast<uint64_t*>(rec);
  const uint32_t* row = hist + (long long)c * P;
  for (int b = threadIdx.x; b < P; b += CT) cur[b] = bstart[b] + row[b];
  for (int t0 = 0; t0 < chunk; t0 += kBdMaxChunk) {
    const long long base = (long long)c * chunk + t0 + threadIdx.x;
    const int per = min(chunk - t0, kBdMaxChunk) / CT;
    uint64_t k[(kBdMaxChunk / CT)];
#pragma unroll
    for (int e = 0; e < (kBdMaxChunk / CT); ++e) {
      const long long j = base + e * CT;
      k[e] = (e < per && j < n) ? keys[j] : kEmptyKey;
    }
    __syncthreads();  // first tile: cursors initialised
#pragma unroll
    for (int e = 0; e < (kBdMaxChunk / CT); ++e) {
      const long long j = base + e * CT;
      if (e < per && j < n) {
        uint32_t pos = kBdInvalid, b = kBdInvalid;
        if (k[e] != kEmptyKey) {
          b = bd_bucket(k[e], rs, (uint32_t)Pd);
          pos = atomicAdd(&cur[b], 1u);
          // the key travels to its bucket position beside its sample index,
          // so the dedup reads its bucket's keys coalesced instead of
          // gathering keys[pj[p]] (a 64-byte line per occurrence).  Measured
          // standalone: scatter 119 -> 163 us, dedup 213 -> 123 us; N>1
          // engine path 1.211 -> 1.169 ms/step, one GPU neutral.
          // record exchange: the key and its occurrence at send-segment
          // positions (the keys are the send segment)
          if (skeys) {
            skeys[pos] = k[e];
            spj[pos] = (uint32_t)j;
          } else {
            if (narrow)
              rk32[pos] = (uint32_t)k[e];
            else
              rk64[pos] = k[e];
            pj[pos] = (uint32_t)j;
          }
        }
        // the BdIndex (j -> bucket position, bucket) only for its consumers
        if (pos_of) pos_of[j] = pos;
        if (bkt) bkt[j] = b;
      }
    }
  }
}

// 4'. the same bucket-ordered list, written through LDS (12- and 8-byte
// records; SS_BD_SORT=0: the kernel above).  One random 8-byte store per key
// left a partial 32-byte sector per record: the scatter wrote 288 MB per
// bench step for 82 MB of records + 41 MB of pos_of (WRITE_SIZE), and the L2
// does not merge a (chunk, bucket) run's stores across tiles (the same bytes
// at 32, 64 and 128 chunks).  Here each tile is counting-sorted by bucket in
// LDS (tile histogram, scan over the P buckets, staged SoA records) and
// written out in bucket order: consecutive lanes store consecutive positions
// of a bucket's run, so one store instruction covers whole sectors of the
// runs it touches.  The longer a tile, the longer each (tile, bucket) run:
// KT keys per thread for 8-byte records (two staged words per key; the
// write-out re-hashes the key for its bucket instead of staging it), KT / 2
// for 12-byte ones.  LDS: (2P + 1) words + 2 * KT * 1024 words.
template <int KT>
__global__ __launch_bounds__(1024) void k_bd_scatter_s(const uint64_t* __restrict__ keys,
                                                       long long n, RouteSpec rs, int Pd, int P,
                                                       int chunk,
                                                       const uint32_t* __restrict__ hist,
                                                       const uint32_t* __restrict__ bstart,
                                                       uint32_t* __restrict__ pos_of,
                                                       uint32_t* __restrict__ bkt,
                                                       uint32_t* __restrict__ rec,
                                                       const uint32_t* __restrict__ wfin,
                                                       int xcd, uint64_t* __restrict__ skeys,
                                                       uint32_t* __restrict__ spj,
                                                       uint32_t* __restrict__ pj) {
  constexpr int CT = 1024;
  extern __shared__ unsigned int sm[];
  unsigned int* cur = sm;           // [P] the chunk's cursor per bucket
  unsigned int* toff = sm + P;      // [P + 1] tile counts, then tile offsets
  uint32_t* stage = toff + P + 1;   // [2 * KT * CT] staged records, SoA
  __shared__ unsigned int wsum[16];
  __shared__ unsigned int tot;
  const int t = threadIdx.x;
  int c = blockIdx.x;
  if (xcd) {
    const int g = (int)gridDim.x, x = c & 7;
    c = x * (g >> 3) + min(x, g & 7) + (c >> 3);
  }
  const bool narrow = wfin && *wfin == 0u;
  // 8-byte records: (key, sample) in two arrays of T; 12-byte: three of T
  const int T = narrow ? KT * CT : (KT / 2) * CT;
  uint32_t* sx = stage;
  uint32_t* sy = stage + T;                  // key high words (12-byte records)
  uint32_t* sz = stage + (narrow ? T : 2 * T);
  const uint32_t* row = hist + (long long)c * P;
  for (int b = t; b < P; b += CT) cur[b] = bstart[b] + row[b];
  const int per = (P + CT - 1) / CT;  // scan: buckets per thread
  const int b0 = t * per, b1 = min(P, b0 + per);
  for (int t0 = 0; t0 < chunk; t0 += T) {
    for (int b = t; b < P; b += CT) toff[b] = 0u;
    __syncthreads();
    const long long base = (long long)c * chunk + t0 + t;
    const int kt = min(chunk - t0, T) / CT;
    uint64_t k[KT];
    uint32_t br[KT];  // bucket << 16 | rank within the tile's bucket (P, T <= 65536)
#pragma unroll
    for (int e = 0; e < KT; ++e) {
      const long long j = base + (long long)e * CT;
      k[e] = (e < kt && j < n) ? keys[j] : kEmptyKey;
    }
#pragma unroll
    for (int e = 0; e < KT; ++e)
      if (k[e] != kEmptyKey) {
        const uint32_t b = bd_bucket(k[e], rs, (uint32_t)Pd);
        br[e] = b << 16 | atomicAdd(&toff[b], 1u);
      }
    __syncthreads();
    unsigned int sum = 0;
    for (int b = b0; b < b1; ++b) sum += toff[b];
    unsigned int o = block_excl_scan_1024(sum, wsum, &tot);
    for (int b = b0; b < b1; ++b) {
      const unsigned int v = toff[b];
      toff[b] = o;
      o += v;
    }
    if (t == 0) toff[P] = tot;
    __syncthreads();
#pragma unroll
    for (int e = 0; e < KT; ++e) {
      const long long j = base + (long long)e * CT;
      if (e < kt && j < n) {
        uint32_t pos = kBdInvalid, b = kBdInvalid;
        if (k[e] != kEmptyKey) {
          b = br[e] >> 16;
          const uint32_t r = br[e] & 0xFFFFu;
          const uint32_t i = toff[b] + r;
          sx[i] = (uint32_t)k[e];
          if (!narrow) sy[i] = (uint32_t)(k[e] >> 32);
          sz[i] = (uint32_t)j;
          pos = cur[b] + r;
        }
        if (pos_of) pos_of[j] = pos;
        if (bkt) bkt[j] = b;
      }
    }
    __syncthreads();
    const unsigned int nt = tot;
    // keys (4 or 8 bytes) and j into two arrays at the bucket positions
    // (the record exchange: the send segment's keys and spj)
    uint32_t* const qj = skeys ? spj : pj;
    if (narrow) {
      uint32_t* rk32 = reinterpret_cast<uint32_t*>(rec);
      for (unsigned int i = t; i < nt; i += CT) {
        const uint32_t key = sx[i];
        const uint32_t b = bd_bucket((uint64_t)key, rs, (uint32_t)Pd);
        const uint32_t q = cur[b] + (i - toff[b]);
        if (skeys)
          skeys[q] = key;
        else
          rk32[q] = key;
        qj[q] = sz[i];
      }
    } else {
      uint64_t* rk64 = reinterpret_cast<uint64_t*>(rec);
      for (unsigned int i = t; i < nt; i += CT) {
        const uint64_t key = (uint64_t)sx[i] | ((uint64_t)sy[i] << 32);
        const uint32_t b = bd_bucket(key, rs, (uint32_t)Pd);
        const uint32_t q = cur[b] + (i - toff[b]);
        (skeys ? skeys : rk64)[q] = key;
        qj[q] = sz[i];
      }
    }
    __syncthreads();
    for (int b = t; b < P; b += CT) cur[b] += toff[b + 1] - toff[b];
    __syncthreads();
  }
}

// 5. one workgroup per bucket: LDS hash dedup -> bucket-local unique ids
template <int RW>
__global__ __launch_bounds__(kBdDT) void k_bd_dedup(const uint64_t* __restrict__ keys,
                                                   uint32_t* __restrict__ pj,
                                                   const uint32_t* __restrict__ bstart,
                                                   uint32_t* __restrict__ luid,
                                                   uint64_t* __restrict__ bkeys,
                                                   uint32_t* __restrict__ unum,
                                                   uint32_t* __restrict__ err, int Pd,
                                                   long long ucap,
                                                   uint32_t* __restrict__ ubase,
                                                   unsigned long long* __restrict__ ucount,
                                                   const void* __restrict__ rec,
                                                   unsigned long long* __restrict__ dbg,
                                                   uint64_t* __restrict__ ukeys,
                                                   float* __restrict__ ugrad, int gdim,
                                                   uint8_t* __restrict__ usingle, int msub,
                                                   uint32_t* __restrict__ usub,
                                                   const uint32_t* __restrict__ wfin, int rbits) {
  // dbg (optional): per bucket wall-clock stamps of the phases (profiling)
#define BD_STAMP(i) \
  if (dbg && t == 0) dbg[(long long)b * 8 + (i)] = wall_clock64();
  __shared__ unsigned long long tab[kBdTS];
  __shared__ unsigned int lid[kBdTS];
  __shared__ uint8_t dupf[kBdTS];
  __shared__ unsigned int wsum[16];
  __shared__ unsigned int tot;
  __shared__ int bad;
  __shared__ unsigned int hsub[kBdMaxSub];  // msub > 1: keys per server sub-bucket, then offsets
  const int t = threadIdx.x, b = blockIdx.x;
  const uint32_t p0 = bstart[b], p1 = bstart[b + 1];
  // the hash table sized to the bucket (load <= 1/2 of its occurrences, 64
  // slots at least): small buckets (word2vec's ~200 occurrences, split-role
  // layouts) do not pay for initialising and compacting all 4096 slots
  const uint32_t ts = lds_table_size(p1 - p0, kBdTS);
  if (t == 0) bad = 0;
  if (t < kBdMaxSub) hsub[t] = 0u;
  for (uint32_t s = t; s < ts; s += kBdDT) {
    tab[s] = kEmptyKey;
    dupf[s] = 0;
  }
  // the first kBdRegs occurrences of each thread keep their slot in
  // registers; a hot bucket's excess parks it in luid[] (rewritten below)
  uint32_t slot[kBdRegs];
  uint64_t kk[kBdRegs];
  // the bucket's keys read coalesced (the scatter wrote pj beside them)
  const bool narrow = RW == 3 && wfin && *wfin == 0u;  // 4-byte keys
  const uint32_t* rk32 = reinterpret_cast<const uint32_t*>(rec);
  const uint64_t* rk64 = reinterpret_cast<const uint64_t*>(rec);
  auto load = [&](uint32_t p) -> uint64_t { return narrow ? (uint64_t)rk32[p] : rk64[p]; };
#pragma unroll
  for (int r = 0; r < kBdRegs; ++r) {
    const uint32_t p = p0 + t + r * kBdDT;
    kk[r] = p < p1 ? load(p) : kEmptyKey;
  }
  __syncthreads();
  BD_STAMP(0)
  // dupf[s]: the key of slot s occurs more than once in the bucket (set by
  // every occurrence but the inserting one: a plain, idempotent LDS store)
  auto insert = [&](uint64_t key) -> uint32_t {
    uint32_t s = (uint32_t)dedup_hash(key) & (ts - 1);
    for (uint32_t k = 0; k < ts; ++k) {
      const unsigned long long v = tab[s];
      if (v == key) {
        dupf[s] = 1;
        return s;
      }
      if (v == kEmptyKey) {
        const unsigned long long prev = atomicCAS(&tab[s], kEmptyKey, (unsigned long long)key);
        if (prev == kEmptyKey) return s;
        if (prev == key) {
          dupf[s] = 1;
          return s;
        }
      }
      s = (s + 1) & (ts - 1);
    }
    bad = 1;
    return kBdInvalid;
  };
#pragma unroll
  for (int r = 0; r < kBdRegs; ++r) slot[r] = kk[r] != kEmptyKey ? insert(kk[r]) : kBdInvalid;
  // hot buckets (Zipf heads): the excess in rounds of kBdRegs occurrences per
  // thread, all loads of a round in flight together; slots park in luid[]
  for (uint32_t q = p0 + t + kBdRegs * kBdDT; q < p1; q += kBdRegs * kBdDT) {
    uint64_t k2[kBdRegs];
#pragma unroll
    for (int r = 0; r < kBdRegs; ++r) {
      const uint32_t p = q + r * kBdDT;
      k2[r] = p < p1 ? load(p) : kEmptyKey;
    }
#pragma unroll
    for (int r = 0; r < kBdRegs; ++r) {
      const uint32_t p = q + r * kBdDT;
      if (p < p1) luid[p] = k2[r] != kEmptyKey ? insert(k2[r]) : kBdInvalid;
    }
  }
  __syncthreads();
  BD_STAMP(1)
  // compaction in slot order: thread t owns slots [per*t, per*(t+1));
  // msub > 1 (N>1 xGMI rounds): grouped by the server's sub-bucket first, so
  // a server sub-bucket's keys from this bucket are one contiguous range
  // (offsets in usub) and the server reads exactly its keys — no re-read of
  // the whole run per sub-bucket, no hashing pass to count them
  constexpr int kPerT = kBdTS / kBdDT;
  const uint32_t per = ts >= (uint32_t)kBdDT ? ts / kBdDT : 1u;
  // slot k of this thread's run (kEmptyKey past the table)
  auto own = [&](int k) -> unsigned long long {
    const uint32_t s = (uint32_t)t * per + (uint32_t)k;
    return (uint32_t)k < per && s < ts ? tab[s] : kEmptyKey;
  };
  unsigned int o = 0;
  uint8_t sb[kPerT];
  uint16_t rk[kPerT];
  // the server's sub-bucket of a key: region buckets (rbits) split each
  // bucket's regions further, floor(region * Pd * msub / R) - k * msub, so a
  // server sub-bucket is whole regions of the server's table too (its pull
  // claims inserts, table.hip k_pull_claim_bk); else a dedup_hash split
  auto sub_of = [&](uint64_t v) -> uint32_t {
    if (rbits) {
      const uint64_t region = table_hash(v) >> (64 - rbits);
      const uint32_t f = (uint32_t)((region * (uint64_t)Pd * (uint64_t)msub) >> rbits);
      return f - (uint32_t)(b % Pd) * (uint32_t)msub;
    }
    return srv_sub(v, msub);
  };
  if (msub > 1) {
#pragma unroll
    for (int k = 0; k < kPerT; ++k) {
      const unsigned long long v = own(k);
      sb[k] = v != kEmptyKey ? (uint8_t)sub_of(v) : 0;
      rk[k] = v != kEmptyKey ? (uint16_t)atomicAdd(&hsub[sb[k]], 1u) : 0;
    }
    __syncthreads();
    if (t == 0) {
      unsigned int e = 0;
      for (int i = 0; i < msub; ++i) {
        const unsigned int c = hsub[i];
        hsub[i] = e;
        e += c;
      }
      tot = e;
    }
  } else {
    unsigned int occ = 0;
#pragma unroll
    for (int k = 0; k < kPerT; ++k) occ += own(k) != kEmptyKey;
    o = block_excl_scan<kBdDT / 64>(occ, wsum, &tot);
  }
  // the bucket's unique ids: one device-scope add per bucket reserves them in
  // its destination's segment (ucount[d], zeroed by k_bd_count) — no scan
  // over the buckets, and the keys go straight to the alltoallv send layout
  const int d = b / Pd;
  __shared__ unsigned long long sbase;
  if (t == 0) {
    const unsigned long long base = atomicAdd(&ucount[d], (unsigned long long)tot);
    sbase = (unsigned long long)d * (unsigned long long)ucap + base;
    ubase[b] = (uint32_t)sbase;
    unum[b] = tot;
    if (bad) atomicOr(err, 1u);
  }
  __syncthreads();
  if (msub > 1 && usub && t < msub) usub[(long long)b * msub + t] = hsub[t];
  const unsigned long long ub = sbase;
#pragma unroll
  for (int k = 0; k < kPerT; ++k) {
    const uint32_t s = (uint32_t)t * per + (uint32_t)k;
    const unsigned long long v = own(k);
    if (v != kEmptyKey) {
      const unsigned int q = msub > 1 ? hsub[sb[k]] + rk[k] : o++;
      lid[s] = q;
      if (bkeys) bkeys[p0 + q] = v;  // staged in the bucket's own occurrence range
      if (ukeys) ukeys[ub + q] = v;
      if (usingle) usingle[ub + q] = dupf[s] ? 0 : 1;  // one occurrence in the batch
    }
  }
  if (ugrad)  // zeroed gradient rows for consumers that scatter-add into them
    for (unsigned int e = t; e < tot * (unsigned int)gdim; e += kBdDT)
      ugrad[ub * (unsigned long long)gdim + e] = 0.f;
  __syncthreads();
  BD_STAMP(2)
#pragma unroll
  for (int r = 0; r < kBdRegs; ++r) {
    const uint32_t p = p0 + t + r * kBdDT;
    if (p < p1) luid[p] = slot[r] == kBdInvalid ? kBdInvalid : lid[slot[r]];
  }
  for (uint32_t p = p0 + t + kBdRegs * kBdDT; p < p1; p += kBdDT) {
    const uint32_t s = luid[p];
    luid[p] = s == kBdInvalid ? kBdInvalid : lid[s];
  }
  __syncthreads();
  BD_STAMP(3)
#undef BD_STAMP
}

// 7. inverse index in occurrence order
__global__ __launch_bounds__(256) void k_bd_inv(BdIndex ix, long long n,
                                                uint32_t* __restrict__ inv) {
  const long long j = (long long)blockIdx.x * 256 + threadIdx.x;
  if (j < n) inv[j] = ix.uid(j);
}

// occurrence-position parameters for scalar rows: occ[p] = uvals[uid] of the
// occurrence at bucket position p (0 where it has no unique id).  One
// workgroup per bucket: the bucket's unique rows (one contiguous range of
// <= 4096 floats) are staged in LDS with coalesced loads, then luid is
// streamed and occ written in bucket order.  The LR forward then reads one
// random word per occurrence, occ[pos_of[j]], instead of the dependent pair
// luid[pos_of[j]] -> uvals[ubase + luid].
template <int FT>
__global__ __launch_bounds__(FT) void k_bd_fill_occ(const uint32_t* __restrict__ bstart,
                                                    const uint32_t* __restrict__ ubase,
                                                    const uint32_t* __restrict__ unum,
                                                    const uint32_t* __restrict__ luid,
                                                    const float* __restrict__ uvals,
                                                    float* __restrict__ occ, int osi,
                                                    const uint32_t* __restrict__ pj,
                                                    SelfSeg self) {
  // pj: write sample order instead, occ[pj[p]] (the forward then streams occ)
  __shared__ float sv[kBdTS];
  const int b = blockIdx.x;
  const uint32_t p0 = bstart[b], p1 = bstart[b + 1];
  const uint32_t base = osi ? p0 : ubase[b];
  const uint32_t nu = min(unum[b], (uint32_t)kBdTS);
  for (uint32_t l = threadIdx.x; l < nu; l += FT) sv[l] = uvals[base + l];
  __syncthreads();
  for (uint32_t pb = p0 + threadIdx.x; pb < p1; pb += 4 * FT) {
    uint32_t l[4], q[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const uint32_t p = pb + r * FT;
      l[r] = p < p1 ? luid[p] : kBdInvalid;
      q[r] = p < p1 ? (pj ? pj[p] : p) : 0u;
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const uint32_t p = pb + r * FT;
      if (p < p1) self.pick(occ, (long long)q[r])[q[r]] = l[r] < nu ? sv[l[r]] : 0.f;
    }
  }
}

// K7 for scalar rows (sparse LR): one workgroup per bucket sums the gradients
// of its unique keys in LDS — per-occurrence g = gs[j / F] * x[j] gathered
// from the per-sample gradient (L2-resident) — and stores each row once:
// no zero-fill, no global atomics.
// OCC: occurrences per thread in flight (all their loads issued before the
// first LDS atomic), and unique rows per thread per pass of the fused update
template <int RT, int OCC = 2>
__global__ __launch_bounds__(RT) void k_bd_reduce(const uint32_t* __restrict__ bstart,
                                                    const uint32_t* __restrict__ ubase,
                                                    const uint32_t* __restrict__ unum,
                                                    const uint32_t* __restrict__ pj,
                                                    const uint32_t* __restrict__ luid,
                                                    const float* __restrict__ gs,
                                                    const float* __restrict__ xval, int F,
                                                    float* __restrict__ ugrad, int osi,
                                                    const uint8_t* __restrict__ usingle,
                                                    DevTable t, const long long* __restrict__ slots,
                                                    const float2* __restrict__ snap, OptParams op,
                                                    SelfSeg self,
                                                    const int* __restrict__ slots32 = nullptr,
                                                    float* __restrict__ lacc = nullptr,
                                                    float* __restrict__ lacc_out = nullptr,
                                                    int lacc_n = 0,
                                                    const uint64_t* __restrict__ bkeys = nullptr,
                                                    int dbg = 0) {
  __shared__ float acc[kBdTS];
  const int b = blockIdx.x;
  // the step's loss accumulator (added by the forward, ordered before this
  // launch) moves to lacc_out and is left zero: no zero-fill launch per step
  if (lacc)
    for (int i = b * RT + threadIdx.x; i < lacc_n; i += gridDim.x * RT) {
      lacc_out[i] = lacc[i];
      lacc[i] = 0.f;
    }
  const uint32_t p0 = bstart[b], p1 = bstart[b + 1], nu = unum[b];
  const uint32_t base = osi ? p0 : ubase[b];  // rows in occurrence space or compact
  for (uint32_t l = threadIdx.x; l < nu; l += RT) acc[l] = 0.f;
  __syncthreads();
  // OCC occurrences per thread in flight (loads before the LDS atomics)
  for (uint32_t pb = p0 + threadIdx.x; pb < p1; pb += OCC * RT) {
    uint32_t l[OCC], j[OCC];
    float g[OCC];
#pragma unroll
    for (int r = 0; r < OCC; ++r) {
      const uint32_t p = pb + r * RT;
      l[r] = p < p1 ? luid[p] : kBdInvalid;  // bucket-local unique id
      j[r] = p < p1 ? pj[p] : 0u;
    }
#pragma unroll
    for (int r = 0; r < OCC; ++r) {
      g[r] = l[r] != kBdInvalid ? ((dbg & 2) ? 1.f : self.grad(gs, j[r], (uint32_t)F)) : 0.f;
      if (xval && l[r] != kBdInvalid) g[r] *= xval[j[r]];
    }
    // keys occurring once in the batch (usingle, from the dedup): a plain
    // LDS store — LDS float atomics are this kernel's cost (~6 us per 1M)
#pragma unroll
    for (int r = 0; r < OCC; ++r) {
      if (l[r] == kBdInvalid) continue;
      if ((dbg & 1) || (usingle && !(dbg & 8) && usingle[ubase[b] + l[r]]))
        acc[l[r]] = g[r];
      else
        atomicAdd(&acc[l[r]], g[r]);
    }
  }
  __syncthreads();
  if (slots || slots32) {
    // fused K5 (scalar AdaGrad rows): the merged gradient goes straight into
    // the optimizer update — from the (w, h) the pull snapshot (coalesced,
    // then one blind 8-byte store per key), or read from the row when no
    // snapshot is valid (N>1 servers with pull-ahead: a read-modify-write).
    // slots32: the pull stored 4-byte slot indices (tables under 2^31 slots)
    // bkeys (claimed pulls, k_pull_claim_bk): the slot of a new key holds
    // nothing yet — store the whole [w | h | key] slot in one 16-byte store
    // (the key of a found key is rewritten unchanged), the bucket's unique
    // keys read coalesced from the dedup's staging
    // OCC rows per thread: every row's slot, snapshot and key loads in
    // flight before the first store
    for (uint32_t l0 = threadIdx.x; l0 < nu; l0 += OCC * RT) {
      long long sl[OCC];
      float2 wh[OCC];
      uint64_t key[OCC];
#pragma unroll
      for (int r = 0; r < OCC; ++r) {
        const uint32_t l = l0 + r * RT;
        sl[r] = l < nu ? (slots32 ? (long long)slots32[base + l] : slots[base + l]) : -1;
        if (snap && l < nu) wh[r] = snap[base + l];
        key[r] = bkeys && l < nu ? bkeys[p0 + l] : 0ull;
      }
#pragma unroll
      for (int r = 0; r < OCC; ++r) {
        const uint32_t l = l0 + r * RT;
        if (sl[r] < 0 || (dbg & 4)) continue;
        if (!snap) wh[r] = *reinterpret_cast<const float2*>(slot_row(t, sl[r]));
        float s2 = 0.f;
        opt_update(op, wh[r].x, wh[r].y, s2, acc[l]);
        if (bkeys) {
          *reinterpret_cast<uint4*>(t.base + (uint64_t)sl[r] * 16) =
              make_uint4(__float_as_uint(wh[r].x), __float_as_uint(wh[r].y), (uint32_t)key[r],
                         (uint32_t)(key[r] >> 32));
        } else {
          *reinterpret_cast<float2*>(slot_row(t, sl[r])) = wh[r];
        }
      }
    }
    return;
  }
  for (uint32_t l = threadIdx.x; l < nu; l += RT) ugrad[base + l] = acc[l];
}

// SS_BD_ROCC: occurrences per thread in flight in k_bd_reduce (2, 4 or 8);
// SS_BD_RT: its workgroup size (256, 512, 1024)
static int bd_rocc() {
  static const int v = [] {
    const char* e = std::getenv("SS_BD_ROCC");
    const int x = e ? std::atoi(e) : 4;
    return x == 2 || x == 8 ? x : 4;
  }();
  return v;
}
static int bd_rt() {
  static const int v = [] {
    const char* e = std::getenv("SS_BD_RT");
    const int x = e ? std::atoi(e) : 1024;
    return x == 256 || x == 512 ? x : 1024;
  }();
  return v;
}
// one launch of k_bd_reduce over P buckets at the (SS_BD_RT, SS_BD_ROCC)
// shape: (1024, 2 / 4), (512, 2 / 4 / 8), (256, 2); others fall back to (1024, 4)
// SS_BD_DBG (measurement only; wrong results): 1 = plain LDS stores for
// every occurrence, 2 = no gradient gather, 4 = no table stores, 8 = atomics
// for single-occurrence keys too
static int bd_dbg() {
  static const int v = [] {
    const char* e = std::getenv("SS_BD_DBG");
    const int d = e ? std::atoi(e) : 0;
    if (d)
      std::fprintf(stderr, "swiftsnails_amd: SS_BD_DBG=%d — k_bd_reduce runs a timing-only "
                           "variant, training results are WRONG\n", d);
    return d;
  }();
  return v;
}
template <typename... A>
static void bd_reduce_launch(int P, hipStream_t st, A... a) {
  const int rt = bd_rt(), oc = bd_rocc(), dbg = bd_dbg();
  if (rt == 512 && oc == 8)
    hipLaunchKernelGGL((k_bd_reduce<512, 8>), dim3(P), dim3(512), 0, st, a..., dbg);
  else if (rt == 512 && oc == 4)
    hipLaunchKernelGGL((k_bd_reduce<512, 4>), dim3(P), dim3(512), 0, st, a..., dbg);
  else if (rt == 512)
    hipLaunchKernelGGL((k_bd_reduce<512, 2>), dim3(P), dim3(512), 0, st, a..., dbg);
  else if (rt == 256)
    hipLaunchKernelGGL((k_bd_reduce<256, 2>), dim3(P), dim3(256), 0, st, a..., dbg);
  else if (oc == 2)
    hipLaunchKernelGGL((k_bd_reduce<1024, 2>), dim3(P), dim3(1024), 0, st, a..., dbg);
  else
    hipLaunchKernelGGL((k_bd_reduce<1024, 4>), dim3(P), dim3(1024), 0, st, a..., dbg);
}

// K7 for FM rows [w | v_1..v_K]: per unique key u with occurrences in samples
// S(u):  grad = [G0, G_f - v_uf * G0],  G0 = sum gs[s],  G_f = sum gss[s][f].
// Columns are accumulated in LDS, as many per pass over the bucket's
// occurrences (L2-resident) as fit next to G0 in 160 KB: every column in one
// pass up to K = 8 (9 x 16 KB), so the occurrence list is read once; then
// each row is stored once.
template <int K>
struct FmCols {
  static constexpr int v = (K + 1) * kBdTS * 4 <= 150 * 1024 ? K : 8;
};
// Fused K5 for a DIM-wide row whose merged gradient is in registers: the
// optimizer update as one read-modify-write of the row (one thread per row;
// the DIM coordinates and their state stay in registers).  The model kernels
// below call it instead of storing ugrad when the engine fuses the apply
// (PSEngine.fuse_apply: one GPU, compact unique ids).
// FM k = 8 rows in fp32 keyfirst slots (80 bytes: [key | w_0..w_8 | s_0..s_8]
// with one state word per coordinate, AdaGrad / SGD-state layouts): the 72-byte
// row moves as one 8-byte and four 16-byte accesses per thread, all five loads
// in flight together, instead of 18 dependent-address 4-byte row_ld / row_st
// (the one-thread-per-row update that measured 0.62 -> 1.04 ms per FM step)
__device__ __forceinline__ bool fm9_vec_ok(const DevTable& t, const OptParams& op) {
  return !t.bf16 && t.dim == 9 && t.stride == 80 && t.row_off == 8 &&
         opt_state_per_coord(op.kind) == 1;
}
__device__ __forceinline__ void fm9_row_update(const DevTable& t, long long slot,
                                               const float (&g)[9], const OptParams& op) {
  float* row = slot_row(t, (uint64_t)slot);  // 8-byte aligned; row + 2 is 16-byte aligned
  float r[18];
  const float2 a = *reinterpret_cast<const float2*>(row);
  const float4* q4 = reinterpret_cast<const float4*>(row + 2);
  float4 q[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) q[i] = q4[i];
  r[0] = a.x, r[1] = a.y;
#pragma unroll
  for (int i = 0; i < 4; ++i)
    r[2 + 4 * i] = q[i].x, r[3 + 4 * i] = q[i].y, r[4 + 4 * i] = q[i].z, r[5 + 4 * i] = q[i].w;
  float s2 = 0.f;
#pragma unroll
  for (int j = 0; j < 9; ++j) opt_update(op, r[j], r[9 + j], s2, g[j]);
  *reinterpret_cast<float2*>(row) = make_float2(r[0], r[1]);
  float4* o4 = reinterpret_cast<float4*>(row + 2);
#pragma unroll
  for (int i = 0; i < 4; ++i)
    o4[i] = make_float4(r[2 + 4 * i], r[3 + 4 * i], r[4 + 4 * i], r[5 + 4 * i]);
}

template <int DIM>
__device__ __forceinline__ void fused_row_update(const DevTable& t, long long slot,
                                                 const float (&g)[DIM], const OptParams& op) {
  if (slot < 0) return;
  if constexpr (DIM == 9) {
    if (fm9_vec_ok(t, op)) {
      fm9_row_update(t, slot, g, op);
      return;
    }
  }
  const int ns = opt_state_per_coord(op.kind);
  float w[DIM], s1[DIM], s2[DIM];
#pragma unroll
  for (int j = 0; j < DIM; ++j) {
    w[j] = row_ld(t, slot, j);
    s1[j] = ns > 0 ? row_ld(t, slot, DIM + j) : 0.f;
    s2[j] = ns > 1 ? row_ld(t, slot, 2 * DIM + j) : 0.f;
  }
#pragma unroll
  for (int j = 0; j < DIM; ++j) {
    opt_update(op, w[j], s1[j], s2[j], g[j]);
    row_st(t, slot, j, w[j], true);
    if (ns > 0) row_st(t, slot, DIM + j, s1[j], true);
    if (ns > 1) row_st(t, slot, 2 * DIM + j, s2[j], true);
  }
}

template <int DIM, int NCOLS = 0>
__global__ __launch_bounds__(1024) void k_bd_reduce_fm(const uint32_t* __restrict__ bstart,
                                                       const uint32_t* __restrict__ ubase,
                                                       const uint32_t* __restrict__ unum,
                                                       const uint32_t* __restrict__ pj,
                                                       const uint32_t* __restrict__ luid,
                                                       const float* __restrict__ gs,
                                                       const float* __restrict__ gss, int F,
                                                       const float* __restrict__ uvals,
                                                       float* __restrict__ ugrad,
                                                       const uint32_t* __restrict__ blist,
                                                       DevTable t = DevTable{},
                                                       const long long* __restrict__ slots = nullptr,
                                                       OptParams op = OptParams{}) {
  constexpr int K = DIM - 1;
  constexpr int NC = NCOLS > 0 ? (NCOLS < K ? NCOLS : K) : FmCols<K>::v;
  __shared__ float g0[kBdTS];
  __shared__ float acc[NC][kBdTS];
  // blist: only the buckets listed there ({count, b...}, the sorted kernel's
  // overflow list), one per workgroup
  if (blist && blockIdx.x >= blist[0]) return;
  const int b = blist ? (int)blist[1 + blockIdx.x] : (int)blockIdx.x;
  const uint32_t p0 = bstart[b], p1 = bstart[b + 1], nu = unum[b], base = ubase[b];
  // gridDim.y > 1: workgroup y of the bucket takes column group y alone (the
  // bucket's column passes run on different CUs); each accumulates G0 itself
  const int cstart = gridDim.y > 1 ? (int)blockIdx.y * NC : 0;
  const int cend = gridDim.y > 1 ? min(K, cstart + NC) : K;
  for (int c0 = cstart; c0 < cend; c0 += NC) {
    const bool first = c0 == cstart;
    for (uint32_t l = threadIdx.x; l < nu; l += 1024) {
      if (first) g0[l] = 0.f;
#pragma unroll
      for (int c = 0; c < NC; ++c) acc[c][l] = 0.f;
    }
    __syncthreads();
    // two occurrences per thread in flight: every load of both issued before
    // the first LDS atomic (the loop is a latency chain otherwise)
    constexpr int RB = 2;
    for (uint32_t pb = p0 + threadIdx.x; pb < p1; pb += 1024 * RB) {
      uint32_t l[RB], sm[RB];
#pragma unroll
      for (int r = 0; r < RB; ++r) {
        const uint32_t p = pb + r * 1024;
        l[r] = p < p1 ? luid[p] : kBdInvalid;  // bucket-local unique id
        sm[r] = p < p1 ? pj[p] : 0u;
      }
      float g[RB], v[RB][NC];
#pragma unroll
      for (int r = 0; r < RB; ++r) {
        const uint32_t s = sm[r] / (uint32_t)F;
        g[r] = (first && l[r] != kBdInvalid) ? gs[s] : 0.f;
        if constexpr (NC == K && K % 4 == 0) {
          // whole 32-B-aligned row of the sample: 16-B vector loads
          const float4* g4 = reinterpret_cast<const float4*>(gss + (size_t)s * K);
#pragma unroll
          for (int q = 0; q < K / 4; ++q) {
            const float4 x = l[r] != kBdInvalid ? g4[q] : make_float4(0.f, 0.f, 0.f, 0.f);
            v[r][4 * q] = x.x, v[r][4 * q + 1] = x.y, v[r][4 * q + 2] = x.z, v[r][4 * q + 3] = x.w;
          }
        } else {
#pragma unroll
          for (int c = 0; c < NC; ++c)
            v[r][c] = (l[r] != kBdInvalid && c0 + c < K) ? gss[(size_t)s * K + c0 + c] : 0.f;
        }
      }
#pragma unroll
      for (int r = 0; r < RB; ++r) {
        if (l[r] == kBdInvalid) continue;
        if (first) atomicAdd(&g0[l[r]], g[r]);
#pragma unroll
        for (int c = 0; c < NC; ++c)
          if (c0 + c < K) atomicAdd(&acc[c][l[r]], v[r][c]);
      }
    }
    __syncthreads();
    // rows out element-major (consecutive lanes -> consecutive floats of the
    // bucket's contiguous [nu][DIM] block): coalesced uvals reads / ugrad stores
    const uint32_t ncol = c0 == 0 ? 1u + (uint32_t)min(NC, K - c0) : (uint32_t)min(NC, K - c0);
    const uint32_t col0 = c0 == 0 ? 0u : 1u + (uint32_t)c0;
    if (ncol == (uint32_t)DIM) {
      const size_t r0 = (size_t)base * DIM;
      for (uint32_t e = threadIdx.x; e < nu * (uint32_t)DIM; e += 1024) {
        const uint32_t l = e / (uint32_t)DIM, c = e - l * (uint32_t)DIM;
        const float G0 = g0[l];
        ugrad[r0 + e] = c == 0 ? G0 : acc[c - 1][l] - uvals[r0 + e] * G0;
      }
    } else {
      for (uint32_t e = threadIdx.x; e < nu * ncol; e += 1024) {
        const uint32_t l = e / ncol, c = col0 + (e - l * ncol);
        const size_t r = (size_t)(base + l) * DIM + c;
        const float G0 = g0[l];
        ugrad[r] = c == 0 ? G0 : acc[c - 1 - c0][l] - uvals[r] * G0;
      }
    }
    __syncthreads();
  }
  if (slots) {
    // fused K5 (single column pass group, gridDim.y == 1): this workgroup's
    // rows of ugrad are complete after the barrier above
    for (uint32_t l = threadIdx.x; l < nu; l += 1024) {
      float g[DIM];
#pragma unroll
      for (int j = 0; j < DIM; ++j) g[j] = ugrad[(size_t)(base + l) * DIM + j];
      fused_row_update<DIM>(t, slots[base + l], g, op);
    }
  }
}

// compact unique rows (ubase[b] + l, the alltoallv layout) -> occurrence-space
// rows (bstart[b] + l): the N>1 pull returns rows compact, the osi consumers
// (LR forward through osi_inv) read them in occurrence space
__global__ __launch_bounds__(256) void k_bd_unplace(const uint32_t* __restrict__ bstart,
                                                    const uint32_t* __restrict__ unum,
                                                    const uint32_t* __restrict__ ubase,
                                                    const float* __restrict__ src,
                                                    float* __restrict__ dst, int dim) {
  const int b = blockIdx.x;
  const unsigned int n = unum[b] * (unsigned int)dim;
  const float* s = src + (size_t)ubase[b] * dim;
  float* d = dst + (size_t)bstart[b] * dim;
  for (unsigned int e = threadIdx.x; e < n; e += 256) d[e] = s[e];
}

// K7 for FM rows without float atomics.  Measured: the LDS form above is
// bound by its 1 + K ds_add_f32 per occurrence (212 us per 2.56M keys at
// K = 8; 63 us with plain stores in their place).  Here each bucket's
// occurrences are grouped by unique id with a counting sort in LDS (two
// integer LDS atomics per occurrence), then every unique key's occurrence
// list is summed in registers — one thread per short list, one wave per list
// longer than kFmLong (Zipf heads: thousands of occurrences) — and its row
// is stored once.  Buckets with more than kFmOcc occurrences are listed in
// `ovf` for the LDS-atomic kernel above.
static constexpr int kFmOcc = 10240;  // occurrences sorted in LDS per bucket (76 KB: 2 per CU)
static constexpr int kFmLong = 16;    // longer lists: one wave each
template <int DIM>
__global__ __launch_bounds__(1024) void k_bd_reduce_fm_sorted(
    const uint32_t* __restrict__ bstart, const uint32_t* __restrict__ ubase,
    const uint32_t* __restrict__ unum, const uint32_t* __restrict__ pj,
    const uint32_t* __restrict__ luid, const float* __restrict__ gs,
    const float* __restrict__ gss, int F, const float* __restrict__ uvals,
    float* __restrict__ ugrad, uint32_t* __restrict__ ovf, DevTable t,
    const long long* __restrict__ slots, OptParams op) {
  constexpr int K = DIM - 1;
  __shared__ uint32_t cnt[kBdTS];      // counts, then placement cursors
  __shared__ uint32_t seg[kBdTS + 1];  // list starts (exclusive scan of the counts)
  __shared__ uint32_t ord[kFmOcc];     // sample index of each occurrence, grouped by id
  __shared__ uint32_t longl[kFmOcc / (kFmLong + 1) + 1];
  __shared__ uint32_t nlong;
  __shared__ unsigned int wsum[16];
  __shared__ unsigned int tot;
  const int b = blockIdx.x, tid = threadIdx.x;
  const uint32_t p0 = bstart[b], p1 = bstart[b + 1], nu = unum[b], base = ubase[b];
  if (p1 - p0 > (uint32_t)kFmOcc) {  // workgroup-uniform
    if (tid == 0) ovf[1 + atomicAdd(&ovf[0], 1u)] = (uint32_t)b;
    return;
  }
  for (uint32_t l = tid; l < nu; l += 1024) cnt[l] = 0u;
  if (tid == 0) nlong = 0u;
  __syncthreads();
  for (uint32_t p = p0 + tid; p < p1; p += 1024) {
    const uint32_t l = luid[p];
    if (l != kBdInvalid) atomicAdd(&cnt[l], 1u);
  }
  __syncthreads();
  // exclusive scan of the nu <= 4096 counts, 4 per thread
  uint32_t c4[4], sum = 0;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const uint32_t l = 4 * tid + k;
    c4[k] = l < nu ? cnt[l] : 0u;
    sum += c4[k];
  }
  uint32_t e = block_excl_scan<16>(sum, wsum, &tot);
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const uint32_t l = 4 * tid + k;
    if (l < nu) {
      seg[l] = e;
      cnt[l] = e;
      if (c4[k] > (uint32_t)kFmLong) longl[atomicAdd(&nlong, 1u)] = l;
    }
    e += c4[k];
  }
  if (tid == 0) seg[nu] = tot;
  __syncthreads();
  for (uint32_t p = p0 + tid; p < p1; p += 1024) {
    const uint32_t l = luid[p];
    if (l != kBdInvalid) ord[atomicAdd(&cnt[l], 1u)] = pj[p] / (uint32_t)F;
  }
  __syncthreads();
  // one unique key's sums over sample rows [q0, q1) of its list, step `st`
  auto accumulate = [&](uint32_t q0, uint32_t q1, uint32_t st, float& g0, float* a) {
    for (uint32_t q = q0; q < q1; q += st) {
      const uint32_t sm = ord[q];
      g0 += gs[sm];
      if constexpr (K % 4 == 0) {
        const float4* g4 = reinterpret_cast<const float4*>(gss + (size_t)sm * K);
#pragma unroll
        for (int k = 0; k < K / 4; ++k) {
          const float4 x = g4[k];
          a[4 * k] += x.x, a[4 * k + 1] += x.y, a[4 * k + 2] += x.z, a[4 * k + 3] += x.w;
        }
      } else {
#pragma unroll
        for (int k = 0; k < K; ++k) a[k] += gss[(size_t)sm * K + k];
      }
    }
  };
  auto store_row = [&](uint32_t l, float g0, const float* a) {
    const size_t r = (size_t)(base + l) * DIM;
    if (slots) {  // fused K5: the row's update instead of its gradient store
      float g[DIM];
      g[0] = g0;
#pragma unroll
      for (int k = 0; k < K; ++k) g[1 + k] = a[k] - uvals[r + 1 + k] * g0;
      fused_row_update<DIM>(t, slots[base + l], g, op);
      return;
    }
    ugrad[r] = g0;
#pragma unroll
    for (int k = 0; k < K; ++k) ugrad[r + 1 + k] = a[k] - uvals[r + 1 + k] * g0;
  };
  // fused FM k = 8 update with vector rows: the key's slot, its table row
  // and its pulled v go out BEFORE the occurrence gathers, so the row's
  // read latency overlaps the sum instead of following it
  bool vec9 = false;
  if constexpr (DIM == 9) vec9 = slots != nullptr && fm9_vec_ok(t, op);
  // short lists: a thread per unique key
  for (uint32_t l = tid; l < nu; l += 1024) {
    const uint32_t q0 = seg[l], q1 = seg[l + 1];
    if (q1 - q0 > (uint32_t)kFmLong) continue;
    float g0 = 0.f, a[K];
#pragma unroll
    for (int k = 0; k < K; ++k) a[k] = 0.f;
    if constexpr (DIM == 9) {
      if (vec9) {
        const long long slot = slots[base + l];
        const size_t r = (size_t)(base + l) * DIM;
        float v[K], row[18];
#pragma unroll
        for (int k = 0; k < K; ++k) v[k] = uvals[r + 1 + k];
        float* rp = slot >= 0 ? slot_row(t, (uint64_t)slot) : nullptr;
        if (rp) {
          const float2 x = *reinterpret_cast<const float2*>(rp);
          const float4* q4 = reinterpret_cast<const float4*>(rp + 2);
          row[0] = x.x, row[1] = x.y;
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const float4 y = q4[i];
            row[2 + 4 * i] = y.x, row[3 + 4 * i] = y.y, row[4 + 4 * i] = y.z, row[5 + 4 * i] = y.w;
          }
        }
        accumulate(q0, q1, 1u, g0, a);
        if (!rp) continue;
        float s2 = 0.f;
        opt_update(op, row[0], row[9], s2, g0);
#pragma unroll
        for (int k = 0; k < K; ++k) opt_update(op, row[1 + k], row[10 + k], s2, a[k] - v[k] * g0);
        *reinterpret_cast<float2*>(rp) = make_float2(row[0], row[1]);
        float4* o4 = reinterpret_cast<float4*>(rp + 2);
#pragma unroll
        for (int i = 0; i < 4; ++i)
          o4[i] = make_float4(row[2 + 4 * i], row[3 + 4 * i], row[4 + 4 * i], row[5 + 4 * i]);
        continue;
      }
    }
    accumulate(q0, q1, 1u, g0, a);
    store_row(l, g0, a);
  }
  // long lists: a wave per unique key, lanes stride the list, wave-reduced
  const int lane = tid & 63, w = tid >> 6;
  for (uint32_t i = w; i < nlong; i += 16) {
    const uint32_t l = longl[i];
    float g0 = 0.f, a[K];
#pragma unroll
    for (int k = 0; k < K; ++k) a[k] = 0.f;
    accumulate(seg[l] + lane, seg[l + 1], 64u, g0, a);
    for (int o = 32; o > 0; o >>= 1) {
      g0 += __shfl_xor(g0, o, 64);
#pragma unroll
      for (int k = 0; k < K; ++k) a[k] += __shfl_xor(a[k], o, 64);
    }
    if (lane == 0) store_row(l, g0, a);
  }
}

// grouped record layout: the per-bucket regroup after the scatter (defined
// with the record-exchange kernels below)
static constexpr int kRgT = 512;
__global__ __launch_bounds__(kRgT) void k_rec_group(const uint32_t* __restrict__ rstart,
                                                    const uint32_t* __restrict__ rnum,
                                                    const uint64_t* __restrict__ gkeys,
                                                    const uint32_t* __restrict__ gspj,
                                                    uint64_t* __restrict__ skeys,
                                                    uint32_t* __restrict__ spj,
                                                    uint32_t* __restrict__ pos_of,
                                                    uint32_t* __restrict__ usub, int msub, int Pd,
                                                    int rbits);

// ------------------------------------------------------------- launchers
int launch_bd_dedup(const uint64_t* keys, long long n, RouteSpec rs, long long ucap,
                    uint32_t* scratch, uint32_t* pj, uint32_t* pos_of, uint32_t* bkt,
                    uint32_t* luid, uint64_t* bkeys, unsigned long long* ucount, uint64_t* ukeys,
                    float* ugrad, int gdim, uint32_t* inv, int place, hipStream_t st,
                    unsigned long long* dbg, uint32_t* rec, uint8_t* usingle, int ndest,
                    long long lay_n, int msub, uint32_t* usub, uint32_t* spj, uint64_t* gkeys,
                    uint32_t* gspj) {
  if (rs.nranks < 1 || rs.nranks > kMaxSeg) throw_error("bdedup: bad nranks");
  // spj (record exchange): no dedup — count, column scan into send-segment
  // positions (d * ucap + ...) with the run tables and per-destination
  // counts, then the scatter writes every occurrence's key into ukeys and its
  // index into spj at that position (the servers dedup what they receive)
  // grouped records (kBdRecGroup, msub > 1): the scatter writes into the
  // staging (gkeys, gspj) and k_rec_group moves each bucket's run into the
  // send segment grouped by the servers' sub-bucket
  const bool grouped = spj && (ndest & kBdRecGroup) && msub > 1;
  if (spj && (!ukeys || !ucount || rs.nranks > kRecMaxDest || !pos_of ||
              !(ndest & kBdRecLayout) || (msub != 1 && !grouped) ||
              (grouped && (!gkeys || !gspj || !usub))))
    throw_error("bdedup: the record exchange needs ukeys, ucount, pos_of, <= 64 ranks and the "
                "record layout; sub-buckets only grouped (with the staging and offsets)");
  if (rs.rbits < 0 || rs.rbits > 20) throw_error("bdedup: region bits 0..20");
  if (msub < 1 || msub > kBdMaxSub || (msub > 1 && !usub))
    throw_error("bdedup: server sub-buckets 1..64 (and their offset table)");
  // lay_n (N>1 engines): the bucket layout is that of a call of lay_n keys
  // whatever this call's n, so every rank splits a destination's keys into
  // the same Pd buckets (the servers merge bucket k of all sources); an empty
  // call then still writes an all-empty layout
  if (lay_n > 0 && lay_n < n) throw_error("bdedup: lay_n below the call's key count");
  const long long ln = lay_n > 0 ? lay_n : n;
  if (ln <= 0) {
    check_hip(hipMemsetAsync(ucount, 0, sizeof(unsigned long long) * rs.nranks, st), "ucount");
    return 0;
  }
  if (ucap < n) throw_error("bdedup: per-destination capacity must be >= n");
  if ((unsigned long long)rs.nranks * (unsigned long long)ucap >= 0x7FFFFFFFull)
    throw_error("bdedup: nranks*ucap overflows 31-bit unique ids");
  if (!rec) throw_error("bdedup: the bucket-ordered key buffer is required");
  const BdLayout L = bd_layout(ln, rs.nranks, ndest);
  if ((long long)L.Pd * bd_clamp_ndest(rs.nranks, ndest) > kBdMaxBuckets + kMaxSeg ||
      ln > bd_max_keys())
    throw_error("bdedup: too many keys per call (max ~45M)");
  // region buckets: only when every (server sub-)bucket gets >= 4 regions,
  // so the floor(region * Pd * msub / R) split keeps buckets within ~25% of
  // the target (a region's keys cannot be split over buckets); else
  // dedup-hash buckets.  A function of the layout only: every rank of an
  // N>1 job decides the same
  if (rs.rbits && 4ll * L.Pd * msub > (1ll << rs.rbits)) rs.rbits = 0;
  // ... and only when the fullest bucket — ceil(R / Pd) whole regions of a
  // destination's keys — still fits the dedup's 4096-slot LDS table with
  // every key distinct (R / Pd just above 4 puts 5 regions, 1.25x the target,
  // into some buckets: ~4480 occurrences at the one-rank target).  The hash
  // buckets' sizes vary by ~2 %; 3800 leaves that margin
  if (rs.rbits) {
    const long long R = 1ll << rs.rbits;
    const long long per_dest = (ln + bd_clamp_ndest(rs.nranks, ndest) - 1) /
                               bd_clamp_ndest(rs.nranks, ndest);
    if ((R + L.Pd - 1) / L.Pd * per_dest > 3800ll * R) rs.rbits = 0;
  }
  uint32_t* S = scratch;
  const size_t lds = sizeof(unsigned int) * (size_t)L.P;
  // workgroup sizes (256/512/1024): count (SS_BD_CNT), column scan
  // (SS_BD_CS), scatter (SS_BD_CT).  Measured in the pipelined bench, where
  // the route stream shares the chip with the pull/forward kernels
  auto wg_env = [](const char* name, int def) {
    const char* e = std::getenv(name);
    const int v = e ? std::atoi(e) : def;
    return (v == 256 || v == 512 || v == 1024) ? v : def;
  };
  static const int ct = wg_env("SS_BD_CT", 1024);
  // count: 1024 threads.  (256 on the N>1 path paid while its rounds pulled
  // ahead — the count then ran beside the server pull and waited for 16 free
  // wave slots on one CU; with synchronous rounds 1024 measured better: 8
  // ranks on one GPU 8.66-8.74 vs 8.71-9.26 ms per 8-rank step, the 1-rank
  // N>1 path 1.076-1.103 vs 1.109-1.169 ms)
  static const int cnt = wg_env("SS_BD_CNT", 1024);
  static const int cs = wg_env("SS_BD_CS", 1024);
  // key width of the hand-off (SS_BD_REC): auto (default: 4 bytes when
  // every key of the call fits 32 bits, else 8) or 8
  static const bool narrow_ok = [] {
    const char* e = std::getenv("SS_BD_REC");
    return !(e && std::atoi(e) >= 8);
  }();
  uint32_t* wacc = narrow_ok ? S + L.wacc : nullptr;
  uint32_t* wfin = S + L.wfin;
#define SS_BD_CT_DISPATCH(ct, KERNEL, ...)                                                    \
  switch (ct) {                                                                               \
    case 256: hipLaunchKernelGGL(KERNEL<256>, dim3(L.nch), dim3(256), lds, st, __VA_ARGS__); break; \
    case 512: hipLaunchKernelGGL(KERNEL<512>, dim3(L.nch), dim3(512), lds, st, __VA_ARGS__); break; \
    default: hipLaunchKernelGGL(KERNEL<1024>, dim3(L.nch), dim3(1024), lds, st, __VA_ARGS__);     \
  }
#define SS_BD_CT_DISPATCH2(ct, RW, KERNEL, ...)                                                  \
  switch (ct) {                                                                               \
    case 256: hipLaunchKernelGGL((KERNEL<256, RW>), dim3(L.nch), dim3(256), lds, st, __VA_ARGS__); break; \
    case 512: hipLaunchKernelGGL((KERNEL<512, RW>), dim3(L.nch), dim3(512), lds, st, __VA_ARGS__); break; \
    default: hipLaunchKernelGGL((KERNEL<1024, RW>), dim3(L.nch), dim3(1024), lds, st, __VA_ARGS__);     \
  }
  SS_BD_CT_DISPATCH(cnt, k_bd_count, keys, n, rs, L.Pd, L.P, L.chunk, S + L.hist, ucount, wacc);
  RecLay rl{};
  if (spj) rl = RecLay{ucap, L.Pd, ucount, S + L.ubase, S + L.unum, S};
  check_launch("k_bd_count");
  switch (cs) {
#define SS_BD_CS_CASE(CS)                                                                      \
  case CS:                                                                                     \
    hipLaunchKernelGGL(k_bd_colscan<CS>, dim3((L.P + 63) / 64), dim3(CS), 0, st, S + L.hist,   \
                       L.nch, L.P, S + L.btot, S + L.bstart, S + L.ctr, wacc, wfin, rl);       \
    break;
    SS_BD_CS_CASE(256)
    SS_BD_CS_CASE(512)
    SS_BD_CS_CASE(1024)
#undef SS_BD_CS_CASE
  }
  check_launch("k_bd_colscan");
  // the LDS-sorted scatter (12- / 8-byte records): the largest tile whose
  // workgroup fits the LDS (a P of up to ~16K buckets takes 2048-key tiles)
  static const bool sorted = [] {
    const char* e = std::getenv("SS_BD_SORT");
    return !(e && e[0] == '0');
  }();
  auto s_lds = [&](int kt) { return sizeof(unsigned int) * (2 * (size_t)L.P + 1 + 2 * (size_t)kt * 1024); };
  const size_t kLdsMax = 160 * 1024 - 256;
  // SS_BD_SKT: the largest keys-per-thread tile to try (16 measured best)
  static const int skt_max = [] {
    const char* e = std::getenv("SS_BD_SKT");
    return e ? std::atoi(e) : 16;
  }();
  int skt = 0;
  for (int kt = 16; kt >= 2 && !skt; kt /= 2)
    if (kt <= skt_max && s_lds(kt) <= kLdsMax) skt = kt;
  if (sorted && skt && L.P < 65536) {
    if (L.chunk % 1024) throw_error("bdedup: chunk not a multiple of 1024");
    switch (skt) {
#define SS_BD_S_CASE(KT)                                                                          \
  case KT: {                                                                                      \
    static const bool attr = (check_hip(hipFuncSetAttribute((const void*)k_bd_scatter_s<KT>,       \
                                                            hipFuncAttributeMaxDynamicSharedMemorySize, \
                                                            (int)kLdsMax),                        \
                                        "k_bd_scatter_s LDS"),                                    \
                              true);                                                              \
    (void)attr;                                                                                   \
    hipLaunchKernelGGL(k_bd_scatter_s<KT>, dim3(L.nch), dim3(1024), s_lds(KT), st, keys, n, rs,  \
                       L.Pd, L.P, L.chunk, S + L.hist, S + L.bstart, pos_of, bkt, rec, wfin,      \
                       bd_xcd(), spj ? (grouped ? gkeys : ukeys) : nullptr,                       \
                       grouped ? gspj : spj, pj);                                                 \
  } break;
      SS_BD_S_CASE(16)
      SS_BD_S_CASE(8)
      SS_BD_S_CASE(4)
      SS_BD_S_CASE(2)
#undef SS_BD_S_CASE
    }
  } else
    SS_BD_CT_DISPATCH2(ct, 3, k_bd_scatter, keys, n, rs, L.Pd, L.P, L.chunk, S + L.hist,
                       S + L.bstart, pj, pos_of, bkt, rec, wfin,
                       bd_xcd(), spj ? (grouped ? gkeys : ukeys) : nullptr, grouped ? gspj : spj)
#undef SS_BD_CT_DISPATCH
#undef SS_BD_CT_DISPATCH2
  check_launch("k_bd_scatter");
  if (grouped) {
    hipLaunchKernelGGL(k_rec_group, dim3(L.P), dim3(kRgT), 0, st, S + L.ubase, S + L.unum, gkeys,
                       gspj, ukeys, spj, pos_of, usub, msub, L.Pd, rs.rbits);
    check_launch("k_rec_group");
  }
  if (spj) return rs.rbits;  // record exchange: the servers dedup
  // place: unique keys straight into the per-destination send segments
  // (+ zeroed gradient rows), reserved with one atomic per bucket
  hipLaunchKernelGGL(k_bd_dedup<3>, dim3(L.P), dim3(kBdDT), 0, st, keys, pj, S + L.bstart, luid,
                     bkeys, S + L.unum, S, L.Pd, ucap, S + L.ubase, ucount, rec, dbg,
                     place ? ukeys : nullptr, place ? ugrad : nullptr, gdim, usingle, msub, usub,
                     wfin, rs.rbits);
  check_launch("k_bd_dedup");
  if (inv && n > 0) {
    if (!pos_of || !bkt) throw_error("bdedup: the compact inverse needs pos_of and bkt");
    BdIndex ix{pos_of, luid, bkt, S + L.ubase};
    hipLaunchKernelGGL(k_bd_inv, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, ix, n, inv);
    check_launch("k_bd_inv");
  }
  return rs.rbits;  // the region bits the buckets follow (0: dedup-hash buckets)
}

// ---- record exchange, worker side (N>1 scalar rows; bd_set_record_layout)
//
// The rows of a step come back at the send-segment positions of its
// occurrences, so the forward reads occ[pos_of[j]] from the rows mailbox —
// its own destination's rows from a cached buffer the server fill wrote
// instead (SelfSeg) — and its per-sample gradient goes out per occurrence:
// grec[p] = gs[spj[p] / F] * x[spj[p]] at the same positions, except for the
// own destination, whose server merge reads gs through spj itself.
// The servers merge them per distinct key with the update fused (server.hip):
// no worker dedup, no worker merge.  The destinations' ranges
// [d * gap, d * gap + ucount[d]) are walked as one flat list.
// skip: a destination whose range is left out (-1: none)
__device__ __forceinline__ void rec_ranges(const unsigned long long* __restrict__ ucount, int nd,
                                           long long gap, long long* cs, int skip = -1) {
  if (threadIdx.x == 0) {
    long long a = 0;
    for (int d = 0; d < nd; ++d) {
      cs[d] = a;
      if (d != skip) a += (long long)min(ucount[d], (unsigned long long)gap);
    }
    cs[nd] = a;
  }
  __syncthreads();
}
// grouped record layout (kBdRecGroup, N>1 with server sub-buckets): one
// workgroup per bucket b moves its run [ubase[b], ubase[b] + unum[b]) from the
// scatter's staging (gkeys, gspj: the same send-segment positions) into the
// send segment grouped by the server's sub-bucket — the split the unique
// dedup makes of its keys (region-based with region buckets, so a server
// sub-bucket is whole regions and its pull can claim) — writing the groups'
// offsets into usub and every record's final position into pos_of (the
// scatter wrote the staging positions, and kBdInvalid for empty keys, first)
__global__ __launch_bounds__(kRgT) void k_rec_group(const uint32_t* __restrict__ rstart,
                                                    const uint32_t* __restrict__ rnum,
                                                    const uint64_t* __restrict__ gkeys,
                                                    const uint32_t* __restrict__ gspj,
                                                    uint64_t* __restrict__ skeys,
                                                    uint32_t* __restrict__ spj,
                                                    uint32_t* __restrict__ pos_of,
                                                    uint32_t* __restrict__ usub, int msub, int Pd,
                                                    int rbits) {
  __shared__ unsigned int cnt[kBdMaxSub];
  __shared__ unsigned int cur[kBdMaxSub];
  const int t = threadIdx.x, b = blockIdx.x;
  // the bucket's run from the run tables the column scan wrote: in the
  // gapped record layout bstart[b + 1] of a destination's last bucket is the
  // next destination's first, d * gap away — past the run, into staging the
  // scatter never wrote
  const uint32_t p0 = rstart[b], p1 = p0 + rnum[b];
  if (t < msub) cnt[t] = 0u;
  __syncthreads();
  auto sub_of = [&](uint64_t v) -> uint32_t {
    if (rbits) {
      const uint64_t region = table_hash(v) >> (64 - rbits);
      const uint32_t f = (uint32_t)((region * (uint64_t)Pd * (uint64_t)msub) >> rbits);
      return f - (uint32_t)(b % Pd) * (uint32_t)msub;
    }
    return srv_sub(v, msub);
  };
  // a wave's lanes grouped by sub-bucket without same-address LDS atomics:
  // a Zipf-hot key puts thousands of a bucket's records into one sub-bucket,
  // and one returning LDS atomic per record on that counter serialised them
  // (9 ms per call at 2 ranks).  Per distinct sub-bucket g of the wave (a
  // leader lane's, found by ballot): one atomic adds the lanes that share it,
  // each lane's rank among them is the popcount of the lower matching lanes
  const int lane = (int)(threadIdx.x & 63);
  auto wave_slot = [&](bool valid, uint32_t g, unsigned int* ctr, bool ret) -> uint32_t {
    uint64_t todo = __ballot(valid);
    uint32_t mine = 0u;
    while (todo) {
      const int leader = __ffsll((unsigned long long)todo) - 1;
      const uint32_t gl = __shfl(g, leader, 64);
      const uint64_t mask = __ballot(valid && g == gl);
      uint32_t base = 0u;
      if (lane == leader) {
        const unsigned int c = (unsigned int)__popcll(mask);
        base = ret ? atomicAdd(&ctr[gl], c) : (atomicAdd(&ctr[gl], c), 0u);
      }
      base = __shfl(base, leader, 64);
      if (valid && g == gl)
        mine = base + (uint32_t)__popcll(mask & ((1ull << lane) - 1ull));
      todo &= ~mask;
    }
    return mine;
  };
  // pass 1: records per sub-bucket (4 per thread in flight); the loop is
  // wave-uniform (every lane runs the ballots)
  const uint32_t n = p1 - p0;
  const uint32_t nr = (n + kRgT - 1) / kRgT;  // rounds of one record per thread
  for (uint32_t r0 = 0; r0 < nr; r0 += 4) {
    uint64_t k[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const uint32_t p = p0 + (r0 + r) * kRgT + t;
      k[r] = (r0 + r < nr && p < p1) ? gkeys[p] : kEmptyKey;
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const bool v = k[r] != kEmptyKey;
      wave_slot(v, v ? min(sub_of(k[r]), (uint32_t)msub - 1) : 0u, cnt, false);
    }
  }
  __syncthreads();
  if (t == 0) {
    unsigned int e = 0;
    for (int i = 0; i < msub; ++i) {
      cur[i] = e;
      usub[(long long)b * msub + i] = e;
      e += cnt[i];
    }
  }
  __syncthreads();
  // pass 2: every record to its group (the run is re-read from L2)
  for (uint32_t r0 = 0; r0 < nr; r0 += 4) {
    uint64_t k[4];
    uint32_t j[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const uint32_t p = p0 + (r0 + r) * kRgT + t;
      const bool in = r0 + r < nr && p < p1;
      k[r] = in ? gkeys[p] : kEmptyKey;
      j[r] = in ? gspj[p] : kBdInvalid;
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const bool v = j[r] != kBdInvalid;
      const uint32_t g = v && k[r] != kEmptyKey ? min(sub_of(k[r]), (uint32_t)msub - 1) : 0u;
      const uint32_t q = p0 + wave_slot(v, g, cur, true);
      if (v) {
        skeys[q] = k[r];
        spj[q] = j[r];
        pos_of[j[r]] = q;
      }
    }
  }
}

__device__ __forceinline__ long long rec_pos(const long long* cs, int nd, long long gap,
                                             long long f) {
  int d = 0;
  while (d + 1 < nd && f >= cs[d + 1]) ++d;
  return (long long)d * gap + (f - cs[d]);
}

__global__ __launch_bounds__(256) void k_rec_grad(const unsigned long long* __restrict__ ucount,
                                                  int nd, long long gap,
                                                  const uint32_t* __restrict__ spj,
                                                  const float* __restrict__ gs,
                                                  const float* __restrict__ xval, int F,
                                                  float* __restrict__ grec,
                                                  float* __restrict__ lacc,
                                                  float* __restrict__ lacc_out, int lacc_n,
                                                  int skip) {
  __shared__ long long cs[kRecMaxDest + 1];
  // the step's loss accumulator (the forward's, stream-ordered before this
  // launch) moves to lacc_out and is left zero, as k_bd_reduce does
  if (lacc)
    for (int i = blockIdx.x * 256 + threadIdx.x; i < lacc_n; i += gridDim.x * 256) {
      lacc_out[i] = lacc[i];
      lacc[i] = 0.f;
    }
  // skip: this rank's own destination, whose server merge reads the
  // per-sample gradient through spj itself (SelfSeg::grad)
  rec_ranges(ucount, nd, gap, cs, skip);
  const long long tot = cs[nd], stride = (long long)gridDim.x * 256 * 4;
  for (long long f0 = (long long)blockIdx.x * 1024 + threadIdx.x; f0 < tot; f0 += stride) {
    long long p[4];
    uint32_t j[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const long long f = f0 + r * 256;
      p[r] = f < tot ? rec_pos(cs, nd, gap, f) : -1;
      j[r] = p[r] >= 0 ? spj[p[r]] : 0u;
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      if (p[r] < 0) continue;
      float g = gs[j[r] / (uint32_t)F];
      if (xval) g *= xval[j[r]];
      grec[p[r]] = g;
    }
  }
}

static int rec_grid(long long cap, int nd) {
  const long long work = (cap * nd + 1023) / 1024;  // the ranges' upper bound (nd may be 0)
  return (int)std::max<long long>(1, std::min<long long>(work, 2048));
}

void launch_rec_grad(const unsigned long long* ucount, int nd, long long gap, const uint32_t* spj,
                     const float* gs, const float* xval, int F, float* grec, hipStream_t st,
                     float* lacc, float* lacc_out, int lacc_n, int skip) {
  if (nd < 1 || nd > kRecMaxDest || gap < 1 || F < 1) throw_error("rec_grad: bad layout");
  if (lacc && (!lacc_out || lacc_n <= 0)) throw_error("rec_grad: loss hand-off needs its output");
  if (skip >= nd) throw_error("rec_grad: skipped destination out of range");
  // the grid covers the ranges walked: none at one rank with its own skipped
  // (the launch then only hands the loss off)
  int grid = rec_grid(gap, skip >= 0 ? nd - 1 : nd);
  // ... and at least one thread per accumulator word for the hand-off (one
  // workgroup walking 8192 words took 16 us of dependent load -> store)
  if (lacc) grid = std::max(grid, (lacc_n + 255) / 256);
  hipLaunchKernelGGL(k_rec_grad, dim3(grid), dim3(256), 0, st, ucount, nd, gap, spj, gs, xval, F,
                     grec, lacc, lacc_out, lacc_n, skip);
  check_launch("k_rec_grad");
}

void launch_bd_fill_occ(long long n, int nranks, const uint32_t* scratch, const uint32_t* luid,
                        const float* uvals, float* occ, int osi, hipStream_t st, int ndest,
                        const uint32_t* pj) {
  if (n <= 0) return;
  const BdLayout L = bd_layout(n, nranks, ndest);
  hipLaunchKernelGGL(k_bd_fill_occ<512>, dim3(L.P), dim3(512), 0, st, scratch + L.bstart,
                     scratch + L.ubase, scratch + L.unum, luid, uvals, occ, osi, pj, SelfSeg{});
  check_launch("k_bd_fill_occ");
}

void launch_bd_unplace(long long n, int nranks, const uint32_t* scratch, const float* src,
                       float* dst, int dim, hipStream_t st, int ndest) {
  if (n <= 0) return;
  const BdLayout L = bd_layout(n, nranks, ndest);
  hipLaunchKernelGGL(k_bd_unplace, dim3(L.P), dim3(256), 0, st, scratch + L.bstart,
                     scratch + L.unum, scratch + L.ubase, src, dst, dim);
  check_launch("k_bd_unplace");
}

void launch_bd_reduce(long long n, int nranks, const uint32_t* scratch, const uint32_t* pj,
                      const uint32_t* luid, const float* gs, const float* xval, int F,
                      float* ugrad, hipStream_t st, int osi, const uint8_t* usingle,
                      const DevTable* t, const long long* slots, const float* snap,
                      const OptParams* op, int ndest, int slot32, float* lacc, float* lacc_out,
                      int lacc_n, const uint64_t* bkeys) {
  if (n <= 0) return;
  if (lacc && (!lacc_out || lacc_n <= 0)) throw_error("bd_reduce: loss hand-off needs its output");
  if (F < 1) throw_error("bd_reduce: F must be >= 1");
  // slot32: `slots` holds 4-byte indices (k_pull_unique_bk's slot32 form)
  const int* s32 = slot32 ? reinterpret_cast<const int*>(slots) : nullptr;
  if (slot32) slots = nullptr;
  DevTable tv{};
  OptParams opv{};
  if (slots || s32) {
    if (!t || !op || osi || t->bf16 || op->kind != kOptAdaGrad || t->dim != 1 || t->width != 2 ||
        t->row_off % 8 != 0 || t->stride % 8 != 0)
      throw_error("bd_reduce: fused apply needs scalar AdaGrad rows and compact ids");
    tv = *t;
    opv = *op;
  }
  if (bkeys && (!(slots || s32) || !snap || t->stride != 16 || t->key_off != 8 || t->row_off != 0))
    throw_error("bd_reduce: slot stores with keys need a snapshot merge into 16-byte [w|h|key] slots");
  const float2* sn = reinterpret_cast<const float2*>(snap);
  const BdLayout L = bd_layout(n, nranks, ndest);
  const uint32_t* S = scratch;
  // workgroup shape: SS_BD_RT / SS_BD_ROCC (bd_reduce_launch)
  bd_reduce_launch(L.P, st, S + L.bstart, S + L.ubase, S + L.unum, pj, luid, gs, xval, F, ugrad,
                   osi, usingle, tv, slots, sn, opv, SelfSeg{}, s32, lacc, lacc_out, lacc_n, bkeys);
  check_launch("k_bd_reduce");
}

// explicit-layout forms (server.hip: the server's merge of received keys has
// its own bucket arrays instead of a BdLayout scratch)
void launch_bd_reduce_p(int P, const uint32_t* bstart, const uint32_t* ubase, const uint32_t* unum,
                        const uint32_t* pj, const uint32_t* luid, const float* gs, int F,
                        float* ugrad, const DevTable* t, const long long* slots,
                        const float* snap, const OptParams* op, hipStream_t st, SelfSeg self,
                        int slot32, const uint64_t* bkeys) {
  if (P <= 0) return;
  DevTable tv{};
  OptParams opv{};
  const int* s32 = slot32 ? reinterpret_cast<const int*>(slots) : nullptr;
  if (slot32) slots = nullptr;
  if (slots || s32) {
    if (!t || !op || t->bf16 || op->kind != kOptAdaGrad || t->dim != 1 || t->width != 2 ||
        t->row_off % 8 != 0 || t->stride % 8 != 0)
      throw_error("bd_reduce_p: fused apply needs scalar AdaGrad rows");
    tv = *t;
    opv = *op;
  }
  if (bkeys && (!(slots || s32) || !snap || t->stride != 16 || t->key_off != 8 || t->row_off != 0))
    throw_error("bd_reduce_p: slot stores with keys need a snapshot merge into [w|h|key] slots");
  bd_reduce_launch(P, st, bstart, ubase, unum, pj, luid, gs, static_cast<const float*>(nullptr), F,
                   ugrad, 0, static_cast<const uint8_t*>(nullptr), tv, slots,
                   reinterpret_cast<const float2*>(snap), opv, self, s32,
                   static_cast<float*>(nullptr), static_cast<float*>(nullptr), 0, bkeys);
  check_launch("k_bd_reduce_p");
}

void launch_bd_fill_occ_p(int P, const uint32_t* bstart, const uint32_t* ubase,
                          const uint32_t* unum, const uint32_t* luid, const float* uvals,
                          float* occ, const uint32_t* pj, hipStream_t st, SelfSeg self) {
  if (P <= 0) return;
  hipLaunchKernelGGL(k_bd_fill_occ<512>, dim3(P), dim3(512), 0, st, bstart, ubase, unum, luid,
                     uvals, occ, 0, pj, self);
  check_launch("k_bd_fill_occ_p");
}

long long bd_fm_ovf_words(long long n) { return n / kFmOcc + 2; }

void launch_bd_reduce_fm(long long n, int nranks, const uint32_t* scratch, const uint32_t* pj,
                         const uint32_t* luid, const float* gs, const float* gss, int F, int dim,
                         const float* uvals, float* ugrad, hipStream_t st, uint32_t* ovf,
                         const DevTable* t, const long long* slots, const OptParams* op,
                         int ndest) {
  if (n <= 0) return;
  DevTable tv{};
  OptParams opv{};
  if (slots) {
    if (!t || !op || !ovf || t->dim != (uint32_t)dim)
      throw_error("bd_reduce_fm: fused apply needs the table, the optimizer, the sorted path");
    tv = *t;
    opv = *op;
  }
  const BdLayout L = bd_layout(n, nranks, ndest);
  const uint32_t* S = scratch;
  // default: sorted lists (no float atomics) + LDS-atomic form for overflow
  // buckets; ovf = {count, bucket ids} scratch of bd_fm_ovf_words(n) words
  static const bool sorted = [] {
    const char* e = std::getenv("SS_FM_REDUCE");
    return !(e && std::string(e) == "atomic");
  }();
  if (slots && !(ovf && sorted))
    throw_error("bd_reduce_fm: fused apply runs on the sorted path only (SS_FM_REDUCE)");
  if (ovf && sorted) {
    const int novf = (int)(n / kFmOcc) + 1;  // an overflow bucket holds > kFmOcc keys
    check_hip(hipMemsetAsync(ovf, 0, sizeof(uint32_t), st), "fm ovf count");
    switch (dim) {
#define SS_BDFMS_CASE(DD)                                                                      \
  case DD:                                                                                     \
    hipLaunchKernelGGL(k_bd_reduce_fm_sorted<DD>, dim3(L.P), dim3(1024), 0, st, S + L.bstart,  \
                       S + L.ubase, S + L.unum, pj, luid, gs, gss, F, uvals, ugrad, ovf, tv,   \
                       slots, opv);                                                            \
    hipLaunchKernelGGL(k_bd_reduce_fm<DD>, dim3(novf), dim3(1024), 0, st, S + L.bstart,         \
                       S + L.ubase, S + L.unum, pj, luid, gs, gss, F, uvals, ugrad, ovf, tv,   \
                       slots, opv);                                                            \
    break;
      SS_BDFMS_CASE(2)
      SS_BDFMS_CASE(5)
      SS_BDFMS_CASE(9)
      SS_BDFMS_CASE(17)
#undef SS_BDFMS_CASE
      default:
        throw_error("bd_reduce_fm: dim must be 1+K with K in {1,4,8,16}");
    }
    check_launch("k_bd_reduce_fm_sorted");
    return;
  }
  switch (dim) {
#define SS_BDFM_CASE(DD)                                                                       \
  case DD:                                                                                     \
    hipLaunchKernelGGL(k_bd_reduce_fm<DD>, dim3(L.P), dim3(1024), 0, st, S + L.bstart,        \
                       S + L.ubase, S + L.unum, pj, luid, gs, gss, F, uvals, ugrad, nullptr);   \
    break;
    SS_BDFM_CASE(2)
    SS_BDFM_CASE(5)
    SS_BDFM_CASE(9)
    SS_BDFM_CASE(17)
#undef SS_BDFM_CASE
    default:
      throw_error("bd_reduce_fm: dim must be 1+K with K in {1,4,8,16}");
  }
  check_launch("k_bd_reduce_fm");
}

}  // namespace ss
