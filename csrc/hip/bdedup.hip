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
//   2 colscan  per-bucket exclusive scan down the chunks + bucket totals
//   3 bstart   bucket start offsets (one workgroup)
//   4 scatter  bucket-ordered occurrence list pj[pos] = j, and pos_of[j]
//   5 dedup    one workgroup per bucket: LDS hash insert, compaction, then a
//              decoupled look-back over the destination's earlier buckets for
//              the unique-id base (single pass, no extra scan launch); writes
//              the send-segment keys, per-position unique ids and ucount[d]
//   6 inverse  inv[j] = luid[pos_of[j]] (coalesced writes, gathered reads)
//
// Measured (profiles/): random 4-12 B stores cost ~5x their bytes in write
// requests (partial 64 B lines from 8 L2s), so the design stores every
// permuted array with as few random stores as possible (only pj) and turns the
// rest into coalesced stores plus gathered loads.
//
// Bucket b = d * Pd + fastrange32(dedup_hash(key) >> 32, Pd) with
// d = map[fmix64(key) % frag_num] (hashfrag.h:48-53).  Pd is chosen so a
// bucket holds ~2048 occurrences; its unique count is then far below the
// 4096-slot LDS table (overflow is detected and reported, never silent).
#include "scan.h"
#include "ss_device.h"
#include "ss_launch.h"

namespace ss {

static constexpr uint32_t kBdInvalid = 0xFFFFFFFFu;
static constexpr int kBdMaxChunk = 8192;  // occurrences per count/scatter workgroup
static constexpr int kBdPer = kBdMaxChunk / 1024;
static constexpr int kBdTarget = 2048;  // target occurrences per bucket
static constexpr int kBdTS = 4096;      // LDS hash slots per bucket
static constexpr int kBdRegs = 4;       // occurrences per thread kept in registers
static constexpr int kBdMaxBuckets = 16384;

__device__ __forceinline__ uint32_t bd_bucket(uint64_t key, const RouteSpec& rs, uint32_t Pd) {
  const uint32_t d =
      rs.nranks == 1 ? 0u : (uint32_t)rs.frag_map[fmix64(key) % (uint64_t)rs.frag_num];
  const uint32_t h = (uint32_t)(dedup_hash(key) >> 32);
  return d * Pd + __umulhi(h, Pd);
}

// ---- layout of the int scratch (u32 words), a function of (n, nranks) only
struct BdLayout {
  int P, Pd, nch, chunk;
  long long hist, btot, bstart, ubase, unum, total;
};

static BdLayout bd_layout(long long n, int nranks) {
  BdLayout L{};
  long long target = kBdTarget;
  if (n > (long long)kBdMaxBuckets * kBdTarget) target = (n + kBdMaxBuckets - 1) / kBdMaxBuckets;
  long long pd = (n + (long long)nranks * target - 1) / ((long long)nranks * target);
  if (pd < 1) pd = 1;
  L.Pd = (int)pd;
  L.P = (int)(pd * nranks);
  // chunk count a multiple of the 256 CUs (balanced waves), chunk <= 8192
  const long long waves = (n + 256ll * kBdMaxChunk - 1) / (256ll * kBdMaxChunk);
  const long long per = (n + 256 * waves - 1) / (256 * waves);
  L.chunk = (int)(((per + 1023) / 1024) * 1024);
  L.nch = (int)((n + L.chunk - 1) / L.chunk);
  if (L.nch < 1) L.nch = 1;
  long long o = 1;  // word 0: sticky error flag (fixed position for any n)
  L.hist = o; o += (long long)L.P * L.nch;
  L.btot = o; o += L.P;
  L.bstart = o; o += L.P + 1;
  L.ubase = o; o += L.P;
  L.unum = o; o += L.P;
  L.total = o;
  return L;
}

long long bd_scratch_words(long long n, int nranks) {
  return bd_layout(n < 1 ? 1 : n, nranks).total;
}
int bd_buckets(long long n, int nranks) { return bd_layout(n < 1 ? 1 : n, nranks).P; }
long long bd_ubase_offset(long long n, int nranks) {
  return bd_layout(n < 1 ? 1 : n, nranks).ubase;
}

// 1. per-chunk bucket histogram (dynamic LDS: P words), chunk-major output
__global__ __launch_bounds__(1024) void k_bd_count(const uint64_t* __restrict__ keys, long long n,
                                                   RouteSpec rs, int Pd, int P, int chunk,
                                                   uint32_t* __restrict__ hist) {
  extern __shared__ unsigned int h[];
  for (int b = threadIdx.x; b < P; b += 1024) h[b] = 0u;
  __syncthreads();
  const long long base = (long long)blockIdx.x * chunk + threadIdx.x;
  const int per = chunk >> 10;
  uint64_t k[kBdPer];
#pragma unroll
  for (int e = 0; e < kBdPer; ++e) {
    const long long j = base + e * 1024;
    k[e] = (e < per && j < n) ? keys[j] : kEmptyKey;
  }
#pragma unroll
  for (int e = 0; e < kBdPer; ++e)
    if (k[e] != kEmptyKey) atomicAdd(&h[bd_bucket(k[e], rs, (uint32_t)Pd)], 1u);
  __syncthreads();
  uint32_t* row = hist + (long long)blockIdx.x * P;
  for (int b = threadIdx.x; b < P; b += 1024) row[b] = h[b];
}

// 2. column scan of the [nch][P] histogram: 64 buckets x 16 chunk segments
//    per workgroup; two passes of independent loads, no serial chain
__global__ __launch_bounds__(1024) void k_bd_colscan(uint32_t* __restrict__ hist, int nch, int P,
                                                     uint32_t* __restrict__ btot) {
  __shared__ unsigned int ss[16][64];
  const int col = threadIdx.x & 63, seg = threadIdx.x >> 6;
  const int b = blockIdx.x * 64 + col;
  const int R = (nch + 15) / 16;
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
    if (seg == 15) btot[b] = off;
  }
}

// 3. exclusive scan of bucket totals -> bucket start offsets (P <= ~16K)
__global__ __launch_bounds__(1024) void k_bd_bstart(const uint32_t* __restrict__ btot, int P,
                                                    uint32_t* __restrict__ bstart) {
  __shared__ unsigned int wsum[16];
  __shared__ unsigned int tot;
  const int per = (P + 1023) / 1024;
  const int b0 = threadIdx.x * per;
  unsigned int s = 0;
  for (int k = 0; k < per; ++k)
    if (b0 + k < P) s += btot[b0 + k];
  unsigned int e = block_excl_scan_1024(s, wsum, &tot);
  for (int k = 0; k < per; ++k)
    if (b0 + k < P) {
      bstart[b0 + k] = e;
      e += btot[b0 + k];
    }
  if (threadIdx.x == 0) bstart[P] = tot;
}

// 4. bucket-ordered occurrence list (dynamic LDS: P words)
__global__ __launch_bounds__(1024) void k_bd_scatter(const uint64_t* __restrict__ keys, long long n,
                                                     RouteSpec rs, int Pd, int P, int chunk,
                                                     const uint32_t* __restrict__ hist,
                                                     const uint32_t* __restrict__ bstart,
                                                     uint32_t* __restrict__ pj,
                                                     uint32_t* __restrict__ pos_of) {
  extern __shared__ unsigned int cur[];
  const int c = blockIdx.x;
  const uint32_t* row = hist + (long long)c * P;
  for (int b = threadIdx.x; b < P; b += 1024) cur[b] = bstart[b] + row[b];
  const long long base = (long long)c * chunk + threadIdx.x;
  const int per = chunk >> 10;
  uint64_t k[kBdPer];
#pragma unroll
  for (int e = 0; e < kBdPer; ++e) {
    const long long j = base + e * 1024;
    k[e] = (e < per && j < n) ? keys[j] : kEmptyKey;
  }
  __syncthreads();
#pragma unroll
  for (int e = 0; e < kBdPer; ++e) {
    const long long j = base + e * 1024;
    if (e < per && j < n) {
      uint32_t pos = kBdInvalid;
      if (k[e] != kEmptyKey) {
        pos = atomicAdd(&cur[bd_bucket(k[e], rs, (uint32_t)Pd)], 1u);
        pj[pos] = (uint32_t)j;
      }
      pos_of[j] = pos;
    }
  }
}

// look-back flag word: [epoch:30][state:2][value:32]; state 1 = bucket
// aggregate, 2 = inclusive prefix within the destination
__device__ __forceinline__ unsigned long long bd_flag(uint32_t epoch, uint32_t st, uint32_t v) {
  return ((unsigned long long)(epoch & 0x3FFFFFFFu) << 34) | ((unsigned long long)st << 32) | v;
}

struct BdOut {
  uint64_t* ukeys;
  uint32_t* luid;
  uint32_t* ubase;
  uint32_t* unum;
  unsigned long long* ucount;
  float* ugrad;
  int gdim;
  long long ucap;
};

// 5. one workgroup per bucket (taken in start order from a ticket counter so
//    the look-back only ever waits on workgroups that are already running)
__global__ __launch_bounds__(1024) void k_bd_dedup(const uint64_t* __restrict__ keys,
                                                   const uint32_t* __restrict__ pj,
                                                   const uint32_t* __restrict__ bstart, int P,
                                                   int Pd, uint32_t epoch,
                                                   unsigned long long* __restrict__ flags,
                                                   unsigned long long* __restrict__ ticket,
                                                   BdOut out, uint32_t* __restrict__ err,
                                                   unsigned long long* __restrict__ dbg) {
  // dbg (optional): per bucket 8 wall-clock stamps of the phases (profiling)
#define BD_STAMP(i) \
  if (dbg && t == 0) dbg[(long long)sb * 8 + (i)] = wall_clock64();
  __shared__ unsigned long long tab[kBdTS];
  __shared__ unsigned int lid[kBdTS];
  __shared__ unsigned int wsum[16];
  __shared__ unsigned int tot;
  __shared__ int sb;
  __shared__ unsigned int sbase;
  __shared__ int bad;
  const int t = threadIdx.x;
  if (t == 0) {
    const unsigned long long tk = atomicAdd(ticket, 1ull);
    if (tk == (unsigned long long)P - 1) atomicExch(ticket, 0ull);  // every ticket taken
    sb = (int)tk;
    bad = 0;
  }
  for (int s = t; s < kBdTS; s += 1024) tab[s] = kEmptyKey;
  __syncthreads();
  BD_STAMP(0)
  const int b = sb;
  const uint32_t p0 = bstart[b], p1 = bstart[b + 1];
  // insert: the first kBdRegs occurrences of each thread keep their slot in
  // registers; a hot bucket's excess parks it in luid[] (rewritten below)
  uint32_t slot[kBdRegs];
  uint64_t kk[kBdRegs];
#pragma unroll
  for (int r = 0; r < kBdRegs; ++r) {
    const uint32_t p = p0 + t + r * 1024;
    kk[r] = p < p1 ? keys[pj[p]] : kEmptyKey;
  }
  if (dbg && t == 0) dbg[(long long)sb * 8 + 1] = wall_clock64() + (kk[0] & 0);
  auto insert = [&](uint64_t key) -> uint32_t {
    uint32_t s = (uint32_t)dedup_hash(key) & (kBdTS - 1);
    for (int k = 0; k < kBdTS; ++k) {
      const unsigned long long v = tab[s];
      if (v == key) return s;
      if (v == kEmptyKey) {
        const unsigned long long prev = atomicCAS(&tab[s], kEmptyKey, (unsigned long long)key);
        if (prev == kEmptyKey || prev == key) return s;
      }
      s = (s + 1) & (kBdTS - 1);
    }
    bad = 1;
    return kBdInvalid;
  };
#pragma unroll
  for (int r = 0; r < kBdRegs; ++r) slot[r] = kk[r] != kEmptyKey ? insert(kk[r]) : kBdInvalid;
  for (uint32_t p = p0 + t + kBdRegs * 1024; p < p1; p += 1024) out.luid[p] = insert(keys[pj[p]]);
  __syncthreads();
  BD_STAMP(2)
  // compaction in slot order: thread t owns slots [4t, 4t+4)
  constexpr int kPerT = kBdTS / 1024;
  unsigned int occ = 0;
#pragma unroll
  for (int k = 0; k < kPerT; ++k) occ += tab[t * kPerT + k] != kEmptyKey;
  unsigned int o = block_excl_scan_1024(occ, wsum, &tot);
#pragma unroll
  for (int k = 0; k < kPerT; ++k) {
    const int s = t * kPerT + k;
    if (tab[s] != kEmptyKey) lid[s] = o++;
  }
  // decoupled look-back within the destination's buckets, 64 predecessors
  // per step (one flag per lane of wave 0)
  __syncthreads();
  BD_STAMP(3)
  if (t < 64) {
    const int d = b / Pd, first = d * Pd;
    const uint32_t ep = epoch & 0x3FFFFFFFu;
    if (t == 0)
      __hip_atomic_store(&flags[b], bd_flag(epoch, b == first ? 2u : 1u, tot), __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
    unsigned int excl = 0;
    int hi = b - 1;  // next predecessor to examine
    while (hi >= first) {
      const int q = hi - t;
      unsigned long long f = 0;
      uint32_t stt = 2;  // lanes past the destination start act as "inclusive 0"
      if (q >= first) {
        for (;;) {
          f = __hip_atomic_load(&flags[q], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          stt = (uint32_t)(f >> 32) & 3u;
          if ((uint32_t)(f >> 34) == ep && stt != 0) break;
          __builtin_amdgcn_s_sleep(1);
        }
      }
      // closest predecessor holding an inclusive prefix
      const unsigned long long incl = __ballot(stt == 2u);
      const int stop = incl ? __builtin_ctzll(incl) : 64;
      unsigned int v = (t <= stop && q >= first) ? (uint32_t)f : 0u;
      for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
      excl += v;
      if (incl) break;
      hi -= 64;
    }
    if (t == 0) {
      if (b != first)
        __hip_atomic_store(&flags[b], bd_flag(epoch, 2, excl + tot), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
      const unsigned int base = (unsigned int)((long long)d * out.ucap + excl);
      sbase = base;
      out.ubase[b] = base;
      out.unum[b] = tot;
      if (b == first + Pd - 1) out.ucount[d] = excl + tot;
      if (bad) atomicOr(err, 1u);
    }
  }
  __syncthreads();
  BD_STAMP(4)
  const unsigned int base = sbase;
#pragma unroll
  for (int k = 0; k < kPerT; ++k) {
    const int s = t * kPerT + k;
    const unsigned long long v = tab[s];
    if (v != kEmptyKey) out.ukeys[base + lid[s]] = v;
  }
  if (out.ugrad)
    for (uint32_t e = t; e < tot * (uint32_t)out.gdim; e += 1024)
      out.ugrad[(unsigned long long)base * out.gdim + e] = 0.f;
#pragma unroll
  for (int r = 0; r < kBdRegs; ++r) {
    const uint32_t p = p0 + t + r * 1024;
    if (p < p1) out.luid[p] = slot[r] == kBdInvalid ? kBdInvalid : base + lid[slot[r]];
  }
  for (uint32_t p = p0 + t + kBdRegs * 1024; p < p1; p += 1024) {
    const uint32_t s = out.luid[p];
    out.luid[p] = s == kBdInvalid ? kBdInvalid : base + lid[s];
  }
  __syncthreads();
  BD_STAMP(5)
#undef BD_STAMP
}

// 6. inverse index in occurrence order
__global__ __launch_bounds__(256) void k_bd_inv(const uint32_t* __restrict__ pos_of, long long n,
                                                const uint32_t* __restrict__ luid,
                                                uint32_t* __restrict__ inv) {
  const long long j = (long long)blockIdx.x * 256 + threadIdx.x;
  if (j < n) {
    const uint32_t p = pos_of[j];
    inv[j] = p == kBdInvalid ? kBdInvalid : luid[p];
  }
}

// K7 for scalar rows (sparse LR): one workgroup per bucket sums the gradients
// of its unique keys in LDS — per-occurrence g = gs[j / F] * x[j] gathered
// from the per-sample gradient (L2-resident) — and stores each row once:
// no zero-fill, no global atomics.
__global__ __launch_bounds__(1024) void k_bd_reduce(const uint32_t* __restrict__ bstart,
                                                    const uint32_t* __restrict__ ubase,
                                                    const uint32_t* __restrict__ unum,
                                                    const uint32_t* __restrict__ pj,
                                                    const uint32_t* __restrict__ luid,
                                                    const float* __restrict__ gs,
                                                    const float* __restrict__ xval, int F,
                                                    float* __restrict__ ugrad) {
  __shared__ float acc[kBdTS];
  const int b = blockIdx.x;
  const uint32_t p0 = bstart[b], p1 = bstart[b + 1], nu = unum[b], base = ubase[b];
  for (uint32_t l = threadIdx.x; l < nu; l += 1024) acc[l] = 0.f;
  __syncthreads();
  for (uint32_t p = p0 + threadIdx.x; p < p1; p += 1024) {
    const uint32_t u = luid[p];
    if (u != kBdInvalid) {
      const uint32_t j = pj[p];
      const float g = gs[j / (uint32_t)F];
      atomicAdd(&acc[u - base], xval ? g * xval[j] : g);
    }
  }
  __syncthreads();
  for (uint32_t l = threadIdx.x; l < nu; l += 1024) ugrad[base + l] = acc[l];
}

// K7 for FM rows [w | v_1..v_K]: per unique key u with occurrences in samples
// S(u):  grad = [G0, G_f - v_uf * G0],  G0 = sum gs[s],  G_f = sum gss[s][f].
// Columns are accumulated in LDS a few at a time (kFmCols per pass over the
// bucket's occurrences, which are L2-resident), so any unique count up to the
// 4096-slot table fits; each row is then stored once.
static constexpr int kFmCols = 3;
template <int DIM>
__global__ __launch_bounds__(1024) void k_bd_reduce_fm(const uint32_t* __restrict__ bstart,
                                                       const uint32_t* __restrict__ ubase,
                                                       const uint32_t* __restrict__ unum,
                                                       const uint32_t* __restrict__ pj,
                                                       const uint32_t* __restrict__ luid,
                                                       const float* __restrict__ gs,
                                                       const float* __restrict__ gss, int F,
                                                       const float* __restrict__ uvals,
                                                       float* __restrict__ ugrad) {
  constexpr int K = DIM - 1;
  __shared__ float g0[kBdTS];
  __shared__ float acc[kFmCols][kBdTS];
  const int b = blockIdx.x;
  const uint32_t p0 = bstart[b], p1 = bstart[b + 1], nu = unum[b], base = ubase[b];
  for (int c0 = 0; c0 < K; c0 += kFmCols) {
    for (uint32_t l = threadIdx.x; l < nu; l += 1024) {
      if (c0 == 0) g0[l] = 0.f;
#pragma unroll
      for (int c = 0; c < kFmCols; ++c) acc[c][l] = 0.f;
    }
    __syncthreads();
    for (uint32_t p = p0 + threadIdx.x; p < p1; p += 1024) {
      const uint32_t u = luid[p];
      if (u == kBdInvalid) continue;
      const uint32_t l = u - base, s = pj[p] / (uint32_t)F;
      if (c0 == 0) atomicAdd(&g0[l], gs[s]);
#pragma unroll
      for (int c = 0; c < kFmCols; ++c)
        if (c0 + c < K) atomicAdd(&acc[c][l], gss[(size_t)s * K + c0 + c]);
    }
    __syncthreads();
    for (uint32_t l = threadIdx.x; l < nu; l += 1024) {
      const size_t r = (size_t)(base + l) * DIM;
      const float G0 = g0[l];
      if (c0 == 0) ugrad[r] = G0;
#pragma unroll
      for (int c = 0; c < kFmCols; ++c)
        if (c0 + c < K) ugrad[r + 1 + c0 + c] = acc[c][l] - uvals[r + 1 + c0 + c] * G0;
    }
    __syncthreads();
  }
}

// ------------------------------------------------------------- launchers
void launch_bd_dedup(const uint64_t* keys, long long n, RouteSpec rs, long long ucap,
                     uint32_t* scratch, unsigned long long* sync, uint32_t epoch, uint32_t* pj,
                     uint32_t* pos_of, uint32_t* luid, unsigned long long* ucount,
                     uint64_t* ukeys, float* ugrad, int gdim, uint32_t* inv, hipStream_t st,
                     unsigned long long* dbg) {
  if (rs.nranks < 1 || rs.nranks > kMaxSeg) throw_error("bdedup: bad nranks");
  if (n <= 0) {
    check_hip(hipMemsetAsync(ucount, 0, sizeof(unsigned long long) * rs.nranks, st), "ucount");
    return;
  }
  if (ucap < n) throw_error("bdedup: per-destination capacity must be >= n");
  if ((unsigned long long)rs.nranks * (unsigned long long)ucap >= 0x7FFFFFFFull)
    throw_error("bdedup: nranks*ucap overflows 31-bit unique ids");
  const BdLayout L = bd_layout(n, rs.nranks);
  if (L.P > kBdMaxBuckets + kMaxSeg || n > (long long)kBdMaxBuckets * 2800)
    throw_error("bdedup: too many keys per call (max ~45M)");
  uint32_t* S = scratch;
  const size_t lds = sizeof(unsigned int) * (size_t)L.P;
  hipLaunchKernelGGL(k_bd_count, dim3(L.nch), dim3(1024), lds, st, keys, n, rs, L.Pd, L.P,
                     L.chunk, S + L.hist);
  check_launch("k_bd_count");
  hipLaunchKernelGGL(k_bd_colscan, dim3((L.P + 63) / 64), dim3(1024), 0, st, S + L.hist, L.nch,
                     L.P, S + L.btot);
  check_launch("k_bd_colscan");
  hipLaunchKernelGGL(k_bd_bstart, dim3(1), dim3(1024), 0, st, S + L.btot, L.P, S + L.bstart);
  check_launch("k_bd_bstart");
  hipLaunchKernelGGL(k_bd_scatter, dim3(L.nch), dim3(1024), lds, st, keys, n, rs, L.Pd, L.P,
                     L.chunk, S + L.hist, S + L.bstart, pj, pos_of);
  check_launch("k_bd_scatter");
  BdOut o{ukeys, luid, S + L.ubase, S + L.unum, ucount, ugrad, gdim, ucap};
  hipLaunchKernelGGL(k_bd_dedup, dim3(L.P), dim3(1024), 0, st, keys, pj, S + L.bstart, L.P, L.Pd,
                     epoch, sync, sync + kBdMaxBuckets + kMaxSeg, o, S, dbg);
  check_launch("k_bd_dedup");
  if (inv) {
    hipLaunchKernelGGL(k_bd_inv, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, pos_of, n,
                       luid, inv);
    check_launch("k_bd_inv");
  }
}

long long bd_sync_words() { return (long long)kBdMaxBuckets + kMaxSeg + 1; }

void launch_bd_reduce(long long n, int nranks, const uint32_t* scratch, const uint32_t* pj,
                      const uint32_t* luid, const float* gs, const float* xval, int F,
                      float* ugrad, hipStream_t st) {
  if (n <= 0) return;
  if (F < 1) throw_error("bd_reduce: F must be >= 1");
  const BdLayout L = bd_layout(n, nranks);
  const uint32_t* S = scratch;
  hipLaunchKernelGGL(k_bd_reduce, dim3(L.P), dim3(1024), 0, st, S + L.bstart, S + L.ubase,
                     S + L.unum, pj, luid, gs, xval, F, ugrad);
  check_launch("k_bd_reduce");
}

void launch_bd_reduce_fm(long long n, int nranks, const uint32_t* scratch, const uint32_t* pj,
                         const uint32_t* luid, const float* gs, const float* gss, int F, int dim,
                         const float* uvals, float* ugrad, hipStream_t st) {
  if (n <= 0) return;
  const BdLayout L = bd_layout(n, nranks);
  const uint32_t* S = scratch;
  switch (dim) {
#define SS_BDFM_CASE(DD)                                                                       \
  case DD:                                                                                     \
    hipLaunchKernelGGL(k_bd_reduce_fm<DD>, dim3(L.P), dim3(1024), 0, st, S + L.bstart,          \
                       S + L.ubase, S + L.unum, pj, luid, gs, gss, F, uvals, ugrad);           \
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
