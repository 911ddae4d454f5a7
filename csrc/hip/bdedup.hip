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
//   1 count    per 8192-occurrence chunk: LDS histogram over buckets
//   2 rowscan  (scan.h) per-bucket chunk bases + bucket totals
//   3 bstart   bucket start offsets (one workgroup)
//   4 scatter  occurrence -> bucket-ordered (key, j) arrays
//   5 dedup    one workgroup per bucket: LDS hash insert, compact, local ids
//   6 rowscan  per-destination scan of bucket unique counts -> ucount[d]
//   7 finish   unique keys to their send segment, inverse index, zeroed grads
//
// Bucket b = d * Pd + fastrange32(dedup_hash(key) >> 32, Pd) with
// d = map[fmix64(key) % frag_num] (hashfrag.h:48-53).  Pd is chosen so a
// bucket holds ~1024 occurrences; its unique count is then far below the
// 4096-slot LDS table (overflow is detected and reported, never silent).
#include "scan.h"
#include "ss_device.h"
#include "ss_launch.h"

namespace ss {

static constexpr uint32_t kBdInvalid = 0xFFFFFFFFu;
static constexpr int kBdChunk = 8192;   // occurrences per count/scatter workgroup
static constexpr int kBdPer = kBdChunk / 1024;
static constexpr int kBdTarget = 1024;  // target occurrences per bucket
static constexpr int kBdTS = 4096;      // LDS hash slots per bucket
static constexpr int kBdMaxBuckets = 16384;

__device__ __forceinline__ uint32_t bd_bucket(uint64_t key, const RouteSpec& rs, uint32_t Pd) {
  const uint32_t d = rs.nranks == 1 ? 0u : (uint32_t)rs.frag_map[fmix64(key) % (uint64_t)rs.frag_num];
  const uint32_t h = (uint32_t)(dedup_hash(key) >> 32);
  return d * Pd + __umulhi(h, Pd);
}

// ---- layout of the int scratch (u32 words), a function of (n, nranks) only
struct BdLayout {
  int P, Pd, nch, ng, ngd;
  long long hist, grp, btot, bstart, ucnt, unum, ugrp, err, total;
};

static BdLayout bd_layout(long long n, int nranks) {
  BdLayout L{};
  long long target = kBdTarget;
  if (n > (long long)kBdMaxBuckets * kBdTarget) target = (n + kBdMaxBuckets - 1) / kBdMaxBuckets;
  long long pd = (n + (long long)nranks * target - 1) / ((long long)nranks * target);
  if (pd < 1) pd = 1;
  L.Pd = (int)pd;
  L.P = (int)(pd * nranks);
  L.nch = (int)((n + kBdChunk - 1) / kBdChunk);
  if (L.nch < 1) L.nch = 1;
  L.ng = scan_groups(L.nch);
  L.ngd = scan_groups(L.Pd);
  long long o = 1;  // word 0: sticky error flag (fixed position for any n)
  L.err = 0;
  L.hist = o; o += (long long)L.P * L.nch;
  L.grp = o; o += (long long)L.P * L.ng;
  L.btot = o; o += L.P;
  L.bstart = o; o += L.P + 1;
  L.ucnt = o; o += L.P;
  L.unum = o; o += L.P;
  L.ugrp = o; o += (long long)nranks * L.ngd;
  L.total = o;
  return L;
}

long long bd_scratch_words(long long n, int nranks) { return bd_layout(n < 1 ? 1 : n, nranks).total; }
int bd_buckets(long long n, int nranks) { return bd_layout(n < 1 ? 1 : n, nranks).P; }

// 1. per-chunk bucket histogram (dynamic LDS: P words)
__global__ __launch_bounds__(1024) void k_bd_count(const uint64_t* __restrict__ keys, long long n,
                                                   RouteSpec rs, int Pd, int P,
                                                   uint32_t* __restrict__ hist, int nch) {
  extern __shared__ unsigned int h[];
  for (int b = threadIdx.x; b < P; b += 1024) h[b] = 0u;
  __syncthreads();
  const long long base = (long long)blockIdx.x * kBdChunk + threadIdx.x;
#pragma unroll
  for (int e = 0; e < kBdPer; ++e) {
    const long long j = base + e * 1024;
    if (j < n) {
      const uint64_t key = keys[j];
      if (key != kEmptyKey) atomicAdd(&h[bd_bucket(key, rs, (uint32_t)Pd)], 1u);
    }
  }
  __syncthreads();
  for (int b = threadIdx.x; b < P; b += 1024) hist[(long long)b * nch + blockIdx.x] = h[b];
}

// 3. exclusive scan of bucket totals -> bucket start offsets (P <= 16384)
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

// 4. scatter occurrences into bucket order (dynamic LDS: P words)
__global__ __launch_bounds__(1024) void k_bd_scatter(const uint64_t* __restrict__ keys, long long n,
                                                     RouteSpec rs, int Pd, int P,
                                                     const uint32_t* __restrict__ hist,
                                                     const uint32_t* __restrict__ grp, int nch,
                                                     int ng, const uint32_t* __restrict__ bstart,
                                                     uint64_t* __restrict__ pkeys,
                                                     uint32_t* __restrict__ pj,
                                                     uint32_t* __restrict__ inv) {
  extern __shared__ unsigned int cur[];
  const int c = blockIdx.x;
  for (int b = threadIdx.x; b < P; b += 1024)
    cur[b] = bstart[b] + hist[(long long)b * nch + c] + grp[(long long)b * ng + c / kScanGroup];
  __syncthreads();
  const long long base = (long long)c * kBdChunk + threadIdx.x;
#pragma unroll
  for (int e = 0; e < kBdPer; ++e) {
    const long long j = base + e * 1024;
    if (j < n) {
      const uint64_t key = keys[j];
      if (key == kEmptyKey) {
        inv[j] = kBdInvalid;
      } else {
        const uint32_t pos = atomicAdd(&cur[bd_bucket(key, rs, (uint32_t)Pd)], 1u);
        pkeys[pos] = key;
        pj[pos] = (uint32_t)j;
      }
    }
  }
}

// 5. one workgroup per bucket: LDS hash dedup, compaction, local unique ids
__global__ __launch_bounds__(1024) void k_bd_dedup(const uint64_t* __restrict__ pkeys,
                                                   const uint32_t* __restrict__ bstart,
                                                   uint32_t* __restrict__ luid,
                                                   uint64_t* __restrict__ bkeys,
                                                   uint32_t* __restrict__ ucnt,
                                                   uint32_t* __restrict__ unum,
                                                   uint32_t* __restrict__ err) {
  __shared__ unsigned long long tab[kBdTS];
  __shared__ unsigned int lid[kBdTS];
  __shared__ unsigned int wsum[16];
  __shared__ unsigned int tot;
  __shared__ int bad;
  const int b = blockIdx.x, t = threadIdx.x;
  for (int s = t; s < kBdTS; s += 1024) tab[s] = kEmptyKey;
  if (t == 0) bad = 0;
  __syncthreads();
  const uint32_t p0 = bstart[b], p1 = bstart[b + 1];
  for (uint32_t p = p0 + t; p < p1; p += 1024) {
    const uint64_t key = pkeys[p];
    uint32_t s = (uint32_t)dedup_hash(key) & (kBdTS - 1);
    int k = 0;
    for (; k < kBdTS; ++k) {
      const unsigned long long v = tab[s];
      if (v == key) break;
      if (v == kEmptyKey) {
        const unsigned long long prev = atomicCAS(&tab[s], kEmptyKey, (unsigned long long)key);
        if (prev == kEmptyKey || prev == key) break;
      }
      s = (s + 1) & (kBdTS - 1);
    }
    if (k == kBdTS) {
      bad = 1;
      s = kBdInvalid;
    }
    luid[p] = s;  // slot for now; rewritten to the local id below
  }
  __syncthreads();
  // compaction in slot order: thread t owns slots [4t, 4t+4)
  constexpr int kPerT = kBdTS / 1024;
  unsigned int occ = 0;
#pragma unroll
  for (int k = 0; k < kPerT; ++k) occ += tab[t * kPerT + k] != kEmptyKey;
  unsigned int o = block_excl_scan_1024(occ, wsum, &tot);
#pragma unroll
  for (int k = 0; k < kPerT; ++k) {
    const int s = t * kPerT + k;
    const unsigned long long v = tab[s];
    if (v != kEmptyKey) {
      lid[s] = o;
      bkeys[p0 + o] = v;  // bucket's unique keys, staged in its occurrence range
      ++o;
    }
  }
  __syncthreads();
  for (uint32_t p = p0 + t; p < p1; p += 1024) {
    const uint32_t s = luid[p];
    luid[p] = s == kBdInvalid ? kBdInvalid : lid[s];
  }
  if (t == 0) {
    ucnt[b] = tot;
    unum[b] = tot;
    if (bad) atomicOr(err, 1u);
  }
}

struct BdView {  // where a bucket's unique ids start
  const uint32_t* ucnt;
  const uint32_t* ugrp;
  int Pd, ngd;
  long long ucap;
  __device__ __forceinline__ unsigned long long base(int b) const {
    const int d = b / Pd, c = b - d * Pd;
    return (unsigned long long)d * ucap + ucnt[b] + ugrp[(long long)d * ngd + c / kScanGroup];
  }
};

// 7. unique keys -> send segments, inverse index, zeroed gradient rows
__global__ __launch_bounds__(256) void k_bd_finish(BdView v, const uint32_t* __restrict__ unum,
                                                   const uint32_t* __restrict__ bstart,
                                                   const uint64_t* __restrict__ bkeys,
                                                   const uint32_t* __restrict__ pj,
                                                   const uint32_t* __restrict__ luid,
                                                   uint64_t* __restrict__ ukeys,
                                                   float* __restrict__ ugrad, int gdim,
                                                   uint32_t* __restrict__ inv) {
  const int b = blockIdx.x;
  const unsigned long long base = v.base(b);
  const uint32_t p0 = bstart[b], p1 = bstart[b + 1], nu = unum[b];
  for (uint32_t l = threadIdx.x; l < nu; l += 256) ukeys[base + l] = bkeys[p0 + l];
  if (ugrad)
    for (uint32_t e = threadIdx.x; e < nu * (uint32_t)gdim; e += 256) ugrad[base * gdim + e] = 0.f;
  for (uint32_t p = p0 + threadIdx.x; p < p1; p += 256) {
    const uint32_t l = luid[p];
    inv[pj[p]] = l == kBdInvalid ? kBdInvalid : (uint32_t)(base + l);
  }
}

// K7 for scalar rows (sparse LR): one workgroup per bucket sums the
// per-occurrence gradients of its unique keys in LDS, then stores each row
// once — no zero-fill, no global atomics.
__global__ __launch_bounds__(1024) void k_bd_reduce(BdView v, const uint32_t* __restrict__ unum,
                                                    const uint32_t* __restrict__ bstart,
                                                    const uint32_t* __restrict__ pj,
                                                    const uint32_t* __restrict__ luid,
                                                    const float* __restrict__ gocc,
                                                    float* __restrict__ ugrad) {
  __shared__ float acc[kBdTS];
  const int b = blockIdx.x;
  const uint32_t p0 = bstart[b], p1 = bstart[b + 1], nu = unum[b];
  for (uint32_t l = threadIdx.x; l < nu; l += 1024) acc[l] = 0.f;
  __syncthreads();
  for (uint32_t p = p0 + threadIdx.x; p < p1; p += 1024) {
    const uint32_t l = luid[p];
    if (l != kBdInvalid) atomicAdd(&acc[l], gocc[pj[p]]);
  }
  __syncthreads();
  const unsigned long long base = v.base(b);
  for (uint32_t l = threadIdx.x; l < nu; l += 1024) ugrad[base + l] = acc[l];
}

// ------------------------------------------------------------- launchers
void launch_bd_dedup(const uint64_t* keys, long long n, RouteSpec rs, long long ucap,
                     uint32_t* scratch, uint64_t* pkeys, uint32_t* pj, uint32_t* luid,
                     uint64_t* bkeys, unsigned long long* ucount, uint64_t* ukeys, float* ugrad,
                     int gdim, uint32_t* inv, hipStream_t st) {
  if (rs.nranks < 1 || rs.nranks > kMaxSeg) throw_error("bdedup: bad nranks");
  if (n <= 0) {
    check_hip(hipMemsetAsync(ucount, 0, sizeof(unsigned long long) * rs.nranks, st), "ucount");
    return;
  }
  if (ucap < n) throw_error("bdedup: per-destination capacity must be >= n");
  if ((unsigned long long)rs.nranks * (unsigned long long)ucap >= 0x7FFFFFFFull)
    throw_error("bdedup: nranks*ucap overflows 31-bit unique ids");
  const BdLayout L = bd_layout(n, rs.nranks);
  if (L.P > kBdMaxBuckets * 2 || (long long)L.P * L.nch > (1ll << 31))
    throw_error("bdedup: too many keys per call");
  if (n > (long long)kBdMaxBuckets * 2800) throw_error("bdedup: too many keys per call (max 45M)");
  uint32_t* S = scratch;
  const size_t lds = sizeof(unsigned int) * (size_t)L.P;
  hipLaunchKernelGGL(k_bd_count, dim3(L.nch), dim3(1024), lds, st, keys, n, rs, L.Pd, L.P,
                     S + L.hist, L.nch);
  check_launch("k_bd_count");
  launch_rowscan(S + L.hist, L.P, L.nch, S + L.grp, S + L.btot, nullptr, st);
  check_launch("bd rowscan");
  hipLaunchKernelGGL(k_bd_bstart, dim3(1), dim3(1024), 0, st, S + L.btot, L.P, S + L.bstart);
  check_launch("k_bd_bstart");
  hipLaunchKernelGGL(k_bd_scatter, dim3(L.nch), dim3(1024), lds, st, keys, n, rs, L.Pd, L.P,
                     S + L.hist, S + L.grp, L.nch, L.ng, S + L.bstart, pkeys, pj, inv);
  check_launch("k_bd_scatter");
  hipLaunchKernelGGL(k_bd_dedup, dim3(L.P), dim3(1024), 0, st, pkeys, S + L.bstart, luid, bkeys,
                     S + L.ucnt, S + L.unum, S + L.err);
  check_launch("k_bd_dedup");
  launch_rowscan(S + L.ucnt, rs.nranks, L.Pd, S + L.ugrp, nullptr, ucount, st);
  check_launch("bd uscan");
  BdView v{S + L.ucnt, S + L.ugrp, L.Pd, L.ngd, ucap};
  hipLaunchKernelGGL(k_bd_finish, dim3(L.P), dim3(256), 0, st, v, S + L.unum, S + L.bstart, bkeys,
                     pj, luid, ukeys, ugrad, gdim, inv);
  check_launch("k_bd_finish");
}

void launch_bd_reduce(long long n, int nranks, long long ucap, const uint32_t* scratch,
                      const uint32_t* pj, const uint32_t* luid, const float* gocc, float* ugrad,
                      hipStream_t st) {
  if (n <= 0) return;
  const BdLayout L = bd_layout(n, nranks);
  const uint32_t* S = scratch;
  BdView v{S + L.ucnt, S + L.ugrp, L.Pd, L.ngd, ucap};
  hipLaunchKernelGGL(k_bd_reduce, dim3(L.P), dim3(1024), 0, st, v, S + L.unum, S + L.bstart, pj,
                     luid, gocc, ugrad);
  check_launch("k_bd_reduce");
}

}  // namespace ss
