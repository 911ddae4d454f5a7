// server.hip — a server's merge of the keys one round receives from all
// source ranks (N>1): one table lookup and ONE optimizer update per distinct
// key, whichever workers pushed it.
//
// Reference semantics: the server applies every push request as it arrives
// (server/init.h:115-149, sparsetable.h:181-192) and the push access method
// has a merge hook for duplicate gradients (merge_push_value,
// sparse_access_method.h:39-40).  In a collective round all pushes of the
// round arrive together, so the server merges them first — a key pushed by 8
// workers costs one probe and one row update instead of 8 of each.
//
// Layout contract (bdedup.hip, N>1): every source splits the keys it sends to
// destination d into the same Pd hash buckets (the layout of a lay_n-key
// call), bucket (d, k) placed contiguously in its send segment.  With each
// segment the source sends the per-bucket (ubase, unum) pairs, so bucket k's
// keys from source s are the run
//     rkeys[s*cap + (rbase[s][k] - me*cap) : ... + rnum[s][k]]
// and server bucket k is the union of N runs.  N runs of ~1024 unique keys do
// not fit one 4096-slot LDS table at N=8, so bucket k is further split into m
// sub-buckets by an independent hash (the low word of dedup_hash; the sender
// used the high word): server bucket b = k*m + t.  The sender grouped each
// run by sub-bucket and sent the groups' offsets (bdedup.hip msub), so
// sub-bucket t's keys from source s are one exact range of its run.
//
//   1 k_srv_count  per b: received keys = the sum of its ranges' lengths (no
//                  key is read); the last workgroup scans them -> bstart
//                  (server "occurrence" ranges)
//   3 k_srv_dedup  per b: LDS hash dedup of the sub-bucket's received keys;
//                  writes the received position of each (pj), its local id
//                  (luid), the unique keys staged at bstart[b] (bkeys, what
//                  the bucketed pull reads) and ubase/unum (compact ids)
//
// The outputs have the worker dedup's shape (bstart/ubase/unum/pj/luid), so
// the server reuses the worker kernels: k_pull_unique_bk (lookup-or-init of
// the distinct keys), k_bd_fill_occ with pj (response rows per received
// position, dim 1), k_bd_reduce with F = 1 (gradient merge + fused AdaGrad,
// dim 1).  Wider rows use k_srv_fill_rows / k_srv_merge_rows below.
#include "ss_device.h"
#include "ss_launch.h"
#include "scan.h"

namespace ss {

static constexpr int kSrvTS = 4096;     // LDS hash slots per server bucket
static constexpr int kSrvOcc = 8192;    // received keys per server bucket (LDS parking)
static constexpr int kSrvDT = 512;      // dedup workgroup
static constexpr int kSrvRegs = 8;      // received keys per dedup thread in flight
static constexpr int kSrvMaxSrc = 64;   // sources of a round
static constexpr uint32_t kSrvInv = 0xFFFFFFFFu;

struct SrvRuns {
  const uint64_t* rkeys;   // [nsrc * cap] received keys, segment s at s*cap
  const uint32_t* rbase;   // [nsrc][Pd] the sources' bucket bases (their send layout)
  const uint32_t* rnum;    // [nsrc][Pd] the sources' bucket sizes
  long long cap;           // per-source segment capacity (== every source's ucap)
  int nsrc, Pd, m, me;
  // [nsrc][Pd][m] (m > 1): where sub-bucket t starts in source s's run k
  // (the sender grouped each run by sub-bucket, bdedup.hip msub)
  const uint32_t* roff;
  SelfSeg self;            // this rank's own keys: the sender's send buffer, not the arena
  __device__ __forceinline__ long long run_start(int s, int k) const {
    return (long long)s * cap + ((long long)rbase[(long long)s * Pd + k] - (long long)me * cap);
  }
  __device__ __forceinline__ uint32_t run_len(int s, int k) const {
    return rnum[(long long)s * Pd + k];
  }
  // the part of run (s, k) server bucket k*m + t reads: the whole run (m ==
  // 1) or the sub-bucket's range (the sender grouped the run)
  __device__ __forceinline__ void part(int s, int k, int t, long long* a, uint32_t* len) const {
    *a = run_start(s, k);
    const uint32_t n = run_len(s, k);
    if (m == 1) {
      *len = n;
      return;
    }
    const uint32_t* o = roff + ((long long)s * Pd + k) * m;
    const uint32_t lo = min(o[t], n), hi = t + 1 < m ? min(o[t + 1], n) : n;
    *a += lo;
    *len = hi > lo ? hi - lo : 0u;
  }
};

// 1+2. received keys per server bucket, kSrvCntK buckets k per workgroup;
//    the LAST workgroup to finish (arrival counter) scans the counts into
//    bstart and zeroes the distinct-key counter — no separate
//    single-workgroup launch.  (One workgroup per k measured 70 us: ~5000
//    arrivals on one counter serialise at ~12 ns each.)
static constexpr int kSrvCntK = 64;

__global__ __launch_bounds__(256) void k_srv_count(SrvRuns R, uint32_t* __restrict__ cnt,
                                                   uint32_t* __restrict__ bstart,
                                                   unsigned long long* __restrict__ ucount,
                                                   unsigned int* __restrict__ ctr) {
  __shared__ unsigned int wsum[16];
  __shared__ unsigned int tot;
  __shared__ bool last;
  const int t = threadIdx.x;
  const int k0 = blockIdx.x * kSrvCntK, k1 = min(R.Pd, k0 + kSrvCntK);
  // the run (or sub-range) lengths are the counts: one thread per bucket
  for (int b = k0 * R.m + t; b < k1 * R.m; b += 256) {
    unsigned int c = 0;
    for (int s = 0; s < R.nsrc; ++s) {
      long long a;
      uint32_t len;
      R.part(s, b / R.m, b % R.m, &a, &len);
      c += len;
    }
    __hip_atomic_store(&cnt[b], c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (t == 0) last = atomicAdd(ctr, 1u) == gridDim.x - 1;
  __syncthreads();
  if (!last) return;  // workgroup-uniform
  const int P = R.Pd * R.m;
  const int per = (P + 255) / 256;
  const int b0 = t * per;
  unsigned int sum = 0;
  for (int i = 0; i < per; ++i)
    if (b0 + i < P) sum += __hip_atomic_load(&cnt[b0 + i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  unsigned int e = block_excl_scan<4>(sum, wsum, &tot);
  for (int i = 0; i < per; ++i)
    if (b0 + i < P) {
      bstart[b0 + i] = e;
      e += __hip_atomic_load(&cnt[b0 + i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  if (t == 0) {
    bstart[P] = tot;
    *ucount = 0ull;
    *ctr = 0u;  // ready for the next call (stream-ordered)
  }
}

// 3. one workgroup per server bucket b = k*m + t
__global__ __launch_bounds__(kSrvDT) void k_srv_dedup(SrvRuns R, const uint32_t* __restrict__ bstart,
                                                      uint32_t* __restrict__ pj,
                                                      uint32_t* __restrict__ luid,
                                                      uint64_t* __restrict__ bkeys,
                                                      uint32_t* __restrict__ ubase,
                                                      uint32_t* __restrict__ unum,
                                                      unsigned long long* __restrict__ ucount,
                                                      uint32_t* __restrict__ err) {
  __shared__ unsigned long long tab[kSrvTS];
  __shared__ unsigned int lid[kSrvTS];
  __shared__ unsigned short park[kSrvOcc];
  __shared__ unsigned int wsum[16];
  __shared__ long long sa[kSrvMaxSrc];      // where each source's part starts
  __shared__ unsigned int so[kSrvMaxSrc + 1];  // its first flat index
  __shared__ unsigned int tot;
  __shared__ int bad;
  const int t = threadIdx.x;
  const int b = blockIdx.x, k = b / R.m;
  const uint32_t sub = (uint32_t)(b % R.m);
  const uint32_t p0 = bstart[b], p1 = bstart[b + 1];
  // the table sized to the bucket's received keys (load <= 1/2): small
  // buckets (word2vec) skip initialising and compacting 4096 slots
  const uint32_t ts = lds_table_size(p1 - p0, kSrvTS);
  for (uint32_t s = t; s < ts; s += kSrvDT) tab[s] = kEmptyKey;
  if (t < R.nsrc) {  // every source's part, looked up in parallel
    long long a;
    uint32_t len;
    R.part(t, k, (int)sub, &a, &len);
    sa[t] = a;
    so[t + 1] = len;
  }
  __syncthreads();
  if (t == 0) {
    so[0] = 0u;
    for (int s = 0; s < R.nsrc; ++s) so[s + 1] += so[s];
    bad = so[R.nsrc] != p1 - p0 ? 2 : 0;  // 2: the runs disagree with the count
  }
  __syncthreads();
  auto insert = [&](uint64_t key) -> uint32_t {
    // slot from the high word's low bits: the sender's bucket fixed the high
    // word's top bits, the sub-bucket the low word's
    uint32_t s = (uint32_t)(dedup_hash(key) >> 32) & (ts - 1);
    for (uint32_t i = 0; i < ts; ++i) {
      const unsigned long long v = tab[s];
      if (v == key) return s;
      if (v == kEmptyKey) {
        const unsigned long long prev = atomicCAS(&tab[s], kEmptyKey, (unsigned long long)key);
        if (prev == kEmptyKey || prev == key) return s;
      }
      s = (s + 1) & (ts - 1);
    }
    atomicOr(&bad, 1);  // 1: the LDS table is full
    return kSrvInv;
  };
  // the sources' parts as one flat list [0, nall): position p0 + f holds
  // flat key f.  kSrvRegs keys per thread are loaded before any is inserted
  // (one load latency per round instead of one per source).  The first
  // kSrvOcc keys park their LDS slot; the rest (a Zipf-head bucket of the
  // record exchange, whose sources ship every occurrence) probe the table
  // again after the compaction
  const uint32_t nall = min(so[R.nsrc], p1 - p0);
  const uint32_t n = min(nall, (uint32_t)kSrvOcc);
  auto flat_pos = [&](uint32_t f) -> long long {
    int s = 0;
    while (s + 1 < R.nsrc && f >= so[s + 1]) ++s;
    return sa[s] + (f - so[s]);
  };
  for (uint32_t f0 = 0; f0 < nall; f0 += kSrvDT * kSrvRegs) {
    uint64_t kk[kSrvRegs];
#pragma unroll
    for (int r = 0; r < kSrvRegs; ++r) {
      const uint32_t f = f0 + (uint32_t)(r * kSrvDT + t);
      kk[r] = kEmptyKey;
      if (f < nall) {
        const long long pos = flat_pos(f);
        kk[r] = R.self.pick(R.rkeys, pos)[pos];
        pj[p0 + f] = (uint32_t)pos;
      }
    }
#pragma unroll
    for (int r = 0; r < kSrvRegs; ++r) {
      const uint32_t f = f0 + (uint32_t)(r * kSrvDT + t);
      if (f < nall) {
        const uint32_t sl = insert(kk[r]);
        if (f < n) park[f] = (unsigned short)sl;
      }
    }
  }
  __syncthreads();
  // compaction in slot order: thread t owns slots [per*t, per*(t+1))
  constexpr int kPerT = kSrvTS / kSrvDT;
  const uint32_t per = ts >= (uint32_t)kSrvDT ? ts / kSrvDT : 1u;
  auto own = [&](int i) -> unsigned long long {
    const uint32_t s = (uint32_t)t * per + (uint32_t)i;
    return (uint32_t)i < per && s < ts ? tab[s] : kEmptyKey;
  };
  unsigned int occ = 0;
#pragma unroll
  for (int i = 0; i < kPerT; ++i) occ += own(i) != kEmptyKey;
  unsigned int o = block_excl_scan<kSrvDT / 64>(occ, wsum, &tot);
  __shared__ unsigned long long sbase;
  if (t == 0) {
    sbase = atomicAdd(ucount, (unsigned long long)tot);
    ubase[b] = (uint32_t)sbase;
    unum[b] = tot;
    if (bad) atomicOr(err, (uint32_t)bad);
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < kPerT; ++i) {
    const uint32_t s = (uint32_t)t * per + (uint32_t)i;
    const unsigned long long v = own(i);
    if (v != kEmptyKey) {
      lid[s] = o;
      bkeys[p0 + o] = v;  // staged in the bucket's own range (k_pull_unique_bk reads it)
      ++o;
    }
  }
  __syncthreads();
  for (uint32_t q = t; q < n; q += kSrvDT) {
    const uint32_t sl = park[q] == 0xFFFFu ? kSrvInv : park[q];
    luid[p0 + q] = sl == kSrvInv || sl >= ts ? kSrvInv : lid[sl];
  }
  // keys past the parking area: their slot by a read-only probe of the
  // compacted table (every key of the bucket was inserted above)
  for (uint32_t f = n + t; f < nall; f += kSrvDT) {
    const long long pos = flat_pos(f);
    const uint64_t key = R.self.pick(R.rkeys, pos)[pos];
    uint32_t sl = (uint32_t)(dedup_hash(key) >> 32) & (ts - 1), id = kSrvInv;
    for (uint32_t i = 0; i < ts; ++i) {
      const unsigned long long v = tab[sl];
      if (v == key) {
        id = lid[sl];
        break;
      }
      if (v == kEmptyKey) break;
      sl = (sl + 1) & (ts - 1);
    }
    luid[p0 + f] = id;
  }
  // a bucket whose counts disagree with its runs (error flagged above): the
  // positions past the sources' runs still get an in-range pj and no local
  // id, so the fill and merge kernels (which walk [p0, p1)) write zero rows
  // to real positions and skip the gradients instead of reading / writing
  // through unset entries
  for (uint32_t f = nall + t; f < p1 - p0; f += kSrvDT) {
    pj[p0 + f] = 0u;
    luid[p0 + f] = kSrvInv;
  }
}

// lanes per row for rows of n 16-byte chunks: the next power of two, <= 64
__device__ __forceinline__ int srv_group(int n) {
  return n <= 1 ? 1 : n <= 2 ? 2 : n <= 4 ? 4 : n <= 8 ? 8 : n <= 16 ? 16 : n <= 32 ? 32 : 64;
}

// response rows of width D > 1: out[pj[p]] = rows[ubase[b] + luid[p]].  A
// group of lanes per received row moving it as 16-byte chunks (D % 4 == 0;
// word2vec's 512-byte rows: one 32-lane group each), 4-byte words otherwise
__global__ __launch_bounds__(256) void k_srv_fill_rows(const uint32_t* __restrict__ bstart,
                                                       const uint32_t* __restrict__ ubase,
                                                       const uint32_t* __restrict__ pj,
                                                       const uint32_t* __restrict__ luid,
                                                       const float* __restrict__ rows,
                                                       float* __restrict__ out, int D,
                                                       SelfSeg self) {
  const int b = blockIdx.x, t = threadIdx.x;
  const uint32_t p0 = bstart[b], p1 = bstart[b + 1], base = ubase[b];
  const bool vec = (D & 3) == 0;
  const int W = vec ? D >> 2 : D;  // chunks per row
  const int G = srv_group(W), lg = t % G, ng = 256 / G;
  // gridDim.y workgroups share a bucket (few, large buckets: word2vec)
  for (uint32_t p = p0 + blockIdx.y * ng + t / G; p < p1; p += gridDim.y * ng) {
    const uint32_t l = luid[p];
    const long long o = (long long)pj[p] * W, r = ((long long)base + l) * W;
    float* outp = self.pick(out, (long long)pj[p]);
    if (vec) {
      float4* dst = reinterpret_cast<float4*>(outp) + o;
      const float4* src = reinterpret_cast<const float4*>(rows) + r;
      for (int c = lg; c < W; c += G) dst[c] = l == kSrvInv ? make_float4(0.f, 0.f, 0.f, 0.f) : src[c];
    } else {
      for (int c = lg; c < W; c += G) outp[o + c] = l == kSrvInv ? 0.f : rows[r + c];
    }
  }
}

// gradient merge of rows of width D: grads received at positions pj[p] are
// summed per distinct key into merged[ubase[b] + l].  Per bucket the
// positions are counting-sorted by local id in LDS (tables sized by the
// bucket's distinct keys, not the 4096-slot maximum: word2vec buckets hold
// ~30), then a lane group per key sums its rows (lane-consecutive words; no
// atomics).  `slots`: the merged row goes straight into the
// optimizer update of the key's table row (each lane updates its
// coordinates and their state) — no merged-row round trip, no apply launch
__global__ __launch_bounds__(512) void k_srv_merge_rows(const uint32_t* __restrict__ bstart,
                                                        const uint32_t* __restrict__ ubase,
                                                        const uint32_t* __restrict__ unum,
                                                        const uint32_t* __restrict__ pj,
                                                        const uint32_t* __restrict__ luid,
                                                        const float* __restrict__ grads,
                                                        float* __restrict__ merged, int D,
                                                        DevTable tab,
                                                        const long long* __restrict__ slots,
                                                        OptParams op, SelfSeg self) {
  __shared__ unsigned int off[kSrvTS + 1];
  __shared__ unsigned int cur[kSrvTS];
  __shared__ unsigned short ord[kSrvOcc];
  __shared__ unsigned int wsum[16];
  const int b = blockIdx.x, t = threadIdx.x;
  const uint32_t p0 = bstart[b], p1 = bstart[b + 1], nu = min(unum[b], (uint32_t)kSrvTS);
  const uint32_t base = ubase[b];
  const uint32_t np = min(p1 - p0, (uint32_t)kSrvOcc);
  if (nu == 0) return;  // workgroup-uniform
  if (np == nu) {
    // every distinct key received once (one source, or no overlap between
    // the sources in this bucket): key l's position is the q with luid = l,
    // no counting sort
    for (uint32_t l = t; l <= nu; l += 512) off[l] = l;
    for (uint32_t q = t; q < np; q += 512) {
      const uint32_t l = luid[p0 + q];
      if (l < nu) ord[l] = (unsigned short)q;
    }
    __syncthreads();
  } else {
    for (uint32_t l = t; l <= nu; l += 512) off[l] = 0u;
    __syncthreads();
    for (uint32_t q = t; q < np; q += 512) {
      const uint32_t l = luid[p0 + q];
      if (l < nu) atomicAdd(&off[l + 1], 1u);
    }
    __syncthreads();
    // inclusive scan of off[1..nu]: thread t owns `per` consecutive entries
    const uint32_t per = (nu + 511) / 512;  // <= kSrvTS / 512
    unsigned int sum = 0;
    for (uint32_t i = 0; i < per; ++i) {
      const uint32_t l = 1 + t * per + i;
      if (l <= nu) sum += off[l];
    }
    unsigned int e = block_excl_scan<8>(sum, wsum, nullptr);
    for (uint32_t i = 0; i < per; ++i) {
      const uint32_t l = 1 + t * per + i;
      if (l <= nu) {
        e += off[l];
        off[l] = e;
      }
    }
    __syncthreads();
    // placement: a second counter pass (cursor = off[l], advanced atomically)
    for (uint32_t l = t; l < nu; l += 512) cur[l] = off[l];
    __syncthreads();
    for (uint32_t q = t; q < np; q += 512) {
      const uint32_t l = luid[p0 + q];
      if (l < nu) ord[atomicAdd(&cur[l], 1u)] = (unsigned short)q;
    }
    __syncthreads();
  }
  const int ns = opt_state_per_coord(op.kind);
  // a group of G lanes per key; lane lg owns coordinates lg + i*G, so every
  // load / store instruction of the group covers G consecutive words (the
  // table row and the gradient rows alike; 16-byte chunks per lane left each
  // instruction a strided 512-byte span)
  const int G = srv_group((D + 3) / 4), lg = t % G;
  const uint32_t kpp = 512 / G;       // keys in flight per workgroup
  // gridDim.y workgroups share a bucket (each sorted the bucket's positions
  // above; few, large buckets: word2vec at one rank has ~50)
  for (uint32_t l = blockIdx.y * kpp + (uint32_t)(t / G); l < nu; l += gridDim.y * kpp) {
    const uint32_t a = off[l], z = off[l + 1];
    const long long slot = slots ? slots[(long long)base + l] : -1;
    const bool upd = slots && slot >= 0;
    for (int c0 = 0; c0 < D; c0 += 4 * G) {
      // fused update: the row (and state) loads go out before the gradient
      // sum, their latency overlaps the gathers instead of following them
      float wv[4], s1[4], s2[4], acc[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int c = c0 + lg + i * G;
        const bool on = upd && c < D;
        wv[i] = on ? row_ld(tab, slot, c) : 0.f;
        s1[i] = on && ns > 0 ? row_ld(tab, slot, D + c) : 0.f;
        s2[i] = on && ns > 1 ? row_ld(tab, slot, 2 * D + c) : 0.f;
      }
      for (uint32_t q = a; q < z; ++q) {
        const long long gp = pj[p0 + ord[q]];
        const float* g = self.pick(grads, gp) + gp * D;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int c = c0 + lg + i * G;
          if (c < D) acc[i] += g[c];
        }
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int c = c0 + lg + i * G;
        if (c >= D) continue;
        if (!slots) {
          merged[((long long)base + l) * D + c] = acc[i];
        } else if (upd) {
          opt_update(op, wv[i], s1[i], s2[i], acc[i]);
          row_st(tab, slot, c, wv[i], true);
          if (ns > 0) row_st(tab, slot, D + c, s1[i], true);
          if (ns > 1) row_st(tab, slot, 2 * D + c, s2[i], true);
        }
      }
    }
  }
}

// ------------------------------------------------------------- launchers
// workgroups per server bucket of the wide-row fill / merge: enough for ~1024
// workgroups in all (word2vec's ~50 buckets of ~500 keys left 200 CUs idle)
static int srv_share(int P) {
  const int y = 1024 / (P < 1 ? 1 : P);
  return y < 1 ? 1 : (y > 8 ? 8 : y);
}

int srv_sub_buckets(int nsrc, long long lay_n, int ndest) {
  // SS_SRV_SUB=m: a fixed count (A/B)
  static const int fixed = [] {
    const char* e = std::getenv("SS_SRV_SUB");
    return e ? std::atoi(e) : 0;
  }();
  if (fixed > 0) return fixed > 64 ? 64 : fixed;
  // one source: its bucket's unique keys passed the worker dedup's own
  // 4096-slot table, so they fit a server table as they are
  if (nsrc <= 1) return 1;
  // N sources x the layout's occurrences per source bucket (lay_n keys per
  // call: ~bd_target_dist() for large calls, fewer for small ones such as
  // word2vec's; <= ~1.25x that with hash imbalance, every occurrence counted
  // as a distinct key) per bucket k, at most ~3000 distinct keys per
  // 4096-slot table
  long long per = bd_target_dist();
  if (lay_n > 0) {
    const int P = bd_buckets(lay_n, nsrc, ndest > 0 ? ndest : nsrc);
    const int nd = ndest > 0 && ndest < nsrc ? ndest : nsrc;
    per = (lay_n + (long long)(P / nsrc) * nd - 1) / ((long long)(P / nsrc) * nd);
  }
  const long long need = (long long)nsrc * per * 5 / 4;
  int m = (int)((need + 2999) / 3000);
  return m < 1 ? 1 : (m > 64 ? 64 : m);
}

void launch_srv_dedup(const uint64_t* rkeys, const uint32_t* rbase, const uint32_t* rnum,
                      long long cap, int nsrc, int Pd, int m, int me, uint32_t* cnt,
                      uint32_t* bstart, uint32_t* pj, uint32_t* luid, uint64_t* bkeys,
                      uint32_t* ubase, uint32_t* unum, unsigned long long* ucount, uint32_t* err,
                      hipStream_t st, const uint32_t* roff, SelfSeg self) {
  if (nsrc < 1 || nsrc > kSrvMaxSrc || Pd < 1 || m < 1 || m > 64) throw_error("srv_dedup: bad layout");
  if (m > 1 && !roff) throw_error("srv_dedup: sub-buckets need the senders' offsets (msub)");
  SrvRuns R{rkeys, rbase, rnum, cap, nsrc, Pd, m, me, roff, self};
  const int P = Pd * m;
  // cnt has P + 1 words: the last is the count kernel's arrival counter
  // (zeroed once at allocation, reset by the kernel)
  hipLaunchKernelGGL(k_srv_count, dim3((Pd + kSrvCntK - 1) / kSrvCntK), dim3(256), 0, st, R, cnt,
                     bstart, ucount, cnt + P);
  check_launch("k_srv_count");
  hipLaunchKernelGGL(k_srv_dedup, dim3(P), dim3(kSrvDT), 0, st, R, bstart, pj, luid, bkeys,
                     ubase, unum, ucount, err);
  check_launch("k_srv_dedup");
}

void launch_srv_fill_rows(int P, const uint32_t* bstart, const uint32_t* ubase,
                          const uint32_t* pj, const uint32_t* luid, const float* rows, float* out,
                          int D, hipStream_t st, SelfSeg self) {
  if (P <= 0) return;
  hipLaunchKernelGGL(k_srv_fill_rows, dim3(P, srv_share(P)), dim3(256), 0, st, bstart, ubase, pj,
                     luid, rows, out, D, self);
  check_launch("k_srv_fill_rows");
}

void launch_srv_merge_rows(int P, const uint32_t* bstart, const uint32_t* ubase,
                           const uint32_t* unum, const uint32_t* pj, const uint32_t* luid,
                           const float* grads, float* merged, int D, hipStream_t st,
                           const DevTable* t, const long long* slots, const OptParams* op,
                           SelfSeg self) {
  if (P <= 0) return;
  if (slots && (!t || !op || (int)t->dim != D ||
                (int)t->width != D * (1 + opt_state_per_coord(op->kind))))
    throw_error("srv_merge_rows: a fused update needs the table of these rows");
  if (!slots && !merged) throw_error("srv_merge_rows: merged rows or a fused update");
  hipLaunchKernelGGL(k_srv_merge_rows, dim3(P, srv_share(P)), dim3(512), 0, st, bstart, ubase,
                     unum, pj, luid,
                     grads, merged, D, t ? *t : DevTable{}, slots, op ? *op : OptParams{}, self);
  check_launch("k_srv_merge_rows");
}

}  // namespace ss
