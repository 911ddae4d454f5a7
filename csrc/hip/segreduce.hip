// segreduce.hip — atomic-light duplicate-key gradient reduction (K7) for
// scalar-per-key models (sparse LR).
//
// The reference merges duplicate-key gradients on the worker
// (GradPramProcMethod::merge_grad, /root/reference/src/core/parameter/
// global_param_cache.h:14-15; PushAccessMethod::merge_push_value,
// sparse_access_method.h:39-40).  The first version here scattered one float
// atomicAdd per key occurrence: 2.56M atomics = 164 us/step, because on
// MI355X every device-scope atomic executes at the memory side (~18 G/s for
// one-lane-per-address adds, tools/mb_atomics.hip).
//
// Replacement = one radix-partition pass + LDS accumulation:
//   route stream (off the critical path, right after dedup):
//     count      per 8192-occurrence chunk, histogram of bin(cu) in LDS
//                (cu = compact unique id, bin = cu >> 13)
//     scan       exclusive scan over [bin][chunk] through LDS tiles, then a
//                work list: each bin cut into <= 8192-pair items, so a bin
//                holding the batch's hot keys (dedup numbers them first) is
//                spread over many workgroups instead of serialising one
//     positions  every occurrence gets its slot in the bin-ordered pair array
//   main stream:
//     the model's forward kernel writes (cu & 8191, grad) at that slot
//     reduce     one workgroup per work item: LDS atomics into 8192
//                accumulators, then one coalesced row-shaped atomicAdd per
//                touched unique key (full-rate atomic shape, ~10 MB/step)
#include <cstdlib>
#include <string>

#include "sample_group.h"
#include "scan.h"

#include "ss_device.h"
#include "ss_launch.h"

namespace ss {

static constexpr uint32_t kInvS = 0xFFFFFFFFu;
static constexpr int kBinShift = 13;
static constexpr int kBinW = 1 << kBinShift;  // unique ids per bin (LDS floats)
static constexpr int kChunk = 8192;           // occurrences per count/positions block
static constexpr int kItem = 8192;            // pairs per reduce work item
static constexpr int kMaxBins = 4096;
static constexpr int kPer = kChunk / 1024;    // occurrences per thread (1024-thread blocks)

// compact id <-> layout id: uid = d*ucap + local, cu = prefix[d] + local
struct CuMap {
  const unsigned long long* ucount;
  int nranks;
  long long ucap;
};

__device__ __forceinline__ void load_prefix(const CuMap& m, unsigned int* pre) {
  if (threadIdx.x == 0) {
    unsigned int a = 0;
    for (int d = 0; d < m.nranks; ++d) {
      pre[d] = a;
      a += (unsigned int)m.ucount[d];
    }
    pre[m.nranks] = a;
  }
  __syncthreads();
}
__device__ __forceinline__ unsigned int cu_of(const CuMap& m, const unsigned int* pre, uint32_t uid) {
  if (m.nranks == 1) return uid;
  const uint32_t d = uid / (uint32_t)m.ucap;  // uid < 2^31: 32-bit divide
  return pre[d] + (uid - d * (uint32_t)m.ucap);
}

__global__ __launch_bounds__(1024) void k_sr_count(const uint32_t* __restrict__ inv, long long n,
                                                   CuMap m, uint32_t* __restrict__ hist, int nbins,
                                                   int nchunks) {
  __shared__ unsigned int pre[kMaxSeg + 1];
  __shared__ unsigned int h[kMaxBins];
  for (int b = threadIdx.x; b < nbins; b += 1024) h[b] = 0;
  load_prefix(m, pre);
  const long long a = (long long)blockIdx.x * kChunk + threadIdx.x;
  uint32_t u[kPer];
#pragma unroll
  for (int k = 0; k < kPer; ++k) u[k] = a + k * 1024 < n ? inv[a + k * 1024] : kInvS;
#pragma unroll
  for (int k = 0; k < kPer; ++k)
    if (u[k] != kInvS) atomicAdd(&h[cu_of(m, pre, u[k]) >> kBinShift], 1u);
  __syncthreads();
  for (int b = threadIdx.x; b < nbins; b += 1024) hist[(long long)b * nchunks + blockIdx.x] = h[b];
}

// Bin starts (exclusive scan of the per-bin totals from the row scan, single
// workgroup over <= 4096 values) and the reduce work list:
// items[k] = (bin, first pair, end pair), <= kItem pairs each.
__global__ __launch_bounds__(1024) void k_sr_scan(const uint32_t* __restrict__ btot, int nbins,
                                                  uint32_t* __restrict__ bstart,
                                                  uint4* __restrict__ items,
                                                  uint32_t* __restrict__ nitems) {
  __shared__ unsigned int wsum[16];
  __shared__ unsigned int tot;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  unsigned int carry = 0;
  for (int b0 = 0; b0 < nbins; b0 += 1024) {
    const int b = b0 + t;
    const unsigned int v = b < nbins ? btot[b] : 0u;
    const unsigned int e = block_excl_scan_1024(v, wsum, &tot);
    if (b < nbins) bstart[b] = carry + e;
    carry += tot;
  }
  if (t == 0) bstart[nbins] = carry;
  __syncthreads();
  // ---- work list: per bin ceil(pairs / kItem) items; block scan over bins
  unsigned int off = 0;
  for (int b0 = 0; b0 < nbins; b0 += 1024) {
    const int b = b0 + t;
    unsigned int st = 0, en = 0, cnt = 0;
    if (b < nbins) {
      st = bstart[b];
      en = bstart[b + 1];
      cnt = (en - st + kItem - 1) / kItem;
    }
    unsigned int x = cnt;
    for (int o = 1; o < 64; o <<= 1) {
      const unsigned int y = __shfl_up(x, o, 64);
      if (lane >= o) x += y;
    }
    if (lane == 63) wsum[w] = x;
    __syncthreads();
    if (w == 0) {
      unsigned int ws = lane < 16 ? wsum[lane] : 0u;
      for (int o = 1; o < 16; o <<= 1) {
        const unsigned int y = __shfl_up(ws, o, 64);
        if (lane >= o) ws += y;
      }
      if (lane < 16) wsum[lane] = ws;
    }
    __syncthreads();
    unsigned int k0 = off + (w ? wsum[w - 1] : 0u) + x - cnt;
    for (unsigned int q = 0; q < cnt; ++q) {
      const unsigned int a = st + q * kItem;
      items[k0 + q] = make_uint4((unsigned)b, a, a + kItem < en ? a + kItem : en, 0u);
    }
    off += wsum[15];
    __syncthreads();
  }
  if (t == 0) *nitems = off;
}

__global__ __launch_bounds__(1024) void k_sr_positions(const uint32_t* __restrict__ inv, long long n,
                                                       CuMap m, const uint32_t* __restrict__ hist,
                                                       const uint32_t* __restrict__ grp,
                                                       const uint32_t* __restrict__ bstart,
                                                       int nbins, int nchunks,
                                                       uint2* __restrict__ plan) {
  __shared__ unsigned int pre[kMaxSeg + 1];
  __shared__ unsigned int cur[kMaxBins];
  const int ng = scan_groups(nchunks), g = blockIdx.x / kScanGroup;
  for (int b = threadIdx.x; b < nbins; b += 1024)
    cur[b] = bstart[b] + hist[(long long)b * nchunks + blockIdx.x] + grp[(long long)b * ng + g];
  load_prefix(m, pre);
  const long long a = (long long)blockIdx.x * kChunk + threadIdx.x;
  uint32_t u[kPer];
#pragma unroll
  for (int k = 0; k < kPer; ++k) u[k] = a + k * 1024 < n ? inv[a + k * 1024] : kInvS;
#pragma unroll
  for (int k = 0; k < kPer; ++k) {
    const long long j = a + k * 1024;
    if (j < n && u[k] != kInvS) {
      const unsigned int cu = cu_of(m, pre, u[k]);
      const unsigned int p = atomicAdd(&cur[cu >> kBinShift], 1u);
      plan[p] = make_uint2((uint32_t)j, cu & (kBinW - 1));  // bin order: (occurrence, cu_lo)
    }
  }
}

// One workgroup per work item; plan[p] = (occurrence j, cu & (kBinW-1)), the
// gradient value is gocc[j] (written coalesced by the model's forward).
// ugrad must be zeroed for the round's unique keys (dedup does it).
__global__ __launch_bounds__(1024) void k_sr_reduce(const uint2* __restrict__ plan,
                                                    const float* __restrict__ gocc,
                                                    const uint4* __restrict__ items,
                                                    const uint32_t* __restrict__ nitems, CuMap m,
                                                    float* __restrict__ ugrad) {
  __shared__ unsigned int pre[kMaxSeg + 1];
  __shared__ float acc[kBinW];
  if (blockIdx.x >= *nitems) return;  // block-uniform
  const uint4 it = items[blockIdx.x];
  for (int c = threadIdx.x; c < kBinW; c += 1024) acc[c] = 0.f;
  load_prefix(m, pre);
  for (uint32_t p = it.y + threadIdx.x; p < it.z; p += 1024) {
    const uint2 pr = plan[p];
    atomicAdd(&acc[pr.y], gocc[pr.x]);
  }
  __syncthreads();
  const unsigned int total = pre[m.nranks];
  for (int c = threadIdx.x; c < kBinW; c += 1024) {
    const unsigned int cu = (it.x << kBinShift) + (unsigned)c;
    const float v = acc[c];
    if (cu >= total || v == 0.f) continue;
    int d = 0;
    while (d + 1 < m.nranks && cu >= pre[d + 1]) ++d;
    atomicAdd(ugrad + (unsigned long long)d * m.ucap + (cu - pre[d]), v);
  }
}

// ---- LR forward: per-sample dot/sigmoid/logloss; the gradient is written
// either per occurrence (g*x COALESCED to g[j], the bin-plan reduce gathers
// it) or per sample (g[s] = p - y, 4 B per sample; the bucketed reduce of
// bdedup.hip gathers it L2-resident and multiplies by x itself).
// Parameter of occurrence j: uvals[inv[j]], uvals[ix.uid(j)] (two dependent
// gathers: luid, then the row), or — `occ`, filled per bucket by
// k_bd_fill_occ — occ[ix.pos_of[j]]: one gather per occurrence
__device__ __forceinline__ float lr_param(long long j, const uint32_t* __restrict__ inv,
                                          const BdIndex& ix, const float* __restrict__ occ,
                                          const float* __restrict__ uvals) {
  if (occ) {
    if (!ix.pos_of) return occ[j];  // filled in sample order (k_bd_fill_occ with pj)
    const uint32_t p = ix.pos_of[j];
    return p == kInvS ? 0.f : occ[p];
  }
  const uint32_t u = inv ? inv[j] : ix.uid(j);  // bucketed dedup: no materialised inverse
  return u == kInvS ? 0.f : uvals[u];
}

__global__ __launch_bounds__(256) void k_lr_fwd_g_lds(const uint32_t* __restrict__ inv,
                                                  BdIndex ix,
                                                  const float* __restrict__ xval,
                                                  const float* __restrict__ labels, int B, int F,
                                                  const float* __restrict__ uvals,
                                                  float* __restrict__ gocc, int per_sample,
                                                  float* __restrict__ loss_sum,
                                                  float* __restrict__ pred,
                                                  const float* __restrict__ occ) {
  __shared__ float sval[256];
  __shared__ float sdot[256];
  __shared__ float sg[256];
  __shared__ float sloss[4];
  const int spb = F >= 256 ? 1 : 256 / F;
  const int t = threadIdx.x, ls = t / F;
  const long long s0 = (long long)blockIdx.x * spb;
  const bool active = ls < spb && s0 + ls < B;
  const long long j = s0 * F + t;
  float x = 0.f, wx = 0.f;
  if (active) {
    x = xval ? xval[j] : 1.f;
    wx = lr_param(j, inv, ix, occ, uvals) * x;
  }
  packed_sample_sums(wx, F, spb, sval, sdot);  // per-sample dots, no LDS atomics
  float l = 0.f;
  if (t < spb && s0 + t < B) {
    const float z = sdot[t];
    const float y = labels[s0 + t];
    const float p = 1.f / (1.f + __expf(-z));
    sg[t] = p - y;
    if (per_sample) gocc[s0 + t] = p - y;
    if (pred) pred[s0 + t] = p;
    l = fmaxf(z, 0.f) + __logf(1.f + __expf(-fabsf(z))) - y * z;
  }
  for (int o = 32; o > 0; o >>= 1) l += __shfl_down(l, o, 64);
  if ((t & 63) == 0) sloss[t >> 6] = l;
  __syncthreads();
  if (t == 0 && loss_sum) ctr_addf(loss_sum, sloss[0] + sloss[1] + sloss[2] + sloss[3]);
  if (active && !per_sample) gocc[j] = sg[ls] * x;
}

// k_lr_fwd_g_lds over R groups of spb samples per workgroup, for the
// bucketed one-gather mode (occ + pos_of, per-sample gradients): every
// thread issues its R pos_of loads, then its R occ gathers, before the first
// LDS sum — R dependent-load chains in flight per thread instead of one, and
// R x fewer 256-thread workgroups (43691 at the bench shape, each one chain
// deep).  Needs R * spb <= 256 (the per-sample tail runs one sample per thread).
template <int R>
__global__ __launch_bounds__(256) void k_lr_fwd_occ(const uint32_t* __restrict__ pos_of,
                                                    const float* __restrict__ xval,
                                                    const float* __restrict__ labels, int B, int F,
                                                    float* __restrict__ gs,
                                                    float* __restrict__ loss_sum,
                                                    float* __restrict__ pred,
                                                    const float* __restrict__ occ,
                                                    SelfSeg oself) {
  __shared__ float sval[R * 256];
  __shared__ float sdot[256];
  __shared__ float sloss[4];
  const int spb = F >= 256 ? 1 : 256 / F;
  const int t = threadIdx.x, ls = t / F;
  const long long sb = (long long)blockIdx.x * spb * R;  // first sample of the workgroup
  uint32_t p[R];
  float x[R];
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const long long s = sb + (long long)r * spb + ls;
    const bool active = ls < spb && s < B;
    const long long j = (sb + (long long)r * spb) * F + t;
    p[r] = active ? (pos_of ? pos_of[j] : (uint32_t)j) : kInvS;  // null: occ in sample order
    x[r] = active ? (xval ? xval[j] : 1.f) : 0.f;
  }
#pragma unroll
  for (int r = 0; r < R; ++r)
    sval[r * 256 + t] = p[r] == kInvS ? 0.f : oself.pick(occ, (long long)p[r])[p[r]] * x[r];
  __syncthreads();
  // R * spb sample sums, tps threads per sample (as packed_sample_sums)
  const int ns = R * spb;
  int tps = 8;
  while (tps > 1 && tps * ns > 256) tps >>= 1;
  const int gi = t / tps, k = t - gi * tps;
  float z = 0.f;
  if (gi < ns) {
    const float* v = sval + (gi / spb) * 256 + (gi % spb) * F;
    for (int f = k; f < F; f += tps) z += v[f];
  }
  for (int o = tps >> 1; o > 0; o >>= 1) z += __shfl_xor(z, o, 64);
  if (gi < ns && k == 0) sdot[gi] = z;
  __syncthreads();
  float l = 0.f;
  if (t < ns && sb + t < B) {  // group r's sample ls2 is sample sb + r * spb + ls2 = sb + t
    const float zz = sdot[t];
    const float y = labels[sb + t];
    const float pr = 1.f / (1.f + __expf(-zz));
    gs[sb + t] = pr - y;
    if (pred) pred[sb + t] = pr;
    l = fmaxf(zz, 0.f) + __logf(1.f + __expf(-fabsf(zz))) - y * zz;
  }
  for (int o = 32; o > 0; o >>= 1) l += __shfl_down(l, o, 64);
  if ((t & 63) == 0) sloss[t >> 6] = l;
  __syncthreads();
  if (t == 0 && loss_sum) ctr_addf(loss_sum, sloss[0] + sloss[1] + sloss[2] + sloss[3]);
}

// Same contract, one sample per lane group (F <= 64, sample_group.h).
__global__ __launch_bounds__(256) void k_lr_fwd_g(const uint32_t* __restrict__ inv,
                                                  BdIndex ix,
                                                  const float* __restrict__ xval,
                                                  const float* __restrict__ labels, int B, int F,
                                                  int L, const float* __restrict__ uvals,
                                                  float* __restrict__ gocc, int per_sample,
                                                  float* __restrict__ loss_sum,
                                                  float* __restrict__ pred,
                                                  const float* __restrict__ occ) {
  __shared__ float sloss[4];
  const int t = threadIdx.x, f = t & (L - 1);
  const long long s = (long long)blockIdx.x * (256 / L) + t / L;
  const bool active = f < F && s < B;
  const long long j = s * F + f;
  float x = 0.f, v = 0.f;
  if (active) {
    x = xval ? xval[j] : 1.f;
    v = lr_param(j, inv, ix, occ, uvals) * x;
  }
  const float z = group_sum(v, L);
  float l = 0.f, g = 0.f;
  if (s < B) {
    const float y = labels[s];
    const float p = 1.f / (1.f + __expf(-z));
    g = p - y;
    if (f == 0) {
      if (per_sample) gocc[s] = g;
      if (pred) pred[s] = p;
      l = fmaxf(z, 0.f) + __logf(1.f + __expf(-fabsf(z))) - y * z;
    }
  }
  const float bl = block_sum_256(l, sloss);
  if (t == 0 && loss_sum) ctr_addf(loss_sum, bl);
  if (active && !per_sample) gocc[j] = g * x;
}

// -------------------------------------------------------------- launchers
int sr_nbins(long long max_unique) { return (int)((max_unique + kBinW - 1) >> kBinShift); }
int sr_nchunks(long long n) { return (int)((n + kChunk - 1) / kChunk); }
int sr_max_items(long long n) { return sr_nbins(n) + sr_nchunks(n) + 1; }
// hist buffer: [nbins][nchunks] counts | [nbins][ngroups] group bases |
//              btot[nbins] | bstart[nbins + 1]
long long sr_hist_words(long long n) {
  const long long nb = sr_nbins(n), nch = sr_nchunks(n);
  return nb * nch + nb * scan_groups((int)nch) + 2 * nb + 1;
}

void launch_sr_plan(const uint32_t* inv, long long n, const unsigned long long* ucount,
                    int nranks, long long ucap, uint32_t* hist, int nbins, void* plan,
                    void* items, uint32_t* nitems, hipStream_t st) {
  if (n <= 0) {
    check_hip(hipMemsetAsync(nitems, 0, 4, st), "nitems");
    return;
  }
  if (nbins > kMaxBins || nbins < 1) throw_error("segreduce: too many unique keys per call");
  if ((unsigned long long)nranks * (unsigned long long)ucap >= 0x80000000ull)
    throw_error("segreduce: unique-id space exceeds 31 bits");
  const int nch = sr_nchunks(n), ng = scan_groups(nch);
  uint32_t* grp = hist + (long long)nbins * nch;
  uint32_t* btot = grp + (long long)nbins * ng;
  uint32_t* bstart = btot + nbins;
  CuMap m{ucount, nranks, ucap};
  hipLaunchKernelGGL(k_sr_count, dim3(nch), dim3(1024), 0, st, inv, n, m, hist, nbins, nch);
  check_launch("k_sr_count");
  launch_rowscan(hist, nbins, nch, grp, btot, nullptr, st);
  check_launch("sr rowscan");
  hipLaunchKernelGGL(k_sr_scan, dim3(1), dim3(1024), 0, st, btot, nbins, bstart,
                     reinterpret_cast<uint4*>(items), nitems);
  check_launch("k_sr_scan");
  hipLaunchKernelGGL(k_sr_positions, dim3(nch), dim3(1024), 0, st, inv, n, m, hist, grp, bstart,
                     nbins, nch, reinterpret_cast<uint2*>(plan));
  check_launch("k_sr_positions");
}

void launch_sr_reduce(const void* plan, const float* gocc, const void* items,
                      const uint32_t* nitems, long long n, const unsigned long long* ucount,
                      int nranks, long long ucap, float* ugrad, hipStream_t st) {
  if (n <= 0) return;
  CuMap m{ucount, nranks, ucap};
  hipLaunchKernelGGL(k_sr_reduce, dim3(sr_max_items(n)), dim3(1024), 0, st,
                     reinterpret_cast<const uint2*>(plan), gocc,
                     reinterpret_cast<const uint4*>(items), nitems, m, ugrad);
  check_launch("k_sr_reduce");
}

void launch_lr_fwd_g(const uint32_t* inv, const BdIndex& ix, const float* xval,
                     const float* labels, int B, int F, const float* uvals, float* gocc,
                     int per_sample, float* loss_sum, float* pred, hipStream_t st,
                     const float* occ, SelfSeg occ_self) {
  if (!occ && !inv && !(ix.pos_of && ix.luid && ix.bkt && ix.ubase))
    throw_error("lr_fwd_g: need inv, a complete BdIndex, or occ (bucket order with pos_of, "
                "else sample order)");
  if (B <= 0) return;
  if (F < 1 || F > 256) throw_error("lr_fwd_g: F must be in [1,256]");
  // layout: one sample per lane group unless that leaves over a quarter of
  // the lanes idle (F = 39 -> 64-lane groups, 61% busy), then the packed one
  // (256/F samples per workgroup, 91% busy at F = 39: 192 vs 202 us per 10.2M
  // keys).  SS_LR_FWD=packed|group forces one (experiment knob).
  static const int force = [] {
    const char* e = std::getenv("SS_LR_FWD");
    if (!e) return 0;
    return std::string(e) == "packed" ? 1 : (std::string(e) == "group" ? 2 : 0);
  }();
  const bool packed = force == 1 || (force == 0 && 4 * F < 3 * group_lanes(F));
  // occ_self (positions read from a second buffer): the one-gather kernel only
  if (occ_self.ptr && !(occ && per_sample))
    throw_error("lr_fwd_g: an own-row buffer needs the one-gather per-sample form");
  if (F <= kGroupMaxF && !packed && !occ_self.ptr) {
    const int L = group_lanes(F), spb = 256 / L;
    hipLaunchKernelGGL(k_lr_fwd_g, dim3((B + spb - 1) / spb), dim3(256), 0, st, inv, ix, xval,
                       labels, B, F, L, uvals, gocc, per_sample, loss_sum, pred, occ);
    check_launch("k_lr_fwd_g");
    return;
  }
  const int spb = F >= 256 ? 1 : 256 / F;
  // the one-gather mode with per-sample gradients: R sample groups per
  // workgroup (SS_LR_FWD_R: 1 / 2 / 4)
  static const int fr = [] {
    const char* e = std::getenv("SS_LR_FWD_R");
    const int v = e ? std::atoi(e) : 4;
    return (v == 1 || v == 2 || v == 8) ? v : 4;
  }();
  if (occ && per_sample && ((fr > 1 && fr * spb <= 256) || occ_self.ptr)) {
    const int r = fr * spb <= 256 ? fr : 1;
    const int g = r * spb;
    if (r == 8)
      hipLaunchKernelGGL(k_lr_fwd_occ<8>, dim3((B + g - 1) / g), dim3(256), 0, st, ix.pos_of, xval,
                         labels, B, F, gocc, loss_sum, pred, occ, occ_self);
    else if (r == 4)
      hipLaunchKernelGGL(k_lr_fwd_occ<4>, dim3((B + g - 1) / g), dim3(256), 0, st, ix.pos_of, xval,
                         labels, B, F, gocc, loss_sum, pred, occ, occ_self);
    else if (r == 2)
      hipLaunchKernelGGL(k_lr_fwd_occ<2>, dim3((B + g - 1) / g), dim3(256), 0, st, ix.pos_of, xval,
                         labels, B, F, gocc, loss_sum, pred, occ, occ_self);
    else
      hipLaunchKernelGGL(k_lr_fwd_occ<1>, dim3((B + g - 1) / g), dim3(256), 0, st, ix.pos_of, xval,
                         labels, B, F, gocc, loss_sum, pred, occ, occ_self);
    check_launch("k_lr_fwd_occ");
    return;
  }
  hipLaunchKernelGGL(k_lr_fwd_g_lds, dim3((B + spb - 1) / spb), dim3(256), 0, st, inv, ix, xval,
                     labels, B, F, uvals, gocc, per_sample, loss_sum, pred, occ);
  check_launch("k_lr_fwd_g_lds");
}

}  // namespace ss
