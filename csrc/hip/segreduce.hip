// segreduce.hip — atomic-free duplicate-key gradient reduction (K7) for
// scalar-per-key models (sparse LR).
//
// The reference merges duplicate-key gradients on the worker
// (GradPramProcMethod::merge_grad, /root/reference/src/core/parameter/
// global_param_cache.h:14-15; PushAccessMethod::merge_push_value,
// sparse_access_method.h:39-40).  The first version here scattered one float
// atomicAdd per key occurrence: 2.56M atomics = 164 us/step, because on
// MI355X every device-scope atomic executes at the memory side (~18 G/s).
//
// Replacement = one radix-partition pass + an LDS accumulation:
//   route stream (off the critical path, right after dedup):
//     count      per chunk of 8192 occurrences, histogram of bin(cu) in LDS,
//                where cu = compact unique id and bin = cu >> 13
//     scan       exclusive scan over [bin][chunk] (one workgroup)
//     positions  every occurrence gets its slot in the bin-ordered pair array
//                (LDS cursor per bin, no global atomics)
//   main stream:
//     the model's forward kernel writes (cu & 8191, grad) at that slot
//     reduce     one workgroup per bin: LDS atomics into 8192 accumulators,
//                then ONE coalesced store per unique key (also zero-fills the
//                keys with no contribution, so dedup need not zero grads)
#include "ss_device.h"
#include "ss_launch.h"

namespace ss {

static constexpr uint32_t kInvS = 0xFFFFFFFFu;
static constexpr int kBinShift = 13;
static constexpr int kBinW = 1 << kBinShift;  // unique ids per bin (LDS floats)
static constexpr int kChunk = 8192;           // occurrences per count/positions block
static constexpr int kMaxBins = 4096;

// compact id <-> layout id: uid = d*ucap + local, cu = prefix[d] + local
struct CuMap {
  const unsigned long long* ucount;
  int nranks;
  long long ucap;
};

__device__ __forceinline__ void load_prefix(const CuMap& m, unsigned long long* pre) {
  if (threadIdx.x == 0) {
    unsigned long long a = 0;
    for (int d = 0; d < m.nranks; ++d) {
      pre[d] = a;
      a += m.ucount[d];
    }
    pre[m.nranks] = a;
  }
  __syncthreads();
}
__device__ __forceinline__ unsigned long long cu_of(const CuMap& m, const unsigned long long* pre,
                                                    uint32_t uid) {
  const unsigned long long d = uid / (unsigned long long)m.ucap;
  return pre[d] + (uid - d * (unsigned long long)m.ucap);
}

__global__ __launch_bounds__(256) void k_sr_count(const uint32_t* __restrict__ inv, long long n,
                                                  CuMap m, uint32_t* __restrict__ hist, int nbins,
                                                  int nchunks) {
  __shared__ unsigned long long pre[kMaxSeg + 1];
  __shared__ unsigned int h[kMaxBins];
  for (int b = threadIdx.x; b < nbins; b += 256) h[b] = 0;
  load_prefix(m, pre);
  const long long a = (long long)blockIdx.x * kChunk;
  const long long e = a + kChunk < n ? a + kChunk : n;
  for (long long j = a + threadIdx.x; j < e; j += 256) {
    const uint32_t u = inv[j];
    if (u != kInvS) atomicAdd(&h[cu_of(m, pre, u) >> kBinShift], 1u);
  }
  __syncthreads();
  for (int b = threadIdx.x; b < nbins; b += 256) hist[(long long)b * nchunks + blockIdx.x] = h[b];
}

// In-place exclusive scan of len values (single workgroup); total -> data[len].
__global__ __launch_bounds__(1024) void k_scan_flat(uint32_t* __restrict__ data, long long len) {
  __shared__ unsigned int wsum[16];
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const long long per = (len + 1023) / 1024;
  const long long a = t * per, e = a + per < len ? a + per : len;
  unsigned int s = 0;
  for (long long i = a; i < e; ++i) s += data[i];
  unsigned int x = s;
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
  unsigned int run = (w ? wsum[w - 1] : 0u) + x - s;
  for (long long i = a; i < e; ++i) {
    const unsigned int v = data[i];
    data[i] = run;
    run += v;
  }
  if (t == 1023) data[len] = wsum[15];
}

__global__ __launch_bounds__(256) void k_sr_positions(const uint32_t* __restrict__ inv, long long n,
                                                      CuMap m, const uint32_t* __restrict__ hist,
                                                      int nbins, int nchunks,
                                                      uint32_t* __restrict__ pos) {
  __shared__ unsigned long long pre[kMaxSeg + 1];
  __shared__ unsigned int cur[kMaxBins];
  for (int b = threadIdx.x; b < nbins; b += 256)
    cur[b] = hist[(long long)b * nchunks + blockIdx.x];
  load_prefix(m, pre);
  const long long a = (long long)blockIdx.x * kChunk;
  const long long e = a + kChunk < n ? a + kChunk : n;
  for (long long j = a + threadIdx.x; j < e; j += 256) {
    const uint32_t u = inv[j];
    pos[j] = u == kInvS ? kInvS : atomicAdd(&cur[cu_of(m, pre, u) >> kBinShift], 1u);
  }
}

// One workgroup per bin. pairs[i] = (cu & (kBinW-1), grad bits).
__global__ __launch_bounds__(1024) void k_sr_reduce(const uint2* __restrict__ pairs,
                                                    const uint32_t* __restrict__ hist, int nbins,
                                                    int nchunks, CuMap m,
                                                    float* __restrict__ ugrad) {
  __shared__ unsigned long long pre[kMaxSeg + 1];
  __shared__ float acc[kBinW];
  const int bin = blockIdx.x;
  for (int c = threadIdx.x; c < kBinW; c += blockDim.x) acc[c] = 0.f;
  load_prefix(m, pre);
  const uint32_t a = hist[(long long)bin * nchunks];
  const uint32_t e = hist[(long long)(bin + 1) * nchunks];  // bin+1 == nbins -> total slot
  for (uint32_t p = a + threadIdx.x; p < e; p += blockDim.x) {
    const uint2 pr = pairs[p];
    atomicAdd(&acc[pr.x], __uint_as_float(pr.y));
  }
  __syncthreads();
  const unsigned long long total = pre[m.nranks];
  for (int c = threadIdx.x; c < kBinW; c += blockDim.x) {
    const unsigned long long cu = ((unsigned long long)bin << kBinShift) + c;
    if (cu >= total) break;
    int d = 0;
    while (d + 1 < m.nranks && cu >= pre[d + 1]) ++d;
    ugrad[(unsigned long long)d * m.ucap + (cu - pre[d])] = acc[c];
  }
}

// ---- LR forward writing bin-ordered (cu_lo, grad) pairs instead of atomics
__global__ __launch_bounds__(256) void k_lr_fwd_pairs(const uint32_t* __restrict__ inv,
                                                      const float* __restrict__ xval,
                                                      const float* __restrict__ labels, int B, int F,
                                                      const float* __restrict__ uvals, CuMap m,
                                                      const uint32_t* __restrict__ pos,
                                                      uint2* __restrict__ pairs,
                                                      float* __restrict__ loss_sum,
                                                      float* __restrict__ pred) {
  __shared__ unsigned long long pre[kMaxSeg + 1];
  __shared__ float sdot[256];
  __shared__ float sg[256];
  __shared__ float sloss[4];
  const int spb = F >= 256 ? 1 : 256 / F;
  const int t = threadIdx.x, ls = t / F;
  const long long s0 = (long long)blockIdx.x * spb;
  if (t < spb) sdot[t] = 0.f;
  load_prefix(m, pre);
  const bool active = ls < spb && s0 + ls < B;
  const long long j = s0 * F + t;
  uint32_t u = kInvS;
  float x = 0.f;
  if (active) {
    u = inv[j];
    x = xval ? xval[j] : 1.f;
    if (u != kInvS) atomicAdd(&sdot[ls], uvals[u] * x);
  }
  __syncthreads();
  float l = 0.f;
  if (t < spb && s0 + t < B) {
    const float z = sdot[t];
    const float y = labels[s0 + t];
    const float p = 1.f / (1.f + __expf(-z));
    sg[t] = p - y;
    if (pred) pred[s0 + t] = p;
    l = fmaxf(z, 0.f) + __logf(1.f + __expf(-fabsf(z))) - y * z;
  }
  for (int o = 32; o > 0; o >>= 1) l += __shfl_down(l, o, 64);
  if ((t & 63) == 0) sloss[t >> 6] = l;
  __syncthreads();
  if (t == 0 && loss_sum) ctr_addf(loss_sum, sloss[0] + sloss[1] + sloss[2] + sloss[3]);
  if (active && u != kInvS) {
    const unsigned long long cu = cu_of(m, pre, u);
    pairs[pos[j]] = make_uint2((uint32_t)(cu & (kBinW - 1)), __float_as_uint(sg[ls] * x));
  }
}

// -------------------------------------------------------------- launchers
int sr_nbins(long long max_unique) { return (int)((max_unique + kBinW - 1) >> kBinShift); }
int sr_nchunks(long long n) { return (int)((n + kChunk - 1) / kChunk); }

void launch_sr_plan(const uint32_t* inv, long long n, const unsigned long long* ucount,
                    int nranks, long long ucap, uint32_t* hist, int nbins, uint32_t* pos,
                    hipStream_t st) {
  if (n <= 0) return;
  if (nbins > kMaxBins || nbins < 1) throw_error("segreduce: too many unique keys per call");
  const int nch = sr_nchunks(n);
  CuMap m{ucount, nranks, ucap};
  hipLaunchKernelGGL(k_sr_count, dim3(nch), dim3(256), 0, st, inv, n, m, hist, nbins, nch);
  check_launch("k_sr_count");
  hipLaunchKernelGGL(k_scan_flat, dim3(1), dim3(1024), 0, st, hist, (long long)nbins * nch);
  check_launch("k_scan_flat");
  hipLaunchKernelGGL(k_sr_positions, dim3(nch), dim3(256), 0, st, inv, n, m, hist, nbins, nch,
                     pos);
  check_launch("k_sr_positions");
}

void launch_sr_reduce(const void* pairs, const uint32_t* hist, int nbins, long long n,
                      const unsigned long long* ucount, int nranks, long long ucap, float* ugrad,
                      hipStream_t st) {
  if (n <= 0) return;
  CuMap m{ucount, nranks, ucap};
  hipLaunchKernelGGL(k_sr_reduce, dim3(nbins), dim3(1024), 0, st,
                     reinterpret_cast<const uint2*>(pairs), hist, nbins, sr_nchunks(n), m, ugrad);
  check_launch("k_sr_reduce");
}

void launch_lr_fwd_pairs(const uint32_t* inv, const float* xval, const float* labels, int B, int F,
                         const float* uvals, const unsigned long long* ucount, int nranks,
                         long long ucap, const uint32_t* pos, void* pairs, float* loss_sum,
                         float* pred, hipStream_t st) {
  if (B <= 0) return;
  if (F < 1 || F > 256) throw_error("lr_fwd_pairs: F must be in [1,256]");
  const int spb = F >= 256 ? 1 : 256 / F;
  CuMap m{ucount, nranks, ucap};
  hipLaunchKernelGGL(k_lr_fwd_pairs, dim3((B + spb - 1) / spb), dim3(256), 0, st, inv, xval, labels,
                     B, F, uvals, m, pos, reinterpret_cast<uint2*>(pairs), loss_sum, pred);
  check_launch("k_lr_fwd_pairs");
}

}  // namespace ss
