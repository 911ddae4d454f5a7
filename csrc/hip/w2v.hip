// w2v.hip — word2vec skip-gram with negative sampling on the parameter server.
//
// The reference names a word2vec app as its default binary but does not ship
// it (/root/reference/src/tools/copy_exec.sh:4-9, distribute.sh:9); its test
// corpus generator is src/tools/gen-word2vec-data.py and its dense helper is
// utils/vec1.h (Vec::dot, randInit (rand/RAND_MAX-0.5)/size).  This is that
// workload designed for CDNA4:
//
//   * keys: center words in the input namespace (syn0 = word id), context
//     and negative words in the output namespace (syn1neg = id | 1<<40,
//     zero-initialised through InitParams.zero_bit);
//   * one 256-thread workgroup = a tile of T=64 centers, each with C context
//     words, plus S=64 negatives SHARED by the tile ("shared negative
//     sampling"): the negative part becomes three small GEMMs —
//         S  = V·Nᵀ   (64×64, K=D)      scores
//         gV = G·N    (64×D,  K=64)     center grads
//         gN = Gᵀ·V   (64×D,  K=64)     negative grads
//     run on the f32-input MFMA (v_mfma_f32_32x32x2_f32, exact fp32) out of
//     LDS (rows padded by one float: conflict-free column reads);
//   * positive (center, context) pairs are row dot products (wave shuffle
//     reduce), context-row gradients go out as coalesced row atomics;
//   * all gradient rows leave the kernel as float atomics shaped as whole
//     128-B row segments (the full-rate atomic shape on MI355X).
#include "ss_device.h"
#include "ss_launch.h"
#include "scan.h"
#include "ss/w2v_window.h"

#include <algorithm>
#include <cstdlib>
#include <string>

namespace ss {

static constexpr uint32_t kInv = 0xFFFFFFFFu;
static constexpr int kT = 64;  // centers per tile
static constexpr int kS = 64;  // shared negatives per tile
static constexpr int kMaxC = 16;  // contexts per center held in registers (window <= 8)
// 8 waves per workgroup: the LDS tiles (~116 KB at D = 128) allow one
// workgroup per CU, and the positive-pair loop is a per-wave latency chain
// (one context-row round trip per center), so 8 waves halve it per wave and
// double the loads in flight per CU (4 waves: 223 us per 16K-center step)
static constexpr int kNW = 8;
static constexpr int kWG = 64 * kNW;
typedef float f32x16 __attribute__((ext_vector_type(16)));

__device__ __forceinline__ float softplus(float x) {
  return fmaxf(x, 0.f) + __logf(1.f + __expf(-fabsf(x)));
}
__device__ __forceinline__ float sigm(float x) { return 1.f / (1.f + __expf(-x)); }

// 32x32 C/D map of v_mfma_f32_32x32x* (cdna_hip_programming.md §3):
// col = lane&31, row = (r&3) + 8*(r>>2) + 4*(lane>>5)
__device__ __forceinline__ int mrow(int r, int lane) { return (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5); }

template <int D>
__global__ __launch_bounds__(kWG) void k_w2v_sgns(const uint32_t* __restrict__ inv_c,
                                                  const uint32_t* __restrict__ inv_x,
                                                  const uint32_t* __restrict__ inv_n, int B, int C,
                                                  float neg_scale, const float* __restrict__ uvals,
                                                  float* __restrict__ ugrad,
                                                  float* __restrict__ loss_sum) {
  constexpr int P = D + 1;  // padded LDS row
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* Vs = smem;              // [T][P] center rows
  float* Ns = Vs + kT * P;       // [S][P] negative rows
  float* Gv = Ns + kS * P;       // [T][P] positive-part center grads
  float* Gs = Gv + kT * P;       // [T][S+1] negative score grads
  float* red = Gs + kT * (kS + 1);  // [kNW] loss partials

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const long long t0 = (long long)blockIdx.x * kT;
  __shared__ uint32_t rc[kT], rn[kS];
  if (tid < kT) rc[tid] = (t0 + tid < B) ? inv_c[t0 + tid] : kInv;
  else if (tid < kT + kS) rn[tid - kT] = inv_n[(long long)blockIdx.x * kS + (tid - kT)];
  __syncthreads();
  // gather center / negative rows into LDS, zero the positive-grad tile
  for (int e = tid; e < kT * D; e += kWG) {
    const int r = e / D, d = e - r * D;
    Vs[r * P + d] = rc[r] == kInv ? 0.f : uvals[(long long)rc[r] * D + d];
    Ns[r * P + d] = rn[r] == kInv ? 0.f : uvals[(long long)rn[r] * D + d];
    Gv[r * P + d] = 0.f;
  }
  __syncthreads();

  float loss = 0.f;
  // ---- negative scores S = V·Nᵀ: wave w < 4 owns quadrant (w>>1, w&1)
  if (w < 4) {
    const int i0 = (w >> 1) * 32, j0 = (w & 1) * 32;
    f32x16 acc = {};
    const int ar = i0 + (lane & 31), kk = lane >> 5;
#pragma unroll 8
    for (int k0 = 0; k0 < D; k0 += 2)
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(Vs[ar * P + k0 + kk], Ns[(j0 + (lane & 31)) * P + k0 + kk],
                                                 acc, 0, 0, 0);
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int row = i0 + mrow(r, lane), col = j0 + (lane & 31);
      const bool ok = rc[row] != kInv && rn[col] != kInv;
      const float s = acc[r];
      Gs[row * (kS + 1) + col] = ok ? neg_scale * sigm(s) : 0.f;  // d/ds softplus(s)
      if (ok) loss += neg_scale * softplus(s);
    }
  }
  // ---- positive pairs: wave w owns centers [kT/kNW * w, kT/kNW * (w+1)).  All C context
  // rows of a center are loaded before any is used (one memory round trip
  // per center instead of one per pair: the first version's per-pair loads
  // made this loop the kernel's latency chain, 160 dependent loads per wave).
  {
    constexpr int R = (D + 63) / 64;  // row floats per lane
    constexpr int TW = kT / kNW;
    for (int t = w * TW; t < w * TW + TW; ++t) {
      if (rc[t] == kInv) continue;  // wave-uniform
      const uint32_t xid = lane < C ? inv_x[(t0 + t) * (long long)C + lane] : kInv;
      float u[kMaxC][R];
#pragma unroll
      for (int j = 0; j < kMaxC; ++j) {
        const uint32_t x = __shfl(xid, j, 64);
#pragma unroll
        for (int r = 0; r < R; ++r) {
          const int d = lane + 64 * r;
          u[j][r] = (j < C && x != kInv && d < D) ? uvals[(long long)x * D + d] : 0.f;
        }
      }
      float v[R], gv[R];
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const int d = lane + 64 * r;
        v[r] = d < D ? Vs[t * P + d] : 0.f;
        gv[r] = 0.f;
      }
#pragma unroll
      for (int j = 0; j < kMaxC; ++j) {
        const uint32_t x = __shfl(xid, j, 64);
        if (j >= C || x == kInv) continue;  // wave-uniform
        float part = 0.f;
#pragma unroll
        for (int r = 0; r < R; ++r) part += v[r] * u[j][r];
        for (int o = 32; o > 0; o >>= 1) part += __shfl_xor(part, o, 64);
        const float g = sigm(part) - 1.f;  // d/ds softplus(-s)
        if (lane == 0) loss += softplus(-part);
        float* gu = ugrad + (long long)x * D;
#pragma unroll
        for (int r = 0; r < R; ++r) {
          const int d = lane + 64 * r;
          if (d < D) {
            atomicAdd(gu + d, g * v[r]);
            gv[r] += g * u[j][r];
          }
        }
      }
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const int d = lane + 64 * r;
        if (d < D) Gv[t * P + d] += gv[r];
      }
    }
  }
  __syncthreads();
  // ---- gV = G·N (+ positive part) and gN = Gᵀ·V: (2 x D/32) tiles each
  constexpr int NT = 2 * (D / 32);
  for (int tt = w; tt < 2 * NT; tt += kNW) {
    const bool center = tt < NT;
    const int q = center ? tt : tt - NT;
    const int ti = q / (D / 32), tj = q % (D / 32);
    f32x16 acc = {};
    const int kk = lane >> 5, li = lane & 31;
    if (center) {
#pragma unroll 8
      for (int k0 = 0; k0 < kS; k0 += 2)  // A[i][k]=G[ti*32+i][k], B[k][j]=N[k][tj*32+j]
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(Gs[(ti * 32 + li) * (kS + 1) + k0 + kk],
                                                   Ns[(k0 + kk) * P + tj * 32 + li], acc, 0, 0, 0);
    } else {
#pragma unroll 8
      for (int k0 = 0; k0 < kT; k0 += 2)  // A[i][k]=G[k][ti*32+i], B[k][j]=V[k][tj*32+j]
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(Gs[(k0 + kk) * (kS + 1) + ti * 32 + li],
                                                   Vs[(k0 + kk) * P + tj * 32 + li], acc, 0, 0, 0);
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int row = ti * 32 + mrow(r, lane), col = tj * 32 + li;
      const uint32_t dst = center ? rc[row] : rn[row];
      if (dst == kInv) continue;
      const float v = acc[r] + (center ? Gv[row * P + col] : 0.f);
      atomicAdd(ugrad + (long long)dst * D + col, v);  // lanes 0-31 / 32-63: two 128-B rows
    }
  }
  for (int o = 32; o > 0; o >>= 1) loss += __shfl_down(loss, o, 64);
  if (lane == 0) red[w] = loss;
  __syncthreads();
  if (tid == 0 && loss_sum) {
    float tot = 0.f;
#pragma unroll
    for (int i = 0; i < kNW; ++i) tot += red[i];
    ctr_addf(loss_sum, tot);
  }
}

// ---------------------------------------------------------------------------
// The same tile on the bf16 MFMA (v_mfma_f32_32x32x16_bf16, fp32 accumulate).
// What it buys is occupancy, not MFMA rate: the fp32 tile's LDS (116 KB at
// D = 128) allows one 8-wave workgroup per CU, and the kernel is a memory /
// atomic latency chain (SQ_WAIT_ANY ~80% of wave cycles).  With the center and
// negative rows and the score gradients staged as bf16 (rows padded by 16 B:
// 16-B aligned fragments, rows spread over the banks) the tile needs 77 KB,
// two workgroups per CU.  The positive pairs stay fp32: each wave reads its
// centers' rows from global (L2-hot) next to the context rows.
// Lane map (cdna_hip_programming.md §3): lane l (r = l&31, h = l>>5) holds
// A[r][8h + j] and B[8h + j][r], j = 0..7; C/D as the fp32 form (mrow).
typedef short bf16x8 __attribute__((ext_vector_type(8)));
__device__ __forceinline__ unsigned short f2bf(float f) {
  uint32_t u = __float_as_uint(f);
  u += 0x7FFFu + ((u >> 16) & 1u);  // round to nearest even (finite inputs)
  return (unsigned short)(u >> 16);
}

template <int D>
struct W2vBf16Smem {
  static constexpr int PB = D + 8;    // bf16 row stride of the V / N tiles
  static constexpr int GB = kS + 8;   // bf16 row stride of the score-gradient tile
  static constexpr int P = D + 1;     // fp32 row stride of the positive-grad tile
  static constexpr size_t bytes = sizeof(unsigned short) * ((size_t)(kT + kS) * PB + (size_t)kT * GB) +
                                  sizeof(float) * ((size_t)kT * P + kNW);
};

template <int D>
__global__ __launch_bounds__(kWG, 4) void k_w2v_sgns_bf16(
    const uint32_t* __restrict__ inv_c, const uint32_t* __restrict__ inv_x,
    const uint32_t* __restrict__ inv_n, int B, int C, float neg_scale,
    const float* __restrict__ uvals, float* __restrict__ ugrad, float* __restrict__ loss_sum) {
  using L = W2vBf16Smem<D>;
  constexpr int PB = L::PB, GB = L::GB, P = L::P;
  extern __shared__ __attribute__((aligned(16))) unsigned short smem16[];
  unsigned short* Vb = smem16;            // [T][PB] center rows (bf16)
  unsigned short* Nb = Vb + kT * PB;      // [S][PB] negative rows (bf16)
  unsigned short* Gb = Nb + kS * PB;      // [T][GB] score gradients (bf16)
  float* Gv = reinterpret_cast<float*>(Gb + kT * GB);  // [T][P] positive-part center grads
  float* red = Gv + kT * P;                             // [kNW] loss partials

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  __shared__ uint32_t rc[kT], rn[kS];
  const int ntiles = (B + kT - 1) / kT;
  float loss = 0.f;
  // a grid smaller than the tile count walks tiles (as in k_w2v_win_bf16)
  for (int tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const long long t0 = (long long)tile * kT;
    if (tid < kT) rc[tid] = (t0 + tid < B) ? inv_c[t0 + tid] : kInv;
    else if (tid < kT + kS) rn[tid - kT] = inv_n[(long long)tile * kS + (tid - kT)];
    __syncthreads();
    // rows -> bf16 tiles, 4 coordinates per thread (16-B loads, 8-B LDS stores)
    for (int e = tid; e < kT * D / 4; e += kWG) {
      const int r = e / (D / 4), d = 4 * (e - r * (D / 4));
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f), n = v;
      if (rc[r] != kInv) v = *reinterpret_cast<const float4*>(uvals + (long long)rc[r] * D + d);
      if (rn[r] != kInv) n = *reinterpret_cast<const float4*>(uvals + (long long)rn[r] * D + d);
      const uint2 pv = make_uint2(f2bf(v.x) | ((uint32_t)f2bf(v.y) << 16),
                                  f2bf(v.z) | ((uint32_t)f2bf(v.w) << 16));
      const uint2 pn = make_uint2(f2bf(n.x) | ((uint32_t)f2bf(n.y) << 16),
                                  f2bf(n.z) | ((uint32_t)f2bf(n.w) << 16));
      *reinterpret_cast<uint2*>(Vb + r * PB + d) = pv;
      *reinterpret_cast<uint2*>(Nb + r * PB + d) = pn;
    }
    for (int e = tid; e < kT * P; e += kWG) Gv[e] = 0.f;
    __syncthreads();

    const int r32 = lane & 31, h = lane >> 5;
    // ---- S = V·Nᵀ: wave w < 4 owns quadrant (w>>1, w&1)
    if (w < 4) {
      const int i0 = (w >> 1) * 32, j0 = (w & 1) * 32;
      f32x16 acc = {};
#pragma unroll
      for (int k0 = 0; k0 < D; k0 += 16) {
        const bf16x8 a = *reinterpret_cast<const bf16x8*>(Vb + (i0 + r32) * PB + k0 + 8 * h);
        const bf16x8 b = *reinterpret_cast<const bf16x8*>(Nb + (j0 + r32) * PB + k0 + 8 * h);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc, 0, 0, 0);
      }
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = i0 + mrow(r, lane), col = j0 + r32;
        const bool ok = rc[row] != kInv && rn[col] != kInv;
        const float sc = acc[r];
        Gb[row * GB + col] = f2bf(ok ? neg_scale * sigm(sc) : 0.f);
        if (ok) loss += neg_scale * softplus(sc);
      }
    }
    // ---- positive pairs (fp32): wave w owns centers [kT/kNW * w, +kT/kNW); the
    // center row comes from global with the context rows (one round trip)
    {
      constexpr int R = (D + 63) / 64;
      constexpr int TW = kT / kNW;
      for (int t = w * TW; t < w * TW + TW; ++t) {
        if (rc[t] == kInv) continue;  // wave-uniform
        const uint32_t xid = lane < C ? inv_x[(t0 + t) * (long long)C + lane] : kInv;
        float u[kMaxC][R], v[R], gv[R];
#pragma unroll
        for (int r = 0; r < R; ++r) {
          const int d = lane + 64 * r;
          v[r] = d < D ? uvals[(long long)rc[t] * D + d] : 0.f;
          gv[r] = 0.f;
        }
#pragma unroll
        for (int j = 0; j < kMaxC; ++j) {
          const uint32_t x = __shfl(xid, j, 64);
#pragma unroll
          for (int r = 0; r < R; ++r) {
            const int d = lane + 64 * r;
            u[j][r] = (j < C && x != kInv && d < D) ? uvals[(long long)x * D + d] : 0.f;
          }
        }
#pragma unroll
        for (int j = 0; j < kMaxC; ++j) {
          const uint32_t x = __shfl(xid, j, 64);
          if (j >= C || x == kInv) continue;  // wave-uniform
          float part = 0.f;
#pragma unroll
          for (int r = 0; r < R; ++r) part += v[r] * u[j][r];
          for (int o = 32; o > 0; o >>= 1) part += __shfl_xor(part, o, 64);
          const float g = sigm(part) - 1.f;
          if (lane == 0) loss += softplus(-part);
          float* gu = ugrad + (long long)x * D;
#pragma unroll
          for (int r = 0; r < R; ++r) {
            const int d = lane + 64 * r;
            if (d < D) {
              atomicAdd(gu + d, g * v[r]);
              gv[r] += g * u[j][r];
            }
          }
        }
#pragma unroll
        for (int r = 0; r < R; ++r) {
          const int d = lane + 64 * r;
          if (d < D) Gv[t * P + d] += gv[r];
        }
      }
    }
    __syncthreads();
    // ---- gV = G·N (+ positive part) and gN = Gᵀ·V, K = 64 in 4 steps of 16.
    // Row-major fragments (G's rows for gV's A) are one 16-B LDS read; the
    // k-strided ones (N for gV's B, G and V for gN) are gathered per element.
    constexpr int NT = 2 * (D / 32);
    for (int tt = w; tt < 2 * NT; tt += kNW) {
      const bool center = tt < NT;
      const int q = center ? tt : tt - NT;
      const int ti = q / (D / 32), tj = q % (D / 32);
      f32x16 acc = {};
#pragma unroll
      for (int k0 = 0; k0 < 64; k0 += 16) {
        bf16x8 a, b;
        const int kb = k0 + 8 * h;
        if (center) {  // A[i][k] = G[ti*32+i][k], B[k][j] = N[k][tj*32+j]
          a = *reinterpret_cast<const bf16x8*>(Gb + (ti * 32 + r32) * GB + kb);
#pragma unroll
          for (int j = 0; j < 8; ++j) b[j] = (short)Nb[(kb + j) * PB + tj * 32 + r32];
        } else {       // A[i][k] = G[k][ti*32+i], B[k][j] = V[k][tj*32+j]
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            a[j] = (short)Gb[(kb + j) * GB + ti * 32 + r32];
            b[j] = (short)Vb[(kb + j) * PB + tj * 32 + r32];
          }
        }
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc, 0, 0, 0);
      }
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = ti * 32 + mrow(r, lane), col = tj * 32 + r32;
        const uint32_t dst = center ? rc[row] : rn[row];
        if (dst == kInv) continue;
        const float v = acc[r] + (center ? Gv[row * P + col] : 0.f);
        atomicAdd(ugrad + (long long)dst * D + col, v);
      }
    }
    __syncthreads();  // the next tile overwrites the LDS tiles
  }
  for (int o = 32; o > 0; o >>= 1) loss += __shfl_down(loss, o, 64);
  if (lane == 0) red[w] = loss;
  __syncthreads();
  if (tid == 0 && loss_sum) {
    float tot = 0.f;
#pragma unroll
    for (int i = 0; i < kNW; ++i) tot += red[i];
    ctr_addf(loss_sum, tot);
  }
}

// ---------------------------------------------------------------------------

// log-uniform ("Zipf-like") word id in [0, V) from a 64-bit hash
__device__ __forceinline__ uint64_t w2v_zipf(uint64_t r, long long V, double logV) {
  const double u = (double)(r >> 11) * (1.0 / 9007199254740992.0);
  long long v = (long long)exp(u * logV) - 1;
  return (uint64_t)(v < 0 ? 0 : (v >= V ? V - 1 : v));
}

// negative samples: word2vec's noise distribution, the unigram distribution
// to the 3/4 — for the log-uniform corpus above P(k) ~ (k + 1)^-3/4, drawn by
// inverting its continuous CDF ((x^(1/4) - 1) / ((V + 1)^(1/4) - 1) on
// [1, V + 1)).  Flatter head than the corpus: the most frequent word is ~0.6%
// of the draws at V = 1M instead of ~5%
__device__ __forceinline__ uint64_t w2v_noise(uint64_t r, long long V) {
  const double u = (double)(r >> 11) * (1.0 / 9007199254740992.0);
  const double q = sqrt(sqrt((double)V + 1.0));
  const double x = 1.0 + u * (q - 1.0);
  long long v = (long long)((x * x) * (x * x)) - 1;
  return (uint64_t)(v < 0 ? 0 : (v >= V ? V - 1 : v));
}

// Synthetic skip-gram batches. Centers are Zipf-like (log-uniform) over V
// words; a context sits within +-W ids of its center (words with nearby ids
// co-occur: learnable structure) except with probability `noise`; negatives
// are drawn from the same unigram-like distribution.  keys = [centers B]
// [contexts B*C][negatives ntile*S], contexts/negatives in namespace 1<<40.
__global__ __launch_bounds__(256) void k_w2v_gen(uint64_t seed, long long base, int B, int C, int W,
                                                 long long nneg, long long V, double logV,
                                                 float noise, uint64_t* __restrict__ keys,
                                                 const long long* __restrict__ step_dev,
                                                 long long step_mul, long long step_add) {
  if (step_dev) base = *step_dev * step_mul + step_add;  // hipGraph replays (models.hip k_gen_ctr)
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const long long n = (long long)B + (long long)B * C + nneg;
  if (i >= n) return;
  auto zipf = [&](uint64_t r) -> uint64_t { return w2v_zipf(r, V, logV); };
  const uint64_t kOut = 1ull << 40;
  if (i < B) {
    keys[i] = zipf(splitmix64(seed ^ ((uint64_t)(base + i) * 0xA24BAED4963EE407ull)));
  } else if (i < B + (long long)B * C) {
    const long long p = i - B, b = p / C;
    const uint64_t c = zipf(splitmix64(seed ^ ((uint64_t)(base + b) * 0xA24BAED4963EE407ull)));
    const uint64_t r = splitmix64(seed ^ 0xC0FFEEull ^ ((uint64_t)(base * C + p) * 0x9E3779B97F4A7C15ull));
    uint64_t x;
    if (u01(r) < noise) {
      x = zipf(splitmix64(r));
    } else {
      const long long off = 1 + (long long)(splitmix64(r ^ 1) % (uint64_t)W);
      const long long s = (r >> 7) & 1 ? off : -off;
      x = (uint64_t)((((long long)c + s) % V + V) % V);
    }
    keys[i] = x | kOut;
  } else {
    const long long q = i - B - (long long)B * C;
    // (base, q) hashed apart: a step's negatives never repeat another's,
    // whatever their count per step
    keys[i] = w2v_noise(splitmix64(seed ^ 0xBADC0DEull ^ splitmix64((uint64_t)base) ^
                                   ((uint64_t)q * 0xD1B54A32D192ED03ull)), V) | kOut;
  }
}


// ---------------------------------------------------------------------------
// Windowed skip-gram tile: the batch layout of ss/w2v_window.h (a run of
// B + 2W consecutive stream positions; centers are the middle B, contexts
// are the neighbouring positions of the run).  One 512-thread workgroup per
// tile of T = 64 consecutive centers; the tile's window rows are the 64 + 2W
// run positions around them (padded to kWU = 96), so the positive pairs are a
// band of the 64 x 96 score matrix and the whole tile is five small GEMMs on
// the bf16 MFMA (fp32 accumulate):
//     S+ = V·Uᵀ (64 x 96)   S- = V·Nᵀ (64 x 64)            scores
//     gV = G+·U + G-·N      gU = G+ᵀ·V (96 x D)   gN = G-ᵀ·V  gradients
// G+ is σ(s) - 1 on the band's valid pairs (same sentence, |Δ| <= the
// center's reduced window, both positions unmasked) and 0 elsewhere; G- is
// σ(s) weighted n_t·K/S for a center with n_t pairs (each pair's K negatives
// drawn from the tile's S shared ones).  A context row now leaves the tile
// once (96 row atomics per tile) instead of once per pair (640 at W = 5 in
// the pairs layout), and the batch carries B + 2W context keys instead of
// 2W·B: the dedup, pull and apply of a step shrink with it.
static constexpr int kWU = 96;  // window rows per tile: 64 + 2W (W <= 15), 3 x 32

template <int D>
struct W2vWinSmem {
  static constexpr int PB = D + 8;     // bf16 row stride of the V / U / N tiles
  static constexpr int GPB = kWU + 8;  // bf16 row stride of G+
  static constexpr int GB = kS + 8;    // bf16 row stride of G-
  static constexpr size_t bytes =
      sizeof(unsigned short) * ((size_t)(kT + kWU + kS) * PB + (size_t)kT * GPB + (size_t)kT * GB);
};

template <int D>
__global__ __launch_bounds__(kWG, 4) void k_w2v_win_bf16(
    const uint32_t* __restrict__ inv_c, const uint32_t* __restrict__ inv_w,
    const uint32_t* __restrict__ inv_n, const int32_t* __restrict__ meta, int B, int W,
    float neg_per_pair, const float* __restrict__ uvals, float* __restrict__ ugrad,
    float* __restrict__ loss_sum, float* __restrict__ pair_sum,
    float* __restrict__ ograd, float* __restrict__ otail) {
  using L = W2vWinSmem<D>;
  constexpr int PB = L::PB, GPB = L::GPB, GB = L::GB, TJ = D / 32;
  extern __shared__ __attribute__((aligned(16))) unsigned short smem16[];
  unsigned short* Vb = smem16;         // [T][PB]   center rows (syn0), bf16
  unsigned short* Ub = Vb + kT * PB;   // [kWU][PB] window rows (syn1neg): rows 0.. = run positions t0..
  unsigned short* Nb = Ub + kWU * PB;  // [S][PB]   shared negatives (syn1neg)
  unsigned short* Gp = Nb + kS * PB;   // [T][GPB]  G+
  unsigned short* Gn = Gp + kT * GPB;  // [T][GB]   G-
  __shared__ uint32_t rc[kT], rw[kWU], rn[kS];
  __shared__ int32_t mw[kWU];
  __shared__ int uany[kWU];
  __shared__ float cwt[kT];  // n_t * K / S
  constexpr int NW = kNW;
  __shared__ float red[NW];

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const long long R = (long long)B + 2 * W;
  const int ntiles = (B + kT - 1) / kT;
  float loss = 0.f, npairs = 0.f;
  // a grid smaller than the tile count walks tiles (SS_W2V_WIN_GRID: leaves
  // CUs to the route stream's kernels)
  for (int tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const long long t0 = (long long)tile * kT;  // first center; its run position is t0 + W
    if (tid < kWU) {  // window row l = run position t0 + l
      const long long q = t0 + tid;
      const bool in = tid < kT + 2 * W && q < R;
      const int32_t m = in ? meta[q] : -1;
      mw[tid] = m;
      rw[tid] = m >= 0 ? inv_w[q] : kInv;
      uany[tid] = 0;
    } else if (tid < kWU + kS) {
      rn[tid - kWU] = inv_n[(long long)tile * kS + (tid - kWU)];
    }
    __syncthreads();
    if (tid < kT) {  // center t sits at window row t + W
      const int32_t mc = mw[tid + W];
      const bool ok = t0 + tid < B && mc >= 0;
      int n = 0;
      if (ok)
        for (int dq = -W; dq <= W; ++dq) n += w2v_pair_ok(mc, mw[tid + W + dq], dq) ? 1 : 0;
      rc[tid] = ok && n > 0 ? inv_c[t0 + tid] : kInv;  // a center without pairs does not train
      cwt[tid] = (float)n * neg_per_pair;
      npairs += (float)n;
    }
    __syncthreads();
    // rows -> bf16 tiles (V, U, N are consecutive rows of stride PB).  Every
    // load of the thread is issued before the first LDS store (one memory
    // round trip per tile instead of one per loop trip: the loop form
    // serialised 14 dependent gathers per thread at D = 128).  A center row
    // without pairs (rc = kInv) stays zero: its G+ and G- rows are zero.
    {
      constexpr int NE = (kT + kWU + kS) * (D / 4), PER = (NE + (64 * NW) - 1) / (64 * NW);
      float4 v[PER];
#pragma unroll
      for (int i = 0; i < PER; ++i) {
        const int e = tid + i * (64 * NW), r = e / (D / 4), d = 4 * (e - r * (D / 4));
        const uint32_t id = e >= NE ? kInv : r < kT ? rc[r] : r < kT + kWU ? rw[r - kT] : rn[r - kT - kWU];
        v[i] = id != kInv ? *reinterpret_cast<const float4*>(uvals + (long long)id * D + d)
                          : make_float4(0.f, 0.f, 0.f, 0.f);
      }
#pragma unroll
      for (int i = 0; i < PER; ++i) {
        const int e = tid + i * (64 * NW), r = e / (D / 4), d = 4 * (e - r * (D / 4));
        if (e < NE)
          *reinterpret_cast<uint2*>(smem16 + r * PB + d) =
              make_uint2(f2bf(v[i].x) | ((uint32_t)f2bf(v[i].y) << 16),
                         f2bf(v[i].z) | ((uint32_t)f2bf(v[i].w) << 16));
      }
    }
    __syncthreads();

    const int r32 = lane & 31, h = lane >> 5;
    // ---- scores: 6 tiles of S+ (2 x 3) and 4 of S- (2 x 2)
    for (int k = w; k < 10; k += NW) {
      const bool pos = k < 6;
      const int ti = pos ? k / 3 : (k - 6) >> 1, tj = pos ? k % 3 : (k - 6) & 1;
      const unsigned short* Bm = pos ? Ub : Nb;
      f32x16 acc = {};
#pragma unroll
      for (int k0 = 0; k0 < D; k0 += 16) {
        const bf16x8 a = *reinterpret_cast<const bf16x8*>(Vb + (ti * 32 + r32) * PB + k0 + 8 * h);
        const bf16x8 b = *reinterpret_cast<const bf16x8*>(Bm + (tj * 32 + r32) * PB + k0 + 8 * h);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc, 0, 0, 0);
      }
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = ti * 32 + mrow(r, lane), col = tj * 32 + r32;
        const float sc = acc[r];
        if (pos) {
          const bool ok = rc[row] != kInv && rw[col] != kInv &&
                          w2v_pair_ok(mw[row + W], mw[col], col - (row + W));
          Gp[row * GPB + col] = f2bf(ok ? sigm(sc) - 1.f : 0.f);  // d/ds softplus(-s)
          if (ok) {
            loss += softplus(-sc);
            uany[col] = 1;
          }
        } else {
          const bool ok = rc[row] != kInv && rn[col] != kInv;
          const float cw = cwt[row];
          Gn[row * GB + col] = f2bf(ok ? cw * sigm(sc) : 0.f);  // d/ds softplus(s), weighted
          if (ok) loss += cw * softplus(sc);
        }
      }
    }
    __syncthreads();
    // ---- gradients: gV (2 x TJ tiles), gU (3 x TJ), gN (2 x TJ)
    for (int tt = w; tt < 7 * TJ; tt += NW) {
      const int kind = tt < 2 * TJ ? 0 : (tt < 5 * TJ ? 1 : 2);
      const int q = tt - (kind == 0 ? 0 : (kind == 1 ? 2 * TJ : 5 * TJ));
      const int ti = q / TJ, tj = q % TJ;
      f32x16 acc = {};
      if (kind == 0) {  // gV = G+·U (K = window rows) + G-·N (K = negatives)
#pragma unroll
        for (int k0 = 0; k0 < kWU; k0 += 16) {
          const int kb = k0 + 8 * h;
          const bf16x8 a = *reinterpret_cast<const bf16x8*>(Gp + (ti * 32 + r32) * GPB + kb);
          bf16x8 b;
#pragma unroll
          for (int j = 0; j < 8; ++j) b[j] = (short)Ub[(kb + j) * PB + tj * 32 + r32];
          acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc, 0, 0, 0);
        }
#pragma unroll
        for (int k0 = 0; k0 < kS; k0 += 16) {
          const int kb = k0 + 8 * h;
          const bf16x8 a = *reinterpret_cast<const bf16x8*>(Gn + (ti * 32 + r32) * GB + kb);
          bf16x8 b;
#pragma unroll
          for (int j = 0; j < 8; ++j) b[j] = (short)Nb[(kb + j) * PB + tj * 32 + r32];
          acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc, 0, 0, 0);
        }
      } else {  // gU = G+ᵀ·V, gN = G-ᵀ·V (K = centers)
        const unsigned short* G = kind == 1 ? Gp : Gn;
        const int GS = kind == 1 ? GPB : GB;
#pragma unroll
        for (int k0 = 0; k0 < kT; k0 += 16) {
          const int kb = k0 + 8 * h;
          bf16x8 a, b;
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            a[j] = (short)G[(kb + j) * GS + ti * 32 + r32];
            b[j] = (short)Vb[(kb + j) * PB + tj * 32 + r32];
          }
          acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc, 0, 0, 0);
        }
      }
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = ti * 32 + mrow(r, lane), col = tj * 32 + r32;
        if (ograd) {
          // occurrence rows, plain stores (k_w2v_oreduce sums them per key).
          // Every row the tile covers is written (a row without pairs has a
          // zero gradient).  Window row l >= 64 of a tile other than the
          // last is also row l - 64 of the next tile: it goes to the tail
          // buffer instead, so no occurrence row has two writers.
          long long orow = -1;
          if (kind == 0) {
            if (t0 + row < B) orow = t0 + row;
          } else if (kind == 1) {
            const long long q = t0 + row;
            if (row < kT + 2 * W && q < R) {
              if (row < kT || tile == ntiles - 1)
                orow = B + q;
              else
                otail[((long long)tile * 2 * W + (row - kT)) * D + col] = acc[r];
            }
          } else {
            orow = B + R + (long long)tile * kS + row;
          }
          if (orow >= 0) ograd[orow * D + col] = acc[r];
          continue;
        }
        const uint32_t dst = kind == 0 ? rc[row] : (kind == 1 ? (uany[row] ? rw[row] : kInv) : rn[row]);
        if (dst == kInv) continue;  // lanes 0-31 / 32-63: one 128-B row segment each
        atomicAdd(ugrad + (long long)dst * D + col, acc[r]);
      }
    }
    __syncthreads();  // the next tile overwrites the LDS tiles
  }
  for (int o = 32; o > 0; o >>= 1) loss += __shfl_down(loss, o, 64);
  if (lane == 0) red[w] = loss;
  __syncthreads();
  if (tid == 0 && loss_sum) {
    float tot = 0.f;
#pragma unroll
    for (int i = 0; i < NW; ++i) tot += red[i];
    ctr_addf(loss_sum, tot);
  }
  if (w == 0 && pair_sum) {  // centers' pair counts live in wave 0 (tid < kT)
    for (int o = 32; o > 0; o >>= 1) npairs += __shfl_down(npairs, o, 64);
    if (lane == 0) ctr_addf(pair_sum, npairs);  // valid positive pairs
  }
}

// ---- atomic-free gradient merge of the windowed tile (SS_W2V_GRAD=reduce)
//
// Measured: the tile's row atomics (~52K rows of 512 B per 16K-center step,
// two 64-lane float atomics per row) took 71 of its 71 us standalone -> 32 us
// with the same rows as plain stores; the per-CU atomic issue rate, not
// memory, bounds them.  So the tile stores occurrence rows (ograd: one row per
// key position, otail: the 2W window rows a tile shares with the next one)
// and the rows are summed per unique key here.
//
// k_w2v_osort (route stream: depends on the key layout only, so it runs a
// round ahead beside the dedup) groups each dedup bucket's occurrences by
// unique key with a counting sort in LDS and cuts every key's list into items
// of <= kOsCh occurrences, written into the bucket's own occurrence range of
// `items` (a bucket has at most as many items as occurrences: no global scan).
// k_w2v_oreduce (main stream) sums one item per wave, <= 8 rows in flight, and
// stores the key's gradient row — or adds it with row atomics when a Zipf-head
// key has several items (its row was zeroed by the dedup): a head key's
// thousands of occurrences spread over many waves instead of serialising one.
static constexpr int kOsT = 256;
static constexpr int kOsMaxU = 4096;      // unique keys per dedup bucket (bdedup.hip kBdTS)
static constexpr uint32_t kOsCh = 32;     // occurrences per reduce item

__global__ __launch_bounds__(kOsT) void k_w2v_osort(const uint32_t* __restrict__ bstart,
                                                    const uint32_t* __restrict__ unum,
                                                    const uint32_t* __restrict__ ubase,
                                                    const uint32_t* __restrict__ pj,
                                                    const uint32_t* __restrict__ luid,
                                                    uint32_t* __restrict__ ord,
                                                    uint4* __restrict__ items,
                                                    uint8_t* __restrict__ uhot) {
  __shared__ uint32_t cnt[kOsMaxU];
  __shared__ uint32_t ifirst[kOsMaxU];  // a single-occurrence key's item slot
  __shared__ unsigned int wsum[kOsT / 64];
  __shared__ unsigned int tot, toti;
  const int b = blockIdx.x, tid = threadIdx.x;
  const uint32_t p0 = bstart[b], p1 = bstart[b + 1], base = ubase[b];
  const uint32_t nu = min(unum[b], (uint32_t)kOsMaxU);
  for (uint32_t l = tid; l < nu; l += kOsT) cnt[l] = 0u;
  __syncthreads();
  // loops with wave-uniform bounds: the hottest key of each wave's 64
  // occurrences (lane-first match) takes one LDS atomic for all its lanes —
  // a Zipf-head key (thousands of occurrences in one bucket: the negatives
  // of a per-pair step) otherwise serialises its bucket's workgroup on one
  // LDS word
  const int lane = tid & 63;
  for (uint32_t q = p0 + (tid & ~63u); q < p1; q += kOsT) {
    const uint32_t p = q + lane;
    const uint32_t l = p < p1 ? luid[p] : kInv;
    const bool ok = l < nu;
    const unsigned long long m = __ballot(ok);
    if (!m) continue;  // wave-uniform
    const int lead = __ffsll((long long)m) - 1;
    const uint32_t lh = __shfl(l, lead, 64);
    const unsigned long long same = __ballot(ok && l == lh);
    if (lane == lead) atomicAdd(&cnt[lh], (uint32_t)__popcll(same));
    else if (ok && l != lh) atomicAdd(&cnt[l], 1u);
  }
  __syncthreads();
  constexpr int PT = kOsMaxU / kOsT;  // counts per thread, consecutive keys
  uint32_t c[PT], sc = 0, si = 0;
#pragma unroll
  for (int k = 0; k < PT; ++k) {
    const uint32_t l = (uint32_t)tid * PT + k;
    c[k] = l < nu ? cnt[l] : 0u;
    sc += c[k];
    si += (c[k] + kOsCh - 1) / kOsCh;
  }
  uint32_t e = block_excl_scan<kOsT / 64>(sc, wsum, &tot);
  uint32_t ei = block_excl_scan<kOsT / 64>(si, wsum, &toti);
#pragma unroll
  for (int k = 0; k < PT; ++k) {
    const uint32_t l = (uint32_t)tid * PT + k;
    if (l < nu) {
      cnt[l] = e;  // placement cursor
      ifirst[l] = (p0 + ei) | (c[k] == 1 ? 0x80000000u : 0u);
      const uint32_t nit = (c[k] + kOsCh - 1) / kOsCh;
      // uhot: the key's row sums over several items (row atomics into ugrad):
      // its optimizer update runs after the reduce (launch_apply `only`)
      if (uhot) uhot[base + l] = nit > 1 ? 1 : 0;
      if (c[k] > 1)  // (a single-occurrence item is written at placement, below)
        for (uint32_t m = 0; m < nit; ++m)
          items[p0 + ei + m] = make_uint4(p0 + e + m * kOsCh, min(kOsCh, c[k] - m * kOsCh),
                                          base + l, nit > 1 ? 1u : 0u);
      ei += nit;
    }
    e += c[k];
  }
  for (uint32_t q = p0 + toti + tid; q < p1; q += kOsT) items[q] = make_uint4(0u, 0u, 0u, 0u);
  __syncthreads();
  for (uint32_t q = p0 + (tid & ~63u); q < p1; q += kOsT) {
    const uint32_t p = q + lane;
    const uint32_t l = p < p1 ? luid[p] : kInv;
    const bool ok = l < nu;
    const unsigned long long m = __ballot(ok);
    if (!m) continue;  // wave-uniform
    const int lead = __ffsll((long long)m) - 1;
    const uint32_t lh = __shfl(l, lead, 64);
    const bool hot = ok && l == lh;
    const unsigned long long same = __ballot(hot);
    uint32_t o = 0;
    if (lane == lead) o = atomicAdd(&cnt[lh], (uint32_t)__popcll(same));
    o = __shfl(o, lead, 64) + (uint32_t)__popcll(same & ((1ull << lane) - 1ull));
    if (ok && !hot) o = atomicAdd(&cnt[l], 1u);
    if (!ok) continue;
    const uint32_t j = pj[p];
    ord[p0 + o] = j;
    // most keys occur once: their item carries the key position itself
    // (flag 2), so the reduce skips the dependent `ord` load
    if (ifirst[l] & 0x80000000u) items[ifirst[l] & 0x7FFFFFFFu] = make_uint4(j, 1u, base + l, 2u);
  }
}

template <int V>
struct OVec;  // V consecutive floats moved as one access
template <>
struct OVec<4> {
  using T = float4;
  __device__ static float get(const T& x, int v) { return v == 0 ? x.x : v == 1 ? x.y : v == 2 ? x.z : x.w; }
};
template <>
struct OVec<2> {
  using T = float2;
  __device__ static float get(const T& x, int v) { return v == 0 ? x.x : x.y; }
};
template <>
struct OVec<1> {
  using T = float;
  __device__ static float get(const T& x, int) { return x; }
};

// `gnc` (per-pair negatives): occurrence j >= `negbase` is the negative row
// gn * v_c, stored by k_w2v_pp as the pair (gn, c) — 8 bytes instead of a
// D-float row — and expanded here from the center row uvals[c] (the step's
// center rows: a few MB, cache-resident).  SC: the per-pair form; the window
// tile's reduce (no scaled rows) keeps its one-phase loop.
template <int D, bool SC>
__global__ __launch_bounds__(256) void k_w2v_oreduce(const uint4* __restrict__ items, long long n,
                                                     const uint32_t* __restrict__ ord,
                                                     const float* __restrict__ ograd,
                                                     const float* __restrict__ otail, int B,
                                                     int W, int ntiles,
                                                     float* __restrict__ ugrad,
                                                     const float2* __restrict__ gnc,
                                                     long long negbase,
                                                     const float* __restrict__ uvals,
                                                     float* __restrict__ lacc,
                                                     float* __restrict__ lacc_out, int lacc_n,
                                                     DevTable tab,
                                                     const long long* __restrict__ slots,
                                                     OptParams op, int early_slot) {
  // the step's loss / pair accumulators (the tile kernel's, ordered before
  // this launch on the stream) move to acc_out and are left zero for the next
  // step's tile: no zero-fill launch per step
  if (lacc)
    for (int i = blockIdx.x * 256 + threadIdx.x; i < lacc_n; i += gridDim.x * 256) {
      lacc_out[i] = lacc[i];
      lacc[i] = 0.f;
    }
  // one item per half-wave: 32 lanes x V floats cover a row (512 B at D =
  // 128 as 16-B loads), two independent item chains per wave
  constexpr int V = D / 32;
  constexpr int QF = 8;  // rows in flight per half-wave
  using VT = typename OVec<V>::T;
  const int lane = threadIdx.x & 63, hl = lane & 31;
  const long long R = (long long)B + 2 * W;
  const long long s = ((long long)blockIdx.x * 4 + (threadIdx.x >> 6)) * 2 + (lane >> 5);
  const uint4 it = s < n ? items[s] : make_uint4(0u, 0u, 0u, 0u);
  if (it.y == 0) return;  // half-wave-uniform (the shuffles below stay inside a half)
  // the tail copy of run position j (row l - 64 of the previous tile), or -1
  auto tail_of = [&](long long j) -> long long {
    if (!otail || j < B || j >= B + R) return -1;
    const long long rq = j - B;
    if (rq >= kT && rq % kT < 2 * W && rq / kT <= ntiles - 1) return (rq / kT - 1) * 2 * W + rq % kT;
    return -1;
  };
  const uint32_t jl = (it.w & 2u) ? it.x : (hl < (int)it.y ? ord[it.x + hl] : 0u);
  // the fused update's slot index is loaded beside the first gathers (one
  // dependent load off the item's chain; the row itself is read after them —
  // holding it through the gathers cost an occupancy step)
  const long long fslot = (early_slot && slots && !(it.w & 1u)) ? slots[it.z] : -1;
  float acc[V];
#pragma unroll
  for (int v = 0; v < V; ++v) acc[v] = 0.f;
  for (uint32_t k0 = 0; k0 < it.y; k0 += QF) {
    VT x[QF], y[QF];
    if constexpr (!SC) {
#pragma unroll
      for (int r = 0; r < QF; ++r) {
        const uint32_t k = k0 + r;
        const long long j = (long long)__shfl(jl, (int)(k < it.y ? k : 0), 32);
        const long long tq = k < it.y ? tail_of(j) : -1;
        x[r] = k < it.y ? *reinterpret_cast<const VT*>(ograd + j * D + hl * V) : VT{};
        y[r] = tq >= 0 ? *reinterpret_cast<const VT*>(otail + tq * D + hl * V) : VT{};
      }
#pragma unroll
      for (int r = 0; r < QF; ++r)
#pragma unroll
        for (int v = 0; v < V; ++v) acc[v] += OVec<V>::get(x[r], v) + OVec<V>::get(y[r], v);
      continue;
    }
    float sc[QF];
    long long jj[QF];
    float2 e[QF];
    // three phases, so every load of a phase is in flight together: the
    // occurrence ids, then the negatives' (gn, center) pairs, then the rows
#pragma unroll
    for (int r = 0; r < QF; ++r) {
      const uint32_t k = k0 + r;
      const long long jv = (long long)__shfl(jl, (int)(k < it.y ? k : 0), 32);
      jj[r] = k < it.y ? jv : -1;
    }
#pragma unroll
    for (int r = 0; r < QF; ++r)
      e[r] = jj[r] >= negbase ? gnc[jj[r] - negbase] : make_float2(1.f, 0.f);
#pragma unroll
    for (int r = 0; r < QF; ++r) {
      const long long j = jj[r];
      sc[r] = 1.f;
      y[r] = VT{};
      if (j < 0) {
        x[r] = VT{};
      } else if (j >= negbase) {  // a scaled center row (per-pair negative)
        const uint32_t c = __float_as_uint(e[r].y);
        sc[r] = e[r].x;
        x[r] = (c != kInv && e[r].x != 0.f)
                   ? *reinterpret_cast<const VT*>(uvals + (long long)c * D + hl * V) : VT{};
      } else {
        x[r] = *reinterpret_cast<const VT*>(ograd + j * D + hl * V);
      }
    }
#pragma unroll
    for (int r = 0; r < QF; ++r)
#pragma unroll
      for (int v = 0; v < V; ++v) acc[v] += sc[r] * OVec<V>::get(x[r], v);
  }
  if (slots && !(it.w & 1u)) {
    // fused K5 (one GPU): this item is the key's whole gradient row — the
    // optimizer update of its table row right here (parameters, then the
    // state, V consecutive floats per lane) instead of a ugrad row that the
    // apply kernel reads back; keys summed over several items (row atomics
    // below) are updated by the apply kernel afterwards (launch_apply only)
    const long long slot = early_slot ? fslot : slots[it.z];
    if (slot < 0) return;  // half-wave-uniform
    const int ns = opt_state_per_coord(op.kind);
    if (tab.bf16) {
      // compact rows: V bf16 words per lane and array, updated in fp32 and
      // stored with stochastic rounding (row_st's rule)
      unsigned short* r16 = reinterpret_cast<unsigned short*>(slot_row(tab, slot));
      float wf[V], s1f[V], s2f[V];
#pragma unroll
      for (int v = 0; v < V; ++v) {
        const int j = hl * V + v;
        wf[v] = bf16_val(r16[j]);
        s1f[v] = ns > 0 ? bf16_val(r16[D + j]) : 0.f;
        s2f[v] = ns > 1 ? bf16_val(r16[2 * D + j]) : 0.f;
      }
#pragma unroll
      for (int v = 0; v < V; ++v) {
        const int j = hl * V + v;
        opt_update(op, wf[v], s1f[v], s2f[v], acc[v]);
        r16[j] = bf16_bits((uint64_t)slot, j, wf[v], true);
        if (ns > 0) r16[D + j] = bf16_bits((uint64_t)slot, D + j, s1f[v], true);
        if (ns > 1) r16[2 * D + j] = bf16_bits((uint64_t)slot, 2 * D + j, s2f[v], true);
      }
      return;
    }
    float* row = slot_row(tab, slot) + hl * V;
    VT w = *reinterpret_cast<const VT*>(row);
    VT s1 = ns > 0 ? *reinterpret_cast<const VT*>(row + D) : VT{};
    VT s2 = ns > 1 ? *reinterpret_cast<const VT*>(row + 2 * D) : VT{};
    float* wf = reinterpret_cast<float*>(&w);
    float* s1f = reinterpret_cast<float*>(&s1);
    float* s2f = reinterpret_cast<float*>(&s2);
#pragma unroll
    for (int v = 0; v < V; ++v) opt_update(op, wf[v], s1f[v], s2f[v], acc[v]);
    *reinterpret_cast<VT*>(row) = w;
    if (ns > 0) *reinterpret_cast<VT*>(row + D) = s1;
    if (ns > 1) *reinterpret_cast<VT*>(row + 2 * D) = s2;
    return;
  }
  float* g = ugrad + (long long)it.z * D + hl * V;
  if (it.w & 1u) {
#pragma unroll
    for (int v = 0; v < V; ++v) atomicAdd(g + v, acc[v]);
  } else {
    VT o;
    float* of = reinterpret_cast<float*>(&o);
#pragma unroll
    for (int v = 0; v < V; ++v) of[v] = acc[v];
    *reinterpret_cast<VT*>(g) = o;
  }
}

// ---- classic SGNS: K negatives drawn per positive pair (neg_mode per_pair)
//
// The shared-negative tile above trains each center against the 64 negatives
// of its tile, weighted to K per pair; this is word2vec's own objective: every
// (center t, context q) pair has its own K negatives (keys [B centers | run
// positions | B x 2W x K negatives], negative (t, o, k) at B + R + (t*2W + o)*K
// + k, o the offset slot of dq = o - W (o < W) or o - W + 1).  Dot products,
// not GEMMs: each pair touches 1 + K rows once, so there is no tile to put on
// the MFMA.  Gradients as occurrence rows summed per key by k_w2v_oreduce (as
// the window tile's): k_w2v_pp (one wave per center) writes the center row,
// the pair's scalar g+ = sig(v.u) - 1, and for each negative only the pair
// (gn, center id) — the negative's gradient row is gn * v_center, which the
// reduce expands from the (cache-resident) center row: 8 bytes per negative
// occurrence instead of a D-float row (819K x 512 B = 420 MB of stores and as
// many loads per config-3 step); k_w2v_ppctx (one wave per run position)
// gathers g+ * v over the 2W centers that pair with it.
static constexpr int kPpMaxK = 16;
// One wave per center; its 2W pairs run as an S-stage pipeline: pairs o+1 ..
// o+S-1 have their 1 + K rows in flight while pair o computes (the per-pair
// row-load chain, not bandwidth, bounds the kernel).  KT: the compile-time
// bound of K (5, word2vec's default), so the row stages take S x (1 + KT) x
// D/64 registers — at KT = 5, S = 3: two pairs in flight at 5+ waves per
// SIMD, against one pair at 122 VGPRs (4 waves) when every stage was sized
// for 16 negatives (k_w2v_pp16 below, any K).  The wave's center, its
// pairs' context ids and its negatives' ids are wave-uniform: scalar loads,
// no lane shuffles.
template <int D, int KT, int S>
__global__ __launch_bounds__(256) void k_w2v_pp(const uint32_t* __restrict__ inv_c,
                                                const uint32_t* __restrict__ inv_w,
                                                const uint32_t* __restrict__ inv_n,
                                                const int32_t* __restrict__ meta, int B, int W,
                                                int K, const float* __restrict__ uvals,
                                                float* __restrict__ ograd,
                                                float* __restrict__ gpair,
                                                float* __restrict__ loss_sum,
                                                float* __restrict__ pair_sum,
                                                float2* __restrict__ gnc) {
  constexpr int R = (D + 63) / 64;
  __shared__ float red[2][4];
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const long long t = (long long)blockIdx.x * 4 + w;
  float loss = 0.f, npairs = 0.f;
  if (t < B) {  // wave-uniform
    const int P2 = 2 * W;
    const uint32_t c = inv_c[t];
    const int32_t mt = meta[t + W];
    const long long nb0 = t * (long long)P2 * K;
    // pair o's context row id (kInv: not a valid pair); uniform
    auto ctx = [&](int o) -> uint32_t {
      const int dq = o < W ? o - W : o - W + 1;
      const long long q = t + W + dq;
      return (c != kInv && w2v_pair_ok(mt, meta[q], dq)) ? inv_w[q] : kInv;
    };
    float v[R], gv[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const int d = lane + 64 * r;
      v[r] = (d < D && c != kInv) ? uvals[(long long)c * D + d] : 0.f;
      gv[r] = 0.f;
    }
    // rows of pair o into (u, n); nothing when the pair is not valid
    auto issue = [&](int o, uint32_t xq, float (&u)[R], float (&n)[KT][R]) {
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const int d = lane + 64 * r;
        u[r] = (d < D && xq != kInv) ? uvals[(long long)xq * D + d] : 0.f;
      }
      const long long nb = nb0 + (long long)o * K;
#pragma unroll
      for (int k = 0; k < KT; ++k) {
        const uint32_t x = (k < K && xq != kInv) ? inv_n[nb + k] : kInv;
#pragma unroll
        for (int r = 0; r < R; ++r) {
          const int d = lane + 64 * r;
          n[k][r] = (x != kInv && d < D) ? uvals[(long long)x * D + d] : 0.f;
        }
      }
    };
    auto compute = [&](int o, uint32_t xq, const float (&u)[R], const float (&n)[KT][R]) {
      const long long nb = (t * P2 + o) * (long long)K;
      if (xq == kInv) {  // the pair's negatives get a zero entry
        if (lane < K) gnc[nb + lane] = make_float2(0.f, __uint_as_float(kInv));
        if (lane == 0) gpair[t * P2 + o] = 0.f;
        return;
      }
      float sp = 0.f;
#pragma unroll
      for (int r = 0; r < R; ++r) sp += v[r] * u[r];
      for (int m = 32; m > 0; m >>= 1) sp += __shfl_xor(sp, m, 64);
      const float gp = sigm(sp) - 1.f;  // d/ds softplus(-s)
      if (lane == 0) {
        loss += softplus(-sp);
        npairs += 1.f;
        gpair[t * P2 + o] = gp;
      }
#pragma unroll
      for (int r = 0; r < R; ++r) gv[r] += gp * u[r];
      float gk = 0.f;  // lane k < K: negative k's gn
#pragma unroll
      for (int k = 0; k < KT; ++k) {
        if (k >= K) break;
        float sn = 0.f;
#pragma unroll
        for (int r = 0; r < R; ++r) sn += v[r] * n[k][r];
        for (int m = 32; m > 0; m >>= 1) sn += __shfl_xor(sn, m, 64);
        const float gn = sigm(sn);  // d/ds softplus(s)
        if (lane == 0) loss += softplus(sn);
        if (lane == k) gk = gn;
#pragma unroll
        for (int r = 0; r < R; ++r) gv[r] += gn * n[k][r];
      }
      if (lane < K) gnc[nb + lane] = make_float2(gk, __uint_as_float(c));
    };
    float u[S][R], n[S][KT][R];
    uint32_t xs[S];
#pragma unroll
    for (int q = 0; q < S - 1; ++q)
      if (q < P2) {
        xs[q] = ctx(q);
        issue(q, xs[q], u[q], n[q]);
      }
    for (int o0 = 0; o0 < P2; o0 += S) {
#pragma unroll
      for (int q = 0; q < S; ++q) {
        const int o = o0 + q, oi = o + S - 1;
        if (oi < P2) {  // pair oi into the stage pair o - 1 freed
          xs[(q + S - 1) % S] = ctx(oi);
          issue(oi, xs[(q + S - 1) % S], u[(q + S - 1) % S], n[(q + S - 1) % S]);
        }
        if (o < P2) compute(o, xs[q], u[q], n[q]);
      }
    }
#pragma unroll
    for (int r = 0; r < R; ++r)
      if (lane + 64 * r < D) ograd[t * D + lane + 64 * r] = gv[r];
  }
  if (lane == 0) {
    red[0][w] = loss;
    red[1][w] = npairs;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    if (loss_sum) ctr_addf(loss_sum, red[0][0] + red[0][1] + red[0][2] + red[0][3]);
    if (pair_sum) ctr_addf(pair_sum, red[1][0] + red[1][1] + red[1][2] + red[1][3]);
  }
}

static constexpr int kPpIdx = 8;  // negative indices per lane: 2W * K <= 64 * 8
// Any K <= 16 (k_w2v_pp16): one wave per center; the 2W pairs run as a two-stage pipeline: every
// index of the center (contexts, pair validity, all 2W x K negatives) is
// loaded up front, one lane each, and pair o+1's 1 + K rows are in flight
// while pair o computes — one row-load latency per pair instead of an
// index load followed by a row load (measured: the per-pair chain, not
// bandwidth, bounded the kernel).
template <int D>
__global__ __launch_bounds__(256) void k_w2v_pp16(const uint32_t* __restrict__ inv_c,
                                                const uint32_t* __restrict__ inv_w,
                                                const uint32_t* __restrict__ inv_n,
                                                const int32_t* __restrict__ meta, int B, int W,
                                                int K, const float* __restrict__ uvals,
                                                float* __restrict__ ograd,
                                                float* __restrict__ gpair,
                                                float* __restrict__ loss_sum,
                                                float* __restrict__ pair_sum,
                                                float2* __restrict__ gnc) {
  constexpr int R = (D + 63) / 64;
  __shared__ float red[2][4];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const long long t = (long long)blockIdx.x * 4 + w;
  float loss = 0.f, npairs = 0.f;
  if (t < B) {  // wave-uniform
    const int P2 = 2 * W;
    const uint32_t c = inv_c[t];
    // lane o < 2W: pair o's context row id (kInv: the pair is not valid)
    uint32_t xl = kInv;
    if (lane < P2) {
      const int dq = lane < W ? lane - W : lane - W + 1;
      const long long q = t + W + dq;
      if (c != kInv && w2v_pair_ok(meta[t + W], meta[q], dq)) xl = inv_w[q];
    }
    // every negative index of the center: (pair o, k) at o * K + k, lane-strided
    uint32_t ni[kPpIdx];
    const long long nb0 = t * (long long)P2 * K;
#pragma unroll
    for (int i = 0; i < kPpIdx; ++i) {
      const int e = i * 64 + lane;
      ni[i] = e < P2 * K ? inv_n[nb0 + e] : kInv;
    }
    float v[R], gv[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const int d = lane + 64 * r;
      v[r] = (d < D && c != kInv) ? uvals[(long long)c * D + d] : 0.f;
      gv[r] = 0.f;
    }
    auto nidx = [&](int e) -> uint32_t {  // negative e of the center (wave-uniform e)
      uint32_t x = kInv;
#pragma unroll
      for (int i = 0; i < kPpIdx; ++i)
        if (e / 64 == i) x = __shfl(ni[i], e % 64, 64);
      return x;
    };
    // rows of pair o into (u, n); nothing when the pair is not valid
    auto issue = [&](int o, float (&u)[R], float (&n)[kPpMaxK][R]) {
      const uint32_t xq = __shfl(xl, o, 64);
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const int d = lane + 64 * r;
        u[r] = (d < D && xq != kInv) ? uvals[(long long)xq * D + d] : 0.f;
      }
#pragma unroll
      for (int k = 0; k < kPpMaxK; ++k) {
        const uint32_t x = (k < K && xq != kInv) ? nidx(o * K + k) : kInv;
#pragma unroll
        for (int r = 0; r < R; ++r) {
          const int d = lane + 64 * r;
          n[k][r] = (x != kInv && d < D) ? uvals[(long long)x * D + d] : 0.f;
        }
      }
    };
    auto compute = [&](int o, const float (&u)[R], const float (&n)[kPpMaxK][R]) {
      const long long nb = (t * P2 + o) * (long long)K;
      if (__shfl(xl, o, 64) == kInv) {  // the pair's negatives get a zero entry
        if (lane < K) gnc[nb + lane] = make_float2(0.f, __uint_as_float(kInv));
        if (lane == 0) gpair[t * P2 + o] = 0.f;
        return;
      }
      float sp = 0.f;
#pragma unroll
      for (int r = 0; r < R; ++r) sp += v[r] * u[r];
      for (int m = 32; m > 0; m >>= 1) sp += __shfl_xor(sp, m, 64);
      const float gp = sigm(sp) - 1.f;  // d/ds softplus(-s)
      if (lane == 0) {
        loss += softplus(-sp);
        npairs += 1.f;
        gpair[t * P2 + o] = gp;
      }
#pragma unroll
      for (int r = 0; r < R; ++r) gv[r] += gp * u[r];
      float gk = 0.f;  // lane k < K: negative k's gn
#pragma unroll
      for (int k = 0; k < kPpMaxK; ++k) {
        if (k >= K) break;
        float sn = 0.f;
#pragma unroll
        for (int r = 0; r < R; ++r) sn += v[r] * n[k][r];
        for (int m = 32; m > 0; m >>= 1) sn += __shfl_xor(sn, m, 64);
        const float gn = sigm(sn);  // d/ds softplus(s)
        if (lane == 0) loss += softplus(sn);
        if (lane == k) gk = gn;
#pragma unroll
        for (int r = 0; r < R; ++r) gv[r] += gn * n[k][r];
      }
      if (lane < K) gnc[nb + lane] = make_float2(gk, __uint_as_float(c));
    };
    float ua[R], na[kPpMaxK][R], ub[R], nbuf[kPpMaxK][R];
    issue(0, ua, na);
    for (int o = 0; o < P2; o += 2) {
      if (o + 1 < P2) issue(o + 1, ub, nbuf);
      compute(o, ua, na);
      if (o + 1 < P2) {
        if (o + 2 < P2) issue(o + 2, ua, na);
        compute(o + 1, ub, nbuf);
      }
    }
#pragma unroll
    for (int r = 0; r < R; ++r)
      if (lane + 64 * r < D) ograd[t * D + lane + 64 * r] = gv[r];
  }
  if (lane == 0) {
    red[0][w] = loss;
    red[1][w] = npairs;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    if (loss_sum) ctr_addf(loss_sum, red[0][0] + red[0][1] + red[0][2] + red[0][3]);
    if (pair_sum) ctr_addf(pair_sum, red[1][0] + red[1][1] + red[1][2] + red[1][3]);
  }
}

template <int D>
__global__ __launch_bounds__(256) void k_w2v_ppctx(const uint32_t* __restrict__ inv_c,
                                                   const float* __restrict__ gpair, int B, int W,
                                                   const float* __restrict__ uvals,
                                                   float* __restrict__ ograd) {
  constexpr int R = (D + 63) / 64;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const long long Rn = (long long)B + 2 * W;
  const long long q = (long long)blockIdx.x * 4 + w;  // run position
  if (q >= Rn) return;  // wave-uniform
  // lane o < 2W: the pair (center t = q - W - dq, q) of offset slot o, whose
  // g+ k_w2v_pp stored (0 when the pair is not valid)
  uint32_t cl = kInv;
  float gl = 0.f;
  if (lane < 2 * W) {
    const int o = lane, dq = o < W ? o - W : o - W + 1;
    const long long t = q - W - dq;
    if (t >= 0 && t < B) {
      gl = gpair[t * 2 * W + o];
      if (gl != 0.f) cl = inv_c[t];
    }
  }
  float acc[R];
#pragma unroll
  for (int r = 0; r < R; ++r) acc[r] = 0.f;
  for (int o = 0; o < 2 * W; ++o) {
    const uint32_t c = __shfl(cl, o, 64);
    const float g = __shfl(gl, o, 64);
    if (c == kInv) continue;  // wave-uniform
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const int d = lane + 64 * r;
      if (d < D) acc[r] += g * uvals[(long long)c * D + d];
    }
  }
#pragma unroll
  for (int r = 0; r < R; ++r)
    if (lane + 64 * r < D) ograd[(B + q) * D + lane + 64 * r] = acc[r];
}

// Synthetic token stream in the windowed layout: sentences of L tokens, each
// around a Zipf-drawn topic word (a token is the topic +- W ids, or with
// probability `noise` an independent Zipf word), so words with nearby ids
// co-occur — the learnable structure of k_w2v_gen, as a stream.  Position g
// of the rank's stream is a pure function of (seed, g): consecutive runs
// (base = (step * world + rank) * B) overlap by 2W positions consistently.
// keys = [centers B][run positions B + 2W | 1<<40][negatives nneg | 1<<40].
__global__ __launch_bounds__(256) void k_w2v_stream_gen(
    uint64_t seed, long long base, int B, int W, int L, long long nneg, long long V, double logV,
    float noise, uint64_t* __restrict__ keys, int32_t* __restrict__ meta,
    const long long* __restrict__ step_dev, long long step_mul, long long step_add) {
  if (step_dev) base = *step_dev * step_mul + step_add;
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const long long R = (long long)B + 2 * W;
  const uint64_t kOut = 1ull << 40;
  if (i < R) {
    const long long g = base - W + i;
    uint64_t tok = 0;
    int32_t m = -1;
    if (g >= 0) {
      const long long s = g / L;
      const uint64_t c = w2v_zipf(splitmix64(seed ^ ((uint64_t)s * 0xA24BAED4963EE407ull)), V, logV);
      const uint64_t r = splitmix64(seed ^ 0xC0FFEEull ^ ((uint64_t)g * 0x9E3779B97F4A7C15ull));
      if (u01(r) < noise) {
        tok = w2v_zipf(splitmix64(r), V, logV);
      } else {
        const long long off = (long long)(splitmix64(r ^ 1) % (uint64_t)(2 * W + 1)) - W;
        tok = (uint64_t)((((long long)c + off) % V + V) % V);
      }
      m = w2v_meta((uint64_t)s, w2v_reduced_window(seed, (uint64_t)g, W));
    }
    keys[B + i] = tok | kOut;
    meta[i] = m;
    if (i >= W && i < W + B) keys[i - W] = tok;
  } else if (i < R + nneg) {
    const long long q = i - R;
    keys[B + R + q] =
        w2v_noise(splitmix64(seed ^ 0xBADC0DEull ^ splitmix64((uint64_t)base) ^
                             ((uint64_t)q * 0xD1B54A32D192ED03ull)), V) | kOut;
  }
}

size_t w2v_smem_bytes(int D) {
  const int P = D + 1;
  return sizeof(float) * ((size_t)3 * kT * P + (size_t)kT * (kS + 1) + kNW);
}

// Grid of the window tile kernel (k_w2v_win_bf16).  With the gradient rows as
// float atomics: half the CUs, each workgroup walking tiles — one workgroup
// per tile held every CU with an 80+ KB-LDS workgroup for the kernel's whole
// (atomic-bound) run, and the route stream's dedup (53 KB LDS) of the next
// round then ran 5x slower beside it (11 -> 57 us); 16K centers, caps 256 /
// 192 / 160 / 128 / 96 / 64 gave 0.143 / 0.124 / 0.121 / 0.123 / 0.128 /
// 0.148 ms/step.  With occurrence-row stores (the default) the tile takes 29
// us and one workgroup per tile is faster (hipGraph replay, one box: 0.092 vs
// 0.101-0.103 ms/step at half the CUs).  SS_W2V_WIN_GRID overrides (0: one
// workgroup per tile)
static int w2v_tile_grid(int tiles, bool atomics) {
  static const int env = [] {
    const char* e = std::getenv("SS_W2V_WIN_GRID");
    return e ? std::atoi(e) : -1;
  }();
  static const int half = [] {
    int dev = 0, cus = 0;
    check_hip(hipGetDevice(&dev), "hipGetDevice");
    check_hip(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev),
              "CU count");
    return std::max(1, cus / 2);
  }();
  const int cap = env >= 0 ? env : (atomics ? half : 0);
  return cap > 0 ? std::min(tiles, cap) : tiles;
}

// Raise a kernel's dynamic-LDS limit once per process (a driver call per
// launch costs host time on the small-batch path); thread-safe static init.
template <auto Kernel>
static void smem_attr_once(size_t bytes) {
  static const bool done = (check_hip(hipFuncSetAttribute((const void*)Kernel,
                                                          hipFuncAttributeMaxDynamicSharedMemorySize,
                                                          (int)bytes),
                                      "w2v smem attr"),
                            true);
  (void)done;
}

template <int D>
static void launch_w2v_bf16(int tiles, const uint32_t* inv_c, const uint32_t* inv_x,
                            const uint32_t* inv_n, int B, int C, float neg_scale,
                            const float* uvals, float* ugrad, float* loss_sum, hipStream_t st) {
  const size_t sm = W2vBf16Smem<D>::bytes;
  smem_attr_once<k_w2v_sgns_bf16<D>>(sm);
  // one workgroup per tile: the pairs tile is bound by its own ~84 MB of row
  // atomics per 16K-center step and needs every CU (half the CUs, as the
  // window tile uses: 0.272 -> 0.289 ms/step).  Positive pairs in their own
  // one-wave-per-center kernel measured slower (0.307 -> 0.344 ms/step: the
  // pairs are bound by the memory-side rate of their row atomics, not by the
  // tile's occupancy)
  hipLaunchKernelGGL(k_w2v_sgns_bf16<D>, dim3(tiles), dim3(kWG), sm, st, inv_c, inv_x, inv_n, B,
                     C, neg_scale, uvals, ugrad, loss_sum);
}

void launch_w2v_sgns(const uint32_t* inv_c, const uint32_t* inv_x, const uint32_t* inv_n, int B,
                     int C, int D, float neg_scale, const float* uvals, float* ugrad,
                     float* loss_sum, hipStream_t st, int bf16) {
  if (B <= 0) return;
  if (C < 1 || C > kMaxC) throw_error("w2v_sgns: contexts per center must be in [1,16]");
  const int tiles = (B + kT - 1) / kT;
  if (bf16) {
    switch (D) {
#define SS_W2VB_CASE(DD)                                                                     \
  case DD:                                                                                   \
    launch_w2v_bf16<DD>(tiles, inv_c, inv_x, inv_n, B, C, neg_scale, uvals, ugrad,    \
                        loss_sum, st);                                                       \
    break;
      SS_W2VB_CASE(32)
      SS_W2VB_CASE(64)
      SS_W2VB_CASE(128)
#undef SS_W2VB_CASE
      default:
        throw_error("w2v_sgns: D must be 32, 64 or 128");
    }
    check_launch("k_w2v_sgns_bf16");
    return;
  }
  const size_t sm = w2v_smem_bytes(D);
  switch (D) {
#define SS_W2V_CASE(DD)                                                                     \
  case DD:                                                                                  \
    smem_attr_once<k_w2v_sgns<DD>>(sm);                                                     \
    hipLaunchKernelGGL(k_w2v_sgns<DD>, dim3(tiles), dim3(kWG), sm, st, inv_c, inv_x, inv_n, B, C, \
                       neg_scale, uvals, ugrad, loss_sum);                                  \
    break;
    SS_W2V_CASE(32)
    SS_W2V_CASE(64)
    SS_W2V_CASE(128)
#undef SS_W2V_CASE
    default:
      throw_error("w2v_sgns: D must be 32, 64 or 128");
  }
  check_launch("k_w2v_sgns");
}

void launch_w2v_osort(int P, const uint32_t* bstart, const uint32_t* unum, const uint32_t* ubase,
                      const uint32_t* pj, const uint32_t* luid, uint32_t* ord, uint32_t* items,
                      hipStream_t st, uint8_t* uhot) {
  if (P <= 0) return;
  hipLaunchKernelGGL(k_w2v_osort, dim3(P), dim3(kOsT), 0, st, bstart, unum, ubase, pj, luid, ord,
                     reinterpret_cast<uint4*>(items), uhot);
  check_launch("k_w2v_osort");
}

// The per-pair form with TWO items per half-wave (SS_W2V_PP_ITEMS=2): most
// items of a per-pair step are keys drawn once (a tail word's single
// negative occurrence), whose chain — item, (gn, center), center row, slot,
// parameter row, store — holds one row in flight per half-wave in the kernel
// above.  Here each half-wave walks items s and s + nh (nh = half-waves in
// the grid) in lock step, QF2 occurrences of each per round (2: 56 VGPRs at
// D = 128, 8 waves per SIMD — twice the item chains in flight; 4: 78 VGPRs,
// 6 waves, SS_W2V_PP_QF=4).
template <int D, int QF2>
__global__ __launch_bounds__(256) void k_w2v_oreduce_pp2(
    const uint4* __restrict__ items, long long n, const uint32_t* __restrict__ ord,
    const float* __restrict__ ograd, float* __restrict__ ugrad,
    const float2* __restrict__ gnc, long long negbase, const float* __restrict__ uvals,
    float* __restrict__ lacc, float* __restrict__ lacc_out, int lacc_n, DevTable tab,
    const long long* __restrict__ slots, OptParams op) {
  if (lacc)
    for (int i = blockIdx.x * 256 + threadIdx.x; i < lacc_n; i += gridDim.x * 256) {
      lacc_out[i] = lacc[i];
      lacc[i] = 0.f;
    }
  constexpr int V = D / 32;
  using VT = typename OVec<V>::T;
  const int lane = threadIdx.x & 63, hl = lane & 31;
  const long long nh = (long long)gridDim.x * 8;
  const long long s0 = ((long long)blockIdx.x * 4 + (threadIdx.x >> 6)) * 2 + (lane >> 5);
  uint4 it[2];
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const long long s = s0 + u * nh;
    it[u] = s < n ? items[s] : make_uint4(0u, 0u, 0u, 0u);
  }
  if (it[0].y == 0 && it[1].y == 0) return;  // half-wave-uniform
  uint32_t jl[2];
  long long fslot[2];
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    jl[u] = (it[u].w & 2u) ? it[u].x : (hl < (int)it[u].y ? ord[it[u].x + hl] : 0u);
    fslot[u] = (slots && it[u].y && !(it[u].w & 1u)) ? slots[it[u].z] : -1;
  }
  float acc[2][V];
#pragma unroll
  for (int u = 0; u < 2; ++u)
#pragma unroll
    for (int v = 0; v < V; ++v) acc[u][v] = 0.f;
  const uint32_t ymax = max(it[0].y, it[1].y);
  for (uint32_t k0 = 0; k0 < ymax; k0 += QF2) {
    long long jj[2][QF2];
    float2 e[2][QF2];
    VT x[2][QF2];
    float sc[2][QF2];
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int r = 0; r < QF2; ++r) {
        const uint32_t k = k0 + r;
        const long long jv = (long long)__shfl(jl[u], (int)(k < it[u].y ? k : 0), 32);
        jj[u][r] = k < it[u].y ? jv : -1;
      }
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int r = 0; r < QF2; ++r)
        e[u][r] = jj[u][r] >= negbase ? gnc[jj[u][r] - negbase] : make_float2(1.f, 0.f);
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int r = 0; r < QF2; ++r) {
        const long long j = jj[u][r];
        sc[u][r] = 1.f;
        if (j < 0) {
          x[u][r] = VT{};
        } else if (j >= negbase) {  // a scaled center row (per-pair negative)
          const uint32_t c = __float_as_uint(e[u][r].y);
          sc[u][r] = e[u][r].x;
          x[u][r] = (c != kInv && e[u][r].x != 0.f)
                        ? *reinterpret_cast<const VT*>(uvals + (long long)c * D + hl * V) : VT{};
        } else {
          x[u][r] = *reinterpret_cast<const VT*>(ograd + j * D + hl * V);
        }
      }
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int r = 0; r < QF2; ++r)
#pragma unroll
        for (int v = 0; v < V; ++v) acc[u][v] += sc[u][r] * OVec<V>::get(x[u][r], v);
  }
  const int ns = opt_state_per_coord(op.kind);
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    if (it[u].y == 0) continue;  // half-wave-uniform
    if (slots && !(it[u].w & 1u)) {  // fused K5, as in k_w2v_oreduce
      const long long slot = fslot[u];
      if (slot < 0) continue;
      if (tab.bf16) {
        unsigned short* r16 = reinterpret_cast<unsigned short*>(slot_row(tab, slot));
#pragma unroll
        for (int v = 0; v < V; ++v) {
          const int j = hl * V + v;
          float w = bf16_val(r16[j]);
          float a = ns > 0 ? bf16_val(r16[D + j]) : 0.f;
          float b = ns > 1 ? bf16_val(r16[2 * D + j]) : 0.f;
          opt_update(op, w, a, b, acc[u][v]);
          r16[j] = bf16_bits((uint64_t)slot, j, w, true);
          if (ns > 0) r16[D + j] = bf16_bits((uint64_t)slot, D + j, a, true);
          if (ns > 1) r16[2 * D + j] = bf16_bits((uint64_t)slot, 2 * D + j, b, true);
        }
        continue;
      }
      float* row = slot_row(tab, slot) + hl * V;
      VT w = *reinterpret_cast<const VT*>(row);
      VT s1 = ns > 0 ? *reinterpret_cast<const VT*>(row + D) : VT{};
      VT s2 = ns > 1 ? *reinterpret_cast<const VT*>(row + 2 * D) : VT{};
      float* wf = reinterpret_cast<float*>(&w);
      float* s1f = reinterpret_cast<float*>(&s1);
      float* s2f = reinterpret_cast<float*>(&s2);
#pragma unroll
      for (int v = 0; v < V; ++v) opt_update(op, wf[v], s1f[v], s2f[v], acc[u][v]);
      *reinterpret_cast<VT*>(row) = w;
      if (ns > 0) *reinterpret_cast<VT*>(row + D) = s1;
      if (ns > 1) *reinterpret_cast<VT*>(row + 2 * D) = s2;
      continue;
    }
    float* g = ugrad + (long long)it[u].z * D + hl * V;
    if (it[u].w & 1u) {
#pragma unroll
      for (int v = 0; v < V; ++v) atomicAdd(g + v, acc[u][v]);
    } else {
      VT o;
      float* of = reinterpret_cast<float*>(&o);
#pragma unroll
      for (int v = 0; v < V; ++v) of[v] = acc[u][v];
      *reinterpret_cast<VT*>(g) = o;
    }
  }
}

static int pp_qf() {
  static const int v = [] {
    const char* e = std::getenv("SS_W2V_PP_QF");
    return e ? std::atoi(e) : 2;
  }();
  return v;
}
// SS_W2V_PP_ITEMS: items per half-wave of the per-pair reduce, 1 or 2
static int pp_items() {
  static const int v = [] {
    const char* e = std::getenv("SS_W2V_PP_ITEMS");
    return e ? std::atoi(e) : 2;
  }();
  return v;
}

// SS_W2V_EARLY_SLOT=0: the fused update loads its slot index after the
// occurrence gathers instead of beside the first (A/B)
static int early_slot() {
  static const int v = [] {
    const char* e = std::getenv("SS_W2V_EARLY_SLOT");
    return e ? std::atoi(e) : 1;
  }();
  return v;
}

void launch_w2v_oreduce(const uint32_t* items, long long n, const uint32_t* ord, const float* ograd,
                        const float* otail, int B, int W, int D, float* ugrad, hipStream_t st,
                        const float* gnc, long long negbase, const float* uvals, float* acc,
                        float* acc_out, int acc_n, const DevTable* tab, const long long* slots,
                        const OptParams* op) {
  if (gnc && !uvals) throw_error("w2v_oreduce: scaled negative rows need the center rows");
  DevTable tv{};
  OptParams opv{};
  if (slots) {
    const int ns = op ? opt_state_per_coord(op->kind) : 0;
    const int al = tab && tab->bf16 ? 8 : 16;
    if (!tab || !op || (int)tab->dim != D || (int)tab->width != D * (1 + ns) ||
        tab->row_off % al != 0 || tab->stride % al != 0)
      throw_error("w2v_oreduce: a fused update needs aligned rows of this D");
    tv = *tab;
    opv = *op;
  }
  if (acc && (!acc_out || acc_n <= 0)) throw_error("w2v_oreduce: accumulator hand-off needs acc_out");
  if (n <= 0 && !acc) return;
  if (W < 1 || W > kW2vMaxWindow) throw_error("w2v_oreduce: window must be in [1, 15]");
  const int ntiles = (B + kT - 1) / kT;
  // an item per half-wave, no grid stride: the reduce is a chain of
  // dependent loads per item (item -> rows -> store), so every chain of the
  // call runs concurrently
  const int grid = (int)std::max<long long>((n + 7) / 8, acc ? 64 : 1);
  const uint4* it = reinterpret_cast<const uint4*>(items);
  if (gnc && pp_items() == 2) {
    // two items per half-wave: half the grid (s and s + nh per half-wave)
    const int g2 = (int)std::max<long long>((n + 15) / 16, acc ? 64 : 1);
    switch (D) {
#define SS_W2VO2(DD)                                                                            \
  case DD:                                                                                      \
    if (pp_qf() == 4)                                                                           \
      hipLaunchKernelGGL((k_w2v_oreduce_pp2<DD, 4>), dim3(g2), dim3(256), 0, st, it, n, ord,    \
                         ograd, ugrad, reinterpret_cast<const float2*>(gnc), negbase, uvals,    \
                         acc, acc_out, acc_n, tv, slots, opv);                                  \
    else                                                                                        \
      hipLaunchKernelGGL((k_w2v_oreduce_pp2<DD, 2>), dim3(g2), dim3(256), 0, st, it, n, ord,    \
                         ograd, ugrad, reinterpret_cast<const float2*>(gnc), negbase, uvals,    \
                         acc, acc_out, acc_n, tv, slots, opv);                                  \
    break;
      SS_W2VO2(32)
      SS_W2VO2(64)
      SS_W2VO2(128)
#undef SS_W2VO2
      default:
        throw_error("w2v_oreduce: D must be 32, 64 or 128");
    }
    check_launch("k_w2v_oreduce_pp2");
    return;
  }
  switch (D) {
#define SS_W2VO_CASE(DD)                                                                      \
  case DD:                                                                                    \
    if (gnc)                                                                                  \
      hipLaunchKernelGGL((k_w2v_oreduce<DD, true>), dim3(grid), dim3(256), 0, st, it, n, ord,  \
                         ograd, otail, B, W, ntiles, ugrad,                                    \
                         reinterpret_cast<const float2*>(gnc), negbase, uvals, acc, acc_out,   \
                         acc_n, tv, slots, opv, early_slot());                                 \
    else                                                                                      \
      hipLaunchKernelGGL((k_w2v_oreduce<DD, false>), dim3(grid), dim3(256), 0, st, it, n, ord, \
                         ograd, otail, B, W, ntiles, ugrad, nullptr, 0ll, nullptr, acc,        \
                         acc_out, acc_n, tv, slots, opv, early_slot());                        \
    break;
    SS_W2VO_CASE(32)
    SS_W2VO_CASE(64)
    SS_W2VO_CASE(128)
#undef SS_W2VO_CASE
    default:
      throw_error("w2v_oreduce: D must be 32, 64 or 128");
  }
  check_launch("k_w2v_oreduce");
}

void launch_w2v_win(const uint32_t* inv_c, const uint32_t* inv_w, const uint32_t* inv_n,
                    const int32_t* meta, int B, int W, int D, float neg_per_pair,
                    const float* uvals, float* ugrad, float* loss_sum, float* pair_sum,
                    hipStream_t st, float* ograd, float* otail) {
  if (B <= 0) return;
  if (W < 1 || W > kW2vMaxWindow) throw_error("w2v_win: window must be in [1, 15]");
  const int tiles = (B + kT - 1) / kT;
  const int grid = w2v_tile_grid(tiles, ograd == nullptr);
  // 8 waves per tile: 16 (1024 threads) ran the tile alone 29.6 -> 23.1 us
  // but the step 0.083 -> 0.093 ms (its registers fill the CU's SIMDs and
  // nothing else runs beside it)
  switch (D) {
#define SS_W2VW_CASE(DD)                                                                     \
  case DD:                                                                                   \
    smem_attr_once<k_w2v_win_bf16<DD>>(W2vWinSmem<DD>::bytes);                               \
    hipLaunchKernelGGL(k_w2v_win_bf16<DD>, dim3(grid), dim3(512), W2vWinSmem<DD>::bytes, st,     \
                       inv_c, inv_w, inv_n, meta, B, W, neg_per_pair, uvals, ugrad, loss_sum,  \
                       pair_sum, ograd, otail);                                                \
    break;
    SS_W2VW_CASE(32)
    SS_W2VW_CASE(64)
    SS_W2VW_CASE(128)
#undef SS_W2VW_CASE
    default:
      throw_error("w2v_win: D must be 32, 64 or 128");
  }
  check_launch("k_w2v_win_bf16");
}

// SS_W2V_PP_STAGES: pipeline stages of the K <= 5 kernel, 3 (default) or 4;
// 2: the K <= 16 kernel for every K.  Measured (1M vocab, dim 128, K = 5,
// serialised): 110.5 / 122.6 / 171 us; step 0.542 / 0.551 / 0.607-0.610 ms
static int pp_stages() {
  static const int v = [] {
    const char* e = std::getenv("SS_W2V_PP_STAGES");
    return e ? std::atoi(e) : 3;
  }();
  return v;
}

void launch_w2v_pp(const uint32_t* inv_c, const uint32_t* inv_w, const uint32_t* inv_n,
                   const int32_t* meta, int B, int W, int K, int D, const float* uvals,
                   float* ograd, float* gpair, float* loss_sum, float* pair_sum, hipStream_t st,
                   float* gnc) {
  if (B <= 0) return;
  if (!gnc) throw_error("w2v_pp: the (gn, center) buffer of the negatives is required");
  if (W < 1 || W > kW2vMaxWindow) throw_error("w2v_pp: window must be in [1, 15]");
  if (K < 1 || K > kPpMaxK) throw_error("w2v_pp: negatives per pair must be in [1, 16]");
  if (2 * W * K > 64 * kPpIdx) throw_error("w2v_pp: 2W x K must be <= 512");
  const long long Rn = (long long)B + 2 * W;
  switch (D) {
#define SS_W2VP_CASE(DD)                                                                       \
  case DD:                                                                                     \
    if (K <= 5 && pp_stages() == 3)                                                            \
      hipLaunchKernelGGL((k_w2v_pp<DD, 5, 3>), dim3((unsigned)((B + 3) / 4)), dim3(256), 0, st,  \
                         inv_c, inv_w, inv_n, meta, B, W, K, uvals, ograd, gpair, loss_sum,     \
                         pair_sum, reinterpret_cast<float2*>(gnc));                             \
    else if (K <= 5 && pp_stages() > 3)                                                        \
      hipLaunchKernelGGL((k_w2v_pp<DD, 5, 4>), dim3((unsigned)((B + 3) / 4)), dim3(256), 0, st,  \
                         inv_c, inv_w, inv_n, meta, B, W, K, uvals, ograd, gpair, loss_sum,     \
                         pair_sum, reinterpret_cast<float2*>(gnc));                             \
    else                                                                                       \
      hipLaunchKernelGGL(k_w2v_pp16<DD>, dim3((unsigned)((B + 3) / 4)), dim3(256), 0, st,       \
                         inv_c, inv_w, inv_n, meta, B, W, K, uvals, ograd, gpair, loss_sum,     \
                         pair_sum, reinterpret_cast<float2*>(gnc));                             \
    check_launch("k_w2v_pp");                                                                  \
    hipLaunchKernelGGL(k_w2v_ppctx<DD>, dim3((unsigned)((Rn + 3) / 4)), dim3(256), 0, st,       \
                       inv_c, gpair, B, W, uvals, ograd);                                      \
    check_launch("k_w2v_ppctx");                                                               \
    break;
    SS_W2VP_CASE(32)
    SS_W2VP_CASE(64)
    SS_W2VP_CASE(128)
#undef SS_W2VP_CASE
    default:
      throw_error("w2v_pp: D must be 32, 64 or 128");
  }
}

void launch_w2v_stream_gen(uint64_t seed, long long base, int B, int W, int L, long long nneg,
                           long long V, float noise, uint64_t* keys, int32_t* meta,
                           hipStream_t st, const long long* step_dev, long long step_mul,
                           long long step_add) {
  if (W < 1 || W > kW2vMaxWindow) throw_error("w2v_stream_gen: window must be in [1, 15]");
  if (L < 1) throw_error("w2v_stream_gen: sentence length must be >= 1");
  const long long n = (long long)B + 2 * W + nneg;
  if (B <= 0 || n <= 0) return;
  hipLaunchKernelGGL(k_w2v_stream_gen, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, seed,
                     base, B, W, L, nneg, V, log((double)V + 1.0), noise, keys, meta, step_dev,
                     step_mul, step_add);
  check_launch("k_w2v_stream_gen");
}

void launch_w2v_gen(uint64_t seed, long long base, int B, int C, int W, long long nneg,
                    long long V, float noise, uint64_t* keys, hipStream_t st,
                    const long long* step_dev, long long step_mul, long long step_add) {
  const long long n = (long long)B + (long long)B * C + nneg;
  if (n <= 0) return;
  if (W < 1) throw_error("w2v_gen: window must be >= 1");
  hipLaunchKernelGGL(k_w2v_gen, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, seed, base, B,
                     C, W, nneg, V, log((double)V + 1.0), noise, keys, step_dev, step_mul,
                     step_add);
  check_launch("k_w2v_gen");
}

}  // namespace ss
