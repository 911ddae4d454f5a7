// models.hip — fused model kernels for the sparse-LR workload (gfx950).
//
// The reference ships no application code (its scripts name the absent
// src/apps/logistic_regression, /root/reference/src/tools/hadoop-server.sh:7);
// its `train()` hot loop would be a per-sample sparse dot + sigmoid + grad
// scatter over the pulled GlobalParamCache (global_param_cache.h:28-118,
// Vec math in utils/vec1.h:97-104).  Here that loop is one kernel:
//
//   K6+K7  gather w through the dedup inverse index, per-sample dot (LDS
//          segmented sum), sigmoid + logloss, and scatter the per-key
//          gradient (p - y) * x into the unique-key gradient rows that the
//          push round ships to the servers.
//
// Synthetic CTR data is generated on device each step (counter-based RNG), so
// the timed step includes producing its input batch.
#include "sample_group.h"
#include "ss_device.h"
#include "ss_launch.h"

namespace ss {

static constexpr uint32_t kInvalidU = 0xFFFFFFFFu;

// Samples handled by one 256-thread block when a sample has F features.
__host__ __device__ inline int samples_per_block(int F) { return F >= 256 ? 1 : 256 / F; }

// Per-key ground-truth weight of the synthetic generator (labels are drawn
// from a true sparse-LR model so convergence is measurable).
__device__ __forceinline__ float truth_weight(uint64_t key, float scale) {
  return (u01(splitmix64(key ^ 0x5DEECE66Dull)) - 0.5f) * scale;
}

// Keys: field f owns [f*V, (f+1)*V); ids are log-uniform (Zipf-like head, as
// in CTR data) with a `tail_frac` share drawn uniformly over the field (long
// tail that keeps inserting new keys into the table).
__device__ __forceinline__ uint64_t gen_ctr_key(uint64_t seed, uint64_t gs, int f, long long V,
                                                double logV, float tail_frac) {
  const uint64_t r = splitmix64(seed ^ (gs * 0xA24BAED4963EE407ull) ^ ((uint64_t)f << 40));
  const uint64_t r2 = splitmix64(r);
  uint64_t id;
  if (u01(r2) < tail_frac) {
    id = fastrange64(splitmix64(r2 ^ 0x632BE59BD9B4E019ull), (uint64_t)V);
  } else {
    const double u = (double)(r >> 11) * (1.0 / 9007199254740992.0);
    long long v = (long long)exp(u * logV) - 1;
    id = (uint64_t)(v < 0 ? 0 : (v >= V ? V - 1 : v));
  }
  return (uint64_t)f * (uint64_t)V + id;
}

__device__ __forceinline__ float gen_ctr_label(uint64_t seed, uint64_t gs, float z) {
  const float p = 1.f / (1.f + __expf(-z));
  return u01(splitmix64(seed ^ 0xBEEF ^ (gs * 0x9E3779B97F4A7C15ull))) < p ? 1.f : 0.f;
}

// Packed layout (256/F samples per workgroup) with an LDS per-sample sum.  The
// generator is VALU-bound (fp64 exp, 64-bit mixing), so lane utilisation is
// what counts: measured on MI355X the packed layout (91% of lanes busy at
// F = 39) beat the one-sample-per-lane-group layout of the LR forward (61%),
// 55 vs 69 us per 2.56M keys.
// sample_base: first global sample id of the batch; with step_dev (hipGraph
// replays, where kernel arguments are frozen) it is *step_dev * step_mul +
// step_add instead, so every replay generates the next batch
__global__ __launch_bounds__(256) void k_gen_ctr(uint64_t seed, long long sample_base, int B,
                                                     int F, long long V, double logV,
                                                     float tail_frac, float truth_scale,
                                                     float truth_bias, uint64_t* __restrict__ keys,
                                                     float* __restrict__ labels,
                                                     const long long* __restrict__ step_dev,
                                                     long long step_mul, long long step_add) {
  if (step_dev) sample_base = *step_dev * step_mul + step_add;
  __shared__ float sval[256];
  __shared__ float sdot[256];
  const int spb = samples_per_block(F);
  const int t = threadIdx.x;
  const int ls = t / F, f = t - (t / F) * F;
  const long long s0 = (long long)blockIdx.x * spb;
  float wv = 0.f;
  if (ls < spb && s0 + ls < B && F <= 256) {
    const uint64_t key =
        gen_ctr_key(seed, (uint64_t)(sample_base + s0 + ls), f, V, logV, tail_frac);
    keys[(s0 + ls) * F + f] = key;
    wv = truth_weight(key, truth_scale);
  }
  packed_sample_sums(wv, F, spb, sval, sdot);  // per-sample sums, no LDS atomics
  if (t < spb && s0 + t < B)
    labels[s0 + t] = gen_ctr_label(seed, (uint64_t)(sample_base + s0 + t), sdot[t] + truth_bias);
}

// The same generator over R groups of spb samples per workgroup: each
// thread draws its R keys (independent hash / exp chains, all in flight
// together) before the per-sample sums, and R x fewer workgroups are
// dispatched (43691 256-thread workgroups of one key per thread at the bench
// shape).  Bit-identical keys and labels (models/ctr_data.py gen_ctr_np).
template <int R>
__global__ __launch_bounds__(256) void k_gen_ctr_r(uint64_t seed, long long sample_base, int B,
                                                   int F, long long V, double logV,
                                                   float tail_frac, float truth_scale,
                                                   float truth_bias, uint64_t* __restrict__ keys,
                                                   float* __restrict__ labels,
                                                   const long long* __restrict__ step_dev,
                                                   long long step_mul, long long step_add) {
  if (step_dev) sample_base = *step_dev * step_mul + step_add;
  __shared__ float sval[R * 256];
  __shared__ float sdot[256];
  const int spb = samples_per_block(F);
  const int t = threadIdx.x;
  const int ls = t / F, f = t - (t / F) * F;
  const long long sb = (long long)blockIdx.x * spb * R;  // first sample of the workgroup
  float wv[R];
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const long long s = sb + (long long)r * spb + ls;
    wv[r] = 0.f;
    if (ls < spb && s < B) {
      const uint64_t key = gen_ctr_key(seed, (uint64_t)(sample_base + s), f, V, logV, tail_frac);
      keys[s * F + f] = key;
      wv[r] = truth_weight(key, truth_scale);
    }
  }
#pragma unroll
  for (int r = 0; r < R; ++r) sval[r * 256 + t] = wv[r];
  __syncthreads();
  // R * spb sample sums, tps threads per sample (as packed_sample_sums)
  const int ns = R * spb;
  int tps = 8;
  while (tps > 1 && tps * ns > 256) tps >>= 1;
  const int gi = t / tps, k = t - gi * tps;
  float z = 0.f;
  if (gi < ns) {
    const float* v = sval + (gi / spb) * 256 + (gi % spb) * F;
    for (int ff = k; ff < F; ff += tps) z += v[ff];
  }
  for (int o = tps >> 1; o > 0; o >>= 1) z += __shfl_xor(z, o, 64);
  if (gi < ns && k == 0) sdot[gi] = z;
  __syncthreads();
  if (t < ns && sb + t < B)
    labels[sb + t] =
        gen_ctr_label(seed, (uint64_t)(sample_base + sb + t), sdot[t] + truth_bias);
}

// Fused LR forward/backward over B samples x F features (CTR-style fixed
// field count).  inv[j] indexes the pulled unique-key value/gradient rows.
__global__ __launch_bounds__(256) void k_lr_fwd_bwd_lds(const uint32_t* __restrict__ inv,
                                                    const float* __restrict__ xval,
                                                    const float* __restrict__ labels, int B, int F,
                                                    const float* __restrict__ uvals,
                                                    float* __restrict__ ugrad,
                                                    float* __restrict__ loss_sum,
                                                    float* __restrict__ pred) {
  __shared__ float sdot[256];
  __shared__ float sg[256];
  __shared__ float sloss[4];
  const int spb = samples_per_block(F);
  const int t = threadIdx.x;
  const int ls = t / F;
  const long long s0 = (long long)blockIdx.x * spb;
  if (t < spb) sdot[t] = 0.f;
  __syncthreads();
  const bool active = ls < spb && s0 + ls < B;
  const long long j = s0 * F + t;
  uint32_t u = kInvalidU;
  float x = 0.f;
  if (active) {
    u = inv[j];
    x = xval ? xval[j] : 1.f;
    if (u != kInvalidU) atomicAdd(&sdot[ls], uvals[u] * x);
  }
  __syncthreads();
  float l = 0.f;
  if (t < spb && s0 + t < B) {
    const float z = sdot[t];
    const float y = labels[s0 + t];
    const float p = 1.f / (1.f + __expf(-z));
    sg[t] = p - y;
    if (pred) pred[s0 + t] = p;
    // numerically stable logloss: softplus(z) - y*z
    l = fmaxf(z, 0.f) + __logf(1.f + __expf(-fabsf(z))) - y * z;
  }
  // block loss reduce (wave shuffle + LDS)
  for (int o = 32; o > 0; o >>= 1) l += __shfl_down(l, o, 64);
  if ((t & 63) == 0) sloss[t >> 6] = l;
  __syncthreads();
  if (t == 0 && loss_sum) ctr_addf(loss_sum, sloss[0] + sloss[1] + sloss[2] + sloss[3]);
  if (active && u != kInvalidU) atomicAdd(ugrad + u, sg[ls] * x);
}

// Same, one sample per lane group (F <= 64).
__global__ __launch_bounds__(256) void k_lr_fwd_bwd(const uint32_t* __restrict__ inv,
                                                    const float* __restrict__ xval,
                                                    const float* __restrict__ labels, int B, int F,
                                                    int L, const float* __restrict__ uvals,
                                                    float* __restrict__ ugrad,
                                                    float* __restrict__ loss_sum,
                                                    float* __restrict__ pred) {
  __shared__ float sloss[4];
  const int t = threadIdx.x, f = t & (L - 1);
  const long long s = (long long)blockIdx.x * (256 / L) + t / L;
  const bool active = f < F && s < B;
  const long long j = s * F + f;
  uint32_t u = kInvalidU;
  float x = 0.f, v = 0.f;
  if (active) {
    u = inv[j];
    x = xval ? xval[j] : 1.f;
    if (u != kInvalidU) v = uvals[u] * x;
  }
  const float z = group_sum(v, L);
  float l = 0.f, g = 0.f;
  if (s < B) {
    const float y = labels[s];
    const float p = 1.f / (1.f + __expf(-z));
    g = p - y;
    if (f == 0) {
      if (pred) pred[s] = p;
      l = fmaxf(z, 0.f) + __logf(1.f + __expf(-fabsf(z))) - y * z;
    }
  }
  const float bl = block_sum_256(l, sloss);
  if (t == 0 && loss_sum) ctr_addf(loss_sum, bl);
  if (active && u != kInvalidU) atomicAdd(ugrad + u, g * x);
}

// Factorization machine (binary features) fused forward/backward.
// Row of a key = [w | v_0..v_{K-1}] (dim = 1 + K).  Per sample
//   z = sum_i w_i + 1/2 * sum_f [(sum_i v_if)^2 - sum_i v_if^2]
//   dz/dw_i = 1, dz/dv_if = s_f - v_if  with s_f = sum_i v_if
// One lane per (sample, field) occurrence; per-sample sums in LDS; the
// per-key gradient rows (dim contiguous floats) leave as row atomics.
template <int DIM>
__global__ __launch_bounds__(256) void k_fm_fwd_bwd(const uint32_t* __restrict__ inv,
                                                    const float* __restrict__ labels, int B, int F,
                                                    const float* __restrict__ uvals,
                                                    float* __restrict__ ugrad,
                                                    float* __restrict__ loss_sum,
                                                    float* __restrict__ pred) {
  constexpr int K = DIM - 1;
  __shared__ float ssum[256 / 2][K > 0 ? K : 1];  // spb <= 128 (F >= 2)
  __shared__ float sz[128];
  __shared__ float sg[128];
  __shared__ float sloss[4];
  const int spb = samples_per_block(F);
  const int t = threadIdx.x, ls = t / F;
  const long long s0 = (long long)blockIdx.x * spb;
  for (int e = t; e < spb * K; e += 256) ssum[e / K][e % K] = 0.f;
  if (t < spb) sz[t] = 0.f;
  __syncthreads();
  const bool active = ls < spb && s0 + ls < B;
  const long long j = s0 * F + t;
  uint32_t u = kInvalidU;
  float row[DIM];
  if (active) u = inv[j];
  if (active && u != kInvalidU) {
    const float* r = uvals + (long long)u * DIM;
#pragma unroll
    for (int d = 0; d < DIM; ++d) row[d] = r[d];
    float sq = 0.f;
#pragma unroll
    for (int f = 0; f < K; ++f) {
      atomicAdd(&ssum[ls][f], row[1 + f]);
      sq += row[1 + f] * row[1 + f];
    }
    atomicAdd(&sz[ls], row[0] - 0.5f * sq);
  }
  __syncthreads();
  float l = 0.f;
  if (t < spb && s0 + t < B) {
    float z = sz[t];
#pragma unroll
    for (int f = 0; f < K; ++f) z += 0.5f * ssum[t][f] * ssum[t][f];
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
  if (active && u != kInvalidU) {
    const float g = sg[ls];
    float* gr = ugrad + (long long)u * DIM;
    atomicAdd(gr, g);
#pragma unroll
    for (int f = 0; f < K; ++f) atomicAdd(gr + 1 + f, g * (ssum[ls][f] - row[1 + f]));
  }
}

// FM forward, one sample per lane group (F <= 64), no atomics: emits the
// per-sample gradient factors instead of per-occurrence rows —
//   gs[s] = p - y,  gss[s][f] = gs[s] * sum_i v_if
// from which the per-key gradient is  [sum gs,  sum gss_f - v_f * sum gs]
// summed over the key's occurrences (k_bd_reduce_fm in bdedup.hip does that
// per dedup bucket in LDS and stores each unique row once).
template <int DIM>
__global__ __launch_bounds__(256) void k_fm_fwd_g(const uint32_t* __restrict__ inv, BdIndex ix,
                                                  const float* __restrict__ labels, int B, int F,
                                                  int L, const float* __restrict__ uvals,
                                                  float* __restrict__ gs, float* __restrict__ gss,
                                                  float* __restrict__ loss_sum,
                                                  float* __restrict__ pred) {
  constexpr int K = DIM - 1;
  __shared__ float sloss[4];
  const int t = threadIdx.x, f = t & (L - 1);
  const long long s = (long long)blockIdx.x * (256 / L) + t / L;
  const long long j = s * F + f;
  float row[DIM];
#pragma unroll
  for (int d = 0; d < DIM; ++d) row[d] = 0.f;
  if (f < F && s < B) {
    const uint32_t u = inv ? inv[j] : ix.uid(j);
    if (u != kInvalidU) {
      const float* r = uvals + (long long)u * DIM;
#pragma unroll
      for (int d = 0; d < DIM; ++d) row[d] = r[d];
    }
  }
  float sq = 0.f;
#pragma unroll
  for (int k = 0; k < K; ++k) sq += row[1 + k] * row[1 + k];
  float z = group_sum(row[0] - 0.5f * sq, L);
  float ssum[K > 0 ? K : 1];
#pragma unroll
  for (int k = 0; k < K; ++k) {
    ssum[k] = group_sum(row[1 + k], L);
    z += 0.5f * ssum[k] * ssum[k];
  }
  float l = 0.f;
  if (s < B) {
    const float y = labels[s];
    const float p = 1.f / (1.f + __expf(-z));
    const float g = p - y;
    if (f == 0) {
      gs[s] = g;
      if (pred) pred[s] = p;
      l = fmaxf(z, 0.f) + __logf(1.f + __expf(-fabsf(z))) - y * z;
    }
#pragma unroll
    for (int k = 0; k < K; ++k)
      if (f == k) gss[s * K + k] = g * ssum[k];
  }
  const float bl = block_sum_256(l, sloss);
  if (t == 0 && loss_sum) ctr_addf(loss_sum, bl);
}

void launch_fm_fwd_g(const uint32_t* inv, const BdIndex& ix, const float* labels, int B, int F,
                     int dim, const float* uvals, float* gs, float* gss, float* loss_sum,
                     float* pred, hipStream_t st) {
  if (B <= 0) return;
  if (F < 2 || F > kGroupMaxF) throw_error("fm_fwd_g: F must be in [2,64]");
  if (!inv && !(ix.pos_of && ix.luid && ix.bkt && ix.ubase))
    throw_error("fm_fwd_g: need inv or a complete BdIndex");
  const int L = group_lanes(F), spb = 256 / L;
  if (L < dim - 1) throw_error("fm_fwd_g: needs F >= K lanes per sample");
  const int blocks = (B + spb - 1) / spb;
  switch (dim) {
#define SS_FMG_CASE(DD)                                                                      \
  case DD:                                                                                   \
    hipLaunchKernelGGL(k_fm_fwd_g<DD>, dim3(blocks), dim3(256), 0, st, inv, ix, labels, B, F, \
                       L, uvals, gs, gss, loss_sum, pred);                                   \
    break;
    SS_FMG_CASE(2)
    SS_FMG_CASE(5)
    SS_FMG_CASE(9)
    SS_FMG_CASE(17)
#undef SS_FMG_CASE
    default:
      throw_error("fm_fwd_g: dim must be 1+K with K in {1,4,8,16}");
  }
  check_launch("k_fm_fwd_g");
}

void launch_fm_fwd_bwd(const uint32_t* inv, const float* labels, int B, int F, int dim,
                       const float* uvals, float* ugrad, float* loss_sum, float* pred,
                       hipStream_t st) {
  if (B <= 0) return;
  if (F < 2 || F > 256) throw_error("fm_fwd_bwd: F must be in [2,256]");
  const int spb = samples_per_block(F);
  const int blocks = (B + spb - 1) / spb;
  switch (dim) {
#define SS_FM_CASE(DD)                                                                       \
  case DD:                                                                                   \
    hipLaunchKernelGGL(k_fm_fwd_bwd<DD>, dim3(blocks), dim3(256), 0, st, inv, labels, B, F, uvals, \
                       ugrad, loss_sum, pred);                                               \
    break;
    SS_FM_CASE(2)
    SS_FM_CASE(5)
    SS_FM_CASE(9)
    SS_FM_CASE(17)
#undef SS_FM_CASE
    default:
      throw_error("fm_fwd_bwd: dim must be 1+K with K in {1,4,8,16}");
  }
  check_launch("k_fm_fwd_bwd");
}

void launch_gen_ctr(uint64_t seed, long long sample_base, int B, int F, long long vocab_per_field,
                    float tail_frac, float truth_scale, float truth_bias, uint64_t* keys,
                    float* labels, hipStream_t st, const long long* step_dev, long long step_mul,
                    long long step_add) {
  if (B <= 0) return;
  if (F < 1 || F > 256) throw_error("gen_ctr: F must be in [1,256]");
  const double logV = log((double)vocab_per_field + 1.0);
  const int spb = samples_per_block(F);
  // R sample groups per workgroup (SS_GEN_R: 1 / 2 / 4 / 8); 8 measured
  // 0.7227-0.7229 vs 0.7266-0.7278 ms per bench step (4), three A/B pairs
  static const int gr = [] {
    const char* e = std::getenv("SS_GEN_R");
    const int v = e ? std::atoi(e) : 8;
    return (v == 1 || v == 2 || v == 4) ? v : 8;
  }();
  if (gr > 1 && gr * spb <= 256) {
    const int g = gr * spb, nb = (B + g - 1) / g;
    if (gr == 8)
      hipLaunchKernelGGL(k_gen_ctr_r<8>, dim3(nb), dim3(256), 0, st, seed, sample_base, B, F,
                         vocab_per_field, logV, tail_frac, truth_scale, truth_bias, keys, labels,
                         step_dev, step_mul, step_add);
    else if (gr == 4)
      hipLaunchKernelGGL(k_gen_ctr_r<4>, dim3(nb), dim3(256), 0, st, seed, sample_base, B, F,
                         vocab_per_field, logV, tail_frac, truth_scale, truth_bias, keys, labels,
                         step_dev, step_mul, step_add);
    else
      hipLaunchKernelGGL(k_gen_ctr_r<2>, dim3(nb), dim3(256), 0, st, seed, sample_base, B, F,
                         vocab_per_field, logV, tail_frac, truth_scale, truth_bias, keys, labels,
                         step_dev, step_mul, step_add);
    check_launch("k_gen_ctr_r");
    return;
  }
  const int blocks = (B + spb - 1) / spb;
  hipLaunchKernelGGL(k_gen_ctr, dim3(blocks), dim3(256), 0, st, seed, sample_base, B, F,
                     vocab_per_field, logV, tail_frac, truth_scale, truth_bias, keys, labels,
                     step_dev, step_mul, step_add);
  check_launch("k_gen_ctr");
}

void launch_lr_fwd_bwd(const uint32_t* inv, const float* xval, const float* labels, int B, int F,
                       const float* uvals, float* ugrad, float* loss_sum, float* pred,
                       hipStream_t st) {
  if (B <= 0) return;
  if (F < 1 || F > 256) throw_error("lr_fwd_bwd: F must be in [1,256]");
  if (F <= kGroupMaxF) {
    const int L = group_lanes(F), spb = 256 / L;
    hipLaunchKernelGGL(k_lr_fwd_bwd, dim3((B + spb - 1) / spb), dim3(256), 0, st, inv, xval,
                       labels, B, F, L, uvals, ugrad, loss_sum, pred);
    check_launch("k_lr_fwd_bwd");
    return;
  }
  const int spb = samples_per_block(F);
  const int blocks = (B + spb - 1) / spb;
  hipLaunchKernelGGL(k_lr_fwd_bwd_lds, dim3(blocks), dim3(256), 0, st, inv, xval, labels, B, F,
                     uvals, ugrad, loss_sum, pred);
  check_launch("k_lr_fwd_bwd_lds");
}

}  // namespace ss
