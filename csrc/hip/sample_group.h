// sample_group.h — "one sample per lane group" layout for per-sample
// reductions over F <= 64 features (gfx950, wave64).
//
// A sample's F feature lanes form an aligned group of L = next_pow2(F) lanes
// inside one wave, so its sum is log2(L) __shfl_xor steps with no LDS and no
// atomics.  (The first kernels packed samples back to back — 256/F samples per
// workgroup — and summed with LDS float atomics; 39 lanes adding to one LDS
// word serialise, which made the per-sample dot the largest cost of k_gen_ctr
// and the LR forward.)  Lanes f >= F of a group idle: 25 of 64 for the 39-field
// CTR layout, which these memory-bound kernels can afford.
#pragma once
#include <hip/hip_runtime.h>

namespace ss {

static constexpr int kGroupMaxF = 64;

__host__ __device__ inline int group_lanes(int F) {
  int L = 1;
  while (L < F) L <<= 1;
  return L;
}

__device__ __forceinline__ float group_sum(float v, int L) {
  for (int o = L >> 1; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// Per-sample sums in the PACKED layout (256/F samples per 256-thread block,
// sample ls on threads [ls*F, ls*F+F)) without LDS atomics: every thread
// stores its value, then TPS threads per sample add a strided share and
// reduce with shuffles (F lanes adding into one LDS word with atomics
// serialise F-way).  vals: 256 floats of LDS; sums: spb floats of LDS.
// Every thread of the block must call it (two barriers).
__device__ __forceinline__ void packed_sample_sums(float v, int F, int spb, float* vals,
                                                   float* sums) {
  const int t = threadIdx.x;
  vals[t] = v;
  __syncthreads();
  int tps = 8;  // threads per sample: 8, or fewer when samples are many
  while (tps > 1 && tps * spb > 256) tps >>= 1;
  const int gi = t / tps, k = t - gi * tps;
  float s = 0.f;
  if (gi < spb)
    for (int f = k; f < F; f += tps) s += vals[gi * F + f];
  for (int o = tps >> 1; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
  if (gi < spb && k == 0) sums[gi] = s;
  __syncthreads();
}

// block-wide sum of one float per thread (256 threads), added to a sharded
// counter by thread 0
__device__ __forceinline__ float block_sum_256(float v, float* s4) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_down(v, o, 64);
  if ((threadIdx.x & 63) == 0) s4[threadIdx.x >> 6] = v;
  __syncthreads();
  return s4[0] + s4[1] + s4[2] + s4[3];
}

}  // namespace ss
