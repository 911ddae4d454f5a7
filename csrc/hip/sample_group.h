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

// block-wide sum of one float per thread (256 threads), added to a sharded
// counter by thread 0
__device__ __forceinline__ float block_sum_256(float v, float* s4) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_down(v, o, 64);
  if ((threadIdx.x & 63) == 0) s4[threadIdx.x >> 6] = v;
  __syncthreads();
  return s4[0] + s4[1] + s4[2] + s4[3];
}

}  // namespace ss
