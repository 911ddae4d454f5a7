// scan.h — row-wise exclusive scans of small [rows][cols] uint32 matrices
// (per-block counts -> per-block bases), as two PARALLEL phases instead of
// one long single-workgroup pass.  A single-workgroup scan sits on the
// critical path as a chain of dependent global round trips; behind the table
// kernels' random-access traffic each round trip stretches, which made the
// first single-block scans cost 80-150 us per step (profiles/).
//
//   phase 1  grid (ceil(cols/1024), rows): each 1024-wide group of a row is
//            scanned in place (exclusive) and its total stored in G[row][g];
//   phase 2  grid (rows), 64 threads: G[row][*] scanned in place (exclusive,
//            <= 64*kMaxGroupsPerLane groups) and the row total -> total[row].
// A consumer's exclusive prefix of element (r, c) is M[r][c] + G[r][c/1024].
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

namespace ss {

static constexpr int kScanGroup = 1024;

__device__ __forceinline__ unsigned int block_excl_scan_1024(unsigned int v, unsigned int* wsum,
                                                            unsigned int* total) {
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  unsigned int x = v;
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
  const unsigned int r = (w ? wsum[w - 1] : 0u) + x - v;
  if (total) *total = wsum[15];
  __syncthreads();
  return r;
}

// Exclusive scan across a workgroup of NW waves (NW <= 16); *total = sum.
template <int NW>
__device__ __forceinline__ unsigned int block_excl_scan(unsigned int v, unsigned int* wsum,
                                                        unsigned int* total) {
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  unsigned int x = v;
  for (int o = 1; o < 64; o <<= 1) {
    const unsigned int y = __shfl_up(x, o, 64);
    if (lane >= o) x += y;
  }
  if (lane == 63) wsum[w] = x;
  __syncthreads();
  if (w == 0) {
    unsigned int ws = lane < NW ? wsum[lane] : 0u;
    for (int o = 1; o < NW; o <<= 1) {
      const unsigned int y = __shfl_up(ws, o, 64);
      if (lane >= o) ws += y;
    }
    if (lane < NW) wsum[lane] = ws;
  }
  __syncthreads();
  const unsigned int r = (w ? wsum[w - 1] : 0u) + x - v;
  if (total) *total = wsum[NW - 1];
  __syncthreads();
  return r;
}

static __global__ __launch_bounds__(1024) void k_rowscan_p1(uint32_t* __restrict__ m, int cols,
                                                     uint32_t* __restrict__ G, int ngroups) {
  __shared__ unsigned int wsum[16];
  __shared__ unsigned int tot;
  const int row = blockIdx.y, g = blockIdx.x;
  const long long c = (long long)g * kScanGroup + threadIdx.x;
  uint32_t* r = m + (long long)row * cols;
  const unsigned int v = c < cols ? r[c] : 0u;
  const unsigned int e = block_excl_scan_1024(v, wsum, &tot);
  if (c < cols) r[c] = e;
  if (threadIdx.x == 0) G[(long long)row * ngroups + g] = tot;
}

static __global__ __launch_bounds__(64) void k_rowscan_p2(uint32_t* __restrict__ G, int ngroups,
                                                   uint32_t* __restrict__ total32,
                                                   unsigned long long* __restrict__ total64) {
  const int row = blockIdx.x, lane = threadIdx.x;
  uint32_t* g = G + (long long)row * ngroups;
  unsigned int carry = 0;
  for (int b = 0; b < ngroups; b += 64) {
    const unsigned int v = b + lane < ngroups ? g[b + lane] : 0u;
    unsigned int x = v;
    for (int o = 1; o < 64; o <<= 1) {
      const unsigned int y = __shfl_up(x, o, 64);
      if (lane >= o) x += y;
    }
    if (b + lane < ngroups) g[b + lane] = carry + x - v;
    carry += __shfl(x, 63, 64);
  }
  if (lane == 0) {
    if (total32) total32[row] = carry;
    if (total64) total64[row] = carry;
  }
}

__host__ __device__ inline int scan_groups(int cols) {
  return (cols + kScanGroup - 1) / kScanGroup;
}

// Short rows (<= 4 groups of 1024): one 64-thread wave scans a whole row —
// 1024-thread workgroups would wait for whole free CUs behind the table
// kernels on the other stream (measured: 83 us for a 313 x 313 scan).
static __global__ __launch_bounds__(64) void k_rowscan_wave(uint32_t* __restrict__ m, int cols,
                                                            uint32_t* __restrict__ G, int ngroups,
                                                            uint32_t* __restrict__ total32,
                                                            unsigned long long* __restrict__ total64) {
  const int row = blockIdx.x, lane = threadIdx.x;
  uint32_t* r = m + (long long)row * cols;
  unsigned int carry = 0;
  for (int b = 0; b < cols; b += 64) {
    const unsigned int v = b + lane < cols ? r[b + lane] : 0u;
    unsigned int x = v;
    for (int o = 1; o < 64; o <<= 1) {
      const unsigned int y = __shfl_up(x, o, 64);
      if (lane >= o) x += y;
    }
    if (b + lane < cols) r[b + lane] = carry + x - v;
    carry += __shfl(x, 63, 64);
  }
  for (int g = lane; g < ngroups; g += 64) G[(long long)row * ngroups + g] = 0u;
  if (lane == 0) {
    if (total32) total32[row] = carry;
    if (total64) total64[row] = carry;
  }
}

inline void launch_rowscan(uint32_t* m, int rows, int cols, uint32_t* G, uint32_t* total32,
                           unsigned long long* total64, hipStream_t st) {
  const int ng = scan_groups(cols);
  if (cols <= 4 * kScanGroup) {
    hipLaunchKernelGGL(k_rowscan_wave, dim3(rows), dim3(64), 0, st, m, cols, G, ng, total32,
                       total64);
    return;
  }
  hipLaunchKernelGGL(k_rowscan_p1, dim3(ng, rows), dim3(1024), 0, st, m, cols, G, ng);
  hipLaunchKernelGGL(k_rowscan_p2, dim3(rows), dim3(64), 0, st, G, ng, total32, total64);
}

}  // namespace ss
