// mb_atomics.hip — microbenchmark: random-access primitives on a large HBM
// table, to price the hash-table operations (probe load, CAS claim, plain
// claim store, float atomic add, slot RMW) on MI355X.
//
// build: hipcc --offload-arch=gfx950 -O3 tools/mb_atomics.hip -o tools/bin/mb_atomics
// run  : tools/bin/mb_atomics [table_GB=23] [n_ops=1500000]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                     \
  do {                                                                            \
    hipError_t e = (x);                                                           \
    if (e != hipSuccess) {                                                        \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); \
      std::exit(1);                                                               \
    }                                                                             \
  } while (0)

__device__ __forceinline__ unsigned long long mix(unsigned long long x) {
  x ^= x >> 33;
  x *= 0xff51afd7ed558ccdull;
  x ^= x >> 33;
  x *= 0xc4ceb9fe1a85ec53ull;
  x ^= x >> 33;
  return x;
}
__device__ __forceinline__ unsigned long long slot_of(long long i, unsigned long long nslots,
                                                      unsigned long long salt) {
  return __umul64hi(mix((unsigned long long)i * 0x9E3779B97F4A7C15ull + salt), nslots);
}

// slots are 16 B: [f32 w, f32 h, u64 key]
__global__ void k_load(const unsigned long long* t, unsigned long long nslots, long long n,
                       unsigned long long salt, unsigned long long* sink) {
  long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  unsigned long long v = t[2 * slot_of(i, nslots, salt) + 1];
  if (v == 0x123456789ull) sink[0] = v;
}
__global__ void k_store(unsigned long long* t, unsigned long long nslots, long long n,
                        unsigned long long salt) {
  long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  t[2 * slot_of(i, nslots, salt) + 1] = (unsigned long long)i;
}
__global__ void k_cas(unsigned long long* t, unsigned long long nslots, long long n,
                      unsigned long long salt, unsigned long long* sink) {
  long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  unsigned long long prev = atomicCAS(t + 2 * slot_of(i, nslots, salt) + 1, ~0ull, (unsigned long long)i);
  if (prev == 0x123456789ull) sink[0] = prev;
}
__global__ void k_load_cas(unsigned long long* t, unsigned long long nslots, long long n,
                           unsigned long long salt, unsigned long long* sink) {
  long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  unsigned long long* p = t + 2 * slot_of(i, nslots, salt) + 1;
  unsigned long long v = *p;
  if (v == ~0ull) v = atomicCAS(p, ~0ull, (unsigned long long)i);
  if (v == 0x123456789ull) sink[0] = v;
}
__global__ void k_fadd(float* t, unsigned long long nslots, long long n, unsigned long long salt) {
  long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  atomicAdd(t + 4 * slot_of(i, nslots, salt), 1.0f);
}
__global__ void k_rmw(float* t, unsigned long long nslots, long long n, unsigned long long salt) {
  long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  float2* p = reinterpret_cast<float2*>(t + 4 * slot_of(i, nslots, salt));
  float2 v = *p;
  v.y += 1.f;
  v.x -= 0.01f * rsqrtf(v.y);
  *p = v;
}
__global__ void k_fadd_small(float* t, unsigned long long nslots, long long n, unsigned long long salt) {
  long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  atomicAdd(t + slot_of(i, nslots, salt), 1.0f);
}

// one counter atomic per wave / per block onto a single address (the
// table-size / segment-count counters of the hot kernels)
__global__ void k_ctr_wave(unsigned long long* ctr, long long n) {
  long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n && (threadIdx.x & 63) == 0) atomicAdd(ctr, 1ull);
}
__global__ void k_ctr_block(unsigned long long* ctr, long long n) {
  long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n && threadIdx.x == 0) atomicAdd(ctr, 1ull);
}
__global__ void k_ctr_wave_sharded(unsigned long long* ctr, long long n) {
  long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n && (threadIdx.x & 63) == 0) atomicAdd(ctr + 16 * (blockIdx.x & 255), 1ull);
}
__global__ void k_nothing(unsigned long long* ctr, long long n) {
  long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i == n) ctr[1] = 0;
}

int main(int argc, char** argv) {
  double gb = argc > 1 ? atof(argv[1]) : 23.0;
  long long n = argc > 2 ? atoll(argv[2]) : 1500000;
  unsigned long long nslots = (unsigned long long)(gb * 1e9 / 16);
  unsigned long long* t;
  unsigned long long* sink;
  CK(hipMalloc(&t, nslots * 16));
  CK(hipMalloc(&sink, 64));
  CK(hipMemset(t, 0xFF, nslots * 16));
  float* small;
  const unsigned long long small_n = 1500000;
  CK(hipMalloc(&small, small_n * 4));
  CK(hipMemset(small, 0, small_n * 4));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  dim3 grid((unsigned)((n + 255) / 256)), blk(256);
  auto timeit = [&](const char* name, auto launch) {
    launch(1ull);  // warm
    CK(hipDeviceSynchronize());
    float best = 1e30f;
    for (int r = 0; r < 5; ++r) {
      CK(hipEventRecord(a));
      launch(100ull + r);
      CK(hipEventRecord(b));
      CK(hipEventSynchronize(b));
      float ms;
      CK(hipEventElapsedTime(&ms, a, b));
      if (ms < best) best = ms;
    }
    std::printf("%-34s %9.1f us  %7.2f Gop/s\n", name, best * 1e3, n / (best * 1e-3) / 1e9);
  };
  std::printf("table %.1f GB (%llu 16-B slots), %lld random ops per launch\n", gb, nslots, n);
  timeit("load u64 (probe)", [&](unsigned long long s) { hipLaunchKernelGGL(k_load, grid, blk, 0, 0, t, nslots, n, s, sink); });
  timeit("store u64 (plain claim)", [&](unsigned long long s) { hipLaunchKernelGGL(k_store, grid, blk, 0, 0, t, nslots, n, s); });
  CK(hipMemset(t, 0xFF, nslots * 16));
  timeit("CAS u64 (claim, empty slots)", [&](unsigned long long s) { hipLaunchKernelGGL(k_cas, grid, blk, 0, 0, t, nslots, n, s * 7919, sink); });
  timeit("load then CAS if empty", [&](unsigned long long s) { hipLaunchKernelGGL(k_load_cas, grid, blk, 0, 0, t, nslots, n, s * 104729, sink); });
  timeit("f32 atomicAdd (no return)", [&](unsigned long long s) { hipLaunchKernelGGL(k_fadd, grid, blk, 0, 0, (float*)t, nslots, n, s); });
  timeit("slot RMW (adagrad-like, plain)", [&](unsigned long long s) { hipLaunchKernelGGL(k_rmw, grid, blk, 0, 0, (float*)t, nslots, n, s); });
  timeit("f32 atomicAdd into 6 MB array", [&](unsigned long long s) { hipLaunchKernelGGL(k_fadd_small, grid, blk, 0, 0, small, small_n, n, s); });
  unsigned long long* ctr;
  CK(hipMalloc(&ctr, 256 * 128));
  CK(hipMemset(ctr, 0, 256 * 128));
  timeit("empty grid (launch floor)", [&](unsigned long long) { hipLaunchKernelGGL(k_nothing, grid, blk, 0, 0, ctr, n); });
  timeit("1 atomic/wave, one counter", [&](unsigned long long) { hipLaunchKernelGGL(k_ctr_wave, grid, blk, 0, 0, ctr, n); });
  timeit("1 atomic/block, one counter", [&](unsigned long long) { hipLaunchKernelGGL(k_ctr_block, grid, blk, 0, 0, ctr, n); });
  timeit("1 atomic/wave, 256 sharded ctrs", [&](unsigned long long) { hipLaunchKernelGGL(k_ctr_wave_sharded, grid, blk, 0, 0, ctr, n); });
  CK(hipFree(t));
  return 0;
}
