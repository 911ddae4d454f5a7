// mb_zatomic.hip — microbenchmark: pricing a bucket-order LR forward.
//
// The LR forward gathers one parameter per occurrence in sample order
// (occ[pos_of[j]]: a random 4-byte read from a 41 MB array).  The alternative
// is to walk occurrences in bucket order and add each parameter into its
// sample's logit, z[pj[p] / F] (a random 4-byte float atomic into a 1 MB
// array).  This prices both access patterns at the bench shape.
//
// build: hipcc --offload-arch=gfx950 -O3 tools/mb_zatomic.hip -o tools/bin/mb_zatomic
// run  : tools/bin/mb_zatomic [n_occ=10223616] [F=39]
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

// random permutation-like index: j -> (j * a + c) mod n (a odd, n arbitrary:
// not a bijection in general, but a uniform scatter, which is all we need)
__global__ void k_index(unsigned* idx, long long n, unsigned long long a) {
  long long j = blockIdx.x * (long long)blockDim.x + threadIdx.x;
  if (j < n) idx[j] = (unsigned)(((unsigned long long)j * a + 12345ull) % (unsigned long long)n);
}

// gather: out[j] = occ[pos[j]] summed per sample of F (one lane per occurrence)
__global__ __launch_bounds__(256) void k_gather(const unsigned* __restrict__ pos,
                                                const float* __restrict__ occ, float* out,
                                                long long n) {
  long long j = blockIdx.x * (long long)blockDim.x + threadIdx.x;
  if (j < n) out[j] = occ[pos[j]];
}

// atomics: z[pj[p] / F] += v[p] (bucket order, random sample)
template <int SCOPE>
__global__ __launch_bounds__(256) void k_zadd(const unsigned* __restrict__ pj,
                                              const float* __restrict__ v, float* z, long long n,
                                              int F) {
  long long p = blockIdx.x * (long long)blockDim.x + threadIdx.x;
  if (p < n) {
    const unsigned s = pj[p] / (unsigned)F;
    if (SCOPE == 0)
      atomicAdd(&z[s], v[p]);
    else
      __hip_atomic_fetch_add(&z[s], v[p], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// atomics without return, unsafe-fp path
__global__ __launch_bounds__(256) void k_zadd_nr(const unsigned* __restrict__ pj,
                                                 const float* __restrict__ v, float* z, long long n,
                                                 int F) {
  long long p = blockIdx.x * (long long)blockDim.x + threadIdx.x;
  if (p < n) unsafeAtomicAdd(&z[pj[p] / (unsigned)F], v[p]);
}

int main(int argc, char** argv) {
  const long long n = argc > 1 ? std::atoll(argv[1]) : 10223616ll;
  const int F = argc > 2 ? std::atoi(argv[2]) : 39;
  const long long B = (n + F - 1) / F;
  unsigned *pos, *pj;
  float *occ, *out, *v, *z;
  CK(hipMalloc(&pos, n * 4));
  CK(hipMalloc(&pj, n * 4));
  CK(hipMalloc(&occ, n * 4));
  CK(hipMalloc(&out, n * 4));
  CK(hipMalloc(&v, n * 4));
  CK(hipMalloc(&z, B * 4));
  const int T = 256;
  const long long G = (n + T - 1) / T;
  k_index<<<G, T>>>(pos, n, 2654435761ull);
  k_index<<<G, T>>>(pj, n, 40503ull * 65537ull + 2);
  CK(hipMemset(occ, 0, n * 4));
  CK(hipMemset(v, 0, n * 4));
  CK(hipDeviceSynchronize());
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  auto run = [&](const char* name, auto launch) {
    for (int w = 0; w < 3; ++w) launch();
    CK(hipEventRecord(e0));
    const int R = 20;
    for (int r = 0; r < R; ++r) launch();
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    std::printf("%-28s %8.1f us  (%.1f G ops/s)\n", name, 1000.f * ms / R, n / (1e6 * ms / R));
  };
  run("gather occ[pos[j]]", [&] { k_gather<<<G, T>>>(pos, occ, out, n); });
  run("atomicAdd z[pj/F]", [&] {
    CK(hipMemsetAsync(z, 0, B * 4));
    k_zadd<0><<<G, T>>>(pj, v, z, n, F);
  });
  run("agent fetch_add z[pj/F]", [&] {
    CK(hipMemsetAsync(z, 0, B * 4));
    k_zadd<1><<<G, T>>>(pj, v, z, n, F);
  });
  run("unsafeAtomicAdd z[pj/F]", [&] {
    CK(hipMemsetAsync(z, 0, B * 4));
    k_zadd_nr<<<G, T>>>(pj, v, z, n, F);
  });
  run("memset z only", [&] { CK(hipMemsetAsync(z, 0, B * 4)); });
  CK(hipDeviceSynchronize());
  return 0;
}
