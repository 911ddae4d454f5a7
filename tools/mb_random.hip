// mb_random.hip — random small-row access rates on MI355X (table-slot shape):
// one thread per row, rows of 16 B in a large array, indices random.
//   read8  : load one 8-byte key per row
//   rmw16  : load 16 B, update, store 16 B (AdaGrad-style slot update)
//   cas8   : one 64-bit CAS per row (insert of a new key)
//   store8 : one blind 8-byte store per row (the fused LR update's row write)
// Usage: mb_random [GiB=23] [rows=1500000] [regions=0]
//   regions > 0: every run of 1024 consecutive indices (one dedup bucket's
//   unique keys) falls inside one of `regions` equal slices of the table —
//   the access pattern of a table whose slot hash keeps a bucket's keys in
//   one region (TLB / DRAM locality test)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s\n", hipGetErrorString(e)); return 1; } } while (0)

__global__ void k_read8(const unsigned long long* __restrict__ tab, const unsigned long long* __restrict__ idx,
                        long long n, unsigned long long* __restrict__ out) {
  long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = tab[idx[i] * 2 + 1];
}
__global__ void k_rmw16(float4* __restrict__ tab, const unsigned long long* __restrict__ idx,
                        const float* __restrict__ g, long long n) {
  long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) {
    float4 v = tab[idx[i]];
    const float gi = g[i];
    v.y += gi * gi;
    v.x -= 0.05f * gi * rsqrtf(v.y + 1e-8f);
    tab[idx[i]] = v;
  }
}
__global__ void k_cas8(unsigned long long* __restrict__ tab, const unsigned long long* __restrict__ idx,
                       long long n, unsigned long long* __restrict__ out) {
  long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = atomicCAS(tab + idx[i] * 2 + 1, ~0ull, (unsigned long long)i);
}

__global__ void k_store8(unsigned long long* __restrict__ tab,
                         const unsigned long long* __restrict__ idx, long long n) {
  long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) tab[idx[i] * 2] = (unsigned long long)i;
}

int main(int argc, char** argv) {
  const double gib = argc > 1 ? atof(argv[1]) : 23.0;
  const long long n = argc > 2 ? atoll(argv[2]) : 1500000;
  const long long regions = argc > 3 ? atoll(argv[3]) : 0;
  const size_t rows = (size_t)(gib * (1ull << 30) / 16);
  unsigned long long *tab, *idx, *out;
  float* g;
  CK(hipMalloc(&tab, rows * 16));
  CK(hipMemset(tab, 0xFF, rows * 16));
  CK(hipMalloc(&idx, n * 8));
  CK(hipMalloc(&out, n * 8));
  CK(hipMalloc(&g, n * 4));
  std::vector<unsigned long long> h(n);
  unsigned long long x = 88172645463325252ull;
  const size_t rrows = regions > 0 ? rows / (size_t)regions : rows;
  size_t rbase = 0;
  for (long long i = 0; i < n; ++i) {
    x ^= x << 13; x ^= x >> 7; x ^= x << 17;
    if (regions > 0 && i % 1024 == 0) rbase = (x >> 7) % (size_t)regions * rrows;
    x ^= x << 13; x ^= x >> 7; x ^= x << 17;
    h[i] = regions > 0 ? rbase + x % rrows : x % rows;
  }
  CK(hipMemcpy(idx, h.data(), n * 8, hipMemcpyHostToDevice));
  CK(hipMemset(g, 0, n * 4));
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  const int bs = 256, gr = (int)((n + bs - 1) / bs);
  for (int kind = 0; kind < 4; ++kind) {
    float best = 1e9;
    for (int rep = 0; rep < 6; ++rep) {
      if (kind == 2) CK(hipMemset(tab, 0xFF, rows * 16));
      hipEventRecord(a);
      if (kind == 0) hipLaunchKernelGGL(k_read8, gr, bs, 0, 0, tab, idx, n, out);
      if (kind == 1) hipLaunchKernelGGL(k_rmw16, gr, bs, 0, 0, (float4*)tab, idx, g, n);
      if (kind == 2) hipLaunchKernelGGL(k_cas8, gr, bs, 0, 0, tab, idx, n, out);
      if (kind == 3) hipLaunchKernelGGL(k_store8, gr, bs, 0, 0, tab, idx, n);
      hipEventRecord(b);
      hipEventSynchronize(b);
      float ms;
      hipEventElapsedTime(&ms, a, b);
      if (rep && ms < best) best = ms;
    }
    const char* nm[4] = {"read8", "rmw16", "cas8", "store8"};
    printf("%-6s rows=%lld table=%.1f GiB: %.1f us  %.2f G rows/s\n", nm[kind], n, gib, best * 1e3,
           n / (best * 1e-3) / 1e9);
  }
  return 0;
}
