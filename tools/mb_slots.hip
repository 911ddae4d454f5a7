// mb_slots.hip — steady-state cost of the table's per-step random slot
// traffic on MI355X, write-back included: ITER rounds, each a "pull" kernel
// (one random slot read per row, optionally a CAS on a fresh slot) followed by
// an "update" kernel (one random slot write per row), timed over all rounds so
// the L2 / MALL write-back of the stores is paid inside the measurement (a
// single store kernel's time hides it: 3.3M 8-byte stores "cost" 60 us while
// they fit the 256 MB MALL).
//
//   mode read16      : 16-byte read per row (the claimed pull's probe)
//   mode read16+cas8 : + a CAS on an empty slot for 62% of rows (CAS inserts)
//   mode store8      : blind 8-byte store (the old fused merge: w, h)
//   mode store16     : blind 16-byte store ([w | h | key], the claimed merge)
//   stride S         : slot size in bytes (16, 32, 64) — one slot per row, the
//                      store writes S bytes (64: a whole 64-byte line)
//
// Usage: mb_slots [GiB=32] [rows=5300000] [iters=20]
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s\n", hipGetErrorString(e)); return 1; } } while (0)

__global__ void k_read(const char* __restrict__ tab, const unsigned long long* __restrict__ idx,
                       long long n, int stride, float* __restrict__ out) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint4 v = *reinterpret_cast<const uint4*>(tab + idx[i] * stride);
  out[i] = __uint_as_float(v.x ^ v.w);
}
__global__ void k_read_cas(char* __restrict__ tab, const unsigned long long* __restrict__ idx,
                           const unsigned long long* __restrict__ idx2, long long n, int stride,
                           float* __restrict__ out) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint4 v = *reinterpret_cast<const uint4*>(tab + idx[i] * stride);
  float r = __uint_as_float(v.x ^ v.w);
  if ((i * 0x9E3779B1u) % 100 < 62) {  // a new key: claim an empty slot
    unsigned long long* kp = reinterpret_cast<unsigned long long*>(tab + idx2[i] * stride + 8);
    r += (float)(atomicCAS(kp, ~0ull, (unsigned long long)i) & 1);
  }
  out[i] = r;
}
__global__ void k_store(char* __restrict__ tab, const unsigned long long* __restrict__ idx,
                        long long n, int stride, int bytes) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  char* p = tab + idx[i] * stride;
  const uint4 v = make_uint4((unsigned)i, 1u, 2u, 3u);
  if (bytes == 8) {
    *reinterpret_cast<uint2*>(p) = make_uint2((unsigned)i, 1u);
  } else {
    for (int b = 0; b < bytes; b += 16) *reinterpret_cast<uint4*>(p + b) = v;
  }
}

int main(int argc, char** argv) {
  const double gib = argc > 1 ? atof(argv[1]) : 32.0;
  const long long n = argc > 2 ? atoll(argv[2]) : 5300000;
  const int iters = argc > 3 ? atoi(argv[3]) : 20;
  const size_t bytes = (size_t)(gib * (1ull << 30));
  char* tab;
  unsigned long long *idx, *idx2;
  float* out;
  CK(hipMalloc(&tab, bytes));
  CK(hipMemset(tab, 0xFF, bytes));
  CK(hipMalloc(&idx, (size_t)iters * n * 8));
  CK(hipMalloc(&idx2, (size_t)iters * n * 8));
  CK(hipMalloc(&out, n * 4));
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  const int bs = 256, gr = (int)((n + bs - 1) / bs);
  const int strides[3] = {16, 32, 64};
  for (int si = 0; si < 3; ++si) {
    const int stride = strides[si];
    const size_t rows = bytes / stride;
    std::vector<unsigned long long> h((size_t)iters * n), h2((size_t)iters * n);
    unsigned long long x = 88172645463325252ull + stride;
    for (auto& v : h) { x ^= x << 13; x ^= x >> 7; x ^= x << 17; v = x % rows; }
    for (auto& v : h2) { x ^= x << 13; x ^= x >> 7; x ^= x << 17; v = x % rows; }
    CK(hipMemcpy(idx, h.data(), h.size() * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(idx2, h2.data(), h2.size() * 8, hipMemcpyHostToDevice));
    // (pull kind, store bytes): 0 read / 1 read+cas; store 0 = none
    const int cases[6][2] = {{0, 0}, {1, 0}, {0, 8}, {0, 16}, {1, 8}, {0, stride}};
    const char* names[6] = {"read16", "read16+cas8", "read16|store8", "read16|store16",
                            "read16+cas8|store8", "read16|storeS"};
    for (int c = 0; c < 6; ++c) {
      if (c == 5 && stride == 16) continue;
      hipDeviceSynchronize();
      hipEventRecord(a);
      for (int it = 0; it < iters; ++it) {
        const unsigned long long* ix = idx + (size_t)it * n;
        if (cases[c][0] == 0)
          hipLaunchKernelGGL(k_read, gr, bs, 0, 0, tab, ix, n, stride, out);
        else
          hipLaunchKernelGGL(k_read_cas, gr, bs, 0, 0, tab, ix, idx2 + (size_t)it * n, n, stride,
                             out);
        if (cases[c][1])
          hipLaunchKernelGGL(k_store, gr, bs, 0, 0, tab, ix, n, stride, cases[c][1]);
      }
      hipEventRecord(b);
      hipEventSynchronize(b);
      float ms;
      hipEventElapsedTime(&ms, a, b);
      printf("stride %2d %-20s rows=%lld: %7.1f us per round\n", stride, names[c], n,
             ms * 1e3 / iters);
    }
  }
  return 0;
}
