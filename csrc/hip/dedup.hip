// dedup.hip — worker-side batch key dedup + routing (gfx950).
//
// Replaces, per SURVEY §2.9.1:
//   K1  the caller-side std::unordered_set dedup that feeds
//       pull_with_barrier/push_with_barrier
//       (/root/reference/src/core/parameter/global_pull_access.h:40)
//   K2  arrange_local_vals / arrange_local_grads: route every key to
//       map[fmix64(key) % frag_num] and group per destination
//       (global_pull_access.h:58-72, global_push_access.h:80-99,
//        hashfrag.h:48-53)
//   K10 the (key,val) byte-stream serialisation — eliminated: unique keys are
//       written straight into per-destination segments at fixed displacement
//       dest*ucap, which is exactly the alltoallv send layout.
//
// One pass: every occurrence CASes its key into a power-of-two scratch table
// (load <= 0.5, scratch is memset to 0xFF once per round).  The lane that wins
// the CAS is the unique representative: it routes the key, takes a position
// inside its destination segment (LDS counter per destination, one global
// atomic per block and destination), writes the key and zeroes the gradient
// row the model will accumulate into.  A second tiny pass turns each
// occurrence's scratch slot into its unique id (the `inverse` index the model
// kernels gather/scatter through).
#include "ss_device.h"
#include "ss_launch.h"

namespace ss {

static constexpr uint32_t kInvalid = 0xFFFFFFFFu;

__global__ __launch_bounds__(256) void k_dedup_route(
    const uint64_t* __restrict__ keys, long long n, uint64_t* __restrict__ skeys,
    uint32_t* __restrict__ suid, unsigned long long smask, uint32_t* __restrict__ slot_of,
    RouteSpec rs, long long ucap, unsigned long long* __restrict__ ucount,
    uint64_t* __restrict__ ukeys, float* __restrict__ ugrad, int gdim) {
  __shared__ unsigned int lcnt[kMaxSeg];
  __shared__ unsigned long long lbase[kMaxSeg];
  for (int r = threadIdx.x; r < rs.nranks; r += blockDim.x) lcnt[r] = 0;
  __syncthreads();

  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  bool won = false;
  int dest = 0;
  unsigned int loff = 0;
  uint64_t key = kEmptyKey;
  unsigned long long s = 0;
  if (i < n) {
    key = keys[i];
    if (key == kEmptyKey) {
      slot_of[i] = kInvalid;
    } else {
      s = dedup_hash(key) & smask;
      for (;;) {  // terminates: scratch holds >= 2n slots, at most n distinct keys
        const uint64_t k = skeys[s];
        if (k == key) break;
        if (k == kEmptyKey) {
          const unsigned long long prev =
              atomicCAS(reinterpret_cast<unsigned long long*>(skeys + s), kEmptyKey, key);
          if (prev == kEmptyKey) {
            won = true;
            break;
          }
          if (prev == key) break;
        }
        s = (s + 1) & smask;
      }
      slot_of[i] = (uint32_t)s;
      if (won) {
        dest = rs.nranks == 1 ? 0 : rs.frag_map[fmix64(key) % (uint64_t)rs.frag_num];
        loff = atomicAdd(&lcnt[dest], 1u);
      }
    }
  }
  __syncthreads();
  for (int r = threadIdx.x; r < rs.nranks; r += blockDim.x)
    lbase[r] = lcnt[r] ? atomicAdd(&ucount[r], (unsigned long long)lcnt[r]) : 0ull;
  __syncthreads();
  if (won) {
    const unsigned long long uid = (unsigned long long)dest * ucap + lbase[dest] + loff;
    ukeys[uid] = key;
    suid[s] = (uint32_t)uid;
    if (ugrad)
      for (int j = 0; j < gdim; ++j) ugrad[uid * gdim + j] = 0.f;
  }
}

__global__ __launch_bounds__(256) void k_dedup_inverse(const uint32_t* __restrict__ slot_of,
                                                       const uint32_t* __restrict__ suid,
                                                       long long n, uint32_t* __restrict__ inv) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) {
    const uint32_t s = slot_of[i];
    inv[i] = s == kInvalid ? kInvalid : suid[s];
  }
}

__global__ __launch_bounds__(256) void k_route_keys(const uint64_t* __restrict__ keys, long long n,
                                                    RouteSpec rs, int* __restrict__ dest) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) dest[i] = rs.frag_map[fmix64(keys[i]) % (uint64_t)rs.frag_num];
}

// Row gather through an index (model side of K6): out[i] = src[idx[i]].
__global__ __launch_bounds__(256) void k_gather_rows(const float* __restrict__ src,
                                                     const uint32_t* __restrict__ idx, long long n,
                                                     int dim, float* __restrict__ out) {
  const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long e = t; e < n * dim; e += stride) {
    const long long i = e / dim;
    const int j = (int)(e - i * dim);
    const uint32_t r = idx[i];
    out[e] = r == kInvalid ? 0.f : src[(long long)r * dim + j];
  }
}

// Duplicate-merging scatter-add (K7 generic form): out[idx[i]] += src[i].
__global__ __launch_bounds__(256) void k_scatter_add_rows(const float* __restrict__ src,
                                                          const uint32_t* __restrict__ idx,
                                                          long long n, int dim,
                                                          float* __restrict__ out) {
  const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long e = t; e < n * dim; e += stride) {
    const long long i = e / dim;
    const int j = (int)(e - i * dim);
    const uint32_t r = idx[i];
    if (r != kInvalid) atomicAdd(out + (long long)r * dim + j, src[e]);
  }
}

static inline int blocks_for(long long n, int cap = 1 << 30) {
  long long b = (n + 255) / 256;
  if (b < 1) b = 1;
  return (int)(b > cap ? cap : b);
}

void launch_dedup_route(const uint64_t* keys, long long n, uint64_t* scratch_keys,
                        uint32_t* scratch_uid, unsigned long long scratch_cap,
                        uint32_t* slot_of, RouteSpec rs, long long ucap,
                        unsigned long long* ucount, uint64_t* ukeys, float* ugrad, int gdim,
                        hipStream_t st) {
  if (n <= 0) return;
  if ((scratch_cap & (scratch_cap - 1)) != 0 || scratch_cap < 2ull * (unsigned long long)n)
    throw_error("dedup scratch capacity must be a power of two >= 2n");
  if (rs.nranks < 1 || rs.nranks > kMaxSeg) throw_error("dedup: bad nranks");
  if (ucap < n) throw_error("dedup: per-destination capacity must be >= n");
  if ((unsigned long long)rs.nranks * (unsigned long long)ucap >= 0xFFFFFFFFull)
    throw_error("dedup: nranks*ucap overflows 32-bit unique ids");
  hipLaunchKernelGGL(k_dedup_route, dim3(blocks_for(n)), dim3(256), 0, st, keys, n, scratch_keys,
                     scratch_uid, scratch_cap - 1, slot_of, rs, ucap, ucount, ukeys, ugrad, gdim);
  check_launch("k_dedup_route");
}

void launch_dedup_inverse(const uint32_t* slot_of, const uint32_t* scratch_uid, long long n,
                          uint32_t* inv, hipStream_t st) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_dedup_inverse, dim3(blocks_for(n)), dim3(256), 0, st, slot_of, scratch_uid,
                     n, inv);
  check_launch("k_dedup_inverse");
}

void launch_route_keys(const uint64_t* keys, long long n, RouteSpec rs, int* dest,
                       hipStream_t st) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_route_keys, dim3(blocks_for(n)), dim3(256), 0, st, keys, n, rs, dest);
  check_launch("k_route_keys");
}

void launch_gather_rows(const float* src, const uint32_t* idx, long long n, int dim, float* out,
                        hipStream_t st) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_gather_rows, dim3(blocks_for(n * dim, 16384)), dim3(256), 0, st, src, idx,
                     n, dim, out);
  check_launch("k_gather_rows");
}

void launch_scatter_add_rows(const float* src, const uint32_t* idx, long long n, int dim,
                             float* out, hipStream_t st) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_scatter_add_rows, dim3(blocks_for(n * dim, 16384)), dim3(256), 0, st, src,
                     idx, n, dim, out);
  check_launch("k_scatter_add_rows");
}

}  // namespace ss
