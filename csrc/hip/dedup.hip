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
// Four kernels, and no same-address atomics (measured on MI355X: one
// atomic per wave onto a single counter serialises at ~12 ns each — 23K of
// them cost 285 us, more than the whole dedup):
//   1. insert:  every occurrence CASes its key into a power-of-two scratch
//      table (load <= 0.67).  The CAS winner is the key's representative: it
//      routes the key and takes a block-local offset in its destination from
//      an LDS counter; the block writes its per-destination counts with plain
//      stores, and the winner parks (block, dest, offset) in the slot's tag.
//   2+3. scan:  two parallel phases (scan.h) turn the per-block counts into
//      per-block bases and the per-destination totals.
//   4. finish:  every occurrence resolves its unique id from its slot's tag;
//      the winner also writes the key into the send segment, zeroes the
//      gradient row and resets its scratch slot to EMPTY — so the scratch
//      never needs a full memset between rounds.
#include "scan.h"
#include "ss_device.h"
#include "ss_launch.h"

namespace ss {

static constexpr uint32_t kInvalid = 0xFFFFFFFFu;
static constexpr uint32_t kWinBit = 0x80000000u;  // slot_of[i] flag: occurrence i won its key
// tag = (block << 15) | (dest << 9) | local_offset
__device__ __forceinline__ uint32_t mk_tag(uint32_t b, uint32_t d, uint32_t o) {
  return (b << 15) | (d << 9) | o;
}

__global__ __launch_bounds__(256) void k_dedup_insert(const uint64_t* __restrict__ keys, long long n,
                                                      uint64_t* __restrict__ skeys,
                                                      uint32_t* __restrict__ stag,
                                                      unsigned long long smask,
                                                      uint32_t* __restrict__ slot_of, RouteSpec rs,
                                                      uint32_t* __restrict__ blk_cnt, int nblocks) {
  __shared__ unsigned int lcnt[kMaxSeg];
  for (int r = threadIdx.x; r < rs.nranks; r += blockDim.x) lcnt[r] = 0;
  __syncthreads();
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  bool won = false;
  int dest = 0;
  unsigned long long s = 0;
  if (i < n) {
    const uint64_t key = keys[i];
    if (key == kEmptyKey) {
      slot_of[i] = kInvalid;
    } else {
      s = dedup_hash(key) & smask;
      for (;;) {  // terminates: scratch holds > n slots
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
      slot_of[i] = (uint32_t)s | (won ? kWinBit : 0u);
      if (won) dest = (int)rs.dest_of(key);
    }
  }
  unsigned int loff = 0;
  if (won) loff = atomicAdd(&lcnt[dest], 1u);  // LDS atomic (cheap)
  if (won) stag[s] = mk_tag(blockIdx.x, (uint32_t)dest, loff);
  __syncthreads();
  for (int r = threadIdx.x; r < rs.nranks; r += blockDim.x)
    blk_cnt[(long long)r * nblocks + blockIdx.x] = lcnt[r];
}

__global__ __launch_bounds__(256) void k_dedup_finish(const uint64_t* __restrict__ keys, long long n,
                                                      const uint32_t* __restrict__ slot_of,
                                                      const uint32_t* __restrict__ stag,
                                                      uint64_t* __restrict__ skeys,
                                                      const uint32_t* __restrict__ blk_base,
                                                      const uint32_t* __restrict__ grp_base,
                                                      int nblocks, int ngroups, long long ucap,
                                                      uint32_t* __restrict__ inv,
                                                      uint64_t* __restrict__ ukeys,
                                                      float* __restrict__ ugrad, int gdim) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t so = slot_of[i];
  if (so == kInvalid) {
    inv[i] = kInvalid;
    return;
  }
  const uint32_t s = so & ~kWinBit;
  const uint32_t tag = stag[s];
  const uint32_t b = tag >> 15, d = (tag >> 9) & 63u, o = tag & 511u;
  const unsigned long long uid = (unsigned long long)d * ucap +
                                 blk_base[(long long)d * nblocks + b] +
                                 grp_base[(long long)d * ngroups + b / kScanGroup] + o;
  inv[i] = (uint32_t)uid;
  if (so & kWinBit) {
    ukeys[uid] = keys[i];
    skeys[s] = kEmptyKey;  // only this round's winners dirtied the scratch
    if (ugrad)
      for (int j = 0; j < gdim; ++j) ugrad[uid * gdim + j] = 0.f;
  }
}

__global__ __launch_bounds__(256) void k_route_keys(const uint64_t* __restrict__ keys, long long n,
                                                    RouteSpec rs, int* __restrict__ dest) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) dest[i] = rs.frag_map[rs.frag_of(fmix64(keys[i]))];
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

int dedup_blocks(long long n) { return blocks_for(n); }
// blk_cnt buffer: [nranks][nblocks] counts followed by [nranks][ngroups] group bases
long long dedup_cnt_words(long long n, int nranks) {
  const int nb = blocks_for(n);
  return (long long)nranks * ((long long)nb + scan_groups(nb));
}

void launch_dedup_route(const uint64_t* keys, long long n, uint64_t* scratch_keys,
                        uint32_t* scratch_tag, unsigned long long scratch_cap, uint32_t* slot_of,
                        RouteSpec rs, long long ucap, unsigned long long* ucount, uint64_t* ukeys,
                        float* ugrad, int gdim, uint32_t* blk_cnt, uint32_t* inv,
                        hipStream_t st) {
  if (n <= 0) {
    check_hip(hipMemsetAsync(ucount, 0, sizeof(unsigned long long) * rs.nranks, st), "ucount");
    return;
  }
  if ((scratch_cap & (scratch_cap - 1)) != 0 || scratch_cap <= (unsigned long long)n)
    throw_error("dedup scratch capacity must be a power of two > n");
  if (rs.nranks < 1 || rs.nranks > kMaxSeg) throw_error("dedup: bad nranks");
  if (ucap < n) throw_error("dedup: per-destination capacity must be >= n");
  if ((unsigned long long)rs.nranks * (unsigned long long)ucap >= 0x7FFFFFFFull)
    throw_error("dedup: nranks*ucap overflows 31-bit unique ids");
  if (scratch_cap > 0x80000000ull) throw_error("dedup: scratch too large for 31-bit slots");
  const int nb = blocks_for(n);
  if (nb >= (1 << 17)) throw_error("dedup: too many keys per call (max 33M)");
  hipLaunchKernelGGL(k_dedup_insert, dim3(nb), dim3(256), 0, st, keys, n, scratch_keys, scratch_tag,
                     scratch_cap - 1, slot_of, rs, blk_cnt, nb);
  check_launch("k_dedup_insert");
  uint32_t* grp = blk_cnt + (long long)rs.nranks * nb;
  launch_rowscan(blk_cnt, rs.nranks, nb, grp, nullptr, ucount, st);
  check_launch("dedup rowscan");
  hipLaunchKernelGGL(k_dedup_finish, dim3(nb), dim3(256), 0, st, keys, n, slot_of, scratch_tag,
                     scratch_keys, blk_cnt, grp, nb, scan_groups(nb), ucap, inv, ukeys, ugrad,
                     gdim);
  check_launch("k_dedup_finish");
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
