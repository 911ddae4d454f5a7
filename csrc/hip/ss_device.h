// ss_device.h — device-side data structures shared by the gfx950 kernels.
//
// HBM sparse table (replaces the reference's per-shard google::dense_hash_map
// + pthread rwlock, /root/reference/src/core/parameter/sparsetable.h:5-67):
//
//   * one open-addressed table per GPU shard, array-of-slots layout:
//       slot = [ row: `width` fp32 (params then optimizer state) | pad | key u64 ]
//     so a lookup-or-init + row gather touches the same cache line(s): for
//     sparse LR (width 2: w, adagrad-acc) a slot is exactly 16 B and one random
//     HBM access serves probe + gather + update.
//   * linear probing from fastrange(table_hash(key), cap) — capacities need
//     not be powers of two, so a shard can fill whatever HBM it is given.
//   * lock-free: 64-bit CAS on the key word claims a slot; the claiming lane
//     initialises the row. Readers of a freshly inserted row are always in a
//     later kernel (stream order = the happens-before edge), so no per-slot
//     ready flag or spin is needed.
//   * region tables (rbits > 0, scalar LR shards): the slots form R = 2^rbits
//     equal regions and a key probes only inside the region of its hash's top
//     rbits bits (home slot, then linear, wrapping at the region's end).  The
//     1-GPU dedup buckets whole regions (bd_bucket with RouteSpec.rbits), so
//     ONE workgroup owns every insert into a region during a pull: it claims
//     empty slots in LDS instead of with a device-scope CAS, and the fused
//     merge + update stores [w | h | key] in one 16-byte store (table.hip
//     k_pull_claim_bk, bdedup.hip k_bd_reduce) — no atomic, no second write
//     to the claimed line.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>
#include "ss/hash.h"
#include "ss/optim.h"

namespace ss {

static constexpr int kMaxSeg = 64;

// Sharded counters.  Measured on MI355X: one atomic per wave onto a single
// address serialises at ~12 ns (23K wave atomics = 285 us), while the same
// adds spread over 256 cache-line-separated shards cost nothing measurable.
// Every accumulate-only counter (table size, loss sums) is a [256 x 128 B]
// array; readers sum the shards.
static constexpr int kCtrShards = 256;
__device__ __forceinline__ void ctr_add(unsigned long long* base, unsigned long long v) {
  atomicAdd(base + 16 * (blockIdx.x & (kCtrShards - 1)), v);
}
__device__ __forceinline__ void ctr_addf(float* base, float v) {
  atomicAdd(base + 32 * (blockIdx.x & (kCtrShards - 1)), v);
}

struct DevTable {
  char* base;         // cap * stride bytes
  uint64_t cap;       // number of slots
  uint32_t stride;    // bytes per slot (multiple of 8)
  uint32_t key_off;   // byte offset of the key inside a slot
  uint32_t dim;       // parameter floats per row (what pull returns)
  uint32_t width;     // dim + optimizer-state floats
  // 1: every EMPTY slot's row already holds the initial row (key-independent
  // init, filled at allocation), so an insert is the key CAS alone — no
  // second write to the freshly claimed line
  uint32_t prefilled;
  uint32_t row_off;   // byte offset of the row (params, then optimizer state)
  // 1: compact rows — parameters and optimizer state stored as bf16 (half
  // the bytes per slot: capacity for the 10B-key FM table), math in fp32;
  // read / written through row_ld / row_st
  uint32_t bf16;
  // region tables: log2 of the region count (0: one region, the whole
  // table) and slots per region (cap = rlen << rbits)
  uint32_t rbits;
  uint64_t rlen;
};

// The probe sequence of a key: home slot fastrange(table_hash, cap), then
// linear inside [lo, hi) — the key's region (the whole table when rbits is
// 0).  fastrange keeps the home inside the region of the hash's top bits:
// floor(floor(h * cap / 2^64) / rlen) == floor(h * 2^rbits / 2^64) for
// cap == rlen * 2^rbits.
struct ProbeSeq {
  uint64_t s, lo, hi;
  __device__ __forceinline__ void next() { s = (s + 1 == hi) ? lo : s + 1; }
  __device__ __forceinline__ uint64_t len() const { return hi - lo; }
};
__device__ __forceinline__ ProbeSeq probe_seq(const DevTable& t, uint64_t key) {
  const uint64_t h = table_hash(key);
  ProbeSeq p;
  p.s = fastrange64(h, t.cap);
  if (t.rbits) {
    p.lo = (h >> (64 - t.rbits)) * t.rlen;
    p.hi = p.lo + t.rlen;
  } else {
    p.lo = 0;
    p.hi = t.cap;
  }
  return p;
}

__device__ __forceinline__ uint64_t* slot_key(const DevTable& t, uint64_t s) {
  return reinterpret_cast<uint64_t*>(t.base + s * (uint64_t)t.stride + t.key_off);
}
__device__ __forceinline__ float* slot_row(const DevTable& t, uint64_t s) {
  return reinterpret_cast<float*>(t.base + s * (uint64_t)t.stride + t.row_off);
}

// coordinate j of slot s's row as fp32, either storage format.  A bf16 word
// still holding the empty-slot fill (0xFFFF) reads as the fp32 fill
// 0xFFFFFFFF, so "not written yet" (table.hip fresh_or) means the same.
__device__ __forceinline__ float row_ld(const DevTable& t, uint64_t s, uint32_t j) {
  const char* r = t.base + s * (uint64_t)t.stride + t.row_off;
  if (t.bf16) {
    const uint32_t u = reinterpret_cast<const unsigned short*>(r)[j];
    return __uint_as_float(u == 0xFFFFu ? 0xFFFFFFFFu : (u << 16));
  }
  return reinterpret_cast<const float*>(r)[j];
}

// v as a compact row holds it (bf16 round to nearest even), else v: what a
// pull returns for a row it just initialised equals what later pulls read
__device__ __forceinline__ float row_round(const DevTable& t, float v) {
  if (!t.bf16) return v;
  uint32_t u = __float_as_uint(v);
  if ((u & 0x7F800000u) != 0x7F800000u) u += 0x7FFFu + ((u >> 16) & 1u);
  return __uint_as_float(u & 0xFFFF0000u);
}

// v as the bf16 word a compact row stores for coordinate j of slot s:
// rounded stochastically when `sr` (an optimizer step: round-to-nearest would
// drop every update below half an ulp — 1/512 of the weight — so small steps
// would never move a weight), else to nearest even; NaN / Inf keep their top
// bits (the init marker)
__device__ __forceinline__ unsigned short bf16_bits(uint64_t s, uint32_t j, float v, bool sr) {
  uint32_t u = __float_as_uint(v);
  if ((u & 0x7F800000u) != 0x7F800000u) {
    if (sr) {
      // dither from (slot, coordinate, value bits, the wall clock): the
      // clock makes a row that returns to the same value after an update
      // that rounded away draw a fresh dither next time (value bits alone
      // repeat the same rounding forever); no state, works under graph replay
      uint32_t h = (uint32_t)s * 0x9E3779B1u ^ (j * 0x85EBCA77u) ^ u ^
                   ((uint32_t)wall_clock64() * 0xC2B2AE35u);
      h ^= h >> 15;
      h *= 0x2C1B3C6Du;
      h ^= h >> 12;
      u += h & 0xFFFFu;
    } else {
      u += 0x7FFFu + ((u >> 16) & 1u);
    }
  }
  return (unsigned short)(u >> 16);
}
// a stored bf16 word as fp32; the empty-slot fill (0xFFFF) reads as the fp32
// fill 0xFFFFFFFF
__device__ __forceinline__ float bf16_val(uint32_t u16) {
  return __uint_as_float(u16 == 0xFFFFu ? 0xFFFFFFFFu : (u16 << 16));
}

// store v as coordinate j (bf16: bf16_bits, stochastic rounding when `sr`)
__device__ __forceinline__ void row_st(const DevTable& t, uint64_t s, uint32_t j, float v,
                                       bool sr = false) {
  char* r = t.base + s * (uint64_t)t.stride + t.row_off;
  if (!t.bf16) {
    reinterpret_cast<float*>(r)[j] = v;
    return;
  }
  reinterpret_cast<unsigned short*>(r)[j] = bf16_bits(s, j, v, sr);
}

// A list of (offset, count) segments inside one buffer.  The collective
// round engine lays every per-peer message out at a fixed displacement
// (peer * capacity), so the server kernels walk N segments of one buffer
// instead of packing/unpacking.  If `dev_count` is set, the list is a single
// segment at offset 0 whose length lives in device memory (written by an
// earlier kernel in the same stream): no host round-trip on the 1-GPU path.
struct SegList {
  int nseg;
  const long long* dev_count;
  long long off[kMaxSeg];
  long long prefix[kMaxSeg + 1];  // prefix[i] = sum of counts before segment i
};

__device__ __forceinline__ long long seg_total(const SegList& sl) {
  return sl.dev_count ? *sl.dev_count : sl.prefix[sl.nseg];
}
// flat index -> buffer position (and segment id)
__device__ __forceinline__ long long seg_pos(const SegList& sl, long long g, int* seg) {
  if (sl.dev_count) { *seg = 0; return g; }
  int s = 0;
  while (s + 1 < sl.nseg && g >= sl.prefix[s + 1]) ++s;
  *seg = s;
  return sl.off[s] + (g - sl.prefix[s]);
}

// N>1 rounds: a rank's own segment of a mailbox exchange is not copied into
// its arena — the positions [lo, hi) (source / destination == this rank, in
// rows) are read from / written to the local buffer the put would have copied
// (the same row index), every other position from / to the arena
struct SelfSeg {
  char* ptr = nullptr;
  long long lo = 0, hi = 0;
  // record exchange, own gradients (k_bd_reduce at the server): the rank's
  // own records were never written out per occurrence — position p's
  // gradient is ptr[ind[p] / F] (the worker's per-sample gradient) times
  // xv[ind[p]] (file feature values; null: binary features), ind = the
  // worker's spj (send position -> occurrence)
  const uint32_t* ind = nullptr;
  const float* xv = nullptr;
  uint32_t F = 1;
  template <typename T>
  __host__ __device__ __forceinline__ T* pick(T* arena, long long pos) const {
    return (ptr && pos >= lo && pos < hi) ? reinterpret_cast<T*>(ptr) : arena;
  }
  __device__ __forceinline__ bool mine(long long pos) const {
    return ptr && pos >= lo && pos < hi;
  }
  // the scalar gradient at received position j (arena rows are per position;
  // the F of the arena's layout is `af`)
  __device__ __forceinline__ float grad(const float* arena, uint32_t j, uint32_t af) const {
    if (ind && mine(j)) {
      const uint32_t q = ind[j];
      const float g = reinterpret_cast<const float*>(ptr)[q / F];
      return xv ? g * xv[q] : g;
    }
    return pick(arena, (long long)j)[j / af];
  }
};

// slots of a per-workgroup LDS hash table for up to n distinct keys: the
// power of two >= 2n (load <= 1/2), at least 64, at most cap
__device__ __forceinline__ uint32_t lds_table_size(uint32_t n, uint32_t cap) {
  uint32_t ts = 64;
  while (ts < 2 * n && ts < cap) ts <<= 1;
  return ts;
}

// N>1 server sub-bucket of a key (server.hip): the top bits of dedup_hash's
// low word.  The sender's bucket took the high word's top bits and its LDS
// slot the low word's low bits, so the three are independent.
__device__ __forceinline__ uint32_t srv_sub(uint64_t key, int m) {
  return m <= 1 ? 0u : __umulhi((uint32_t)dedup_hash(key), (uint32_t)m);
}

}  // namespace ss
