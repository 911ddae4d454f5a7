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
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>
#include "ss/hash.h"

namespace ss {

static constexpr int kMaxSeg = 64;

struct DevTable {
  char* base;         // cap * stride bytes
  uint64_t cap;       // number of slots
  uint32_t stride;    // bytes per slot (multiple of 8)
  uint32_t key_off;   // byte offset of the key inside a slot
  uint32_t dim;       // parameter floats per row (what pull returns)
  uint32_t width;     // dim + optimizer-state floats
};

__device__ __forceinline__ uint64_t* slot_key(const DevTable& t, uint64_t s) {
  return reinterpret_cast<uint64_t*>(t.base + s * (uint64_t)t.stride + t.key_off);
}
__device__ __forceinline__ float* slot_row(const DevTable& t, uint64_t s) {
  return reinterpret_cast<float*>(t.base + s * (uint64_t)t.stride);
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

enum InitKind : int { kInitZero = 0, kInitUniform = 1, kInitNormal = 2 };
enum OptKind : int { kOptSGD = 0, kOptAdaGrad = 1, kOptFTRL = 2, kOptAdam = 3 };

struct InitParams {
  int kind;
  float scale;      // uniform: (u - 0.5) * scale ; normal: N(0,1) * scale
  float state_init; // initial value for optimizer state (AdaGrad init accumulator)
  uint64_t seed;
};

struct OptParams {
  int kind;
  float lr;
  float l1, l2;
  float eps;
  float beta1, beta2;   // Adam
  float bc1, bc2;       // Adam bias corrections 1/(1-b^t), host-computed per round
  float ftrl_alpha, ftrl_beta;
  float grad_scale;     // multiplies incoming gradients (e.g. 1/global_batch)
  float clip;           // |g| clip, 0 = off
};

__host__ __device__ inline int opt_state_width(int kind, int dim) {
  switch (kind) {
    case kOptSGD: return 0;
    case kOptAdaGrad: return dim;
    case kOptFTRL: return 2 * dim;
    case kOptAdam: return 2 * dim;
  }
  return 0;
}

// Deterministic per-(key, j) initial value: independent of the inserting lane,
// the shard layout and the world size — checkpoints are reproducible.
__device__ __forceinline__ float init_value(const InitParams& ip, uint64_t key, uint32_t j,
                                            uint32_t dim) {
  if (ip.kind == kInitZero) return 0.0f;
  uint64_t r = splitmix64(ip.seed ^ (key * 0x9E3779B97F4A7C15ull) ^ ((uint64_t)j << 48) ^ j);
  if (ip.kind == kInitUniform) {
    // reference word2vec convention: (rand/RAND_MAX - 0.5) / size  (vec1.h:223-226)
    return (u01(r) - 0.5f) * ip.scale;
  }
  float u1 = fmaxf(u01(r), 1e-7f);
  float u2 = u01(splitmix64(r));
  return sqrtf(-2.0f * __logf(u1)) * __cosf(6.2831853f * u2) * ip.scale;
}

// One coordinate of an optimizer step. `row` = params, `st` = state base.
__device__ __forceinline__ void opt_apply(const OptParams& op, float* row, float* st,
                                          uint32_t dim, uint32_t j, float g) {
  g *= op.grad_scale;
  if (op.clip > 0.f) g = fminf(fmaxf(g, -op.clip), op.clip);
  float w = row[j];
  switch (op.kind) {
    case kOptSGD: {
      g += op.l2 * w;
      row[j] = w - op.lr * g;
    } break;
    case kOptAdaGrad: {
      g += op.l2 * w;
      float h = st[j] + g * g;
      st[j] = h;
      row[j] = w - op.lr * g * __frsqrt_rn(h + op.eps);
    } break;
    case kOptFTRL: {
      // FTRL-Proximal (per-coordinate); w is kept materialised in the row.
      float z = st[j], n = st[dim + j];
      float n2 = n + g * g;
      float sigma = (sqrtf(n2) - sqrtf(n)) / op.ftrl_alpha;
      z += g - sigma * w;
      st[j] = z;
      st[dim + j] = n2;
      float az = fabsf(z);
      row[j] = az <= op.l1 ? 0.0f
                           : -(z - copysignf(op.l1, z)) /
                                 ((op.ftrl_beta + sqrtf(n2)) / op.ftrl_alpha + op.l2);
    } break;
    case kOptAdam: {
      g += op.l2 * w;
      float m = op.beta1 * st[j] + (1.f - op.beta1) * g;
      float v = op.beta2 * st[dim + j] + (1.f - op.beta2) * g * g;
      st[j] = m;
      st[dim + j] = v;
      row[j] = w - op.lr * (m * op.bc1) / (sqrtf(v * op.bc2) + op.eps);
    } break;
  }
}

}  // namespace ss
