// table.hip — HBM open-addressed parameter table kernels (gfx950).
//
// Replaces, per SURVEY §2.9.1:
//   K3  server lookup-or-init  (PullAccessAgent::get_pull_value,
//       /root/reference/src/core/parameter/sparsetable.h:142-149)
//   K4  row gather for the pull response (server/init.h:61-68)
//   K5  server push apply      (PushAccessAgent::apply_push_value,
//       sparsetable.h:181-192; server/init.h:119-125)
//   K8  occupied-slot compaction for the text/binary dump
//       (SparseTableShard operator<<, sparsetable.h:49-56)
//
// Work decomposition: a *group* of G lanes (G in {1,4,16,64}) owns one key.
// The group leader walks the probe sequence (one 8-byte key load per step,
// the row sits in the same slot so the following gather is a sequential read
// of the same/adjacent lines); the slot is broadcast with a width-G shuffle
// and the G lanes sweep the row.  G=1 for sparse-LR rows (width 2 = 8 B),
// G=16/64 for embedding rows (word2vec / FM), so a 64-wide wavefront always
// has all lanes busy on HBM traffic.
#include <algorithm>
#include <cstdlib>
#include <stdexcept>

#include "ss_device.h"
#include "ss_launch.h"

namespace ss {

static constexpr int kApplyRegs = 4;  // row coordinates per lane held in registers


__device__ __forceinline__ long long probe_slot(const DevTable& t, uint64_t key, bool insert,
                                                bool* inserted) {
  ProbeSeq ps = probe_seq(t, key);
  for (uint64_t n = 0, len = ps.len(); n < len; ++n, ps.next()) {
    const uint64_t s = ps.s;
    uint64_t* kp = slot_key(t, s);
    // A slot's key only ever changes EMPTY -> key inside a launch, so a stale
    // plain load can only read EMPTY; the CAS below then returns the truth.
    uint64_t k = *kp;
    if (k == key) return (long long)s;
    if (k == kEmptyKey) {
      if (!insert) return -1;
      unsigned long long prev =
          atomicCAS(reinterpret_cast<unsigned long long*>(kp), kEmptyKey, key);
      if (prev == kEmptyKey) {
        *inserted = true;
        return (long long)s;
      }
      if (prev == key) return (long long)s;
    }
  }
  return -1;
}

__device__ __forceinline__ unsigned long long wave_sum_u64(unsigned long long v) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_down(v, o, 64);
  return v;
}

template <int G>
__device__ __forceinline__ void init_row(const DevTable& t, const InitParams& ip, long long slot,
                                         uint64_t key, int lg) {
  if (t.prefilled) return;
  for (uint32_t j = lg; j < t.width; j += G)
    row_st(t, slot, j, j < t.dim ? init_value(ip, key, j, t.dim) : ip.state_init);
}

// K3: lookup-or-init (insert=1) or lookup-only (insert=0). slots_out[pos] = slot | -1.
template <int G>
__global__ __launch_bounds__(256) void k_probe(DevTable t, const uint64_t* __restrict__ keys,
                                               SegList sl, long long* __restrict__ slots_out,
                                               InitParams ip, int insert,
                                               unsigned long long* size_ctr, int* err) {
  const long long total = seg_total(sl);
  const int lg = threadIdx.x % G;
  const long long ngroups = (long long)gridDim.x * (blockDim.x / G);
  unsigned long long ins = 0;
  for (long long g = (long long)blockIdx.x * (blockDim.x / G) + threadIdx.x / G; g < total;
       g += ngroups) {
    int seg;
    const long long pos = seg_pos(sl, g, &seg);
    const uint64_t key = keys[pos];
    long long slot = -1;
    int inserted = 0;
    if (lg == 0) {
      bool b = false;
      if (key != kEmptyKey) slot = probe_slot(t, key, insert != 0, &b);
      inserted = b;
      if (slot < 0 && insert) atomicOr(err, key == kEmptyKey ? 2 : 1);
      slots_out[pos] = slot;
    }
    if (G > 1) {
      slot = __shfl(slot, 0, G);
      inserted = __shfl(inserted, 0, G);
    }
    if (inserted) init_row<G>(t, ip, slot, key, lg);
    ins += (lg == 0 && inserted);
  }
  ins = wave_sum_u64(ins);
  if ((threadIdx.x & 63) == 0 && ins) ctr_add(size_ctr, ins);
}

// K4: gather parameter rows (dim floats) for resolved slots; missing -> 0.
template <int G>
__global__ __launch_bounds__(256) void k_gather(DevTable t, const long long* __restrict__ slots,
                                                SegList sl, float* __restrict__ out) {
  const long long total = seg_total(sl);
  const int lg = threadIdx.x % G;
  const long long ngroups = (long long)gridDim.x * (blockDim.x / G);
  for (long long g = (long long)blockIdx.x * (blockDim.x / G) + threadIdx.x / G; g < total;
       g += ngroups) {
    int seg;
    const long long pos = seg_pos(sl, g, &seg);
    const long long slot = slots[pos];
    float* o = out + pos * (long long)t.dim;
    if (slot < 0) {
      for (uint32_t j = lg; j < t.dim; j += G) o[j] = 0.f;
    } else {
      for (uint32_t j = lg; j < t.dim; j += G) o[j] = row_ld(t, slot, j);
    }
  }
}

// A row read by a lane that FOUND its key may belong to a key another lane of
// the same launch is inserting right now (duplicate keys: the server side of
// an N>1 pull receives the same key from several workers).  Empty slots hold
// the 0xFF fill, so a coordinate still reading 0xFFFFFFFF has not been
// initialised yet: substitute the deterministic initial value the inserting
// lane is writing (init_value depends on (key, j) only).  No arithmetic NaN
// has this bit pattern.
__device__ __forceinline__ float fresh_or(float v, const InitParams& ip, uint64_t key, uint32_t j,
                                          uint32_t dim) {
  return __float_as_uint(v) == 0xFFFFFFFFu ? init_value(ip, key, j, dim) : v;
}

// K3+K4 fused: probe, init if new, and emit the row without a second pass.
// Duplicate keys within the launch are safe (CAS claim + fresh_or above).
// one key of a unique-key pull: probe (insert if new) by the group leader,
// init the row if it was inserted, emit the row to out[pos]
// Scalar (w, h) rows in 16-byte [w | h | key] slots (sparse LR): each probe
// step is ONE 16-byte load that brings the key and the row together, so a
// found key needs no second (dependent) load of its row.  Returns the slot
// (-1: table full) and the row as it was read; `*inserted` when this lane
// claimed an EMPTY slot (the row then is the prefilled / initial row).
__device__ __forceinline__ long long probe_slot16(const DevTable& t, uint64_t key, float2* wh,
                                                  bool* inserted) {
  ProbeSeq ps = probe_seq(t, key);
  for (uint64_t n = 0, len = ps.len(); n < len; ++n, ps.next()) {
    const uint64_t s = ps.s;
    const uint4 v = *reinterpret_cast<const uint4*>(t.base + s * 16);
    const uint64_t k = ((uint64_t)v.w << 32) | v.z;
    if (k == key) {
      *wh = make_float2(__uint_as_float(v.x), __uint_as_float(v.y));
      return (long long)s;
    }
    if (k == kEmptyKey) {
      uint64_t* kp = slot_key(t, s);
      const unsigned long long prev =
          atomicCAS(reinterpret_cast<unsigned long long*>(kp), kEmptyKey, key);
      if (prev == kEmptyKey) {
        *inserted = true;
        return (long long)s;
      }
      if (prev == key) {  // a duplicate of this key claimed it in this launch
        *wh = *reinterpret_cast<const float2*>(slot_row(t, s));
        return (long long)s;
      }
    }
  }
  return -1;
}

template <int G>
__device__ __forceinline__ void pull_one(const DevTable& t, uint64_t key, long long pos,
                                         long long* __restrict__ slots_out, float* __restrict__ out,
                                         const InitParams& ip, int* err, int lg,
                                         unsigned long long& ins,
                                         float2* __restrict__ snap = nullptr, int one16 = 0) {
  if (G == 1 && one16) {
    // 16-byte [w | h | key] slots: one load per probe step (probe_slot16);
    // with `snap` the (w, h) pair also goes to the snapshot.  one16 == 2:
    // the slot indices are stored as 4 bytes (a table under 2^31 slots)
    bool b = false;
    float2 wh = make_float2(0.f, 0.f);
    const long long slot = key != kEmptyKey ? probe_slot16(t, key, &wh, &b) : -1;
    if (slot < 0) atomicOr(err, key == kEmptyKey ? 2 : 1);
    if (slots_out) {
      if (one16 == 2) reinterpret_cast<int*>(slots_out)[pos] = (int)slot;
      else slots_out[pos] = slot;
    }
    float* o = out + pos * (long long)t.dim;
    if (slot < 0) {
      o[0] = 0.f;
      return;
    }
    if (b) {
      wh = make_float2(init_value(ip, key, 0, 1), ip.state_init);
      if (!t.prefilled) *reinterpret_cast<float2*>(slot_row(t, slot)) = wh;
    } else {
      wh.x = fresh_or(wh.x, ip, key, 0, 1);
      if (__float_as_uint(wh.y) == 0xFFFFFFFFu) wh.y = ip.state_init;
    }
    o[0] = wh.x;
    if (snap) snap[pos] = wh;
    ins += b;
    return;
  }
  long long slot = -1;
  int inserted = 0;
  if (lg == 0) {
    bool b = false;
    if (key != kEmptyKey) slot = probe_slot(t, key, true, &b);
    inserted = b;
    if (slot < 0) atomicOr(err, key == kEmptyKey ? 2 : 1);
    if (slots_out) slots_out[pos] = slot;
  }
  if (G > 1) {
    slot = __shfl(slot, 0, G);
    inserted = __shfl(inserted, 0, G);
  }
  float* o = out + pos * (long long)t.dim;
  if (slot < 0) {
    for (uint32_t j = lg; j < t.dim; j += G) o[j] = 0.f;
  } else if (G == 1 && snap) {
    // scalar (w, h) rows, snapshot mode (see k_apply): one 8-byte row read,
    // w to the model, (w, h) to the snapshot the apply updates from
    float2 wh;
    if (inserted) {
      wh = make_float2(init_value(ip, key, 0, 1), ip.state_init);
      if (!t.prefilled) *reinterpret_cast<float2*>(slot_row(t, slot)) = wh;
    } else {
      wh = *reinterpret_cast<const float2*>(slot_row(t, slot));
      wh.x = fresh_or(wh.x, ip, key, 0, 1);
      if (__float_as_uint(wh.y) == 0xFFFFFFFFu) wh.y = ip.state_init;
    }
    o[0] = wh.x;
    snap[pos] = wh;
  } else {
    if (inserted) {
      for (uint32_t j = lg; j < t.width; j += G) {
        const float v = j < t.dim ? init_value(ip, key, j, t.dim) : ip.state_init;
        if (!t.prefilled) row_st(t, slot, j, v);
        if (j < t.dim) o[j] = row_round(t, v);
      }
    } else if (t.dim <= (uint32_t)G * kApplyRegs) {
      // every load before the first store: the compiler cannot prove `o` and
      // `row` disjoint, so a copy loop would be one round trip per coordinate
      float v[kApplyRegs];
#pragma unroll
      for (int r = 0; r < kApplyRegs; ++r) {
        const uint32_t j = lg + r * G;
        if (j < t.dim) v[r] = row_ld(t, slot, j);
      }
#pragma unroll
      for (int r = 0; r < kApplyRegs; ++r) {
        const uint32_t j = lg + r * G;
        if (j < t.dim) o[j] = row_round(t, fresh_or(v[r], ip, key, j, t.dim));
      }
    } else {
      for (uint32_t j = lg; j < t.dim; j += G)
        o[j] = row_round(t, fresh_or(row_ld(t, slot, j), ip, key, j, t.dim));
    }
  }
  ins += (lg == 0 && inserted);
}

template <int G>
__global__ __launch_bounds__(256) void k_pull_unique(DevTable t, const uint64_t* __restrict__ keys,
                                                     SegList sl, long long* __restrict__ slots_out,
                                                     float* __restrict__ out, InitParams ip,
                                                     unsigned long long* size_ctr, int* err) {
  const long long total = seg_total(sl);
  const int lg = threadIdx.x % G;
  const long long ngroups = (long long)gridDim.x * (blockDim.x / G);
  unsigned long long ins = 0;
  for (long long g = (long long)blockIdx.x * (blockDim.x / G) + threadIdx.x / G; g < total;
       g += ngroups) {
    int seg;
    const long long pos = seg_pos(sl, g, &seg);
    pull_one<G>(t, keys[pos], pos, slots_out, out, ip, err, lg, ins);
  }
  ins = wave_sum_u64(ins);
  if ((threadIdx.x & 63) == 0 && ins) ctr_add(size_ctr, ins);
}

// Same, straight from the bucketed dedup's per-bucket staging (bdedup.hip):
// workgroup b pulls bucket b's unique keys bkeys[bstart[b] + l] to unique id
// ubase[b] + l — the colocated 1-GPU path needs no send-segment copy.
template <int G>
__global__ __launch_bounds__(256) void k_pull_unique_bk(DevTable t, const uint64_t* __restrict__ bkeys,
                                                        const uint32_t* __restrict__ bstart,
                                                        const uint32_t* __restrict__ unum,
                                                        const uint32_t* __restrict__ ubase,
                                                        long long* __restrict__ slots_out,
                                                        float* __restrict__ out, InitParams ip,
                                                        unsigned long long* size_ctr, int* err,
                                                        float2* __restrict__ snap, int one16) {
  const int b = blockIdx.x, lg = threadIdx.x % G;
  const uint32_t nu = unum[b], base = ubase[b];
  const uint64_t* src = bkeys + bstart[b];
  unsigned long long ins = 0;
  // gridDim.y workgroups share a bucket (fewer serial probes per lane)
  for (uint32_t l = blockIdx.y * (256 / G) + threadIdx.x / G; l < nu;
       l += gridDim.y * (256 / G))
    pull_one<G>(t, src[l], (long long)base + l, slots_out, out, ip, err, lg, ins, snap, one16);
  ins = wave_sum_u64(ins);
  if ((threadIdx.x & 63) == 0 && ins) ctr_add(size_ctr, ins);
}


// K3 of the one-GPU headline on a REGION table (ss_device.h): one workgroup
// per region-aligned dedup bucket, so the workgroup is the only inserter
// into its regions during this launch.  A key is probed with 16-byte
// [w | h | key] loads; an EMPTY slot is claimed in an LDS set of slot
// indices instead of with a device-scope CAS (those run at the memory side:
// 3.3M new keys per bench step cost more than the probes), and NOTHING is
// written to the table: the pull returns the initial (w, h) of a new key as
// its snapshot, and the fused merge + AdaGrad update stores the whole slot
// [w | h | key] with one 16-byte store (k_bd_reduce with bkeys) — which also
// makes a random initialiser free (the row is written once either way).
// Until that store a claimed slot still reads EMPTY: every consumer of the
// table is stream-ordered after it (PSEngine defers only synchronous
// one-GPU rounds; launch_commit_claims is the fallback writer).
// threads per bucket workgroup (SS_CLAIM_T): 256 measured 0.795-0.798 ms
// per bench step against 0.832-0.835 (512) and 0.843-0.844 (1024) on one
// box — small workgroups interleave with the route stream's kernels
static constexpr int kClaimT = 256;
// LDS claim set of TS slot indices (a power of two >= the <= 4096 keys of a
// bucket, so a claim always finds a free entry): 8192 keeps it at most half
// full; 4096 (SS_CLAIM_TS=4096) halves its LDS — 32 instead of 48 KB per
// workgroup, 5 instead of 3 workgroups per CU — at the price of longer LDS
// probes in buckets with many new keys
static constexpr int kClaimTS = 8192;
template <int TS>
__device__ __forceinline__ bool lds_claim(uint32_t* cl, uint32_t s) {
  constexpr int kBits = TS == 8192 ? 13 : 12;
  static_assert(TS == 1 << kBits, "claim set: 4096 or 8192 entries");
  uint32_t i = (s * 0x9E3779B1u) >> (32 - kBits);
  for (int k = 0; k < TS; ++k) {
    const uint32_t v = cl[i];
    if (v == s) return false;
    if (v == 0xFFFFFFFFu) {
      const uint32_t prev = atomicCAS(&cl[i], 0xFFFFFFFFu, s);
      if (prev == 0xFFFFFFFFu) return true;
      if (prev == s) return false;
    }
    i = (i + 1) & (TS - 1);
  }
  return false;  // unreachable: at most 4096 distinct slots claimed per workgroup
}

// luid / occ (optional, the LR forward's one-gather mode): the bucket's
// parameters also go to occ[p] = w(luid[p]) for its occurrence positions p
// (k_bd_fill_occ fused: the rows staged in LDS, no uvals round trip); `out`
// may then be null.
static constexpr int kClaimMaxU = 4096;  // unique keys of a bucket (the dedup's LDS table)
// KR: keys per thread whose first probe loads are in flight together (a
// bucket's ~1800 unique keys over 256 threads are ~7 keys per thread; the
// workgroup's 48 KB of LDS allows 3 per CU).  The first probe resolves
// almost every key (mean probe length 0.48 at load 0.49,
// profiles/r6_long_region.md); longer probes continue one load at a time.
// KR = 1 (one key at a time) measured fastest: see launch_pull_claim_bk
template <int CT, int KR, int TS = kClaimTS>
__global__ __launch_bounds__(CT) void k_pull_claim_bk(
    DevTable t, const uint64_t* __restrict__ bkeys, const uint32_t* __restrict__ bstart,
    const uint32_t* __restrict__ unum, const uint32_t* __restrict__ ubase,
    int* __restrict__ slots32, float* __restrict__ out, float2* __restrict__ snap, InitParams ip,
    unsigned long long* size_ctr, int* err, const uint32_t* __restrict__ luid,
    float* __restrict__ occ, const uint32_t* __restrict__ pj, SelfSeg self) {
  __shared__ uint32_t cl[TS];
  __shared__ float sv[kClaimMaxU];
  for (int i = threadIdx.x; i < TS; i += CT) cl[i] = 0xFFFFFFFFu;
  __syncthreads();
  const int b = blockIdx.x;
  const uint32_t nu = unum[b], base = ubase[b];
  const uint64_t* src = bkeys + bstart[b];
  unsigned long long ins = 0;
  for (uint32_t l0 = threadIdx.x; l0 < nu; l0 += KR * CT) {
    uint64_t key[KR], s0[KR];
    uint4 v[KR];
#pragma unroll
    for (int r = 0; r < KR; ++r) {
      const uint32_t l = l0 + r * CT;
      key[r] = l < nu ? src[l] : kEmptyKey;
    }
#pragma unroll
    for (int r = 0; r < KR; ++r)
      if (key[r] != kEmptyKey) {
        s0[r] = probe_seq(t, key[r]).s;
        v[r] = *reinterpret_cast<const uint4*>(t.base + s0[r] * 16);
      }
#pragma unroll
    for (int r = 0; r < KR; ++r) {
      const uint32_t l = l0 + r * CT;
      if (l >= nu) continue;
      long long slot = -1;
      bool inserted = false;
      float2 wh = make_float2(0.f, 0.f);
      if (key[r] != kEmptyKey) {
        ProbeSeq ps = probe_seq(t, key[r]);
        uint4 x = v[r];
        for (uint64_t n = 0, len = ps.len(); n < len; ++n) {
          if (n) {
            ps.next();
            x = *reinterpret_cast<const uint4*>(t.base + ps.s * 16);
          }
          const uint64_t k = ((uint64_t)x.w << 32) | x.z;
          if (k == key[r]) {
            slot = (long long)ps.s;
            wh = make_float2(__uint_as_float(x.x), __uint_as_float(x.y));
            break;
          }
          if (k == kEmptyKey && lds_claim<TS>(cl, (uint32_t)ps.s)) {
            slot = (long long)ps.s;
            inserted = true;
            break;
          }
        }
      }
      if (slot < 0) atomicOr(err, key[r] == kEmptyKey ? 2 : 1);  // 1: the key's region is full
      const long long pos = (long long)base + l;
      slots32[pos] = (int)slot;
      if (inserted) {
        wh = make_float2(init_value(ip, key[r], 0, 1), ip.state_init);
      } else if (slot >= 0) {
        // a row written by an older CAS-path insert of a non-prefilled table
        wh.x = fresh_or(wh.x, ip, key[r], 0, 1);
        if (__float_as_uint(wh.y) == 0xFFFFFFFFu) wh.y = ip.state_init;
      }
      if (out) out[pos] = wh.x;
      if (occ && l < (uint32_t)kClaimMaxU) sv[l] = wh.x;
      snap[pos] = wh;
      ins += inserted;
    }
  }
  ins = wave_sum_u64(ins);
  if ((threadIdx.x & 63) == 0 && ins) ctr_add(size_ctr, ins);
  if (occ) {  // workgroup-uniform
    __syncthreads();
    const uint32_t p0 = bstart[b], p1 = bstart[b + 1];
    const uint32_t nv = min(nu, (uint32_t)kClaimMaxU);
    // pj (an N>1 server's fill, k_bd_fill_occ_p fused): the row goes to the
    // received position pj[p] of the response, this rank's own positions
    // straight into its vals arena (self)
    for (uint32_t pb = p0 + threadIdx.x; pb < p1; pb += 4 * CT) {
      uint32_t lu[4], q[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const uint32_t p = pb + r * CT;
        lu[r] = p < p1 ? luid[p] : 0xFFFFFFFFu;
        q[r] = p < p1 ? (pj ? pj[p] : p) : 0u;
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const uint32_t p = pb + r * CT;
        if (p < p1) self.pick(occ, (long long)q[r])[q[r]] = lu[r] < nv ? sv[lu[r]] : 0.f;
      }
    }
  }
}

// The fallback writer of a claimed pull whose fused merge did not run (a
// snapshot invalidated between pull and push): every claimed slot still
// EMPTY gets its key and the snapshot's (initial) row.  A claimed slot that
// holds ANOTHER key by now was taken by an insert that bypassed the claim
// bookkeeping (a direct table insert between the pull and its commit): the
// round's slot indices then point at that key's row, so the sticky error bit
// 4 fails the next check instead of letting the push update the wrong row.
__global__ __launch_bounds__(256) void k_commit_claims(
    DevTable t, const uint64_t* __restrict__ bkeys, const uint32_t* __restrict__ bstart,
    const uint32_t* __restrict__ unum, const uint32_t* __restrict__ ubase,
    const int* __restrict__ slots32, const float2* __restrict__ snap, int* __restrict__ err) {
  const int b = blockIdx.x;
  const uint32_t nu = unum[b], base = ubase[b];
  const uint64_t* src = bkeys + bstart[b];
  for (uint32_t l = threadIdx.x; l < nu; l += 256) {
    const int s = slots32[base + l];
    if (s < 0) continue;
    const uint64_t key = src[l];
    const uint64_t held = *slot_key(t, (uint64_t)s);
    if (held != kEmptyKey) {
      if (held != key && err) atomicOr(err, 4);
      continue;
    }
    const float2 wh = snap[base + l];
    *reinterpret_cast<uint4*>(t.base + (uint64_t)s * 16) =
        make_uint4(__float_as_uint(wh.x), __float_as_uint(wh.y), (uint32_t)key,
                   (uint32_t)(key >> 32));
  }
}


// k_pull_unique_bk for wide fp32 rows (word2vec, D = 32 / 64 / 128): 8 lanes
// per key, each moving D/32 16-byte vectors of the row (a D = 128 row is 32
// float4s: 8 lanes x 4), so a wave has 8 keys' probe -> row chains in flight
// instead of one (a 64-lane group per key left the pull latency-bound: 439K
// distinct 512-B rows of a per-pair step read + written at ~1.3 TB/s).
static constexpr int kPvL = 8;
// 4 consecutive coordinates of a wide row as one vector access: a float4
// (fp32 rows) or 4 packed bf16 words (compact rows, one 8-byte access)
template <bool B16>
__device__ __forceinline__ float4 row4_ld(const char* row, int q) {
  if constexpr (B16) {
    const uint2 x = reinterpret_cast<const uint2*>(row)[q];
    return make_float4(bf16_val(x.x & 0xFFFFu), bf16_val(x.x >> 16), bf16_val(x.y & 0xFFFFu),
                       bf16_val(x.y >> 16));
  } else {
    return reinterpret_cast<const float4*>(row)[q];
  }
}
// ... and stored: bf16 words rounded as row_st does (coordinate j0 + 0..3 of
// slot s; `sr`: stochastically, for optimizer steps)
template <bool B16>
__device__ __forceinline__ void row4_st(char* row, int q, float4 v, uint64_t s, uint32_t j0,
                                        bool sr) {
  if constexpr (B16) {
    const uint32_t a = bf16_bits(s, j0, v.x, sr), b = bf16_bits(s, j0 + 1, v.y, sr);
    const uint32_t c = bf16_bits(s, j0 + 2, v.z, sr), d = bf16_bits(s, j0 + 3, v.w, sr);
    reinterpret_cast<uint2*>(row)[q] = make_uint2(a | (b << 16), c | (d << 16));
  } else {
    reinterpret_cast<float4*>(row)[q] = v;
  }
}
template <int D, bool B16>
__global__ __launch_bounds__(256) void k_pull_rows_bk(DevTable t, const uint64_t* __restrict__ bkeys,
                                                      const uint32_t* __restrict__ bstart,
                                                      const uint32_t* __restrict__ unum,
                                                      const uint32_t* __restrict__ ubase,
                                                      long long* __restrict__ slots_out,
                                                      float* __restrict__ out, InitParams ip,
                                                      unsigned long long* size_ctr, int* err) {
  constexpr int NV = D / (4 * kPvL);  // float4s per lane
  static_assert(NV >= 1 && D % (4 * kPvL) == 0, "D must be a multiple of 32");
  const int b = blockIdx.x, lg = threadIdx.x & (kPvL - 1);
  const uint32_t nu = unum[b], base = ubase[b];
  const uint64_t* src = bkeys + bstart[b];
  unsigned long long ins = 0;
  // block-uniform trip count: every shuffle below runs with the whole wave
  for (uint32_t l0 = blockIdx.y * (256 / kPvL); l0 < nu; l0 += gridDim.y * (256 / kPvL)) {
    const uint32_t l = l0 + threadIdx.x / kPvL;
    const bool act = l < nu;  // uniform inside a lane group
    const uint64_t key = act ? src[l] : kEmptyKey;
    long long slot = -1;
    int inserted = 0;
    if (act && lg == 0) {
      bool bb = false;
      if (key != kEmptyKey) slot = probe_slot(t, key, true, &bb);
      inserted = bb;
      if (slot < 0) atomicOr(err, key == kEmptyKey ? 2 : 1);
      if (slots_out) slots_out[(long long)base + l] = slot;
    }
    slot = __shfl(slot, 0, kPvL);
    inserted = __shfl(inserted, 0, kPvL);
    if (!act) continue;
    float4* o = reinterpret_cast<float4*>(out + ((long long)base + l) * D);
    if (slot < 0) {
#pragma unroll
      for (int k = 0; k < NV; ++k) o[lg + k * kPvL] = make_float4(0.f, 0.f, 0.f, 0.f);
    } else if (inserted) {
      for (uint32_t j = lg; j < t.width; j += kPvL) {
        const float v = j < (uint32_t)D ? init_value(ip, key, j, D) : ip.state_init;
        if (!t.prefilled) row_st(t, slot, j, v);
        // a compact row returns its initial value as stored (row_round)
        if (j < (uint32_t)D) out[((long long)base + l) * D + j] = row_round(t, v);
      }
      ins += (lg == 0);
    } else {
      // (loading the home slot's row beside the probe's key load measured
      // neutral: 148 vs 152 us for the per-pair pull)
      const char* r = reinterpret_cast<const char*>(slot_row(t, slot));
      float4 v[NV];
#pragma unroll
      for (int k = 0; k < NV; ++k) v[k] = row4_ld<B16>(r, lg + k * kPvL);
#pragma unroll
      for (int k = 0; k < NV; ++k) {
        const uint32_t j = 4u * (lg + k * kPvL);
        // (row_round: a compact row's fresh value as it will be stored)
        v[k].x = row_round(t, fresh_or(v[k].x, ip, key, j, D));
        v[k].y = row_round(t, fresh_or(v[k].y, ip, key, j + 1, D));
        v[k].z = row_round(t, fresh_or(v[k].z, ip, key, j + 2, D));
        v[k].w = row_round(t, fresh_or(v[k].w, ip, key, j + 3, D));
        o[lg + k * kPvL] = v[k];
      }
    }
  }
  ins = wave_sum_u64(ins);
  if ((threadIdx.x & 63) == 0 && ins) ctr_add(size_ctr, ins);
}


// k_pull_unique_bk for narrow fp32 rows whose key and parameters share a
// slot's first 64 bytes ([key | params | state], FM's 9 parameters at bytes
// 8..44 of an 80-byte slot): 4 lanes per key, each probe step one 16-byte
// load per lane, so the step that finds the key has already read the row —
// one dependent round trip per key instead of two (key, then row).
static constexpr int kPnL = 4;
__global__ __launch_bounds__(256) void k_pull_narrow_bk(DevTable t, const uint64_t* __restrict__ bkeys,
                                                        const uint32_t* __restrict__ bstart,
                                                        const uint32_t* __restrict__ unum,
                                                        const uint32_t* __restrict__ ubase,
                                                        long long* __restrict__ slots_out,
                                                        float* __restrict__ out, InitParams ip,
                                                        unsigned long long* size_ctr, int* err) {
  const int b = blockIdx.x, lg = threadIdx.x & (kPnL - 1);
  const uint32_t nu = unum[b], base = ubase[b], D = t.dim;
  const uint64_t* src = bkeys + bstart[b];
  unsigned long long ins = 0;
  // block-uniform trip count: the shuffles below run with the whole wave
  for (uint32_t l0 = blockIdx.y * (256 / kPnL); l0 < nu; l0 += gridDim.y * (256 / kPnL)) {
    const uint32_t l = l0 + threadIdx.x / kPnL;
    const bool act = l < nu;  // uniform inside a lane group
    const uint64_t key = act ? src[l] : kEmptyKey;
    long long slot = -1;
    bool inserted = false;
    uint4 v = make_uint4(0u, 0u, 0u, 0u);
    if (act && key != kEmptyKey) {
      ProbeSeq ps = probe_seq(t, key);
      for (uint64_t n = 0, len = ps.len(); n < len; ++n, ps.next()) {  // group-uniform trip count
        const uint64_t s = ps.s;
        v = *reinterpret_cast<const uint4*>(t.base + s * (uint64_t)t.stride + 16 * lg);
        const uint64_t k = ((uint64_t)__shfl(v.y, 0, kPnL) << 32) | __shfl(v.x, 0, kPnL);
        if (k == key) {
          slot = (long long)s;
          break;
        }
        if (k == kEmptyKey) {
          unsigned long long prev = 0;
          if (lg == 0)
            prev = atomicCAS(reinterpret_cast<unsigned long long*>(slot_key(t, s)), kEmptyKey, key);
          prev = __shfl(prev, 0, kPnL);
          if (prev == kEmptyKey || prev == key) {  // claimed (or a duplicate of this key did)
            slot = (long long)s;
            inserted = prev == kEmptyKey;
            break;
          }
        }
      }
    }
    if (!act) continue;
    if (lg == 0) {
      if (slot < 0) atomicOr(err, key == kEmptyKey ? 2 : 1);
      if (slots_out) slots_out[(long long)base + l] = slot;
    }
    float* o = out + ((long long)base + l) * D;
    if (slot < 0) {
      for (uint32_t j = lg; j < D; j += kPnL) o[j] = 0.f;
    } else if (inserted) {
      for (uint32_t j = lg; j < t.width; j += kPnL) {
        const float x = j < D ? init_value(ip, key, j, D) : ip.state_init;
        if (!t.prefilled) row_st(t, (uint64_t)slot, j, x);
        if (j < D) o[j] = x;
      }
      ins += (lg == 0);
    } else {
      // this lane holds slot bytes [16 lg, 16 lg + 16): parameter j is at 8 + 4 j
      const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const int byte = 16 * lg + 4 * c;
        if (byte < 8) continue;
        const uint32_t j = (uint32_t)(byte - 8) >> 2;
        if (j < D) o[j] = fresh_or(__uint_as_float(w[c]), ip, key, j, D);
      }
    }
  }
  ins = wave_sum_u64(ins);
  if ((threadIdx.x & 63) == 0 && ins) ctr_add(size_ctr, ins);
}


// Read-only lookup of a bucket view's unique keys (the N>1 collective
// lookup, PSEngine.lookup: a server answers any worker's keys without
// inserting): out[(ubase[b] + l) * dim + j] = the row of bkeys[bstart[b] + l],
// zeros for a key this shard does not hold.  G lanes per key.
template <int G>
__global__ __launch_bounds__(256) void k_lookup_bk(DevTable t, const uint64_t* __restrict__ bkeys,
                                                   const uint32_t* __restrict__ bstart,
                                                   const uint32_t* __restrict__ unum,
                                                   const uint32_t* __restrict__ ubase,
                                                   float* __restrict__ out) {
  const int b = blockIdx.x, lg = threadIdx.x % G;
  const uint32_t nu = unum[b], base = ubase[b];
  const uint64_t* src = bkeys + bstart[b];
  for (uint32_t l = blockIdx.y * (256 / G) + threadIdx.x / G; l < nu;
       l += gridDim.y * (256 / G)) {  // uniform inside a lane group
    const uint64_t key = src[l];
    long long slot = -1;
    if (lg == 0 && key != kEmptyKey) {
      bool unused = false;
      slot = probe_slot(t, key, false, &unused);
    }
    if (G > 1) slot = __shfl(slot, 0, G);
    float* o = out + ((long long)base + l) * (long long)t.dim;
    for (uint32_t j = lg; j < t.dim; j += G) o[j] = slot < 0 ? 0.f : row_ld(t, slot, j);
  }
}

// ---------------------------------------------------------------------------
// K5: fused optimizer update on resolved slots. Keys inside one launch must be
// unique (the host launches one segment per source rank, in rank order, so
// duplicate keys from different workers are applied sequentially — no lost
// updates, deterministic, and no float atomics on the hot path).
// one row of K5: lane lg of a G-lane group updates its coordinates
template <int G>
__device__ __forceinline__ void apply_row(const DevTable& t, long long slot,
                                          const float* __restrict__ gr, const OptParams& op,
                                          int lg, const float2* __restrict__ snap = nullptr) {
  if (slot < 0) return;
  if (G == 1 && t.dim == 1 && op.kind == kOptAdaGrad && !t.bf16 &&
      t.row_off % 8 == 0 && t.stride % 8 == 0) {
    float* row = slot_row(t, slot);
    // scalar-row AdaGrad (sparse LR): the (w, h) pair as one 8-byte load and
    // one 8-byte store instead of two of each.  With a snapshot (the (w, h)
    // the pull read, valid when nothing else wrote the row in between) the
    // random read goes away: a coalesced read and a blind random store.
    float2 wh = snap ? *snap : *reinterpret_cast<const float2*>(row);
    float s2 = 0.f;
    opt_update(op, wh.x, wh.y, s2, gr[0]);
    *reinterpret_cast<float2*>(row) = wh;
    return;
  }
  if (t.dim <= (uint32_t)G * kApplyRegs) {
    // all of this lane's coordinates loaded first, updated in registers,
    // stored after: one memory round trip per row (a load-update-store loop
    // per coordinate serialised dim/G round trips: FM rows took 3)
    const int ns = opt_state_per_coord(op.kind);
    float w[kApplyRegs], s1[kApplyRegs], s2[kApplyRegs], g[kApplyRegs];
#pragma unroll
    for (int r = 0; r < kApplyRegs; ++r) {
      const uint32_t j = lg + r * G;
      if (j < t.dim) {
        w[r] = row_ld(t, slot, j);
        g[r] = gr[j];
        s1[r] = ns > 0 ? row_ld(t, slot, t.dim + j) : 0.f;
        s2[r] = ns > 1 ? row_ld(t, slot, 2 * t.dim + j) : 0.f;
      }
    }
#pragma unroll
    for (int r = 0; r < kApplyRegs; ++r) {
      const uint32_t j = lg + r * G;
      if (j < t.dim) {
        opt_update(op, w[r], s1[r], s2[r], g[r]);
        row_st(t, slot, j, w[r], true);
        if (ns > 0) row_st(t, slot, t.dim + j, s1[r], true);
        if (ns > 1) row_st(t, slot, 2 * t.dim + j, s2[r], true);
      }
    }
  } else if (t.bf16) {
    const int ns = opt_state_per_coord(op.kind);
    for (uint32_t j = lg; j < t.dim; j += G) {
      float w = row_ld(t, slot, j);
      float s1 = ns > 0 ? row_ld(t, slot, t.dim + j) : 0.f;
      float s2 = ns > 1 ? row_ld(t, slot, 2 * t.dim + j) : 0.f;
      opt_update(op, w, s1, s2, gr[j]);
      row_st(t, slot, j, w, true);
      if (ns > 0) row_st(t, slot, t.dim + j, s1, true);
      if (ns > 1) row_st(t, slot, 2 * t.dim + j, s2, true);
    }
  } else {
    float* row = slot_row(t, slot);
    for (uint32_t j = lg; j < t.dim; j += G) opt_apply(op, row, row + t.dim, t.dim, j, gr[j]);
  }
}

template <int G>
__global__ __launch_bounds__(256) void k_apply(DevTable t, const long long* __restrict__ slots,
                                               const float* __restrict__ grads, SegList sl,
                                               OptParams op, const float2* __restrict__ snap,
                                               int slot32) {
  const long long total = seg_total(sl);
  const int* s32 = reinterpret_cast<const int*>(slots);
  const int lg = threadIdx.x % G;
  const long long ngroups = (long long)gridDim.x * (blockDim.x / G);
  for (long long g = (long long)blockIdx.x * (blockDim.x / G) + threadIdx.x / G; g < total;
       g += ngroups) {
    int seg;
    const long long pos = seg_pos(sl, g, &seg);
    apply_row<G>(t, slot32 ? (long long)s32[pos] : slots[pos], grads + pos * (long long)t.dim, op, lg,
                 snap ? snap + pos : nullptr);
  }
}

// K5 for wide fp32 rows (word2vec, D = 32 / 64 / 128): 8 lanes per key,
// parameters, optimizer state and gradient moved as 16-byte vectors (the
// 64-lane group per key kept one key's load -> update -> store chain per
// wave in flight).
template <int D, bool B16>
__global__ __launch_bounds__(256) void k_apply_rows(DevTable t, const long long* __restrict__ slots,
                                                    const float* __restrict__ grads, SegList sl,
                                                    OptParams op,
                                                    const uint8_t* __restrict__ only) {
  constexpr int NV = D / (4 * kPvL), Q = D / 4;  // float4s per lane / per array
  const long long total = seg_total(sl);
  const int lg = threadIdx.x & (kPvL - 1);
  const long long ngroups = (long long)gridDim.x * (256 / kPvL);
  const int ns = opt_state_per_coord(op.kind);
  for (long long g = (long long)blockIdx.x * (256 / kPvL) + threadIdx.x / kPvL; g < total;
       g += ngroups) {
    int seg;
    const long long pos = seg_pos(sl, g, &seg);
    if (only && !only[pos]) continue;  // the same for the 8 lanes of a key
    const long long slot = slots[pos];
    if (slot < 0) continue;
    char* row = reinterpret_cast<char*>(slot_row(t, slot));
    const float4* gr = reinterpret_cast<const float4*>(grads + pos * D);
    const float4 z = make_float4(0.f, 0.f, 0.f, 0.f);
    float4 w[NV], s1[NV], s2[NV], gv[NV];
#pragma unroll
    for (int k = 0; k < NV; ++k) {
      const int q = lg + k * kPvL;
      w[k] = row4_ld<B16>(row, q);
      gv[k] = gr[q];
      s1[k] = ns > 0 ? row4_ld<B16>(row, Q + q) : z;
      s2[k] = ns > 1 ? row4_ld<B16>(row, 2 * Q + q) : z;
    }
#pragma unroll
    for (int k = 0; k < NV; ++k) {
      opt_update(op, w[k].x, s1[k].x, s2[k].x, gv[k].x);
      opt_update(op, w[k].y, s1[k].y, s2[k].y, gv[k].y);
      opt_update(op, w[k].z, s1[k].z, s2[k].z, gv[k].z);
      opt_update(op, w[k].w, s1[k].w, s2[k].w, gv[k].w);
      const int q = lg + k * kPvL;
      row4_st<B16>(row, q, w[k], (uint64_t)slot, 4u * q, true);
      if (ns > 0) row4_st<B16>(row, Q + q, s1[k], (uint64_t)slot, 4u * (Q + q), true);
      if (ns > 1) row4_st<B16>(row, 2 * Q + q, s2[k], (uint64_t)slot, 4u * (2 * Q + q), true);
    }
  }
}

// K5 for narrow multi-coordinate rows (FM: 9 weights + 9 AdaGrad sums, 4
// lanes per key): the row moves as 8-byte chunks staged through LDS.  The
// per-coordinate form (apply_row) issues a 4-byte access per lane per array
// and coordinate round — 6 loads and 6 stores per key for an FM row, each a
// separate request to the same two or three sectors; here a key's row is 3
// float2 loads and 3 stores (32 contiguous bytes per instruction per key),
// regrouped into (w_j, s_j) pairs in LDS.
static constexpr int kStageMaxW = 48;  // row floats staged per key (dim * (1 + state))
template <int G>
__global__ __launch_bounds__(256) void k_apply_st(DevTable t, const long long* __restrict__ slots,
                                                  const float* __restrict__ grads, SegList sl,
                                                  OptParams op) {
  // even row stride: the load/store phases move float2 pairs as one 8-byte
  // LDS access (an odd stride split them into two 4-byte accesses); 52 floats
  // = 20 mod 32 puts the 8 four-lane groups of a half-wave on disjoint 4-bank
  // slots for the 4-byte update-phase accesses
  __shared__ float2 stage2[256 / G][kStageMaxW / 2 + 2];
  const long long total = seg_total(sl);
  const int lg = threadIdx.x % G, grp = threadIdx.x / G;
  const long long ngroups = (long long)gridDim.x * (256 / G);
  const int dim = (int)t.dim, ns = opt_state_per_coord(op.kind);
  const int W = dim * (1 + ns), nch = W / 2;  // W even (launch_apply checks)
  float2* st2 = stage2[grp];
  float* st = reinterpret_cast<float*>(st2);
  for (long long g = (long long)blockIdx.x * (256 / G) + grp; g < total; g += ngroups) {
    int seg;
    const long long pos = seg_pos(sl, g, &seg);
    const long long slot = slots[pos];
    if (slot < 0) continue;  // the same for the G lanes of a group
    float2* row = reinterpret_cast<float2*>(slot_row(t, slot));
    for (int k = lg; k < nch; k += G) st2[k] = row[k];
    __builtin_amdgcn_wave_barrier();
    for (int j = lg; j < dim; j += G) {
      float w = st[j], s1 = ns > 0 ? st[dim + j] : 0.f, s2 = ns > 1 ? st[2 * dim + j] : 0.f;
      opt_update(op, w, s1, s2, grads[pos * (long long)dim + j]);
      st[j] = w;
      if (ns > 0) st[dim + j] = s1;
      if (ns > 1) st[2 * dim + j] = s2;
    }
    __builtin_amdgcn_wave_barrier();
    for (int k = lg; k < nch; k += G) row[k] = st2[k];
    __builtin_amdgcn_wave_barrier();
  }
}

// Assign full rows (params + state) for keys, inserting when missing
// (checkpoint load / rehash).  `rows` has `width` floats per key.
template <int G>
__global__ __launch_bounds__(256) void k_assign(DevTable t, const uint64_t* __restrict__ keys,
                                                const float* __restrict__ rows, long long n,
                                                unsigned long long* size_ctr, int* err) {
  const int lg = threadIdx.x % G;
  const long long ngroups = (long long)gridDim.x * (blockDim.x / G);
  unsigned long long ins = 0;
  for (long long g = (long long)blockIdx.x * (blockDim.x / G) + threadIdx.x / G; g < n;
       g += ngroups) {
    const uint64_t key = keys[g];
    long long slot = -1;
    int inserted = 0;
    if (lg == 0) {
      bool b = false;
      if (key != kEmptyKey) slot = probe_slot(t, key, true, &b);
      inserted = b;
      if (slot < 0) atomicOr(err, key == kEmptyKey ? 2 : 1);
    }
    if (G > 1) {
      slot = __shfl(slot, 0, G);
      inserted = __shfl(inserted, 0, G);
    }
    if (slot >= 0) {
      const float* src = rows + g * (long long)t.width;
      for (uint32_t j = lg; j < t.width; j += G) row_st(t, slot, j, src[j]);
    }
    ins += (lg == 0 && inserted);
  }
  ins = wave_sum_u64(ins);
  if ((threadIdx.x & 63) == 0 && ins) ctr_add(size_ctr, ins);
}

// K8: compact occupied slots of [s0, s0+n) into (keys_out, rows_out[width]).
// Wave ballot + one atomic per wave for the output cursor.
__global__ __launch_bounds__(256) void k_export(DevTable t, unsigned long long s0, long long n,
                                                uint64_t* __restrict__ keys_out,
                                                float* __restrict__ rows_out,
                                                unsigned long long* cursor) {
  const int lane = threadIdx.x & 63;
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long base = (long long)blockIdx.x * blockDim.x; base < n; base += stride) {
    const long long i = base + threadIdx.x;
    uint64_t key = kEmptyKey;
    if (i < n) key = *slot_key(t, s0 + i);
    const bool occ = key != kEmptyKey;
    const unsigned long long mask = __ballot(occ);
    unsigned long long wbase = 0;
    if (lane == 0 && mask) wbase = atomicAdd(cursor, (unsigned long long)__popcll(mask));
    wbase = __shfl(wbase, 0, 64);
    if (occ) {
      const unsigned long long o = wbase + __popcll(mask & ((1ull << lane) - 1));
      keys_out[o] = key;
      for (uint32_t j = 0; j < t.width; ++j) rows_out[o * t.width + j] = row_ld(t, s0 + i, j);
    }
  }
}

// Probe-length histogram (observability): for every occupied slot
// the distance from its key's home slot, binned [0, nbins-1] (last bin =
// ">= nbins-1").  LDS histogram per workgroup, one global add per bin.
__global__ __launch_bounds__(256) void k_probe_hist(DevTable t, unsigned long long* __restrict__ hist,
                                                    int nbins) {
  __shared__ unsigned int h[256];
  for (int b = threadIdx.x; b < nbins; b += 256) h[b] = 0u;
  __syncthreads();
  const unsigned long long stride = (unsigned long long)gridDim.x * blockDim.x;
  for (unsigned long long s = (unsigned long long)blockIdx.x * blockDim.x + threadIdx.x; s < t.cap;
       s += stride) {
    const uint64_t key = *slot_key(t, s);
    if (key == kEmptyKey) continue;
    const ProbeSeq ps = probe_seq(t, key);  // home slot and the key's region
    const uint64_t home = ps.s;
    const uint64_t d = s >= home ? s - home : s + ps.len() - home;
    atomicAdd(&h[d < (uint64_t)nbins - 1 ? (int)d : nbins - 1], 1u);
  }
  __syncthreads();
  for (int b = threadIdx.x; b < nbins; b += 256)
    if (h[b]) atomicAdd(hist + b, (unsigned long long)h[b]);
}

// ---------------------------------------------------------------- launchers
// cap (workgroups) on the general pull's grid-stride loop: `per_cu`
// 256-thread workgroups per CU, leaving CUs to the other streams' kernels
static int grid_cap_per_cu(int per_cu) {
  int dev = 0, cus = 0;
  check_hip(hipGetDevice(&dev), "hipGetDevice");
  check_hip(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev), "CU count");
  return std::max(1, cus * per_cu);
}

static inline int grid_for(long long groups, int G, int cap_blocks = 16384) {
  long long threads = groups * G;
  long long b = (threads + 255) / 256;
  if (b < 1) b = 1;
  if (b > cap_blocks) b = cap_blocks;
  return (int)b;
}

#define SS_DISPATCH_G(G, ...)                   \
  switch (G) {                                  \
    case 1: { constexpr int kG = 1; __VA_ARGS__; } break;   \
    case 4: { constexpr int kG = 4; __VA_ARGS__; } break;   \
    case 16: { constexpr int kG = 16; __VA_ARGS__; } break; \
    case 64: { constexpr int kG = 64; __VA_ARGS__; } break; \
    default: throw_error("unsupported lane-group size");    \
  }

// the 8-lane / 16-byte forms for wide fp32 rows (SS_PULL_VEC=0: the lane-group forms)
static bool pull_vec_on() {
  static const bool on = [] {
    const char* e = std::getenv("SS_PULL_VEC");
    return !(e && e[0] == '0');
  }();
  return on;
}
// wide rows (word2vec): fp32 rows 16-byte aligned, or compact bf16 rows
// 8-byte aligned (4 coordinates per 8-byte access)
static bool wide_rows(const DevTable& t) {
  const int al = t.bf16 ? 8 : 16;
  return (t.dim == 32 || t.dim == 64 || t.dim == 128) && t.row_off % al == 0 &&
         t.stride % al == 0;
}
// launch_apply takes an `only` mask for this table (the wide-row vector apply)
bool apply_masked_ok(const DevTable& t, const OptParams& op) {
  const uint32_t W = t.dim * (uint32_t)(1 + opt_state_per_coord(op.kind));
  return pull_vec_on() && wide_rows(t) && W == t.width;
}

void launch_probe(const DevTable& t, const uint64_t* keys, const SegList& sl, long long max_n,
                  long long* slots, const InitParams& ip, int insert,
                  unsigned long long* size_ctr, int* err, int G, hipStream_t st) {
  if (max_n <= 0) return;
  SS_DISPATCH_G(G, hipLaunchKernelGGL(k_probe<kG>, dim3(grid_for(max_n, kG)), dim3(256), 0, st, t,
                                      keys, sl, slots, ip, insert, size_ctr, err));
  check_launch("k_probe");
}

void launch_gather(const DevTable& t, const long long* slots, const SegList& sl, long long max_n,
                   float* out, int G, hipStream_t st) {
  if (max_n <= 0) return;
  SS_DISPATCH_G(G, hipLaunchKernelGGL(k_gather<kG>, dim3(grid_for(max_n, kG)), dim3(256), 0, st,
                                      t, slots, sl, out));
  check_launch("k_gather");
}

void launch_pull_unique(const DevTable& t, const uint64_t* keys, const SegList& sl,
                        long long max_n, long long* slots, float* out, const InitParams& ip,
                        unsigned long long* size_ctr, int* err, int G, hipStream_t st) {
  if (max_n <= 0) return;
  // general pull (the N>1 server pull of the received segments): at most 4
  // workgroups per CU, grid-stride beyond, so the route stream's next dedup
  // (count / scatter: few, large workgroups) is not starved beside it (see
  // launch_bd_dedup)
  static const int pull_cap = grid_cap_per_cu(4);
  SS_DISPATCH_G(G, hipLaunchKernelGGL(k_pull_unique<kG>, dim3(grid_for(max_n, kG, pull_cap)),
                                      dim3(256), 0, st, t, keys, sl, slots, out, ip, size_ctr,
                                      err));
  check_launch("k_pull_unique");
}

void launch_pull_unique_bk(const DevTable& t, const uint64_t* bkeys, const uint32_t* bstart,
                           const uint32_t* unum, const uint32_t* ubase, int P, long long* slots,
                           float* out, const InitParams& ip, unsigned long long* size_ctr,
                           int* err, int G, hipStream_t st, float* snap, int slot32) {
  if (P <= 0) return;
  if (snap && (t.bf16 || !(G == 1 && t.dim == 1 && t.width == 2 && t.row_off % 8 == 0 &&
                           t.stride % 8 == 0)))
    throw std::invalid_argument("pull snapshot: scalar (w, h) rows with G = 1 only");
  // workgroups per bucket: 4 — one per ~265 unique keys, so a
  // lane probes about once; measured 1.19 -> 1.13-1.17 ms/step vs 1 (the
  // kernel alone barely changes: smaller workgroups interleave better with
  // the route stream's kernels)
  // FM rows (G = 4): 2, 0.548-0.556 -> 0.541 ms/step (4: 0.544-0.551);
  // word2vec rows (G = 64): 2 — with the occurrence-row reduce and hipGraph
  // replay, 1 / 2 / 4 / 8: 0.0840-0.0848 / 0.0829-0.0830 / 0.0837-0.0844 /
  // 0.0858 ms/step (earlier, atomic-bound: 2 and 4 neutral)
  const int ny = G == 1 ? 4 : 2;
  // wide fp32 rows: 8 lanes per key, 16-byte row accesses (k_pull_rows_bk)
  if (!snap && pull_vec_on() && wide_rows(t) && reinterpret_cast<uintptr_t>(out) % 16 == 0) {
#define SS_PRB(DD, B)                                                                          \
  hipLaunchKernelGGL((k_pull_rows_bk<DD, B>), dim3(P, ny), dim3(256), 0, st, t, bkeys, bstart,   \
                     unum, ubase, slots, out, ip, size_ctr, err)
    switch (t.dim) {
      case 32: if (t.bf16) SS_PRB(32, true); else SS_PRB(32, false); break;
      case 64: if (t.bf16) SS_PRB(64, true); else SS_PRB(64, false); break;
      default: if (t.bf16) SS_PRB(128, true); else SS_PRB(128, false); break;
    }
#undef SS_PRB
    check_launch("k_pull_rows_bk");
    return;
  }
  // narrow fp32 rows with key + parameters in the slot's first 64 bytes (FM)
  if (!snap && pull_vec_on() && !t.bf16 && t.key_off == 0 && t.row_off == 8 &&
      t.stride % 16 == 0 && t.stride >= 64 && t.dim >= 2 && 8 + 4 * t.dim <= 64) {
    hipLaunchKernelGGL(k_pull_narrow_bk, dim3(P, ny), dim3(256), 0, st, t, bkeys, bstart, unum,
                       ubase, slots, out, ip, size_ctr, err);
    check_launch("k_pull_narrow_bk");
    return;
  }
  // snapshot pulls on 16-byte [w | h | key] slots probe with one 16-byte
  // load per step (probe_slot16; key load then row load measured slower)
  int one16 = snap && t.stride == 16 && t.key_off == 8 && t.row_off == 0;
  if (slot32) {
    if (!one16 || G != 1 || t.cap >= (1ull << 31))
      throw std::invalid_argument("pull: 4-byte slots need snapshot 16-byte slots, cap < 2^31");
    one16 = 2;
  }
  SS_DISPATCH_G(G, hipLaunchKernelGGL(k_pull_unique_bk<kG>, dim3(P, ny), dim3(256), 0, st, t,
                                      bkeys, bstart, unum, ubase, slots, out, ip, size_ctr, err,
                                      reinterpret_cast<float2*>(snap), one16));
  check_launch("k_pull_unique_bk");
}

void launch_lookup_bk(const DevTable& t, const uint64_t* bkeys, const uint32_t* bstart,
                      const uint32_t* unum, const uint32_t* ubase, int P, float* out, int G,
                      hipStream_t st) {
  if (P <= 0) return;
  SS_DISPATCH_G(G, hipLaunchKernelGGL(k_lookup_bk<kG>, dim3(P, 2), dim3(256), 0, st, t, bkeys,
                                      bstart, unum, ubase, out));
  check_launch("k_lookup_bk");
}

static void check_claim_table(const DevTable& t) {
  if (!t.rbits || t.bf16 || t.stride != 16 || t.key_off != 8 || t.row_off != 0 || t.dim != 1 ||
      t.width != 2 || t.cap >= (1ull << 31))
    throw std::invalid_argument(
        "claimed pulls: a region table of 16-byte [w|h|key] slots under 2^31 slots");
}

void launch_pull_claim_bk(const DevTable& t, const uint64_t* bkeys, const uint32_t* bstart,
                          const uint32_t* unum, const uint32_t* ubase, int P, int* slots32,
                          float* out, float* snap, const InitParams& ip,
                          unsigned long long* size_ctr, int* err, hipStream_t st,
                          const uint32_t* luid, float* occ, const uint32_t* pj,
                          SelfSeg self) {
  if (P <= 0) return;
  check_claim_table(t);
  if (!slots32 || !(out || occ) || !snap || (occ && !luid))
    throw std::invalid_argument("claimed pull: slots, rows (or occurrence rows + luid), snapshot");
  // workgroup size (SS_CLAIM_T: 256 / 512 / 1024): one workgroup per bucket
  static const int ct = [] {
    const char* e = std::getenv("SS_CLAIM_T");
    const int v = e ? std::atoi(e) : kClaimT;
    return (v == 64 || v == 128 || v == 512 || v == 1024) ? v : 256;
  }();
  // first-probe loads in flight per thread (SS_CLAIM_KR: 1 / 4 / 8; the
  // 256-thread default workgroup only).  Measured slower with more in flight
  // (bench 0.733-0.734 ms at 1, 0.737-0.739 at 4, 0.746-0.748 at 8; pull
  // standalone 209 / 223 / 239 us, raw/r6_claim_kr_ab.txt): the pull is bound
  // by the bytes of its random lines and streams, not by its load chains
  static const int kr = [] {
    const char* e = std::getenv("SS_CLAIM_KR");
    const int v = e ? std::atoi(e) : 1;
    return (v == 4 || v == 8) ? v : 1;
  }();
#define SS_CLAIM_LAUNCH(CT, KR)                                                                 \
  hipLaunchKernelGGL((k_pull_claim_bk<CT, KR>), dim3(P), dim3(CT), 0, st, t, bkeys, bstart, unum, \
                     ubase, slots32, out, reinterpret_cast<float2*>(snap), ip, size_ctr, err, luid, \
                     occ, pj, self)
  static const int cts = [] {
    const char* e = std::getenv("SS_CLAIM_TS");
    return e && std::atoi(e) == 4096 ? 4096 : kClaimTS;
  }();
  if (ct == 256 && kr == 1 && cts == 4096)
    hipLaunchKernelGGL((k_pull_claim_bk<256, 1, 4096>), dim3(P), dim3(256), 0, st, t, bkeys, bstart,
                       unum, ubase, slots32, out, reinterpret_cast<float2*>(snap), ip, size_ctr,
                       err, luid, occ, pj, self);
  else if (ct == 256 && kr == 4) SS_CLAIM_LAUNCH(256, 4);
  else if (ct == 256 && kr == 8) SS_CLAIM_LAUNCH(256, 8);
  else if (ct == 256) SS_CLAIM_LAUNCH(256, 1);
  else if (ct == 64) SS_CLAIM_LAUNCH(64, 1);
  else if (ct == 128) SS_CLAIM_LAUNCH(128, 1);
  else if (ct == 512) SS_CLAIM_LAUNCH(512, 1);
  else SS_CLAIM_LAUNCH(1024, 1);
#undef SS_CLAIM_LAUNCH
  check_launch("k_pull_claim_bk");
}

void launch_commit_claims(const DevTable& t, const uint64_t* bkeys, const uint32_t* bstart,
                          const uint32_t* unum, const uint32_t* ubase, int P, const int* slots32,
                          const float* snap, hipStream_t st, int* err) {
  if (P <= 0) return;
  check_claim_table(t);
  hipLaunchKernelGGL(k_commit_claims, dim3(P), dim3(256), 0, st, t, bkeys, bstart, unum, ubase,
                     slots32, reinterpret_cast<const float2*>(snap), err);
  check_launch("k_commit_claims");
}

void launch_apply(const DevTable& t, const long long* slots, const float* grads,
                  const SegList& sl, long long max_n, const OptParams& op, int G, hipStream_t st,
                  const float* snap, const uint8_t* only, int slot32) {
  if (max_n <= 0) return;
  if (slot32 && (t.dim != 1 || G != 1))
    throw_error("apply: 4-byte slot indices are for scalar rows");
  // one group per key (no grid-stride rounds: a second round is a second
  // random-access latency chain for those lanes) and 8-byte (w, h) accesses;
  // narrow multi-coordinate rows (FM): 8-byte chunks staged through LDS
  // (k_apply_st)
  const int ns = opt_state_per_coord(op.kind);
  const uint32_t W = t.dim * (uint32_t)(1 + ns);
  if (snap && t.bf16) throw_error("apply: snapshot applies need fp32 rows");
  if (!snap && pull_vec_on() && wide_rows(t) && W == t.width &&
      reinterpret_cast<uintptr_t>(grads) % 16 == 0) {
    const long long grid = grid_for(max_n, kPvL, 1 << 22);
#define SS_ARB(DD, B)                                                                          \
  hipLaunchKernelGGL((k_apply_rows<DD, B>), dim3(grid), dim3(256), 0, st, t, slots, grads, sl,   \
                     op, only)
    switch (t.dim) {
      case 32: if (t.bf16) SS_ARB(32, true); else SS_ARB(32, false); break;
      case 64: if (t.bf16) SS_ARB(64, true); else SS_ARB(64, false); break;
      default: if (t.bf16) SS_ARB(128, true); else SS_ARB(128, false); break;
    }
#undef SS_ARB
    check_launch("k_apply_rows");
    return;
  }
  if (only)
    throw_error("apply: the `only` mask needs the wide-row vector apply (dim 32 / 64 / 128, fp32 "
                "or bf16 rows, SS_PULL_VEC=1)");
  if (!snap && !t.bf16 && G > 1 && G <= 16 && t.dim > 1 && W <= (uint32_t)kStageMaxW &&
      W % 2 == 0 && W == t.width && t.row_off % 8 == 0 && t.stride % 8 == 0) {
    SS_DISPATCH_G(G, hipLaunchKernelGGL(k_apply_st<kG>, dim3(grid_for(max_n, kG, 1 << 22)),
                                        dim3(256), 0, st, t, slots, grads, sl, op));
    check_launch("k_apply_st");
    return;
  }
  SS_DISPATCH_G(G, hipLaunchKernelGGL(k_apply<kG>, dim3(grid_for(max_n, kG, 1 << 22)),
                                      dim3(256), 0, st, t, slots, grads, sl, op,
                                      reinterpret_cast<const float2*>(snap), slot32));
  check_launch("k_apply");
}

void launch_assign(const DevTable& t, const uint64_t* keys, const float* rows, long long n,
                   unsigned long long* size_ctr, int* err, int G, hipStream_t st) {
  if (n <= 0) return;
  SS_DISPATCH_G(G, hipLaunchKernelGGL(k_assign<kG>, dim3(grid_for(n, kG)), dim3(256), 0, st, t,
                                      keys, rows, n, size_ctr, err));
  check_launch("k_assign");
}

void launch_probe_hist(const DevTable& t, unsigned long long* hist, int nbins, hipStream_t st) {
  if (nbins < 2 || nbins > 256) throw_error("probe_hist: nbins must be in [2, 256]");
  check_hip(hipMemsetAsync(hist, 0, sizeof(unsigned long long) * nbins, st), "probe_hist");
  hipLaunchKernelGGL(k_probe_hist, dim3(4096), dim3(256), 0, st, t, hist, nbins);
  check_launch("k_probe_hist");
}

void launch_export(const DevTable& t, unsigned long long s0, long long n, uint64_t* keys_out,
                   float* rows_out, unsigned long long* cursor, hipStream_t st) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_export, dim3(grid_for(n, 1, 8192)), dim3(256), 0, st, t, s0, n, keys_out,
                     rows_out, cursor);
  check_launch("k_export");
}

}  // namespace ss
