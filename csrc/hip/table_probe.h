// table_probe.h — device helpers of the scalar-row table probe shared by the
// table kernels (table.hip) and the server's fused pull (server.hip).
#pragma once
#include "ss_device.h"

namespace ss {

__device__ __forceinline__ unsigned long long wave_sum_u64(unsigned long long v) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_down(v, o, 64);
  return v;
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
  uint64_t s = fastrange64(table_hash(key), t.cap);
  for (uint64_t n = 0; n < t.cap; ++n) {
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
    s = (s + 1 == t.cap) ? 0 : s + 1;
  }
  return -1;
}

}  // namespace ss
