// ss/hash.h — key hashing shared by host C++ and gfx950 device code.
//
// Parity: `fmix64` is bit-identical to the reference's `get_hash_code`
// (MurmurHash3 finalizer, /root/reference/src/utils/HashFunction.h:16-24) so that
// key -> fragment -> node routing is reproducible against the reference
// (`to_node_id = map[fmix64(key) % frag_num]`, hashfrag.h:48-53).
//
// The device table and the batch-dedup scratch use *decorrelated* mixes
// (`table_hash`, `dedup_hash`): a shard only ever sees keys whose fmix64 falls
// into one contiguous fragment range, so re-using fmix64 for the in-shard slot
// would cluster the probe sequence.
#pragma once
#include <cstdint>

#if defined(__HIPCC__) || defined(__HIP__)
#define SS_HD __host__ __device__ __forceinline__
#else
#define SS_HD inline
#endif

namespace ss {

// Empty-slot sentinel; mirrors numeric_limits<K>::max() used as the
// dense_hash_map empty key in the reference (sparsetable.h:13).
static constexpr uint64_t kEmptyKey = ~0ull;

SS_HD uint64_t fmix64(uint64_t x) {
  x ^= x >> 33;
  x *= 0xff51afd7ed558ccdull;
  x ^= x >> 33;
  x *= 0xc4ceb9fe1a85ec53ull;
  x ^= x >> 33;
  return x;
}

SS_HD uint64_t table_hash(uint64_t key) { return fmix64(key ^ 0x9E3779B97F4A7C15ull); }
SS_HD uint64_t dedup_hash(uint64_t key) { return fmix64(key + 0xD1B54A32D192ED03ull); }

// splitmix64: counter-based RNG used for synthetic data and deterministic
// per-key parameter initialisation (independent of which lane inserts a key).
SS_HD uint64_t splitmix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

// uniform float in [0, 1) from the top 24 bits.
SS_HD float u01(uint64_t r) { return (float)(r >> 40) * (1.0f / 16777216.0f); }

// Lemire fast range reduction: maps a 64-bit hash onto [0, n) without a
// modulo and without forcing power-of-two table capacities (so a shard can be
// sized to exactly what fits in HBM).
SS_HD uint64_t fastrange64(uint64_t h, uint64_t n) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __umul64hi(h, n);
#else
  return (uint64_t)(((unsigned __int128)h * (unsigned __int128)n) >> 64);
#endif
}

}  // namespace ss
