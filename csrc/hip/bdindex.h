// bdindex.h — occurrence -> unique id through the bucketed dedup's outputs
// (bdedup.hip) without a materialised inverse index:
//   uid(j) = ubase[bkt[j]] + luid[pos_of[j]]
// bkt / pos_of are read coalesced, ubase is L2-resident, luid is one gather.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

namespace ss {

struct BdIndex {
  const uint32_t* pos_of;
  const uint32_t* luid;
  const uint32_t* bkt;
  const uint32_t* ubase;
  __device__ __forceinline__ uint32_t uid(long long j) const {
    const uint32_t p = pos_of[j];
    if (p == 0xFFFFFFFFu) return 0xFFFFFFFFu;
    const uint32_t l = luid[p];
    return l == 0xFFFFFFFFu ? 0xFFFFFFFFu : ubase[bkt[j]] + l;
  }
};

}  // namespace ss
