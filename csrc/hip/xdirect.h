// xdirect.h — a producing kernel's rows stored straight into the peers'
// xGMI mailboxes (the put fused into the kernel that makes the segment).
//
// The put kernel (xgmi.hip k_xput) copies a finished send segment from local
// HBM into every peer's arena: one more read + write of the segment and one
// more launch on the stream's critical chain.  A producer whose output is
// CONTIGUOUS per destination (a bucket's merged gradient rows are one run of
// the destination's segment) can store its rows into the peer arena itself,
// drain them, and arrive: the last of a destination's `blocks_per_dest`
// producing workgroups writes the segment's row count into the receiver's
// header and publishes the (channel, source) ready flag — the same protocol
// as k_xput (uncached arena, stores drained before the flag's system-scope
// add), so the receiver's wait kernel cannot tell the two apart.
// (Scattered rows — the server's response rows at received positions —
// measured slower as direct uncached stores; they keep the bulk put.)
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

namespace ss {

static constexpr int kXDirectMaxRanks = 16;

struct XDirect {
  char* peer[kXDirectMaxRanks];    // every rank's arena in this address space
  long long data_off = 0;          // the region's [nranks][seg_bytes] data area
  long long seg_bytes = 0;         // per-source segment capacity
  long long hdr_off = 0;           // the region's [nranks] i64 row-count header
  long long flag_off = 0;          // byte offset of ready[ch][me] in every arena
  long long ucap = 0;              // rows per destination in the producer's layout
  const unsigned long long* cnt = nullptr;  // rows sent to each destination (device)
  unsigned long long* arrive = nullptr;     // per-destination arrivals (local, monotonic)
  unsigned int* err = nullptr;     // sticky error word (bit 2: a row past its segment)
  int me = 0, nranks = 0, blocks_per_dest = 1, row_bytes = 4;
};

// row r of this rank's segment in destination d's arena (null past the segment)
__device__ __forceinline__ char* xd_row(const XDirect& X, int d, long long r) {
  if (r < 0 || (r + 1) * X.row_bytes > X.seg_bytes) {
    atomicOr(X.err, 2u);
    return nullptr;
  }
  return X.peer[d] + X.data_off + (long long)X.me * X.seg_bytes + r * X.row_bytes;
}

// one thread of a producing workgroup, after the workgroup's stores to
// destination d are drained (s_waitcnt vmcnt(0) + barrier)
__device__ __forceinline__ void xd_arrive(const XDirect& X, int d) {
  const unsigned long long old =
      __hip_atomic_fetch_add(&X.arrive[d], 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if ((old + 1) % (unsigned long long)X.blocks_per_dest != 0) return;
  *reinterpret_cast<volatile long long*>(X.peer[d] + X.hdr_off + 8ll * X.me) = (long long)X.cnt[d];
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __hip_atomic_fetch_add(reinterpret_cast<unsigned long long*>(X.peer[d] + X.flag_off), 1ull,
                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

}  // namespace ss
