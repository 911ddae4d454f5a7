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
static constexpr int kXDirectMaxParts = 4;
// arrivals are counted in two levels: kXDirectGroups group counters per
// destination, then one counter for the groups.  One counter per destination
// serialises every producing workgroup's device-scope add (~12 ns each:
// 1024 buckets = 12 us, the whole kernel at small batches)
static constexpr int kXDirectGroups = 8;
static constexpr int kXDirectLine = 16;  // u64 words per counter (own 128-byte line)
static constexpr int kXDirectDestWords = (kXDirectGroups + 1) * kXDirectLine;

struct XDirect {
  char* peer[kXDirectMaxRanks];    // every rank's arena in this address space
  long long data_off[kXDirectMaxParts] = {};   // each part's [nranks][seg] data area
  long long seg_bytes[kXDirectMaxParts] = {};  // each part's per-source segment capacity
  long long hdr_off = 0;           // part 0's [nranks] i64 row-count header
  long long flag_off = 0;          // byte offset of ready[ch][me] in every arena
  long long ucap = 0;              // part-0 rows per destination in the producer's layout
  const unsigned long long* cnt = nullptr;  // part-0 rows sent to each destination (device)
  unsigned long long* arrive = nullptr;     // [dest][kXDirectDestWords] arrivals (local, monotonic)
  unsigned int* err = nullptr;     // sticky error word (bit 2: a store past its segment)
  int me = 0, nranks = 0, nparts = 0, blocks_per_dest = 1, row_bytes = 4;
};

// byte `off` of this rank's segment of part p in destination d's arena (null,
// and the error bit, past the segment)
__device__ __forceinline__ char* xd_at(const XDirect& X, int p, int d, long long off, int bytes) {
  if (off < 0 || off + bytes > X.seg_bytes[p]) {
    atomicOr(X.err, 2u);
    return nullptr;
  }
  return X.peer[d] + X.data_off[p] + (long long)X.me * X.seg_bytes[p] + off;
}
// row r of part 0
__device__ __forceinline__ char* xd_row(const XDirect& X, int d, long long r) {
  return xd_at(X, 0, d, r * X.row_bytes, X.row_bytes);
}

// one thread of producing workgroup kb (0..blocks_per_dest-1) of destination
// d, after the workgroup's stores there are drained (s_waitcnt vmcnt(0) +
// barrier): the last workgroup of its group arrives at the destination's
// counter, the last group publishes.  The count is read atomically:
// producers may have built it with device-scope adds
__device__ __forceinline__ void xd_arrive(const XDirect& X, int d, int kb) {
  const int B = X.blocks_per_dest;
  const int G = B < kXDirectGroups ? B : kXDirectGroups;
  const int g = kb % G;
  const unsigned long long ng = (unsigned long long)((B - g + G - 1) / G);  // group g's size
  unsigned long long* c = X.arrive + (long long)d * kXDirectDestWords;
  const unsigned long long o1 =
      __hip_atomic_fetch_add(c + g * kXDirectLine, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if ((o1 + 1) % ng != 0) return;
  const unsigned long long o2 = __hip_atomic_fetch_add(c + kXDirectGroups * kXDirectLine, 1ull,
                                                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if ((o2 + 1) % (unsigned long long)G != 0) return;
  const unsigned long long rows =
      __hip_atomic_load(&X.cnt[d], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  *reinterpret_cast<volatile long long*>(X.peer[d] + X.hdr_off + 8ll * X.me) = (long long)rows;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __hip_atomic_fetch_add(reinterpret_cast<unsigned long long*>(X.peer[d] + X.flag_off), 1ull,
                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

}  // namespace ss
