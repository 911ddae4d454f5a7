// comm.h — native RCCL communicator for the collective round engine.
//
// Replaces the reference's ZeroMQ PUSH/PULL full mesh and its RPC layer
// (Listener/Route/Transfer, /root/reference/src/core/transfer/*.h) on the
// data plane.  Every pull/push round is a set of alltoallv exchanges:
//
//   counts  : ncclAllToAll(int64 x 1 per peer)            (M4 phase A)
//   keys    : alltoallv(u64 keys)     worker -> server       (M4 phase B)
//   values  : alltoallv(f32 rows)     server -> worker       (M4 phase C)
//   grads   : alltoallv(f32 rows)     worker -> server       (M5)
//
// alltoallv is a grouped ncclSend/ncclRecv with per-peer displacements, so
// messages are read from / written to fixed segments (peer * capacity) that
// the dedup/route kernel wrote directly — no pack/unpack copies.  On an
// MI355X node every GPU pair has its own xGMI link, so the grouped p2p
// exchange runs all 7 links concurrently (no ring, no per-link serialisation).
// The self segment is a device-to-device hipMemcpyAsync.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>
#include <string>
#include <vector>

struct ncclComm;

namespace ss {

class RcclComm {
 public:
  static std::string unique_id();  // 128-byte ncclUniqueId as raw bytes
  RcclComm(int rank, int nranks, const std::string& uid, int device);
  ~RcclComm();
  RcclComm(const RcclComm&) = delete;
  RcclComm& operator=(const RcclComm&) = delete;

  int rank() const { return rank_; }
  int nranks() const { return nranks_; }

  // Byte-granular alltoallv. counts/displs are in elements of `elem_bytes`.
  void alltoallv(uintptr_t send, const std::vector<long long>& scounts,
                 const std::vector<long long>& sdispls, uintptr_t recv,
                 const std::vector<long long>& rcounts, const std::vector<long long>& rdispls,
                 int elem_bytes, uintptr_t stream, long long send_cap = -1,
                 long long recv_cap = -1);
  // ranks of the communicator as RCCL reports them (ncclCommCount)
  int comm_count() const;
  // Fixed-size alltoall: `count` elements of `elem_bytes` per peer.
  void alltoall(uintptr_t send, uintptr_t recv, long long count, int elem_bytes, uintptr_t stream);
  // dtype: 0=f32 1=f64 2=i32 3=i64 ; op: 0=sum 1=max 2=min
  void allreduce(uintptr_t send, uintptr_t recv, long long count, int dtype, int op,
                 uintptr_t stream);
  void broadcast(uintptr_t buf, long long count, int dtype, int root, uintptr_t stream);
  void allgather(uintptr_t send, uintptr_t recv, long long count, int dtype, uintptr_t stream);
  void abort();

 private:
  ncclComm* comm_ = nullptr;
  int rank_ = 0, nranks_ = 1, device_ = 0;
};

}  // namespace ss
