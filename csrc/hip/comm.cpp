// comm.cpp — RCCL communicator (see comm.h).
#include "comm.h"

#include "ss/a2a_schedule.h"

#include <rccl/rccl.h>

#include <cstring>
#include <stdexcept>

namespace ss {

static void check_nccl(ncclResult_t r, const char* what) {
  if (r != ncclSuccess)
    throw std::runtime_error(std::string("RCCL ") + what + ": " + ncclGetErrorString(r));
}
static void check_hip_c(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
}

static ncclDataType_t to_nccl_dtype(int d) {
  switch (d) {
    case 0: return ncclFloat32;
    case 1: return ncclFloat64;
    case 2: return ncclInt32;
    case 3: return ncclInt64;
    case 4: return ncclUint8;
  }
  throw std::runtime_error("bad dtype");
}
static size_t dtype_size(int d) {
  switch (d) {
    case 0: return 4;
    case 1: return 8;
    case 2: return 4;
    case 3: return 8;
    case 4: return 1;
  }
  return 1;
}

std::string RcclComm::unique_id() {
  ncclUniqueId id;
  check_nccl(ncclGetUniqueId(&id), "ncclGetUniqueId");
  return std::string(reinterpret_cast<const char*>(&id), sizeof(id));
}

RcclComm::RcclComm(int rank, int nranks, const std::string& uid, int device)
    : rank_(rank), nranks_(nranks), device_(device) {
  if (uid.size() != sizeof(ncclUniqueId)) throw std::runtime_error("bad ncclUniqueId size");
  ncclUniqueId id;
  std::memcpy(&id, uid.data(), sizeof(id));
  check_hip_c(hipSetDevice(device), "hipSetDevice");
  ncclComm_t c;
  check_nccl(ncclCommInitRank(&c, nranks, id, rank), "ncclCommInitRank");
  comm_ = c;
}

RcclComm::~RcclComm() {
  if (comm_) ncclCommDestroy(comm_);
}

void RcclComm::abort() {
  if (comm_) {
    ncclCommAbort(comm_);
    comm_ = nullptr;
  }
}

void RcclComm::alltoallv(uintptr_t send, const std::vector<long long>& scounts,
                         const std::vector<long long>& sdispls, uintptr_t recv,
                         const std::vector<long long>& rcounts,
                         const std::vector<long long>& rdispls, int elem_bytes, uintptr_t stream,
                         long long send_cap, long long recv_cap) {
  if (!comm_) throw std::runtime_error("alltoallv on aborted communicator");
  // the whole exchange is validated (sizes, ranges inside the buffers)
  // before anything is enqueued: a bad count must not become a fault
  const std::vector<A2aStep> plan = a2a_schedule(rank_, nranks_, scounts, sdispls, rcounts,
                                                 rdispls, elem_bytes, send_cap, recv_cap);
  auto st = reinterpret_cast<hipStream_t>(stream);
  const char* sb = reinterpret_cast<const char*>(send);
  char* rb = reinterpret_cast<char*>(recv);
  const A2aStep& self = plan[0];
  if (self.send_bytes > 0)
    check_hip_c(hipMemcpyAsync(rb + self.recv_off, sb + self.send_off, self.send_bytes,
                               hipMemcpyDeviceToDevice, st),
                "alltoallv self copy");
  if (nranks_ == 1) return;
  check_nccl(ncclGroupStart(), "groupStart");
  for (size_t i = 1; i < plan.size(); ++i) {
    const A2aStep& x = plan[i];
    if (x.to >= 0)
      check_nccl(ncclSend(sb + x.send_off, x.send_bytes, ncclUint8, x.to, comm_, st), "ncclSend");
    if (x.from >= 0)
      check_nccl(ncclRecv(rb + x.recv_off, x.recv_bytes, ncclUint8, x.from, comm_, st),
                 "ncclRecv");
  }
  check_nccl(ncclGroupEnd(), "groupEnd");
}

int RcclComm::comm_count() const {
  if (!comm_) throw std::runtime_error("comm_count on aborted communicator");
  int n = 0;
  check_nccl(ncclCommCount(comm_, &n), "ncclCommCount");
  return n;
}

void RcclComm::alltoall(uintptr_t send, uintptr_t recv, long long count, int elem_bytes,
                        uintptr_t stream) {
  std::vector<long long> c(nranks_, count), d(nranks_);
  for (int i = 0; i < nranks_; ++i) d[i] = (long long)i * count;
  alltoallv(send, c, d, recv, c, d, elem_bytes, stream, -1, -1);
}

void RcclComm::allreduce(uintptr_t send, uintptr_t recv, long long count, int dtype, int op,
                         uintptr_t stream) {
  ncclRedOp_t o = op == 0 ? ncclSum : (op == 1 ? ncclMax : ncclMin);
  check_nccl(ncclAllReduce(reinterpret_cast<const void*>(send), reinterpret_cast<void*>(recv),
                           count, to_nccl_dtype(dtype), o, comm_,
                           reinterpret_cast<hipStream_t>(stream)),
             "ncclAllReduce");
}

void RcclComm::broadcast(uintptr_t buf, long long count, int dtype, int root, uintptr_t stream) {
  check_nccl(ncclBroadcast(reinterpret_cast<const void*>(buf), reinterpret_cast<void*>(buf), count,
                           to_nccl_dtype(dtype), root, comm_,
                           reinterpret_cast<hipStream_t>(stream)),
             "ncclBroadcast");
}

void RcclComm::allgather(uintptr_t send, uintptr_t recv, long long count, int dtype,
                         uintptr_t stream) {
  (void)dtype_size;
  check_nccl(ncclAllGather(reinterpret_cast<const void*>(send), reinterpret_cast<void*>(recv),
                           count, to_nccl_dtype(dtype), comm_,
                           reinterpret_cast<hipStream_t>(stream)),
             "ncclAllGather");
}

}  // namespace ss
