// comm.cpp — RCCL communicator (see comm.h).
#include "comm.h"

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
                         const std::vector<long long>& rdispls, int elem_bytes, uintptr_t stream) {
  if ((int)scounts.size() != nranks_ || (int)sdispls.size() != nranks_ ||
      (int)rcounts.size() != nranks_ || (int)rdispls.size() != nranks_)
    throw std::runtime_error("alltoallv: count/displ vectors must have nranks entries");
  if (!comm_) throw std::runtime_error("alltoallv on aborted communicator");
  auto st = reinterpret_cast<hipStream_t>(stream);
  const char* sb = reinterpret_cast<const char*>(send);
  char* rb = reinterpret_cast<char*>(recv);
  const size_t eb = (size_t)elem_bytes;
  if (scounts[rank_] != rcounts[rank_])
    throw std::runtime_error("alltoallv: self send/recv counts differ");
  if (scounts[rank_] > 0)
    check_hip_c(hipMemcpyAsync(rb + rdispls[rank_] * eb, sb + sdispls[rank_] * eb,
                               scounts[rank_] * eb, hipMemcpyDeviceToDevice, st),
                "alltoallv self copy");
  check_nccl(ncclGroupStart(), "groupStart");
  for (int k = 1; k < nranks_; ++k) {
    // staggered peer order: rank r talks to r+k and r-k in step k, spreading
    // the first-issued transfers over distinct xGMI links.
    const int to = (rank_ + k) % nranks_;
    const int from = (rank_ - k + nranks_) % nranks_;
    if (scounts[to] > 0)
      check_nccl(ncclSend(sb + sdispls[to] * eb, scounts[to] * eb, ncclUint8, to, comm_, st),
                 "ncclSend");
    if (rcounts[from] > 0)
      check_nccl(ncclRecv(rb + rdispls[from] * eb, rcounts[from] * eb, ncclUint8, from, comm_, st),
                 "ncclRecv");
  }
  check_nccl(ncclGroupEnd(), "groupEnd");
}

void RcclComm::alltoall(uintptr_t send, uintptr_t recv, long long count, int elem_bytes,
                        uintptr_t stream) {
  std::vector<long long> c(nranks_, count), d(nranks_);
  for (int i = 0; i < nranks_; ++i) d[i] = (long long)i * count;
  alltoallv(send, c, d, recv, c, d, elem_bytes, stream);
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
