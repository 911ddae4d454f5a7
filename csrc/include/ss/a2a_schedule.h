// ss/a2a_schedule.h — the peer schedule of one alltoallv exchange, as a pure
// function (host C++, no GPU runtime): which peer a rank sends to and
// receives from in each step, and which byte ranges move.
//
// The RCCL communicator (csrc/hip/comm.cpp) issues exactly these steps
// inside one ncclGroupStart/End; the tests run the schedules of all N ranks
// against each other on the CPU (every message sent once, received once,
// with matching sizes, every range inside its buffer) — the replacement of
// the reference's self-loopback transport test
// (/root/reference/src/unitest/core/transfer/transfer_test.h:13-80).
//
// Staggered order: in step k (1..N-1) rank r sends to r+k and receives from
// r-k, so the first-issued transfers of the N ranks use N distinct xGMI
// links instead of all converging on rank 0.  Step 0 is the self segment
// (a device copy, not a network message).
#pragma once
#include <cstdint>
#include <stdexcept>
#include <string>
#include <vector>

namespace ss {

struct A2aStep {
  int k;                  // step (0 = self copy)
  int to;                 // peer this rank sends to (-1: nothing to send)
  long long send_off;     // byte offset into the send buffer
  long long send_bytes;
  int from;               // peer this rank receives from (-1: nothing to receive)
  long long recv_off;     // byte offset into the receive buffer
  long long recv_bytes;
};

// counts / displacements in elements of `elem_bytes`; send_cap / recv_cap:
// buffer sizes in elements (< 0: unchecked).  Throws std::invalid_argument on
// a malformed exchange (wrong vector sizes, negative counts, a range outside
// its buffer, self counts that differ).
inline std::vector<A2aStep> a2a_schedule(int rank, int nranks,
                                         const std::vector<long long>& scounts,
                                         const std::vector<long long>& sdispls,
                                         const std::vector<long long>& rcounts,
                                         const std::vector<long long>& rdispls, int elem_bytes,
                                         long long send_cap = -1, long long recv_cap = -1) {
  auto fail = [](const std::string& m) { throw std::invalid_argument("alltoallv: " + m); };
  if (nranks < 1 || rank < 0 || rank >= nranks) fail("bad rank/nranks");
  if (elem_bytes < 1) fail("bad element size");
  const size_t n = (size_t)nranks;
  if (scounts.size() != n || sdispls.size() != n || rcounts.size() != n || rdispls.size() != n)
    fail("count/displ vectors must have nranks entries");
  for (int p = 0; p < nranks; ++p) {
    if (scounts[p] < 0 || rcounts[p] < 0 || sdispls[p] < 0 || rdispls[p] < 0)
      fail("negative count or displacement");
    if (send_cap >= 0 && sdispls[p] + scounts[p] > send_cap)
      fail("send range of peer " + std::to_string(p) + " outside the send buffer");
    if (recv_cap >= 0 && rdispls[p] + rcounts[p] > recv_cap)
      fail("recv range of peer " + std::to_string(p) + " outside the receive buffer");
  }
  if (scounts[rank] != rcounts[rank]) fail("self send/recv counts differ");
  const long long eb = elem_bytes;
  std::vector<A2aStep> out;
  out.reserve(n);
  out.push_back({0, scounts[rank] > 0 ? rank : -1, sdispls[rank] * eb, scounts[rank] * eb,
                 rcounts[rank] > 0 ? rank : -1, rdispls[rank] * eb, rcounts[rank] * eb});
  for (int k = 1; k < nranks; ++k) {
    const int to = (rank + k) % nranks;
    const int from = (rank - k + nranks) % nranks;
    out.push_back({k, scounts[to] > 0 ? to : -1, sdispls[to] * eb, scounts[to] * eb,
                   rcounts[from] > 0 ? from : -1, rdispls[from] * eb, rcounts[from] * eb});
  }
  return out;
}

}  // namespace ss
