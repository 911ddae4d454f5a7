// xgmi.hip — peer-to-peer exchange over xGMI with device-side counts.
//
// The RCCL data plane needs every alltoallv's counts on the host (a D2H +
// host wait per round, no hipGraph capture).  Here each rank exports one
// uncached HBM arena through an IPC handle and maps every peer's arena into
// its address space; a `put` kernel stores a round's segments straight into
// the peers' arenas over xGMI (counts read from device memory, written into
// the receiver's header) and bumps a per-(channel, source) counter in the
// receiver's arena; a `wait` kernel on the consumer's stream spins until
// every source's counter has reached the round.  No host synchronisation, no
// per-round host counts: the whole N>1 step can be captured as a graph.
// This is the SURVEY §7.4 "one-sided path (xGMI peer-mapped mailboxes)".
//
// Replaces, on the data plane, the reference's Transfer::send / main_loop
// (/root/reference/src/core/transfer/transfer.h:75-150): a "message" is a
// segment store into the peer's mailbox, its arrival a counter the receiver
// polls, and — like the reference — the receiver learns the payload size
// from the message, not from a separate count exchange.
//
// Arena layout (identical on every rank):
//   [0, 32 KB)       flags: ready[ch][src] u64 counters, one 128-byte line each
//   regions          per (channel, slot): per part a [nranks] i64 count header
//                    (padded to 256 B) and a [nranks][seg_bytes] data area;
//                    source s writes header[s] and data[s]
//
// Ordering: arenas are uncached (hipDeviceMallocUncached), so every store
// into one bypasses the L2s and is complete once acknowledged: each block of
// a put drains its stores (s_waitcnt vmcnt(0)) before it arrives on a local
// counter, and the block that completes a peer's segment then bumps that
// peer's ready counter (a system-scope atomic).  No release / acquire FENCES:
// at system scope they write back / invalidate a whole L2, which measured
// 3x slower for every kernel sharing the chip (1024 put workgroups each
// writing back, a spinning wait invalidating per poll).  The wait kernel
// polls with system-scope (cache-bypassing) relaxed loads; consumers read
// the arena uncached, so no L2 can hold a stale line of a rewritten segment.
//
// Liveness: a wait gives up after `timeout_s` (sticky error word, the
// missing sources' fixed-size parts zeroed so consumers read empty runs), so
// a dead peer ends in an exception at the next check point, not a hung GPU.
// Buffer reuse needs no credits: a slot is rewritten `depth` rounds later,
// after the engine's own event chain has consumed it (parallel/engine.py).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <string>
#include <vector>

#include "ss_launch.h"

namespace ss {

static constexpr int kXMaxRanks = 16;
static constexpr int kXMaxCh = 16;
static constexpr int kXMaxParts = 3;
static constexpr long long kXFlagBytes = (long long)kXMaxCh * kXMaxRanks * 128;
static constexpr int kXPutThreads = 256;

__device__ __forceinline__ unsigned long long* xflag(char* arena, int ch, int src) {
  return reinterpret_cast<unsigned long long*>(arena + ((long long)ch * kXMaxRanks + src) * 128);
}

struct XPart {
  const char* src;                    // local source buffer
  long long sdispl[kXMaxRanks];       // byte offset of destination d's segment in src
  const long long* cnt;               // rows per destination (device, [nranks]) or null
  long long cnt_fixed;                // rows per destination when cnt is null
  long long row_bytes;
  long long hdr_off;                  // arena offset of this part's [nranks] count header
  long long data_off;                 // arena offset of its [nranks][seg_bytes] data
  long long seg_bytes;                // per-source segment capacity
};

struct XPut {
  char* peer[kXMaxRanks];             // every rank's arena in this address space
  int nranks, me, ch, nparts, bpp;    // bpp: blocks per peer
  XPart part[kXMaxParts];
};

__global__ __launch_bounds__(kXPutThreads) void k_xput(XPut P, unsigned long long* arrive,
                                                       unsigned int* err) {
  const int d = blockIdx.y, b = blockIdx.x, t = threadIdx.x;
  char* dst_arena = P.peer[d];
  for (int q = 0; q < P.nparts; ++q) {
    const XPart& x = P.part[q];
    long long rows = x.cnt ? x.cnt[d] : x.cnt_fixed;
    long long bytes = rows * x.row_bytes;
    if (bytes < 0 || bytes > x.seg_bytes) {  // never write past a segment
      if (b == 0 && t == 0) atomicOr(err, 2u);
      bytes = bytes < 0 ? 0 : x.seg_bytes;
      rows = bytes / x.row_bytes;
    }
    const char* s = x.src + x.sdispl[d];
    char* o = dst_arena + x.data_off + (long long)P.me * x.seg_bytes;
    if (b == 0 && t == 0)
      *reinterpret_cast<volatile long long*>(dst_arena + x.hdr_off + 8ll * P.me) = rows;
    const long long stride = (long long)P.bpp * kXPutThreads;
    if ((((uintptr_t)s | (uintptr_t)o) & 15) == 0) {
      const long long n16 = bytes >> 4;
      const int4* s4 = reinterpret_cast<const int4*>(s);
      int4* o4 = reinterpret_cast<int4*>(o);
      for (long long i = (long long)b * kXPutThreads + t; i < n16; i += stride) o4[i] = s4[i];
      for (long long i = (n16 << 2) + (long long)b * kXPutThreads + t; i < (bytes >> 2);
           i += stride)
        reinterpret_cast<int*>(o)[i] = reinterpret_cast<const int*>(s)[i];
    } else {
      for (long long i = (long long)b * kXPutThreads + t; i < (bytes >> 2); i += stride)
        reinterpret_cast<int*>(o)[i] = reinterpret_cast<const int*>(s)[i];
    }
  }
  // drain this block's (uncached) stores to the fabric, then arrive
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (t == 0) {
    const unsigned long long old = __hip_atomic_fetch_add(
        &arrive[d], 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if ((old + 1) % (unsigned long long)P.bpp == 0) {
      // the last block of peer d's segment: every block's stores are
      // acknowledged (they arrived after draining), publish the segment
      __hip_atomic_fetch_add(xflag(dst_arena, P.ch, P.me), 1ull, __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
}

struct XWait {
  int nranks, ch;
  long long timeout_ticks;            // wall_clock64 ticks (100 MHz)
  int nfix;                           // fixed-size parts zeroed for a missing source
  long long fix_data_off[kXMaxParts];
  long long fix_seg_bytes[kXMaxParts];
  long long fix_bytes[kXMaxParts];
  // optional exchange counters, added once the wait is over (no launch of
  // their own): acc[0..2] += sum(sent), sum(recv), bpk * both; xacc += *xval
  const long long* m_sent;
  const long long* m_recv;
  double m_bpk;
  double* m_acc;
  const long long* m_xval;
  double* m_xacc;
};

__global__ __launch_bounds__(64) void k_xwait(char* arena, XWait W,
                                              unsigned long long* waited,
                                              unsigned int* err) {
  const int s = threadIdx.x;
  const unsigned long long target = waited[W.ch] + 1;
  bool ok = true;
  if (s < W.nranks) {
    const unsigned long long* f = xflag(arena, W.ch, s);
    const long long t0 = wall_clock64();
    while (__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) < target) {
      if (wall_clock64() - t0 > W.timeout_ticks) {
        ok = false;
        break;
      }
      __builtin_amdgcn_s_sleep(8);
    }
    if (!ok) {
      atomicOr(err, 1u);
      // the source never arrived: its fixed-size parts (bucket runs) read
      // as empty instead of as whatever the slot held
      for (int q = 0; q < W.nfix; ++q) {
        int* z = reinterpret_cast<int*>(arena + W.fix_data_off[q] + (long long)s * W.fix_seg_bytes[q]);
        for (long long i = 0; i < W.fix_bytes[q] / 4; ++i) z[i] = 0;
      }
    }
  }
  __syncthreads();
  if (s == 0) {
    waited[W.ch] = target;
    if (W.m_acc) {
      long long a = 0, b = 0;
      for (int i = 0; i < W.nranks; ++i) {
        a += W.m_sent[i];
        b += W.m_recv[i];
      }
      W.m_acc[0] += (double)a;
      W.m_acc[1] += (double)b;
      W.m_acc[2] += W.m_bpk * (double)(a + b);
    }
    if (W.m_xacc) W.m_xacc[0] += (double)W.m_xval[0];
  }
}

// ---------------------------------------------------------------- host side
class XgmiArena {
 public:
  XgmiArena(int rank, int nranks, int device, long long bytes)
      : rank_(rank), nranks_(nranks), device_(device), bytes_(bytes) {
    if (nranks < 1 || nranks > kXMaxRanks) throw_error("xgmi: 1..16 ranks");
    if (bytes < kXFlagBytes) throw_error("xgmi: arena smaller than its flag area");
    check_hip(hipSetDevice(device), "hipSetDevice");
    void* p = nullptr;
    check_hip(hipExtMallocWithFlags(&p, (size_t)bytes, hipDeviceMallocUncached),
              "xgmi arena (uncached)");
    base_ = static_cast<char*>(p);
    check_hip(hipMemset(base_, 0, (size_t)kXFlagBytes), "xgmi flags");
    check_hip(hipMalloc(&local_, sizeof(unsigned long long) * (2 * kXMaxCh * kXMaxRanks + 8)),
              "xgmi counters");
    check_hip(hipMemset(local_, 0, sizeof(unsigned long long) * (2 * kXMaxCh * kXMaxRanks + 8)),
              "xgmi counters");
    peers_.assign(nranks, nullptr);
    peers_[rank] = base_;
  }
  ~XgmiArena() {
    hipSetDevice(device_);
    hipDeviceSynchronize();
    for (int r = 0; r < nranks_; ++r)
      if (r != rank_ && peers_[r]) hipIpcCloseMemHandle(peers_[r]);
    if (local_) hipFree(local_);
    if (base_) hipFree(base_);
  }
  XgmiArena(const XgmiArena&) = delete;
  XgmiArena& operator=(const XgmiArena&) = delete;

  std::string ipc_handle() const {
    hipIpcMemHandle_t h;
    check_hip(hipIpcGetMemHandle(&h, base_), "hipIpcGetMemHandle");
    return std::string(reinterpret_cast<const char*>(&h), sizeof(h));
  }
  void open_peers(const std::vector<std::string>& handles) {
    if ((int)handles.size() != nranks_) throw_error("xgmi: one handle per rank");
    check_hip(hipSetDevice(device_), "hipSetDevice");
    for (int r = 0; r < nranks_; ++r) {
      if (r == rank_ || peers_[r]) continue;
      if (handles[r].size() != sizeof(hipIpcMemHandle_t)) throw_error("xgmi: bad IPC handle");
      hipIpcMemHandle_t h;
      std::memcpy(&h, handles[r].data(), sizeof(h));
      void* p = nullptr;
      check_hip(hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess),
                ("hipIpcOpenMemHandle(rank " + std::to_string(r) + ")").c_str());
      peers_[r] = static_cast<char*>(p);
    }
  }
  uintptr_t base() const { return reinterpret_cast<uintptr_t>(base_); }
  long long bytes() const { return bytes_; }
  uintptr_t err_ptr() const { return reinterpret_cast<uintptr_t>(local_ + 2 * kXMaxCh * kXMaxRanks); }

  // parts: (src, sdispl bytes [nranks], cnt dev ptr or 0, cnt_fixed, row_bytes,
  //         hdr_off, data_off, seg_bytes)
  void put(int ch, const std::vector<std::vector<long long>>& parts, int bpp, uintptr_t stream) {
    if (ch < 0 || ch >= kXMaxCh) throw_error("xgmi: bad channel");
    if (parts.empty() || (int)parts.size() > kXMaxParts) throw_error("xgmi: 1..3 parts");
    XPut P{};
    for (int r = 0; r < nranks_; ++r) {
      if (!peers_[r]) throw_error("xgmi: peer arenas not open");
      P.peer[r] = peers_[r];
    }
    P.nranks = nranks_;
    P.me = rank_;
    P.ch = ch;
    P.nparts = (int)parts.size();
    // blocks per peer: sized to the largest segment (~32 KB per block, 8 at
    // least), capped by `bpp`.  Every block drains and arrives on one
    // counter, and those device-scope adds serialise (~12 ns each): 1024
    // blocks for a 1 MB segment cost 12+ us of arrivals alone
    long long maxseg = 0;
    for (const auto& v : parts)
      if (v.size() > 6) maxseg = std::max(maxseg, v[6]);
    const long long want = std::max(8ll, (maxseg + 32767) / 32768);
    P.bpp = (int)std::max(1ll, std::min((long long)(bpp < 1 ? 1 : bpp), want));
    for (size_t q = 0; q < parts.size(); ++q) {
      const auto& v = parts[q];
      if ((int)v.size() != 7 + nranks_) throw_error("xgmi: malformed part");
      XPart& x = P.part[q];
      x.src = reinterpret_cast<const char*>(v[0]);
      x.cnt = reinterpret_cast<const long long*>(v[1]);
      x.cnt_fixed = v[2];
      x.row_bytes = v[3];
      x.hdr_off = v[4];
      x.data_off = v[5];
      x.seg_bytes = v[6];
      if (x.row_bytes < 4 || x.row_bytes % 4) throw_error("xgmi: rows of whole 4-byte words");
      if (x.data_off + (long long)nranks_ * x.seg_bytes > bytes_ || x.hdr_off + 8ll * nranks_ > bytes_ ||
          x.hdr_off < kXFlagBytes || x.data_off < kXFlagBytes)
        throw_error("xgmi: part outside the arena");
      if (!x.cnt && x.cnt_fixed * x.row_bytes > x.seg_bytes)
        throw_error("xgmi: fixed part larger than its segment");
      for (int r = 0; r < nranks_; ++r) x.sdispl[r] = v[7 + r];
    }
    unsigned long long* arrive = local_ + (long long)ch * kXMaxRanks;
    hipLaunchKernelGGL(k_xput, dim3(P.bpp, nranks_), dim3(kXPutThreads), 0,
                       reinterpret_cast<hipStream_t>(stream), P, arrive,
                       reinterpret_cast<unsigned int*>(err_ptr()));
    check_launch("k_xput");
  }

  // fixed: (data_off, seg_bytes, bytes) of the parts zeroed for a missing source
  // metrics: () or (sent, recv, acc, xval, xacc) device pointers (0 = none),
  // bpk: bytes per key of the exchange counter
  void wait(int ch, const std::vector<std::vector<long long>>& fixed, double timeout_s,
            uintptr_t stream, const std::vector<uintptr_t>& metrics, double bpk) {
    if (ch < 0 || ch >= kXMaxCh) throw_error("xgmi: bad channel");
    XWait W{};
    W.nranks = nranks_;
    W.ch = ch;
    W.timeout_ticks = (long long)(timeout_s * 1e8);
    W.nfix = (int)fixed.size();
    if (W.nfix > kXMaxParts) throw_error("xgmi: too many fixed parts");
    for (int q = 0; q < W.nfix; ++q) {
      W.fix_data_off[q] = fixed[q][0];
      W.fix_seg_bytes[q] = fixed[q][1];
      W.fix_bytes[q] = fixed[q][2];
    }
    if (!metrics.empty()) {
      if (metrics.size() != 5) throw_error("xgmi: metrics = (sent, recv, acc, xval, xacc)");
      W.m_sent = reinterpret_cast<const long long*>(metrics[0]);
      W.m_recv = reinterpret_cast<const long long*>(metrics[1]);
      W.m_acc = reinterpret_cast<double*>(metrics[2]);
      W.m_xval = reinterpret_cast<const long long*>(metrics[3]);
      W.m_xacc = reinterpret_cast<double*>(metrics[4]);
      W.m_bpk = bpk;
      if ((W.m_acc && (!W.m_sent || !W.m_recv)) || (W.m_xacc && !W.m_xval))
        throw_error("xgmi: metrics pointers incomplete");
    }
    unsigned long long* waited = local_ + kXMaxCh * kXMaxRanks;
    hipLaunchKernelGGL(k_xwait, dim3(1), dim3(64), 0, reinterpret_cast<hipStream_t>(stream),
                       base_, W, waited, reinterpret_cast<unsigned int*>(err_ptr()));
    check_launch("k_xwait");
  }

 private:
  int rank_, nranks_, device_;
  long long bytes_;
  char* base_ = nullptr;
  unsigned long long* local_ = nullptr;  // arrive[ch][dst], waited[ch], err
  std::vector<char*> peers_;
};

long long xgmi_flag_bytes() { return kXFlagBytes; }

}  // namespace ss

// bindings live here (the class is local to this translation unit)
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>
namespace py = pybind11;

// A torch tensor over device memory this module owns (the arena), through
// DLPack: a capsule whose deleter only frees the descriptor.  ABI of the
// DLPack v0.8 structs (the arena outlives every view: the transport holds it).
namespace {
struct DLDevice_ { int32_t device_type, device_id; };
struct DLDataType_ { uint8_t code, bits; uint16_t lanes; };
struct DLTensor_ {
  void* data;
  DLDevice_ device;
  int32_t ndim;
  DLDataType_ dtype;
  int64_t* shape;
  int64_t* strides;
  uint64_t byte_offset;
};
struct DLManaged_ {
  DLTensor_ t;
  void* ctx;
  void (*deleter)(DLManaged_*);
};
void dl_free(DLManaged_* m) {
  delete[] m->t.shape;
  delete m;
}
}  // namespace

static py::capsule dlpack_view(uintptr_t ptr, std::vector<int64_t> shape, int code, int bits,
                               int device) {
  auto* m = new DLManaged_{};
  m->t.data = reinterpret_cast<void*>(ptr);
  m->t.device = {10 /* kDLROCM */, device};
  m->t.ndim = (int32_t)shape.size();
  m->t.dtype = {(uint8_t)code, (uint8_t)bits, 1};
  m->t.shape = new int64_t[shape.size() ? shape.size() : 1];
  for (size_t i = 0; i < shape.size(); ++i) m->t.shape[i] = shape[i];
  m->t.strides = nullptr;
  m->t.byte_offset = 0;
  m->ctx = nullptr;
  m->deleter = dl_free;
  return py::capsule(m, "dltensor", [](PyObject* cap) {
    // an unconsumed capsule still owns its descriptor
    if (PyCapsule_IsValid(cap, "dltensor")) {
      auto* mm = static_cast<DLManaged_*>(PyCapsule_GetPointer(cap, "dltensor"));
      if (mm) mm->deleter(mm);
    }
  });
}

void bind_xgmi(py::module_& m) {
  m.def("dlpack_view", &dlpack_view, py::arg("ptr"), py::arg("shape"), py::arg("code"),
        py::arg("bits"), py::arg("device"));
  using ss::XgmiArena;
  py::class_<XgmiArena>(m, "XgmiArena", py::module_local())
      .def(py::init<int, int, int, long long>(), py::arg("rank"), py::arg("nranks"),
           py::arg("device"), py::arg("bytes"))
      .def("ipc_handle", [](const XgmiArena& a) { return py::bytes(a.ipc_handle()); })
      .def("open_peers", [](XgmiArena& a, std::vector<py::bytes> hs) {
        std::vector<std::string> v;
        for (auto& h : hs) v.emplace_back(std::string(h));
        a.open_peers(v);
      })
      .def_property_readonly("base", &XgmiArena::base)
      .def_property_readonly("bytes", &XgmiArena::bytes)
      .def_property_readonly("err_ptr", &XgmiArena::err_ptr)
      .def("put", &XgmiArena::put, py::arg("ch"), py::arg("parts"), py::arg("bpp"),
           py::arg("stream"))
      .def("wait", &XgmiArena::wait, py::arg("ch"), py::arg("fixed"), py::arg("timeout_s"),
           py::arg("stream"), py::arg("metrics") = std::vector<uintptr_t>{},
           py::arg("bpk") = 0.0);
  m.def("xgmi_flag_bytes", &ss::xgmi_flag_bytes);
}
