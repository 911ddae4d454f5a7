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
// Ordering (tiers, xgmi.h): arenas are uncached (hipDeviceMallocUncached),
// so a store into one bypasses the L2s and is complete once acknowledged:
// each block of a put drains its stores (s_waitcnt vmcnt(0)) before it
// arrives on a local counter, and the block that completes a peer's segment
// then bumps that peer's ready counter (a system-scope atomic).  This
// fence-free "drain" tier is the default: at system scope a release / acquire
// FENCE writes back / invalidates a whole L2, which measured 3x slower for
// every kernel sharing the chip (1024 put workgroups each writing back, a
// spinning wait invalidating per poll).  The "fenced" tier adds ONE
// system-scope release per block before its arrival (only towards arenas on
// another device) and ONE system-scope acquire after the wait's poll — the
// form that stays correct if an importer's mapping of a peer arena turns out
// to be L2-cached.  parallel/xgmi.py runs a full-size multi-round litmus per
// tier at start-up and uses the first that passes on every rank.  The wait
// kernel polls with system-scope (cache-bypassing) relaxed loads; consumers
// read the arena uncached, so no L2 can hold a stale line of a rewritten
// segment.
//
// Verify mode (SS_XGMI_VERIFY=1): after its payload is drained, each put
// block stores the round number into the receiver's tag area, drains it,
// then arrives; the wait kernel checks every block's tag of every source
// once the flags say the round is complete.  A flag that overtook its data
// shows up as a stale tag: sticky error bit 4 (also in the host-mapped
// error word, which the host reads every round without a sync).
//
// Liveness: a wait gives up after `timeout_s` (sticky error word, the
// missing sources' fixed-size parts zeroed so consumers read empty runs), so
// a dead peer ends in an exception at the next check point, not a hung GPU.
// Buffer reuse needs no credits: a slot is rewritten `depth` rounds later,
// after the engine's own event chain has consumed it (parallel/engine.py).
#include "xgmi.h"

namespace ss {

__device__ __forceinline__ unsigned long long* xflag(char* arena, int ch, int src) {
  return reinterpret_cast<unsigned long long*>(arena + ((long long)ch * kXMaxRanks + src) * 128);
}
__device__ __forceinline__ unsigned* xtag(char* arena, int src, int blk) {
  return reinterpret_cast<unsigned*>(arena + kXFlagBytes) + (long long)src * kXMaxBpp + blk;
}
__device__ __forceinline__ void xdrain() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

__global__ __launch_bounds__(kXPutThreads) void k_xput(XPut P, unsigned long long* arrive,
                                                       unsigned int* err) {
  const int d = blockIdx.y, b = blockIdx.x, t = threadIdx.x;
  char* dst_arena = P.peer[d];
  // this rank's own segment, consumed in place (SelfSeg): block 0 writes the
  // headers and the small parts and publishes; the other blocks have nothing
  // to do and do not arrive
  const bool lite = P.self_lite && d == P.me;
  if (lite && b > 0) return;
  // verify mode: this put's round = rounds put so far + 1 (the counter only
  // moves after every block of the put has read it: ticket below)
  const unsigned round =
      P.verify ? (unsigned)__hip_atomic_load(P.sent, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1u
               : 0u;
  for (int q = 0; q < P.nparts; ++q) {
    const XPart& x = P.part[q];
    long long rows = x.cnt ? x.cnt[d] : x.cnt_fixed;
    long long bytes = rows * x.row_bytes;
    if (bytes < 0 || bytes > x.seg_bytes) {  // never write past a segment
      if (b == 0 && t == 0) atomicOr(err, (unsigned)kXErrSegment);
      bytes = bytes < 0 ? 0 : x.seg_bytes;
      rows = bytes / x.row_bytes;
    }
    const char* s = x.src + x.sdispl[d];
    char* o = dst_arena + x.data_off + (long long)P.me * x.seg_bytes;
    if (b == 0 && t == 0)
      *reinterpret_cast<volatile long long*>(dst_arena + x.hdr_off + 8ll * P.me) = rows;
    if (x.skip_self && d == P.me) continue;  // consumed in place (SelfSeg)
    const long long stride = lite ? (long long)kXPutThreads : (long long)P.bpp * kXPutThreads;
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
  xdrain();
  __syncthreads();
  if (lite) {  // the only block of the own segment: publish it directly
    if (t == 0)
      __hip_atomic_fetch_add(xflag(dst_arena, P.ch, P.me), 1ull, __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_SYSTEM);
    return;
  }
  if (t == 0) {
    const bool fence = P.fenced && ((P.remote >> d) & 1u);
    if (P.verify) {
      // the canary goes after the drained payload, before the arrival
      *reinterpret_cast<volatile unsigned*>(xtag(dst_arena, P.me, b)) = round;
      xdrain();
    }
    if (fence) {
      // fenced tier: make every store of this workgroup (payload, header,
      // tag) visible at system scope before it counts as arrived (the wait
      // after the fence: the fence's own wait can be dropped, guide G16 p.12)
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
      xdrain();
    }
    const unsigned long long old = __hip_atomic_fetch_add(
        &arrive[d], 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if ((old + 1) % (unsigned long long)P.bpp == 0) {
      // the last block of peer d's segment: every block's stores are
      // acknowledged (they arrived after draining), publish the segment
      if (fence) {
        __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "");
        xdrain();
      }
      __hip_atomic_fetch_add(xflag(dst_arena, P.ch, P.me), 1ull, __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_SYSTEM);
    }
    if (P.verify) {
      const unsigned long long total = (unsigned long long)P.bpp * (unsigned long long)P.nranks;
      const unsigned long long tk =
          __hip_atomic_fetch_add(P.ticket, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (tk + 1 == total) {  // every block has read `sent`: the next put's round
        __hip_atomic_store(P.ticket, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_fetch_add(P.sent, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
  }
}

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
      atomicOr(err, (unsigned)kXErrTimeout);
      if (W.host_err) *reinterpret_cast<volatile unsigned*>(W.host_err) |= (unsigned)kXErrTimeout;
      // the source never arrived: its fixed-size parts (bucket runs) read
      // as empty instead of as whatever the slot held
      for (int q = 0; q < W.nfix; ++q) {
        int* z = reinterpret_cast<int*>(arena + W.fix_data_off[q] + (long long)s * W.fix_seg_bytes[q]);
        for (long long i = 0; i < W.fix_bytes[q] / 4; ++i) z[i] = 0;
      }
    }
  }
  if (W.acquire) {
    // fenced tier: one system-scope acquire after the poll, before anything
    // of this round is read (here: the tags; later kernels: the payload)
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
    xdrain();
  }
  if (ok && W.verify && s < W.nranks) {
    const unsigned want = (unsigned)target;
    bool bad = false;
    for (int b = 0; b < W.bpp; ++b)
      bad |= *reinterpret_cast<volatile unsigned*>(xtag(arena, s, b)) != want;
    if (bad) {
      atomicOr(err, (unsigned)kXErrTag);
      if (W.host_err) *reinterpret_cast<volatile unsigned*>(W.host_err) |= (unsigned)kXErrTag;
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

__device__ __forceinline__ int xpattern_word(unsigned seed, long long i) {
  unsigned x = seed ^ ((unsigned)i * 0x9E3779B1u) ^ (unsigned)(i >> 32) * 0x85EBCA77u;
  x ^= x >> 16;
  x *= 0x7FEB352Du;
  x ^= x >> 15;
  x *= 0x846CA68Bu;
  x ^= x >> 16;
  return (int)x;
}

// Received segments out of the (uncached) mailbox into a cached buffer at
// the same offsets: source s's first cnt[s] rows of row_bytes each, at byte
// s * seg_bytes, streamed with 16-byte accesses (every source but `skip`, the
// rank's own segment, which its consumer reads in place).  The server's
// gradient merge then gathers per received position from L2 / MALL instead
// of one uncached memory transaction per 4-byte gather.
__global__ __launch_bounds__(256) void k_xstage(const char* __restrict__ src,
                                                const long long* __restrict__ cnt,
                                                long long seg_bytes, int row_bytes, int skip,
                                                char* __restrict__ dst) {
  const int s = blockIdx.y;
  if (s == skip) return;  // block-uniform
  const long long n = cnt[s] * (long long)row_bytes;
  const long long nv = n / 16;
  const uint4* sv = reinterpret_cast<const uint4*>(src + s * seg_bytes);
  uint4* dv = reinterpret_cast<uint4*>(dst + s * seg_bytes);
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < nv;
       i += (long long)gridDim.x * 256)
    dv[i] = sv[i];
  const long long tail = n - nv * 16;  // whole 4-byte words (row_bytes % 4 == 0)
  if (blockIdx.x == 0 && threadIdx.x < tail / 4)
    reinterpret_cast<uint32_t*>(dst + s * seg_bytes + nv * 16)[threadIdx.x] =
        reinterpret_cast<const uint32_t*>(src + s * seg_bytes + nv * 16)[threadIdx.x];
}

void launch_xstage(const char* src, const long long* cnt, int nsrc, long long seg_bytes,
                   int row_bytes, int skip, char* dst, hipStream_t st) {
  if (nsrc < 1 || row_bytes % 4 || seg_bytes % 16) throw_error("xstage: layout");
  hipLaunchKernelGGL(k_xstage, dim3(128, nsrc), dim3(256), 0, st, src, cnt, seg_bytes, row_bytes,
                     skip, dst);
  check_launch("k_xstage");
}

__global__ __launch_bounds__(256) void k_xpattern(int* dst, long long words, unsigned seed) {
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < words;
       i += (long long)gridDim.x * 256)
    dst[i] = xpattern_word(seed, i);
}

__global__ __launch_bounds__(256) void k_xcheck(const int* src, long long words, unsigned seed,
                                                int* bad) {
  int n = 0;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < words;
       i += (long long)gridDim.x * 256)
    n += src[i] != xpattern_word(seed, i);
  if (n) atomicAdd(bad, n);
}

// one wave busy for `ticks` of the 100 MHz wall clock: a slow device on
// demand (SS_FAULT=gpudelay: a straggler whose GPU work takes longer)
__global__ __launch_bounds__(64) void k_spin(long long ticks) {
  const long long t0 = wall_clock64();
  while (wall_clock64() - t0 < ticks) __builtin_amdgcn_s_sleep(2);
}

void launch_spin(double us, hipStream_t st) {
  if (us <= 0) return;
  hipLaunchKernelGGL(k_spin, dim3(1), dim3(64), 0, st, (long long)(us * 100.0));
  check_launch("k_spin");
}

void launch_xput(const XPut& P, unsigned long long* arrive, unsigned int* err, hipStream_t st) {
  hipLaunchKernelGGL(k_xput, dim3(P.bpp, P.nranks), dim3(kXPutThreads), 0, st, P, arrive, err);
  check_launch("k_xput");
}

void launch_xwait(char* arena, const XWait& W, unsigned long long* waited, unsigned int* err,
                  hipStream_t st) {
  hipLaunchKernelGGL(k_xwait, dim3(1), dim3(64), 0, st, arena, W, waited, err);
  check_launch("k_xwait");
}

static int pattern_grid(long long words) {
  return (int)std::max(1ll, std::min(2048ll, (words + 255) / 256));
}

void launch_xpattern(int* dst, long long words, unsigned seed, hipStream_t st) {
  if (words <= 0) return;
  hipLaunchKernelGGL(k_xpattern, dim3(pattern_grid(words)), dim3(256), 0, st, dst, words, seed);
  check_launch("k_xpattern");
}

void launch_xcheck(const int* src, long long words, unsigned seed, int* bad, hipStream_t st) {
  if (words <= 0) return;
  hipLaunchKernelGGL(k_xcheck, dim3(pattern_grid(words)), dim3(256), 0, st, src, words, seed,
                     bad);
  check_launch("k_xcheck");
}

long long xgmi_head_bytes() { return kXHeadBytes; }

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
      .def_property_readonly("tier", &XgmiArena::tier)
      .def("host_err", &XgmiArena::host_err)
      .def("reset_err", &XgmiArena::reset_err)
      .def("set_tier", &XgmiArena::set_tier, py::arg("tier"), py::arg("remote"),
           py::arg("verify"))
      .def("put", &XgmiArena::put, py::arg("ch"), py::arg("parts"), py::arg("bpp"),
           py::arg("stream"))
      .def("wait", &XgmiArena::wait, py::arg("ch"), py::arg("fixed"), py::arg("timeout_s"),
           py::arg("stream"), py::arg("metrics") = std::vector<uintptr_t>{},
           py::arg("bpk") = 0.0);
  m.def("xgmi_head_bytes", &ss::xgmi_head_bytes);
  m.def("xgmi_pattern", [](uintptr_t dst, long long words, unsigned seed, uintptr_t st) {
    ss::launch_xpattern(reinterpret_cast<int*>(dst), words, seed, reinterpret_cast<hipStream_t>(st));
  });
  m.def("xgmi_check", [](uintptr_t src, long long words, unsigned seed, uintptr_t bad,
                         uintptr_t st) {
    ss::launch_xcheck(reinterpret_cast<const int*>(src), words, seed, reinterpret_cast<int*>(bad),
                      reinterpret_cast<hipStream_t>(st));
  });
  m.def("spin_us", [](double us, uintptr_t st) {
    ss::launch_spin(us, reinterpret_cast<hipStream_t>(st));
  });
  // a stream whose kernels run on `ncus` of the device's CUs only (spread
  // evenly over the CU ids, so every XCD keeps some): the route stream's
  // dedup kernels then leave the other CUs to the main stream's
  // latency-bound table kernels (SS_ROUTE_CUS).  `priority`: the stream's
  // priority (hipStreamCreateWithPriority semantics; 0 = default).  Never
  // destroyed: it lives as long as the engine that wraps it.
  m.def("cu_stream", [](int device, int ncus, int invert) {
    ss::check_hip(hipSetDevice(device), "hipSetDevice");
    int total = 0;
    ss::check_hip(hipDeviceGetAttribute(&total, hipDeviceAttributeMultiprocessorCount, device),
                  "CU count");
    if (ncus < 1 || ncus > total) throw std::invalid_argument("cu_stream: 1..CU count CUs");
    std::vector<uint32_t> mask((total + 31) / 32, invert ? 0xFFFFFFFFu : 0u);
    for (int k = 0; k < ncus; ++k) {
      const int cu = (int)((long long)k * total / ncus);
      if (invert) mask[cu / 32] &= ~(1u << (cu % 32));
      else mask[cu / 32] |= 1u << (cu % 32);
    }
    hipStream_t st = nullptr;
    ss::check_hip(hipExtStreamCreateWithCUMask(&st, (uint32_t)mask.size(), mask.data()),
                  "hipExtStreamCreateWithCUMask");
    return reinterpret_cast<uintptr_t>(st);
  }, py::arg("device"), py::arg("ncus"), py::arg("invert") = 0);
  m.def("device_pci_id", [](int device) {
    char buf[64] = {0};
    ss::check_hip(hipDeviceGetPCIBusId(buf, sizeof(buf), device), "hipDeviceGetPCIBusId");
    return std::string(buf);
  });
}
