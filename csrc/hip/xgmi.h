// xgmi.h — host side of the xGMI peer-mailbox transport (xgmi.hip): the
// arena class the Python transport (parallel/xgmi.py) and the C++ round
// engine (round_engine.cpp) drive, and the put / wait launch descriptors.
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <string>
#include <vector>

#include "ss_launch.h"

namespace ss {

static constexpr int kXMaxRanks = 16;
static constexpr int kXMaxCh = 16;
static constexpr int kXMaxParts = 4;
static constexpr long long kXFlagBytes = (long long)kXMaxCh * kXMaxRanks * 128;
// local counters: put arrivals [ch][dest], waits [ch], error word(s)
static constexpr long long kXLocalWords = 2ll * kXMaxCh * kXMaxRanks + 8;
static constexpr int kXPutThreads = 256;

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

void launch_xput(const XPut& P, unsigned long long* arrive, unsigned int* err, hipStream_t st);
void launch_xwait(char* arena, const XWait& W, unsigned long long* waited, unsigned int* err,
                  hipStream_t st);

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
    check_hip(hipMalloc(&local_, sizeof(unsigned long long) * kXLocalWords), "xgmi counters");
    check_hip(hipMemset(local_, 0, sizeof(unsigned long long) * kXLocalWords), "xgmi counters");
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
    launch_xput(P, arrive, reinterpret_cast<unsigned int*>(err_ptr()),
                reinterpret_cast<hipStream_t>(stream));
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
    launch_xwait(base_, W, waited, reinterpret_cast<unsigned int*>(err_ptr()),
                 reinterpret_cast<hipStream_t>(stream));
  }

 private:
  int rank_, nranks_, device_;
  long long bytes_;
  char* base_ = nullptr;
  unsigned long long* local_ = nullptr;  // arrive[ch][dst], waited[ch], err
  std::vector<char*> peers_;
};

long long xgmi_flag_bytes();

}  // namespace ss
