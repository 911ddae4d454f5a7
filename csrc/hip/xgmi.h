// xgmi.h — host side of the xGMI peer-mailbox transport (xgmi.hip): the
// arena class the Python transport (parallel/xgmi.py) and the C++ round
// engine (round_engine.cpp) drive, and the put / wait launch descriptors.
//
// Publish tiers (XgmiArena::set_tier; parallel/xgmi.py picks the first one
// whose start-up litmus passes on every rank):
//   kTierDrain  — each put block drains its (uncached) stores with
//                 s_waitcnt vmcnt(0), then arrives; the last block of a
//                 segment bumps the receiver's flag (relaxed, system scope).
//                 Correct when the importer's mapping of the peer arena is
//                 uncached (stores are acknowledged by the fabric).
//   kTierFenced — as above plus one system-scope release per block before
//                 its arrival (only for destinations on another device,
//                 `remote` mask) and one system-scope acquire in the wait
//                 kernel: correct also if a peer mapping is L2-cached.
// A job whose litmus fails both tiers falls back to RCCL.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdlib>

#include <algorithm>
#include <cstring>
#include <string>
#include <vector>

#include "ss_launch.h"

namespace ss {

static constexpr int kXMaxRanks = 16;
static constexpr int kXMaxCh = 16;
static constexpr int kXMaxParts = 4;
static constexpr int kXMaxBpp = 1024;  // put workgroups per peer, at most
static constexpr long long kXFlagBytes = (long long)kXMaxCh * kXMaxRanks * 128;
// round tags of the verify mode: [src][put block] u32, after the flags
static constexpr long long kXTagBytes = (long long)kXMaxRanks * kXMaxBpp * 4;
static constexpr long long kXHeadBytes = kXFlagBytes + kXTagBytes;  // regions start here
// local counters: put arrivals [ch][dest], waits [ch], sent rounds [ch],
// put tickets [ch], error word(s)
static constexpr long long kXWaitedOff = (long long)kXMaxCh * kXMaxRanks;
static constexpr long long kXSentOff = kXWaitedOff + kXMaxCh;
static constexpr long long kXTicketOff = kXSentOff + kXMaxCh;
static constexpr long long kXErrOff = 2ll * kXMaxCh * kXMaxRanks;
static constexpr long long kXLocalWords = kXErrOff + 8;
static constexpr int kXPutThreads = 256;

enum XTier { kTierDrain = 0, kTierFenced = 1 };
// sticky error bits (err word; the host-mapped word gets the same bits)
enum XErr { kXErrTimeout = 1, kXErrSegment = 2, kXErrTag = 4 };

struct XPart {
  const char* src;                    // local source buffer
  long long sdispl[kXMaxRanks];       // byte offset of destination d's segment in src
  const long long* cnt;               // rows per destination (device, [nranks]) or null
  long long cnt_fixed;                // rows per destination when cnt is null
  long long row_bytes;
  long long hdr_off;                  // arena offset of this part's [nranks] count header
  long long data_off;                 // arena offset of its [nranks][seg_bytes] data
  long long seg_bytes;                // per-source segment capacity
  int skip_self;                      // this rank's own segment is read in place by its
                                      // consumer (SelfSeg): header and arrival only
};

struct XPut {
  char* peer[kXMaxRanks];             // every rank's arena in this address space
  int nranks, me, ch, nparts, bpp;    // bpp: blocks per peer
  int fenced;                         // kTierFenced: release before each arrival ...
  unsigned remote;                    // ... to the destinations set here
  int verify;                         // write the round tag of each block (SS_XGMI_VERIFY)
  unsigned long long* sent;           // [ch] rounds put (verify mode)
  unsigned long long* ticket;         // [ch] blocks of this put done (verify mode)
  int self_lite;                      // every large part skips d == me: block 0 alone
                                      // serves this rank's own segment and publishes it
  XPart part[kXMaxParts];
};

struct XWait {
  int nranks, ch;
  long long timeout_ticks;            // wall_clock64 ticks (100 MHz)
  int acquire;                        // kTierFenced: system-scope acquire after the poll
  int verify, bpp;                    // check every source's `bpp` round tags
  unsigned* host_err;                 // host-mapped error word (readable without a sync)
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
// litmus patterns: word i of a segment = mix(seed, i); check counts mismatches
void launch_xpattern(int* dst, long long words, unsigned seed, hipStream_t st);
// received rows out of the uncached mailbox into a cached buffer (k_xstage)
void launch_xstage(const char* src, const long long* cnt, int nsrc, long long seg_bytes,
                   int row_bytes, int skip, char* dst, hipStream_t st);
void launch_xcheck(const int* src, long long words, unsigned seed, int* bad, hipStream_t st);
void launch_spin(double us, hipStream_t st);

// put workgroups per peer for segments of at most `maxseg` bytes: ~32 KB per
// block, 8 at least, capped by `cap`.  Every block drains and arrives on one
// counter, and those device-scope adds serialise (~12 ns each): 1024 blocks
// for a 1 MB segment cost 12+ us of arrivals alone
inline int xput_blocks(long long maxseg, int cap) {
  const long long want = std::max(8ll, (maxseg + 32767) / 32768);
  const long long c = std::min<long long>(cap < 1 ? 1 : cap, kXMaxBpp);
  return (int)std::max(1ll, std::min(c, want));
}

class XgmiArena {
 public:
  XgmiArena(int rank, int nranks, int device, long long bytes)
      : rank_(rank), nranks_(nranks), device_(device), bytes_(bytes) {
    if (nranks < 1 || nranks > kXMaxRanks) throw_error("xgmi: 1..16 ranks");
    if (bytes < kXHeadBytes) throw_error("xgmi: arena smaller than its flag and tag area");
    check_hip(hipSetDevice(device), "hipSetDevice");
    void* p = nullptr;
    // SS_XGMI_CACHED=1 (measurement only, one-rank arenas): an ordinary
    // cached allocation — what the uncached mailbox costs its local readers
    static const bool cached = [] {
      const char* e = std::getenv("SS_XGMI_CACHED");
      return e && e[0] == '1';
    }();
    if (cached && nranks == 1)
      check_hip(hipMalloc(&p, (size_t)bytes), "xgmi arena (cached, one rank)");
    else
      check_hip(hipExtMallocWithFlags(&p, (size_t)bytes, hipDeviceMallocUncached),
                "xgmi arena (uncached)");
    base_ = static_cast<char*>(p);
    check_hip(hipMemset(base_, 0, (size_t)kXHeadBytes), "xgmi flags");
    check_hip(hipMalloc(&local_, sizeof(unsigned long long) * kXLocalWords), "xgmi counters");
    check_hip(hipMemset(local_, 0, sizeof(unsigned long long) * kXLocalWords), "xgmi counters");
    // host-mapped error word: the wait kernel stores its error bits here too,
    // so the host can poll it every round without a device synchronisation
    void* h = nullptr;
    check_hip(hipHostMalloc(&h, 64, hipHostMallocMapped | hipHostMallocCoherent),
              "xgmi host error word");
    std::memset(h, 0, 64);
    host_err_ = static_cast<volatile unsigned*>(h);
    check_hip(hipHostGetDevicePointer(reinterpret_cast<void**>(&host_err_dev_),
                                      const_cast<unsigned*>(host_err_), 0),
              "xgmi host error word (device pointer)");
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
    if (host_err_) hipHostFree(const_cast<unsigned*>(host_err_));
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
  uintptr_t err_ptr() const { return reinterpret_cast<uintptr_t>(local_ + kXErrOff); }
  unsigned host_err() const { return *host_err_; }
  // clear the sticky device and host-mapped error words (between start-up
  // litmus tiers: a failed tier's bits must not fail the next one).  Waits
  // for the device first, so no wait kernel of the earlier tier still writes.
  void reset_err() {
    check_hip(hipSetDevice(device_), "hipSetDevice");
    check_hip(hipDeviceSynchronize(), "xgmi reset_err (sync)");
    check_hip(hipMemset(local_ + kXErrOff, 0, sizeof(unsigned long long)), "xgmi reset_err");
    check_hip(hipDeviceSynchronize(), "xgmi reset_err (sync)");
    *host_err_ = 0u;
  }
  int tier() const { return tier_; }
  // tier (XTier), the destinations a fenced put releases to (bit d: rank d's
  // arena is on another device), round-tag verification
  void set_tier(int tier, unsigned remote, bool verify) {
    if (tier != kTierDrain && tier != kTierFenced) throw_error("xgmi: tier 0 (drain) or 1 (fenced)");
    tier_ = tier;
    remote_ = remote;
    verify_ = verify;
  }

  // parts: (src, cnt dev ptr or 0, cnt_fixed, row_bytes, hdr_off, data_off,
  //         seg_bytes, sdispl bytes [nranks] [, skip_self])
  void put(int ch, const std::vector<std::vector<long long>>& parts, int bpp, uintptr_t stream) {
    if (ch < 0 || ch >= kXMaxCh) throw_error("xgmi: bad channel");
    if (parts.empty() || (int)parts.size() > kXMaxParts) throw_error("xgmi: 1..4 parts");
    XPut P{};
    for (int r = 0; r < nranks_; ++r) {
      if (!peers_[r]) throw_error("xgmi: peer arenas not open");
      P.peer[r] = peers_[r];
    }
    P.nranks = nranks_;
    P.me = rank_;
    P.ch = ch;
    P.nparts = (int)parts.size();
    long long maxseg = 0;
    for (const auto& v : parts)
      if (v.size() > 6) maxseg = std::max(maxseg, v[6]);
    P.bpp = xput_blocks(maxseg, bpp);
    P.fenced = tier_ == kTierFenced;
    P.remote = remote_;
    P.verify = verify_;
    P.sent = local_ + kXSentOff + ch;
    P.ticket = local_ + kXTicketOff + ch;
    long long self_bytes = 0;  // what d == me still copies (parts not skipped)
    for (size_t q = 0; q < parts.size(); ++q) {
      const auto& v = parts[q];
      if ((int)v.size() != 7 + nranks_ && (int)v.size() != 8 + nranks_)
        throw_error("xgmi: malformed part");
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
          x.hdr_off < kXHeadBytes || x.data_off < kXHeadBytes)
        throw_error("xgmi: part outside the arena");
      if (!x.cnt && x.cnt_fixed * x.row_bytes > x.seg_bytes)
        throw_error("xgmi: fixed part larger than its segment");
      for (int r = 0; r < nranks_; ++r) x.sdispl[r] = v[7 + r];
      x.skip_self = (int)v.size() == 8 + nranks_ ? (int)v[7 + nranks_] : 0;
      if (!x.skip_self) self_bytes += x.seg_bytes;
    }
    // the own segment's leftovers (bucket-run tables) are small: one block,
    // no arrival counting (the verify tags of the other blocks then stay
    // unwritten, so verify mode keeps the full grid)
    P.self_lite = !verify_ && self_bytes <= (256ll << 10);
    // nothing but the own segment: one block.  (Sizing this grid by the bytes
    // left to copy made the block count differ between the start-up litmus
    // and the production puts of a channel; the arrival counter publishes on
    // every bpp-th arrival, so a put of another geometry could publish before
    // its last block had drained — the grid of a channel must not change.)
    if (P.self_lite && nranks_ == 1) P.bpp = 1;
    // the arrival counters (every destination but a lite own segment) publish
    // on each bpp-th arrival: one geometry per channel for the arena's life
    if (nranks_ > 1 || !P.self_lite) {
      if (!arrive_bpp_[ch]) arrive_bpp_[ch] = P.bpp;
      else if (arrive_bpp_[ch] != P.bpp)
        throw_error("xgmi: a channel's put grid changed (its arrival counter would publish early)");
    }
    // every rank puts to (ch, this arena layout) with the same geometry, so
    // the receiver's tag check uses the block count of its own put
    put_bpp_[ch] = P.bpp;
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
    W.acquire = tier_ == kTierFenced;
    W.verify = verify_ && put_bpp_[ch] > 0;
    W.bpp = put_bpp_[ch];
    W.host_err = host_err_dev_;
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
    unsigned long long* waited = local_ + kXWaitedOff;
    launch_xwait(base_, W, waited, reinterpret_cast<unsigned int*>(err_ptr()),
                 reinterpret_cast<hipStream_t>(stream));
  }

 private:
  int rank_, nranks_, device_;
  long long bytes_;
  char* base_ = nullptr;
  unsigned long long* local_ = nullptr;  // arrive[ch][dst], waited/sent/ticket[ch], err
  volatile unsigned* host_err_ = nullptr;
  unsigned* host_err_dev_ = nullptr;
  std::vector<char*> peers_;
  int tier_ = kTierDrain;
  unsigned remote_ = 0;
  bool verify_ = false;
  int put_bpp_[kXMaxCh] = {};
  int arrive_bpp_[kXMaxCh] = {};  // the block count the channel's arrival counters count in
};

long long xgmi_head_bytes();

}  // namespace ss
