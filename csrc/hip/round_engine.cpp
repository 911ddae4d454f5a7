// round_engine.cpp — the per-round launch sequences of the GPU round engine.
//
// parallel/engine.py decides WHAT a round does (which path, which hooks, the
// snapshot bookkeeping); this class issues HOW — the stream waits, kernels,
// xGMI puts / waits and event records of one stage — as ONE call per stage
// (route end, pull, push) instead of ~4-10 Python-level calls each.  It owns
// the ring's HIP events (route done, pull done, slot free) and their capture
// tags: an event recorded in one hipGraph capture is only waited on inside
// that capture (an earlier replay has completed anyway) — the same rule the
// Python engine applied to torch events.
//
// Paths: the one-GPU path (colocated worker + shard, no exchange) and the
// N>1 xGMI mailbox path (device-side counts; server merge of server.hip).
// Host-count transports (RCCL, gloo, CPU) stay in parallel/engine_host.py.
// Reference parity: the round replaces Transfer::send / the pull and push
// access agents (/root/reference/src/core/transfer/transfer.h:75-150,
// src/core/parameter/global_pull_access.h:40-120, global_push_access.h:36-149).
#include <hip/hip_runtime.h>

#include <array>
#include <cstdlib>
#include <stdexcept>
#include <string>
#include <vector>

#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "ss_launch.h"
#include "xgmi.h"

namespace py = pybind11;

namespace ss {

namespace {
template <typename T>
T* Pt(uintptr_t p) { return reinterpret_cast<T*>(p); }
hipStream_t St(uintptr_t s) { return reinterpret_cast<hipStream_t>(s); }
}  // namespace

// device buffers of one ring slot's server merge (engine._ServerSlot)
struct SrvSlot {
  uint32_t *cnt = nullptr, *bstart = nullptr, *ubase = nullptr, *unum = nullptr;
  uint32_t *pj = nullptr, *luid = nullptr;
  uint64_t* bkeys = nullptr;
  long long* slots = nullptr;
  float* snap = nullptr;
  unsigned long long* ucount = nullptr;
};

// arena offsets of one (channel, part, slot) region
struct XReg {
  long long hdr = 0, data = 0, seg = 0;
};

class RoundEngine {
 public:
  // kGput: this rank's gradients of the slot are put (the main stream's last
  // use of the slot when the server half runs on its own stream)
  enum Kind { kRoute = 0, kPull = 1, kFree = 2, kGput = 3 };

  RoundEngine(int depth, int device) : depth_(depth), device_(device) {
    if (depth < 1 || depth > 16) throw std::invalid_argument("RoundEngine: depth 1..16");
    check_hip(hipSetDevice(device), "hipSetDevice");
    for (auto& k : ev_)
      for (int s = 0; s < depth; ++s) {
        hipEvent_t e;
        check_hip(hipEventCreateWithFlags(&e, hipEventDisableTiming), "hipEventCreate");
        k.push_back(e);
      }
    for (auto& t : tag_) t.assign(depth, -1);
    srv_.resize(depth);
    keys_.resize(depth);
    vals_.resize(depth);
    grads_.resize(depth);
    self_keys_.assign(depth, 0);
    own_vals_.assign(depth, 0);
    srv_done_.assign(depth, 0);
    srv_s32_.assign(depth, 0);
    srv_claim_.assign(depth, 0);
  }
  ~RoundEngine() {
    hipSetDevice(device_);
    // nothing enqueued may still record or wait these events (a graph
    // replay, a stage of this engine on any stream)
    hipDeviceSynchronize();
    for (auto& k : ev_)
      for (auto e : k) hipEventDestroy(e);
  }
  RoundEngine(const RoundEngine&) = delete;
  RoundEngine& operator=(const RoundEngine&) = delete;

  // -------------------------------------------------------------- events
  // tag: the hipGraph capture the call runs in (0 = eager)
  void record(int kind, int slot, uintptr_t stream, int tag) {
    check_slot(slot);
    check_hip(hipEventRecord(ev_.at(kind)[slot], St(stream)), "hipEventRecord");
    tag_.at(kind)[slot] = tag;
  }
  void wait(int kind, int slot, uintptr_t stream, int tag) {
    check_slot(slot);
    if (tag_.at(kind)[slot] == tag)
      check_hip(hipStreamWaitEvent(St(stream), ev_.at(kind)[slot], 0), "hipStreamWaitEvent");
  }
  bool recorded(int kind, int slot) const { return tag_.at(kind).at(slot) >= 0; }
  void forget() {  // a new capture / a reset pipeline: nothing is waitable
    for (auto& t : tag_) t.assign(depth_, -1);
  }

  // ---------------------------------------------------------- N>1 set-up
  // arenas: per ring slot the (keys, vals, grads) mailbox arenas (one IPC
  // allocation each, channel 0 inside; parallel/xgmi.py); regions: keys
  // [depth][3 parts, or 4 with the sub-bucket offsets of a server split (sub
  // > 1)], vals [depth], grads [depth], each (hdr, data, seg) in its arena
  void set_xgmi(std::vector<std::vector<XgmiArena*>> arenas,
                std::vector<std::vector<long long>> keys,
                std::vector<std::vector<long long>> vals, std::vector<std::vector<long long>> grads,
                int nranks, int rank, int Pd, int sub, long long cap, int dim, int bpp,
                double timeout_s) {
    if ((int)arenas.size() != depth_ || (int)keys.size() != depth_ || (int)vals.size() != depth_ ||
        (int)grads.size() != depth_)
      throw std::invalid_argument("set_xgmi: one arena and region set per ring slot");
    ar_.assign(depth_, {nullptr, nullptr, nullptr});
    for (int s = 0; s < depth_; ++s) {
      if (arenas[s].size() != 3) throw std::invalid_argument("set_xgmi: (keys, vals, grads) arenas");
      for (int c = 0; c < 3; ++c) {
        if (!arenas[s][c]) throw std::invalid_argument("set_xgmi: null arena");
        ar_[s][c] = arenas[s][c];
      }
    }
    nkp_ = sub > 1 ? 4 : 3;
    for (int s = 0; s < depth_; ++s) {
      if ((int)keys[s].size() != 3 * nkp_ || vals[s].size() != 3 || grads[s].size() != 3)
        throw std::invalid_argument("set_xgmi: (hdr, data, seg) per part");
      for (int p = 0; p < nkp_; ++p)
        keys_[s][p] = {keys[s][3 * p], keys[s][3 * p + 1], keys[s][3 * p + 2]};
      vals_[s] = {vals[s][0], vals[s][1], vals[s][2]};
      grads_[s] = {grads[s][0], grads[s][1], grads[s][2]};
    }
    nranks_ = nranks;
    rank_ = rank;
    Pd_ = Pd;
    sub_ = sub;
    cap_ = cap;
    dim_ = dim;
    bpp_ = bpp;
    timeout_ = timeout_s;
  }
  // drop the arena pointers (the transport is closing): later N>1 stage
  // calls fail in check_xgmi instead of launching against freed arenas
  void clear_xgmi() { ar_.clear(); }
  void set_server_slot(int slot, std::vector<uintptr_t> p) {
    check_slot(slot);
    if (p.size() != 10) throw std::invalid_argument("set_server_slot: 10 pointers");
    SrvSlot& S = srv_[slot];
    S.cnt = Pt<uint32_t>(p[0]);
    S.bstart = Pt<uint32_t>(p[1]);
    S.ubase = Pt<uint32_t>(p[2]);
    S.unum = Pt<uint32_t>(p[3]);
    S.pj = Pt<uint32_t>(p[4]);
    S.luid = Pt<uint32_t>(p[5]);
    S.bkeys = Pt<uint64_t>(p[6]);
    S.slots = Pt<long long>(p[7]);
    S.snap = Pt<float>(p[8]);
    S.ucount = Pt<unsigned long long>(p[9]);
  }

  // ------------------------------------------------------------ stage 1
  // after the dedup on the route stream: N>1 — the keys + every destination's
  // per-bucket runs (+ their sub-bucket offsets) into the peers' mailboxes;
  // then the route event
  //
  // `srv_ahead` (N>1): the server half that depends on the keys alone —
  // every source's keys in (the keys wait) and the merge of the sources'
  // runs into distinct keys (k_srv_count / k_srv_dedup) — runs here on the
  // route stream too, a round ahead beside the main stream's compute, instead
  // of at the head of the pull; the table lookup stays in the pull (it must
  // see the previous round's update).  `table`: this rank hosts a shard.
  void route_end(int slot, int tag, uintptr_t route, uintptr_t ukeys, uintptr_t ucount,
                 uintptr_t runs_base, uintptr_t runs_num, uintptr_t runs_sub, bool srv_ahead,
                 bool table, uintptr_t rkeys, uintptr_t rbase, uintptr_t rnum,
                 uintptr_t srv_err) {
    check_slot(slot);
    srv_done_[slot] = false;
    if (!ar_.empty()) {
      std::vector<std::vector<long long>> parts;
      parts.push_back(part(ukeys, ucount, 0, 8, keys_[slot][0], cap_, self_bypass()));
      self_keys_[slot] = ukeys;  // the server reads this rank's own keys here
      parts.push_back(part(runs_base, 0, Pd_, 4, keys_[slot][1], Pd_));
      parts.push_back(part(runs_num, 0, Pd_, 4, keys_[slot][2], Pd_));
      if (nkp_ == 4) {
        if (!runs_sub) throw std::invalid_argument("route_end: the sub-bucket offsets");
        parts.push_back(part(runs_sub, 0, (long long)Pd_ * sub_, 4, keys_[slot][3],
                             (long long)Pd_ * sub_));
      }
      ar_[slot][0]->put(0, parts, bpp_, route);
      if (srv_ahead) {
        keys_in(slot, route, table, rkeys, rbase, rnum, srv_err);
        srv_done_[slot] = true;
      }
    }
    record(kRoute, slot, route, tag);
  }

  // ------------------------------------------------------------ stage 2
  // The pull's stream waits for the round's route (unless it IS the route
  // stream) and, pulled ahead, for the push `prev` slots back (staleness
  // bound; prev < 0: none).  One GPU: bucket pull of the dedup's unique keys
  // (+ (w, h) snapshot).  Records the pull event when `ahead`.
  void pull_fast(int slot, int tag, uintptr_t stream, bool wait_route, int prev, bool ahead,
                 const DevTable& t, const InitParams& ip, uintptr_t size_ctr, uintptr_t err, int G,
                 std::vector<uintptr_t> view, int P, uintptr_t uvals, uintptr_t slots,
                 uintptr_t snap, int slot32, bool claim, uintptr_t luid, uintptr_t occ) {
    pull_waits(slot, tag, stream, wait_route, prev);
    if (view.size() != 4) throw std::invalid_argument("pull_fast: (bkeys, bstart, unum, ubase)");
    // claim: region-aligned buckets of a region table — LDS-claimed inserts,
    // the fused merge stores the slots (k_pull_claim_bk)
    if (claim)
      launch_pull_claim_bk(t, Pt<const uint64_t>(view[0]), Pt<const uint32_t>(view[1]),
                           Pt<const uint32_t>(view[2]), Pt<const uint32_t>(view[3]), P,
                           Pt<int>(slots), occ ? nullptr : Pt<float>(uvals), Pt<float>(snap), ip,
                           Pt<unsigned long long>(size_ctr), Pt<int>(err), St(stream),
                           Pt<const uint32_t>(luid), Pt<float>(occ));
    else
      launch_pull_unique_bk(t, Pt<const uint64_t>(view[0]), Pt<const uint32_t>(view[1]),
                            Pt<const uint32_t>(view[2]), Pt<const uint32_t>(view[3]), P,
                            Pt<long long>(slots), Pt<float>(uvals), ip,
                            Pt<unsigned long long>(size_ctr), Pt<int>(err), G, St(stream),
                            Pt<float>(snap), slot32);
    if (ahead) record(kPull, slot, stream, tag);
  }

  // N>1 over the mailboxes: keys in (every source's put of this round),
  // server merge (distinct keys across sources) + lookup, response rows per
  // received position straight into the vals put, rows back; the exchange
  // counters ride on the vals wait.  `table` false: a rank without a shard.
  void pull_xgmi(int slot, int tag, uintptr_t stream, bool wait_route, int prev, bool ahead,
                 bool table, const DevTable& t, const InitParams& ip, uintptr_t size_ctr,
                 uintptr_t err, int G, uintptr_t rkeys, uintptr_t rbase, uintptr_t rnum,
                 uintptr_t srv_err, uintptr_t svals, uintptr_t rvals, bool snap, uintptr_t sent,
                 std::vector<uintptr_t> metrics, bool custom_pull, bool claim,
                 bool insert, uintptr_t srv_stream, uintptr_t own_vals) {
    check_xgmi();
    pull_waits(slot, tag, stream, wait_route, prev);
    // own_vals (record exchange): the rows of this rank's own records go to
    // this cached buffer (cap rows) instead of its uncached vals arena — the
    // forward gathers them per occurrence (SparseLRWorker, lr_fwd_g own=)
    if (own_vals && !self_bypass())
      throw std::invalid_argument("pull_xgmi: own rows need the own-segment bypass (SS_XGMI_SELF)");
    own_vals_[slot] = own_vals;
    // the server half (keys in, merge, lookup, response rows out) on the
    // server stream when the rank has one: a slow compute on the worker's
    // stream no longer holds up the rows every peer waits for.  It follows
    // the round's route (this rank's own keys are read in place) and, in
    // issue order on its stream, the server updates of earlier rounds
    const uintptr_t ss = srv_stream ? srv_stream : stream;
    if (ss != stream) {
      if (custom_pull) throw std::invalid_argument("pull_xgmi: tensor-code pull hooks run on the caller's stream");
      wait(kRoute, slot, ss, tag);
      if (prev >= 0) wait(kFree, prev, ss, tag);
    }
    // the keys in and the server's distinct-key merge, unless the route ran them
    if (!srv_done_[slot]) keys_in(slot, ss, table, rkeys, rbase, rnum, srv_err);
    srv_done_[slot] = false;
    if (table) {
      SrvSlot& S = srv_[slot];
      // snapshot pulls of 16-byte scalar slots in a shard under 2^31 slots
      // store 4-byte slot indices; the push's fused merge reads them back
      srv_s32_[slot] = snap && G == 1 && t.stride == 16 && t.key_off == 8 && t.row_off == 0 &&
                       t.cap < (1ull << 31) && slot32_on();
      // claim: every server sub-bucket is whole regions of this shard (the
      // senders' region buckets): LDS-claimed inserts, the push's fused merge
      // stores [w | h | key] (synchronous snapshot rounds only)
      srv_claim_[slot] = claim && srv_s32_[slot];
      if (!insert) {  // read-only (PSEngine.lookup): nothing inserted, zeros if absent
        if (snap || claim || custom_pull)
          throw std::invalid_argument("pull_xgmi: a read-only lookup takes no snapshot / claim / hook");
        srv_s32_[slot] = srv_claim_[slot] = 0;
        launch_lookup_bk(t, S.bkeys, S.bstart, S.unum, S.ubase, Pd_ * sub_, Pt<float>(svals), G,
                         St(ss));
      } else if (srv_claim_[slot]) {
        // scalar rows: the response fill (rows per received position) fused
        // into the claimed pull — the bucket's rows are staged in its LDS
        // (SS_SRV_FILL_FUSED=0: the separate fill kernel)
        const bool fused = dim_ == 1 && !custom_pull && srv_fill_fused();
        launch_pull_claim_bk(t, S.bkeys, S.bstart, S.unum, S.ubase, Pd_ * sub_,
                             reinterpret_cast<int*>(S.slots), fused ? nullptr : Pt<float>(svals),
                             S.snap, ip, Pt<unsigned long long>(size_ctr), Pt<int>(err), St(ss),
                             fused ? S.luid : nullptr, fused ? Pt<float>(rvals) : nullptr,
                             fused ? S.pj : nullptr, fused ? vals_self(slot) : SelfSeg{});
        if (fused) {
          fill_and_put(slot, ss, 0, rvals, true);
          rows_wait(slot, stream, sent, metrics);
          if (ahead) record(kPull, slot, stream, tag);
          return;
        }
      } else
        launch_pull_unique_bk(t, S.bkeys, S.bstart, S.unum, S.ubase, Pd_ * sub_, S.slots,
                              Pt<float>(svals), ip, Pt<unsigned long long>(size_ctr), Pt<int>(err),
                              G, St(ss), snap ? S.snap : nullptr, srv_s32_[slot]);
      if (custom_pull) return;  // the caller finishes the pull (tensor-code hooks)
      fill_and_put(slot, ss, svals, rvals);
    } else {
      fill_and_put(slot, ss, 0, rvals);
    }
    rows_wait(slot, stream, sent, metrics);
    if (ahead) record(kPull, slot, stream, tag);
  }
  // the second half of pull_xgmi after a tensor-code pull hook ran
  void pull_xgmi_finish(int slot, int tag, uintptr_t stream, bool ahead, uintptr_t svals,
                        uintptr_t rvals, uintptr_t sent, std::vector<uintptr_t> metrics) {
    check_xgmi();
    fill_and_put(slot, stream, svals, rvals);
    rows_wait(slot, stream, sent, metrics);
    if (ahead) record(kPull, slot, stream, tag);
  }



  // ------------------------------------------------------------ stage 3
  // One GPU: the optimizer update at the pulled slots (compact unique ids,
  // count on the device; `snap`: blind store from the pull's snapshot), then
  // the slot-free event on the main stream.  `apply` false: the model's
  // merge kernel already updated the rows (fuse_apply).
  void push_fast(int slot, int tag, uintptr_t stream, bool apply, const DevTable& t,
                 const OptParams& op, int G, uintptr_t slots, uintptr_t grads, uintptr_t ucount,
                 long long max_n, uintptr_t snap, int slot32) {
    check_slot(slot);
    if (apply) {
      SegList sl{};
      sl.nseg = 1;
      sl.dev_count = Pt<const long long>(ucount);
      launch_apply(t, Pt<const long long>(slots), Pt<const float>(grads), sl, max_n, op, G,
                   St(stream), Pt<const float>(snap), nullptr, slot32);
    }
    record(kFree, slot, stream, tag);
  }

  // N>1: gradient rows into the servers' mailboxes, wait for every source's,
  // server merge per distinct key — fused with the AdaGrad update for scalar
  // rows (from the snapshot or the row) or into the row update (wider
  // rows), then the slot-free event; `update`
  // false: merged rows only (`merged`), the caller applies them (the apply
  // kernel, or a tensor-code rule) and releases the slot.
  void push_xgmi(int slot, int tag, uintptr_t stream, uintptr_t grads, uintptr_t ucount,
                 bool table, bool update, const DevTable& t, const OptParams& op, uintptr_t rgrads,
                 bool scalar_fused, bool snap, uintptr_t merged, bool release,
                 uintptr_t srv_stream, uintptr_t gstage, std::vector<uintptr_t> own_grad) {
    // own_grad (record exchange): (per-sample gradient, spj, F, feature
    // values or 0) of this rank's own records, which k_rec_grad did not write
    // out — the server merge reads gs[spj[p] / F] * x for its own positions
    if (!own_grad.empty() && (own_grad.size() != 4 || !own_grad[0] || !own_grad[1] ||
                              own_grad[2] < 1 || !self_bypass() || dim_ != 1))
      throw std::invalid_argument("push_xgmi: own_grad = (gs, spj, F, xval), scalar rows, bypass on");
    check_xgmi();
    std::vector<std::vector<long long>> parts;
    parts.push_back(part(grads, ucount, 0, 4ll * dim_, grads_[slot], cap_, self_bypass()));
    ar_[slot][2]->put(0, parts, bpp_, stream);
    // the server half (gradients in, merge + update, slot free) on the server
    // stream: it follows this put (the worker's last use of the slot)
    const uintptr_t ss = srv_stream ? srv_stream : stream;
    if (ss != stream) {
      if (!(update && release)) throw std::invalid_argument("push_xgmi: the server stream runs fused updates only");
      record(kGput, slot, stream, tag);
      wait(kGput, slot, ss, tag);
    }
    stream = ss;
    ar_[slot][2]->wait(0, {}, timeout_, stream, {}, 0.0);
    if (table) {
      SrvSlot& S = srv_[slot];
      const int Ps = Pd_ * sub_;
      SelfSeg sg = self_seg(grads);  // this rank's own gradient rows, in place
      if (!own_grad.empty()) {
        sg.ptr = reinterpret_cast<char*>(own_grad[0]);
        sg.ind = Pt<const uint32_t>(own_grad[1]);
        sg.F = (uint32_t)own_grad[2];
        sg.xv = Pt<const float>(own_grad[3]);
        if (gstage || !(update && scalar_fused))
          throw std::invalid_argument("push_xgmi: own_grad needs the fused scalar merge, no staging");
      }
      // the peers' gradient rows streamed out of the uncached mailbox into a
      // cached buffer first: the merge gathers them per received position
      if (gstage && nranks_ > 1) {
        launch_xstage(Pt<const char>(rgrads),
                      Pt<const long long>(ar_[slot][2]->base() + grads_[slot].hdr), nranks_,
                      grads_[slot].seg, 4 * dim_, sg.ptr ? rank_ : -1, Pt<char>(gstage),
                      St(stream));
        rgrads = gstage;
      }
      if (srv_s32_[slot] && !(update && scalar_fused && snap))
        throw std::logic_error("push_xgmi: a 4-byte-slot pull needs the fused snapshot merge");
      if (srv_claim_[slot] && !(update && scalar_fused && snap))
        throw std::logic_error("push_xgmi: a claimed pull needs the fused snapshot merge");
      if (update && scalar_fused)
        launch_bd_reduce_p(Ps, S.bstart, S.ubase, S.unum, S.pj, S.luid, Pt<const float>(rgrads),
                           1, nullptr, &t, S.slots, snap ? S.snap : nullptr, &op, St(stream), sg,
                           srv_s32_[slot], srv_claim_[slot] ? S.bkeys : nullptr);
      else if (dim_ == 1)
        launch_bd_reduce_p(Ps, S.bstart, S.ubase, S.unum, S.pj, S.luid, Pt<const float>(rgrads),
                           1, Pt<float>(merged), nullptr, nullptr, nullptr, nullptr, St(stream),
                           sg);
      else if (update)
        launch_srv_merge_rows(Ps, S.bstart, S.ubase, S.unum, S.pj, S.luid,
                              Pt<const float>(rgrads), nullptr, dim_, St(stream), &t, S.slots,
                              &op, sg);
      else
        launch_srv_merge_rows(Ps, S.bstart, S.ubase, S.unum, S.pj, S.luid,
                              Pt<const float>(rgrads), Pt<float>(merged), dim_, St(stream),
                              nullptr, nullptr, nullptr, sg);
    }
    if (release) record(kFree, slot, stream, tag);
  }

 private:
  void check_slot(int slot) const {
    if (slot < 0 || slot >= depth_) throw std::out_of_range("RoundEngine: ring slot");
  }
  void check_xgmi() const {
    if (ar_.empty()) throw std::logic_error("RoundEngine: set_xgmi first");
  }
  void pull_waits(int slot, int tag, uintptr_t stream, bool wait_route, int prev) {
    check_slot(slot);
    if (wait_route) wait(kRoute, slot, stream, tag);
    if (prev >= 0) wait(kFree, prev, stream, tag);
  }
  // one part of a put: (src, per-destination displacements, counts, fixed
  // rows, row bytes) in the arena's layout (XgmiArena::put)
  std::vector<long long> part(uintptr_t src, uintptr_t cnt, long long fixed, long long rb,
                              const XReg& r, long long stride_rows, bool skip_self = false) const {
    std::vector<long long> v = {(long long)src, (long long)cnt, fixed, rb, r.hdr, r.data, r.seg};
    for (int d = 0; d < nranks_; ++d) v.push_back((long long)d * stride_rows * rb);
    v.push_back(skip_self ? 1 : 0);
    return v;
  }
  // every source's keys of the round in (missing sources' fixed-size run
  // tables read as empty), then — a shard — their merge into distinct keys
  void keys_in(int slot, uintptr_t stream, bool table, uintptr_t rkeys, uintptr_t rbase,
               uintptr_t rnum, uintptr_t srv_err) {
    const long long nb = 4ll * Pd_;
    std::vector<std::vector<long long>> fixed = {{keys_[slot][1].data, keys_[slot][1].seg, nb},
                                                 {keys_[slot][2].data, keys_[slot][2].seg, nb}};
    if (nkp_ == 4) fixed.push_back({keys_[slot][3].data, keys_[slot][3].seg, nb * sub_});
    ar_[slot][0]->wait(0, fixed, timeout_, stream, {}, 0.0);
    if (!table) return;
    SrvSlot& S = srv_[slot];
    const uint32_t* roff =
        nkp_ == 4 ? Pt<const uint32_t>(ar_[slot][0]->base() + keys_[slot][3].data) : nullptr;
    launch_srv_dedup(Pt<const uint64_t>(rkeys), Pt<const uint32_t>(rbase),
                     Pt<const uint32_t>(rnum), cap_, nranks_, Pd_, sub_, rank_, S.cnt, S.bstart,
                     S.pj, S.luid, S.bkeys, S.ubase, S.unum, S.ucount, Pt<uint32_t>(srv_err),
                     St(stream), roff, self_seg(self_keys_[slot]));
  }
  // where the server's response rows for this rank's own keys go: its vals
  // arena (same row index), or the record exchange's cached own-row buffer
  SelfSeg vals_self(int slot) const {
    if (!own_vals_[slot]) return self_seg(ar_[slot][1]->base() + vals_[slot].data);
    SelfSeg s = self_seg(own_vals_[slot]);
    s.ptr -= (long long)rank_ * cap_ * 4ll * dim_;  // row index rank*cap + i -> own_vals[i]
    return s;
  }
  // this rank's own segment of a (cap-row) exchange, read in place from `ptr`
  SelfSeg self_seg(uintptr_t ptr) const {
    SelfSeg s;
    if (!self_bypass()) return s;
    s.ptr = reinterpret_cast<char*>(ptr);
    s.lo = (long long)rank_ * cap_;
    s.hi = s.lo + cap_;
    return s;
  }
  // SS_XGMI_SELF=0: copy the rank's own segments into its arena like the
  // peers' (the put kernel's self-copy; A/B)
  static bool self_bypass() {
    static const bool on = [] {
      const char* e = std::getenv("SS_XGMI_SELF");
      return !(e && e[0] == '0');
    }();
    return on;
  }
  // response rows of this round's received keys (per received position)
  // into the vals put, to every source
  // filled: the rows are in place already (the claimed pull's fused fill)
  void fill_and_put(int slot, uintptr_t stream, uintptr_t svals, uintptr_t rvals,
                    bool filled = false) {
    // the rows each source gets back = the keys it sent here (keys header)
    const uintptr_t rc = ar_[slot][0]->base() + keys_[slot][0].hdr;
    // the rows for this rank's own keys go straight into its vals arena (the
    // worker reads them there), the peers' into the response buffer the put
    // sends
    const SelfSeg sv = vals_self(slot);
    if (svals) {
      SrvSlot& S = srv_[slot];
      const int Ps = Pd_ * sub_;
      if (dim_ == 1)
        launch_bd_fill_occ_p(Ps, S.bstart, S.ubase, S.unum, S.luid, Pt<const float>(svals),
                             Pt<float>(rvals), S.pj, St(stream), sv);
      else
        launch_srv_fill_rows(Ps, S.bstart, S.ubase, S.pj, S.luid, Pt<const float>(svals),
                             Pt<float>(rvals), dim_, St(stream), sv);
    }
    std::vector<std::vector<long long>> parts;
    parts.push_back(part(rvals, rc, 0, 4ll * dim_, vals_[slot], cap_,
                         sv.ptr != nullptr && (svals || filled)));
    ar_[slot][1]->put(0, parts, bpp_, stream);
  }
  // wait for every server's rows of this round (+ the exchange counters)
  void rows_wait(int slot, uintptr_t stream, uintptr_t sent, const std::vector<uintptr_t>& metrics) {
    const uintptr_t rc = ar_[slot][0]->base() + keys_[slot][0].hdr;
    std::vector<uintptr_t> m = metrics;
    if (!m.empty()) {
      if (m.size() != 3) throw std::invalid_argument("pull_xgmi: metrics = (acc, xval, xacc)");
      m = {sent, rc, metrics[0], metrics[1], metrics[2]};
    }
    ar_[slot][1]->wait(0, {}, timeout_, stream, m, 8.0 + 8.0 * dim_);
  }

  int depth_, device_;
  std::array<std::vector<hipEvent_t>, 4> ev_;
  std::array<std::vector<int>, 4> tag_;
  std::vector<SrvSlot> srv_;
  std::vector<std::array<XgmiArena*, 3>> ar_;  // per slot: keys, vals, grads
  std::vector<std::array<XReg, 4>> keys_;
  int nkp_ = 3;  // parts of the keys channel
  std::vector<XReg> vals_, grads_;
  std::vector<uintptr_t> self_keys_;  // per slot: this rank's send layout of its keys
  std::vector<uintptr_t> own_vals_;   // per slot: own records' rows (0: the vals arena)
  std::vector<char> srv_done_;        // per slot: the route ran keys_in (srv_ahead)
  std::vector<char> srv_s32_;         // per slot: the server pull stored 4-byte slots
  std::vector<char> srv_claim_;       // per slot: ... and claimed its inserts (no CAS)
  static bool srv_fill_fused() {  // SS_SRV_FILL_FUSED=0: a separate server fill kernel
    static const bool on = [] {
      const char* e = std::getenv("SS_SRV_FILL_FUSED");
      return !(e && e[0] == '0');
    }();
    return on;
  }
  static bool slot32_on() {           // SS_SLOT32=0: 8-byte slot indices
    static const bool on = [] {
      const char* e = std::getenv("SS_SLOT32");
      return !(e && e[0] == '0');
    }();
    return on;
  }
  int nranks_ = 1, rank_ = 0, Pd_ = 1, sub_ = 1, dim_ = 1, bpp_ = 128;
  long long cap_ = 0;
  double timeout_ = 120.0;
};

void bind_round_engine(py::module_& m) {
  py::class_<RoundEngine>(m, "RoundEngine", py::module_local())
      .def(py::init<int, int>(), py::arg("depth"), py::arg("device"))
      .def("record", &RoundEngine::record)
      .def("wait", &RoundEngine::wait)
      .def("recorded", &RoundEngine::recorded)
      .def("forget", &RoundEngine::forget)
      // the engine keeps raw arena pointers: keep the arenas alive with it
      .def("set_xgmi", &RoundEngine::set_xgmi, py::keep_alive<1, 2>())
      .def("clear_xgmi", &RoundEngine::clear_xgmi)
      .def("set_server_slot", &RoundEngine::set_server_slot)
      .def("route_end", &RoundEngine::route_end)
      .def("pull_fast", &RoundEngine::pull_fast)
      .def("pull_xgmi", &RoundEngine::pull_xgmi)
      .def("pull_xgmi_finish", &RoundEngine::pull_xgmi_finish)
      .def("push_fast", &RoundEngine::push_fast)
      .def("push_xgmi", &RoundEngine::push_xgmi);
}

}  // namespace ss
