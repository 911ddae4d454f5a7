// bindings.cpp — pybind11 module `_ss_hip`: the gfx950 kernels and the RCCL
// communicator.  Pointers and streams cross the boundary as integers
// (torch.Tensor.data_ptr(), torch.cuda.Stream.cuda_stream) so the module does
// not compile against torch headers and loads next to whatever torch build is
// present; memory is owned by torch's caching allocator on the Python side.
#include <optional>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "comm.h"
#include "worker.h"
#include "ss_launch.h"

namespace py = pybind11;
using namespace ss;

static hipStream_t S(uintptr_t s) { return reinterpret_cast<hipStream_t>(s); }
template <class T>
static T* P(uintptr_t p) {
  return reinterpret_cast<T*>(p);
}

static SegList make_seglist(const std::vector<long long>& offs, const std::vector<long long>& cnts) {
  if (offs.size() != cnts.size() || offs.empty() || offs.size() > (size_t)kMaxSeg)
    throw std::runtime_error("SegList: need 1..64 (offset, count) pairs");
  SegList sl{};
  sl.nseg = (int)offs.size();
  sl.dev_count = nullptr;
  sl.prefix[0] = 0;
  for (int i = 0; i < sl.nseg; ++i) {
    if (cnts[i] < 0) throw std::runtime_error("SegList: negative count");
    sl.off[i] = offs[i];
    sl.prefix[i + 1] = sl.prefix[i] + cnts[i];
  }
  return sl;
}

static SegList make_seglist_dev(uintptr_t dev_count) {
  SegList sl{};
  sl.nseg = 1;
  sl.dev_count = P<const long long>(dev_count);
  sl.off[0] = 0;
  sl.prefix[0] = 0;
  sl.prefix[1] = 0;
  return sl;
}

static long long seglist_total(const SegList& s) { return s.dev_count ? -1 : s.prefix[s.nseg]; }

static BdIndex make_bdindex(const std::vector<uintptr_t>& v) {
  if (v.empty()) return BdIndex{nullptr, nullptr, nullptr, nullptr};
  if (v.size() != 4) throw std::runtime_error("BdIndex: need (pos_of, luid, bkt, ubase)");
  return BdIndex{P<const uint32_t>(v[0]), P<const uint32_t>(v[1]), P<const uint32_t>(v[2]),
                 P<const uint32_t>(v[3])};
}

void bind_xgmi(py::module_& m);  // xgmi.hip
namespace ss {
void bind_round_engine(py::module_& m);  // round_engine.cpp
}

PYBIND11_MODULE(_ss_hip, m) {
  bind_xgmi(m);
  ss::bind_round_engine(m);
  m.doc() = "SwiftSnails-AMD gfx950 kernels + RCCL communicator";

  py::class_<DevTable>(m, "DevTable", py::module_local())
      .def(py::init([](uintptr_t base, unsigned long long cap, uint32_t stride, uint32_t key_off,
                       uint32_t dim, uint32_t width, uint32_t prefilled, uint32_t row_off,
                       uint32_t bf16, uint32_t rbits) {
             const uint32_t eb = bf16 ? 2u : 4u;
             if (row_off + eb * width > stride || (key_off < row_off + eb * width && key_off + 8 > row_off))
               throw std::invalid_argument("DevTable: row and key overlap inside the slot");
             // region tables: 2^rbits equal regions of >= 64 slots
             if (rbits > 20 || (rbits && (cap % (1ull << rbits) != 0 || (cap >> rbits) < 64)))
               throw std::invalid_argument("DevTable: rbits needs cap = rlen * 2^rbits, rlen >= 64");
             return DevTable{P<char>(base), cap, stride, key_off, dim, width, prefilled, row_off,
                             bf16, rbits, rbits ? (cap >> rbits) : cap};
           }),
           py::arg("base"), py::arg("cap"), py::arg("stride"), py::arg("key_off"), py::arg("dim"),
           py::arg("width"), py::arg("prefilled") = 0, py::arg("row_off") = 0,
           py::arg("bf16") = 0, py::arg("rbits") = 0)
      .def_readonly("rbits", &DevTable::rbits)
      .def_readonly("rlen", &DevTable::rlen)
      .def_readonly("bf16", &DevTable::bf16)
      .def_readonly("row_off", &DevTable::row_off)
      .def_readonly("prefilled", &DevTable::prefilled)
      .def_readonly("cap", &DevTable::cap)
      .def_readonly("stride", &DevTable::stride)
      .def_readonly("key_off", &DevTable::key_off)
      .def_readonly("dim", &DevTable::dim)
      .def_readonly("width", &DevTable::width);

  py::class_<InitParams>(m, "InitParams", py::module_local())
      .def(py::init([](int kind, float scale, float state_init, uint64_t seed, int zero_bit) {
             return InitParams{kind, scale, state_init, seed, zero_bit};
           }),
           py::arg("kind") = 0, py::arg("scale") = 0.f, py::arg("state_init") = 0.f,
           py::arg("seed") = 0, py::arg("zero_bit") = -1);

  py::class_<OptParams>(m, "OptParams", py::module_local())
      .def(py::init([](int kind, float lr, float l1, float l2, float eps, float beta1, float beta2,
                       float bc1, float bc2, float alpha, float beta, float grad_scale,
                       float clip) {
             return OptParams{kind, lr, l1, l2, eps, beta1, beta2, bc1, bc2, alpha, beta,
                              grad_scale, clip};
           }),
           py::arg("kind") = 1, py::arg("lr") = 0.05f, py::arg("l1") = 0.f, py::arg("l2") = 0.f,
           py::arg("eps") = 1e-8f, py::arg("beta1") = 0.9f, py::arg("beta2") = 0.999f,
           py::arg("bc1") = 1.f, py::arg("bc2") = 1.f, py::arg("alpha") = 0.05f,
           py::arg("beta") = 1.f, py::arg("grad_scale") = 1.f, py::arg("clip") = 0.f);

  py::class_<SegList>(m, "SegList", py::module_local())
      .def_static("from_host", &make_seglist)
      .def_static("from_device", &make_seglist_dev)
      .def_property_readonly("total", &seglist_total)
      .def_readonly("nseg", &SegList::nseg);

  m.def("opt_state_width", &opt_state_width);

  // ---- table (K3/K4/K5/K8)
  m.def("probe", [](const DevTable& t, uintptr_t keys, const SegList& sl, long long max_n,
                    uintptr_t slots, const InitParams& ip, int insert, uintptr_t size_ctr,
                    uintptr_t err, int G, uintptr_t st) {
    launch_probe(t, P<const uint64_t>(keys), sl, max_n, P<long long>(slots), ip, insert,
                 P<unsigned long long>(size_ctr), P<int>(err), G, S(st));
  });
  m.def("gather", [](const DevTable& t, uintptr_t slots, const SegList& sl, long long max_n,
                     uintptr_t out, int G, uintptr_t st) {
    launch_gather(t, P<const long long>(slots), sl, max_n, P<float>(out), G, S(st));
  });
  m.def("pull_unique", [](const DevTable& t, uintptr_t keys, const SegList& sl, long long max_n,
                          uintptr_t slots, uintptr_t out, const InitParams& ip, uintptr_t size_ctr,
                          uintptr_t err, int G, uintptr_t st) {
    launch_pull_unique(t, P<const uint64_t>(keys), sl, max_n, P<long long>(slots), P<float>(out),
                       ip, P<unsigned long long>(size_ctr), P<int>(err), G, S(st));
  });
  m.def("pull_unique_bk", [](const DevTable& t, uintptr_t bkeys, uintptr_t bstart, uintptr_t unum,
                             uintptr_t ubase, int P_, uintptr_t slots, uintptr_t out,
                             const InitParams& ip, uintptr_t size_ctr, uintptr_t err, int G,
                             uintptr_t st, uintptr_t snap, int slot32) {
    launch_pull_unique_bk(t, P<const uint64_t>(bkeys), P<const uint32_t>(bstart),
                          P<const uint32_t>(unum), P<const uint32_t>(ubase), P_,
                          P<long long>(slots), P<float>(out), ip, P<unsigned long long>(size_ctr),
                          P<int>(err), G, S(st), P<float>(snap), slot32);
  }, py::arg("t"), py::arg("bkeys"), py::arg("bstart"), py::arg("unum"), py::arg("ubase"),
     py::arg("P"), py::arg("slots"), py::arg("out"), py::arg("ip"), py::arg("size_ctr"),
     py::arg("err"), py::arg("G"), py::arg("st"), py::arg("snap") = 0, py::arg("slot32") = 0);
  m.def("pull_claim_bk", [](const DevTable& t, uintptr_t bkeys, uintptr_t bstart, uintptr_t unum,
                            uintptr_t ubase, int P_, uintptr_t slots32, uintptr_t out,
                            uintptr_t snap, const InitParams& ip, uintptr_t size_ctr,
                            uintptr_t err, uintptr_t st, uintptr_t luid, uintptr_t occ) {
    launch_pull_claim_bk(t, P<const uint64_t>(bkeys), P<const uint32_t>(bstart),
                         P<const uint32_t>(unum), P<const uint32_t>(ubase), P_, P<int>(slots32),
                         P<float>(out), P<float>(snap), ip, P<unsigned long long>(size_ctr),
                         P<int>(err), S(st), P<const uint32_t>(luid), P<float>(occ));
  }, py::arg("t"), py::arg("bkeys"), py::arg("bstart"), py::arg("unum"), py::arg("ubase"),
     py::arg("P"), py::arg("slots32"), py::arg("out"), py::arg("snap"), py::arg("ip"),
     py::arg("size_ctr"), py::arg("err"), py::arg("st"), py::arg("luid") = 0,
     py::arg("occ") = 0);
  m.def("apply_masked_ok", &apply_masked_ok);
  m.def("commit_claims", [](const DevTable& t, uintptr_t bkeys, uintptr_t bstart, uintptr_t unum,
                            uintptr_t ubase, int P_, uintptr_t slots32, uintptr_t snap,
                            uintptr_t st, uintptr_t err) {
    launch_commit_claims(t, P<const uint64_t>(bkeys), P<const uint32_t>(bstart),
                         P<const uint32_t>(unum), P<const uint32_t>(ubase), P_,
                         P<const int>(slots32), P<const float>(snap), S(st), P<int>(err));
  }, py::arg("t"), py::arg("bkeys"), py::arg("bstart"), py::arg("unum"), py::arg("ubase"),
     py::arg("P"), py::arg("slots32"), py::arg("snap"), py::arg("st"), py::arg("err") = 0);
  m.def("apply", [](const DevTable& t, uintptr_t slots, uintptr_t grads, const SegList& sl,
                    long long max_n, const OptParams& op, int G, uintptr_t st, uintptr_t snap,
                    uintptr_t only) {
    launch_apply(t, P<const long long>(slots), P<const float>(grads), sl, max_n, op, G, S(st),
                 P<const float>(snap), P<const uint8_t>(only));
  }, py::arg("t"), py::arg("slots"), py::arg("grads"), py::arg("sl"), py::arg("max_n"),
     py::arg("op"), py::arg("G"), py::arg("st"), py::arg("snap") = 0, py::arg("only") = 0);
  m.def("assign", [](const DevTable& t, uintptr_t keys, uintptr_t rows, long long n,
                     uintptr_t size_ctr, uintptr_t err, int G, uintptr_t st) {
    launch_assign(t, P<const uint64_t>(keys), P<const float>(rows), n,
                  P<unsigned long long>(size_ctr), P<int>(err), G, S(st));
  });
  m.def("export_slots", [](const DevTable& t, unsigned long long s0, long long n, uintptr_t keys,
                           uintptr_t rows, uintptr_t cursor, uintptr_t st) {
    launch_export(t, s0, n, P<uint64_t>(keys), P<float>(rows), P<unsigned long long>(cursor),
                  S(st));
  });

  m.def("probe_hist", [](const DevTable& t, uintptr_t hist, int nbins, uintptr_t st) {
    launch_probe_hist(t, P<unsigned long long>(hist), nbins, S(st));
  });

  // ---- dedup / route (K1/K2/K6/K7)
  m.def("dedup_route", [](uintptr_t keys, long long n, uintptr_t skeys, uintptr_t stag,
                          unsigned long long scap, uintptr_t slot_of, uintptr_t frag_map,
                          int frag_num, int nranks, long long ucap, uintptr_t ucount,
                          uintptr_t ukeys, uintptr_t ugrad, int gdim, uintptr_t blk_cnt,
                          uintptr_t inv, uintptr_t st) {
    RouteSpec rs{P<const int>(frag_map), frag_num, nranks};
    launch_dedup_route(P<const uint64_t>(keys), n, P<uint64_t>(skeys), P<uint32_t>(stag), scap,
                       P<uint32_t>(slot_of), rs, ucap, P<unsigned long long>(ucount),
                       P<uint64_t>(ukeys), P<float>(ugrad), gdim, P<uint32_t>(blk_cnt),
                       P<uint32_t>(inv), S(st));
  });
  m.def("dedup_blocks", &dedup_blocks);
  m.def("bd_max_keys", &bd_max_keys);
  m.def("bd_scratch_words", &bd_scratch_words, py::arg("n"), py::arg("nranks"),
        py::arg("ndest") = 0);
  m.def("bd_ubase_offset", &bd_ubase_offset, py::arg("n"), py::arg("nranks"),
        py::arg("ndest") = 0);
  m.def("bd_offsets", &bd_offsets, py::arg("n"), py::arg("nranks"), py::arg("ndest") = 0);
  m.def("bd_buckets", &bd_buckets, py::arg("n"), py::arg("nranks"), py::arg("ndest") = 0);
  m.def("bd_dedup", [](uintptr_t keys, long long n, uintptr_t frag_map, int frag_num, int nranks,
                       long long ucap, uintptr_t scratch, uintptr_t pj, uintptr_t pos_of,
                       uintptr_t bkt, uintptr_t luid, uintptr_t bkeys, uintptr_t ucount,
                       uintptr_t ukeys, uintptr_t ugrad, int gdim, uintptr_t inv, int place,
                       uintptr_t st, uintptr_t dbg, uintptr_t rec, uintptr_t usingle,
                       int ndest, long long lay_n, int msub, uintptr_t usub, int rbits,
                       uintptr_t spj, uintptr_t gkeys, uintptr_t gspj) {
    RouteSpec rs{P<const int>(frag_map), frag_num, nranks, rbits};
    return launch_bd_dedup(P<const uint64_t>(keys), n, rs, ucap, P<uint32_t>(scratch),
                           P<uint32_t>(pj), P<uint32_t>(pos_of), P<uint32_t>(bkt),
                           P<uint32_t>(luid), P<uint64_t>(bkeys), P<unsigned long long>(ucount),
                           P<uint64_t>(ukeys), P<float>(ugrad), gdim, P<uint32_t>(inv), place,
                           S(st), P<unsigned long long>(dbg), P<uint32_t>(rec),
                           P<uint8_t>(usingle), ndest, lay_n, msub, P<uint32_t>(usub),
                           P<uint32_t>(spj), P<uint64_t>(gkeys), P<uint32_t>(gspj));
  }, py::arg("keys"), py::arg("n"), py::arg("frag_map"), py::arg("frag_num"), py::arg("nranks"),
     py::arg("ucap"), py::arg("scratch"), py::arg("pj"), py::arg("pos_of"), py::arg("bkt"),
     py::arg("luid"), py::arg("bkeys"), py::arg("ucount"), py::arg("ukeys"), py::arg("ugrad"),
     py::arg("gdim"), py::arg("inv"), py::arg("place"), py::arg("st"), py::arg("dbg") = 0,
     py::arg("rec") = 0, py::arg("usingle") = 0, py::arg("ndest") = 0,
     py::arg("lay_n") = 0, py::arg("msub") = 1, py::arg("usub") = 0, py::arg("rbits") = 0,
     py::arg("spj") = 0, py::arg("gkeys") = 0, py::arg("gspj") = 0);
  m.def("bd_record_layout_bit", &bd_record_layout_bit);
  m.def("bd_record_group_bit", &bd_record_group_bit);
  m.def("bd_target_dist", &bd_target_dist);
  m.def("bd_target_for", &bd_target_for, py::arg("nranks"), py::arg("records") = false);
  m.def("rec_grad", [](uintptr_t ucount, int nd, long long gap, uintptr_t spj, uintptr_t gs,
                       uintptr_t xval, int F, uintptr_t grec, uintptr_t st, uintptr_t acc,
                       uintptr_t acc_out, int acc_n, int skip) {
    launch_rec_grad(P<const unsigned long long>(ucount), nd, gap, P<const uint32_t>(spj),
                    P<const float>(gs), P<const float>(xval), F, P<float>(grec), S(st),
                    P<float>(acc), P<float>(acc_out), acc_n, skip);
  }, py::arg("ucount"), py::arg("nd"), py::arg("gap"), py::arg("spj"), py::arg("gs"),
     py::arg("xval"), py::arg("F"), py::arg("grec"), py::arg("st"), py::arg("acc") = 0,
     py::arg("acc_out") = 0, py::arg("acc_n") = 0, py::arg("skip") = -1);
  m.def("bd_reduce", [](long long n, int nranks, uintptr_t scratch, uintptr_t pj, uintptr_t luid,
                        uintptr_t gs, uintptr_t xval, int F, uintptr_t ugrad, uintptr_t st,
                        int osi, uintptr_t usingle, std::optional<DevTable> t, uintptr_t slots,
                        uintptr_t snap, std::optional<OptParams> op, int ndest, int slot32,
                        uintptr_t acc, uintptr_t acc_out, int acc_n, uintptr_t bkeys) {
    launch_bd_reduce(n, nranks, P<const uint32_t>(scratch), P<const uint32_t>(pj),
                     P<const uint32_t>(luid), P<const float>(gs), P<const float>(xval), F,
                     P<float>(ugrad), S(st), osi, P<const uint8_t>(usingle),
                     t ? &*t : nullptr, P<const long long>(slots), P<const float>(snap),
                     op ? &*op : nullptr, ndest, slot32, P<float>(acc), P<float>(acc_out), acc_n,
                     P<const uint64_t>(bkeys));
  }, py::arg("n"), py::arg("nranks"), py::arg("scratch"), py::arg("pj"), py::arg("luid"),
     py::arg("gs"), py::arg("xval"), py::arg("F"), py::arg("ugrad"), py::arg("st"),
     py::arg("osi") = 0, py::arg("usingle") = 0, py::arg("t") = py::none(), py::arg("slots") = 0,
     py::arg("snap") = 0, py::arg("op") = py::none(), py::arg("ndest") = 0,
     py::arg("slot32") = 0, py::arg("acc") = 0, py::arg("acc_out") = 0, py::arg("acc_n") = 0,
     py::arg("bkeys") = 0);
  m.def("bd_unplace", [](long long n, int nranks, uintptr_t scratch, uintptr_t src, uintptr_t dst,
                         int dim, uintptr_t st, int ndest) {
    launch_bd_unplace(n, nranks, P<const uint32_t>(scratch), P<const float>(src), P<float>(dst),
                      dim, S(st), ndest);
  }, py::arg("n"), py::arg("nranks"), py::arg("scratch"), py::arg("src"), py::arg("dst"),
     py::arg("dim"), py::arg("st"), py::arg("ndest") = 0);
  m.def("route_keys", [](uintptr_t keys, long long n, uintptr_t frag_map, int frag_num,
                         int nranks, uintptr_t dest, uintptr_t st) {
    RouteSpec rs{P<const int>(frag_map), frag_num, nranks};
    launch_route_keys(P<const uint64_t>(keys), n, rs, P<int>(dest), S(st));
  });
  m.def("gather_rows", [](uintptr_t src, uintptr_t idx, long long n, int dim, uintptr_t out,
                          uintptr_t st) {
    launch_gather_rows(P<const float>(src), P<const uint32_t>(idx), n, dim, P<float>(out), S(st));
  });
  m.def("scatter_add_rows", [](uintptr_t src, uintptr_t idx, long long n, int dim, uintptr_t out,
                               uintptr_t st) {
    launch_scatter_add_rows(P<const float>(src), P<const uint32_t>(idx), n, dim, P<float>(out),
                            S(st));
  });

  // ---- models
  m.def("csr_batch", [](uintptr_t offs, uintptr_t keys, uintptr_t vals, uintptr_t labels,
                        long long rows, long long cursor, int B, int F, uintptr_t step_dev,
                        long long step_add, uintptr_t out_keys, uintptr_t out_vals,
                        uintptr_t out_labels, uintptr_t st) {
    launch_csr_batch(P<const uint64_t>(offs), P<const uint64_t>(keys), P<const float>(vals),
                     P<const float>(labels), rows, cursor, B, F, P<const long long>(step_dev),
                     step_add, P<uint64_t>(out_keys), P<float>(out_vals), P<float>(out_labels),
                     S(st));
  });
  m.def("w2v_corpus_window", [](uintptr_t tokens, uintptr_t sent_of, long long nsent,
                                uintptr_t table, long long table_size, uintptr_t keep, long long N,
                                uint64_t seed, long long step, uintptr_t step_dev,
                                long long step_add, int B, int W, long long nneg, uint64_t out_bit,
                                uintptr_t keys, uintptr_t meta, uintptr_t st) {
    launch_w2v_corpus_window(P<const uint64_t>(tokens), P<const uint32_t>(sent_of), nsent,
                             P<const uint64_t>(table), table_size, P<const float>(keep), N, seed,
                             step, P<const long long>(step_dev), step_add, B, W, nneg, out_bit,
                             P<uint64_t>(keys), P<int32_t>(meta), S(st));
  });
  m.def("w2v_corpus_batch", [](uintptr_t tokens, uintptr_t sent_offs, uintptr_t sent_of,
                               uintptr_t table, long long table_size, uintptr_t keep, long long N,
                               uint64_t seed, long long step, uintptr_t step_dev,
                               long long step_add, int B, int C, int W, long long nneg,
                               uint64_t out_bit, uintptr_t keys, uintptr_t st) {
    launch_w2v_corpus_batch(P<const uint64_t>(tokens), P<const uint64_t>(sent_offs),
                            P<const uint32_t>(sent_of), P<const uint64_t>(table), table_size,
                            P<const float>(keep), N, seed, step, P<const long long>(step_dev),
                            step_add, B, C, W, nneg, out_bit, P<uint64_t>(keys), S(st));
  });
  m.def("gen_ctr", [](uint64_t seed, long long sample_base, int B, int F, long long V,
                      float tail_frac, float truth_scale, float truth_bias, uintptr_t keys,
                      uintptr_t labels, uintptr_t st, uintptr_t step_dev, long long step_mul,
                      long long step_add) {
    launch_gen_ctr(seed, sample_base, B, F, V, tail_frac, truth_scale, truth_bias,
                   P<uint64_t>(keys), P<float>(labels), S(st), P<const long long>(step_dev),
                   step_mul, step_add);
  }, py::arg("seed"), py::arg("sample_base"), py::arg("B"), py::arg("F"), py::arg("V"),
     py::arg("tail_frac"), py::arg("truth_scale"), py::arg("truth_bias"), py::arg("keys"),
     py::arg("labels"), py::arg("st"), py::arg("step_dev") = 0, py::arg("step_mul") = 0,
     py::arg("step_add") = 0);
  m.def("lr_fwd_bwd", [](uintptr_t inv, uintptr_t xval, uintptr_t labels, int B, int F,
                         uintptr_t uvals, uintptr_t ugrad, uintptr_t loss_sum, uintptr_t pred,
                         uintptr_t st) {
    launch_lr_fwd_bwd(P<const uint32_t>(inv), P<const float>(xval), P<const float>(labels), B, F,
                      P<const float>(uvals), P<float>(ugrad), P<float>(loss_sum), P<float>(pred),
                      S(st));
  });

  m.def("sr_nbins", &sr_nbins);
  m.def("sr_nchunks", &sr_nchunks);
  m.def("sr_max_items", &sr_max_items);
  m.def("sr_hist_words", &sr_hist_words);
  m.def("dedup_cnt_words", &dedup_cnt_words);
  m.def("sr_plan", [](uintptr_t inv, long long n, uintptr_t ucount, int nranks, long long ucap,
                      uintptr_t hist, int nbins, uintptr_t plan, uintptr_t items, uintptr_t nitems,
                      uintptr_t st) {
    launch_sr_plan(P<const uint32_t>(inv), n, P<const unsigned long long>(ucount), nranks, ucap,
                   P<uint32_t>(hist), nbins, P<void>(plan), P<void>(items), P<uint32_t>(nitems),
                   S(st));
  });
  m.def("sr_reduce", [](uintptr_t plan, uintptr_t gocc, uintptr_t items, uintptr_t nitems,
                        long long n, uintptr_t ucount, int nranks, long long ucap, uintptr_t ugrad,
                        uintptr_t st) {
    launch_sr_reduce(P<const void>(plan), P<const float>(gocc), P<const void>(items),
                     P<const uint32_t>(nitems), n, P<const unsigned long long>(ucount), nranks,
                     ucap, P<float>(ugrad), S(st));
  });
  // ix = (pos_of, luid, bkt, ubase) pointers of a bucketed dedup, or () with inv
  m.def("lr_fwd_g", [](uintptr_t inv, uintptr_t xval, uintptr_t labels, int B, int F,
                       uintptr_t uvals, uintptr_t g, int per_sample, uintptr_t loss,
                       uintptr_t pred, uintptr_t st, std::vector<uintptr_t> ix, uintptr_t occ,
                       uintptr_t own, long long own_lo, long long own_hi) {
    // own: the cached buffer holding occ's positions [own_lo, own_hi) (the
    // record exchange's own destination), indexed from own_lo
    SelfSeg os{};
    if (own) {
      if (own_hi <= own_lo || own_lo < 0) throw std::invalid_argument("lr_fwd_g: own range");
      os.ptr = reinterpret_cast<char*>(own) - own_lo * (long long)sizeof(float);
      os.lo = own_lo;
      os.hi = own_hi;
    }
    launch_lr_fwd_g(P<const uint32_t>(inv), make_bdindex(ix), P<const float>(xval),
                    P<const float>(labels), B, F, P<const float>(uvals), P<float>(g), per_sample,
                    P<float>(loss), P<float>(pred), S(st), P<const float>(occ), os);
  }, py::arg("inv"), py::arg("xval"), py::arg("labels"), py::arg("B"), py::arg("F"),
     py::arg("uvals"), py::arg("g"), py::arg("per_sample"), py::arg("loss"), py::arg("pred"),
     py::arg("st"), py::arg("ix") = std::vector<uintptr_t>{}, py::arg("occ") = 0,
     py::arg("own") = 0, py::arg("own_lo") = 0, py::arg("own_hi") = 0);
  m.def("bd_fill_occ", [](long long n, int nranks, uintptr_t scratch, uintptr_t luid,
                          uintptr_t uvals, uintptr_t occ, int osi, uintptr_t st, int ndest,
                          uintptr_t pj) {
    launch_bd_fill_occ(n, nranks, P<const uint32_t>(scratch), P<const uint32_t>(luid),
                       P<const float>(uvals), P<float>(occ), osi, S(st), ndest,
                       P<const uint32_t>(pj));
  }, py::arg("n"), py::arg("nranks"), py::arg("scratch"), py::arg("luid"), py::arg("uvals"),
     py::arg("occ"), py::arg("osi"), py::arg("st"), py::arg("ndest") = 0, py::arg("pj") = 0);
  // server-side merge of a round's received keys (server.hip)
  m.def("srv_sub_buckets", &srv_sub_buckets, py::arg("nsrc"), py::arg("lay_n") = 0,
        py::arg("ndest") = 0);
  m.def("srv_dedup", [](uintptr_t rkeys, uintptr_t rbase, uintptr_t rnum, long long cap, int nsrc,
                        int Pd, int m, int me, uintptr_t cnt, uintptr_t bstart, uintptr_t pj,
                        uintptr_t luid, uintptr_t bkeys, uintptr_t ubase, uintptr_t unum,
                        uintptr_t ucount, uintptr_t err, uintptr_t st, uintptr_t roff) {
    launch_srv_dedup(P<const uint64_t>(rkeys), P<const uint32_t>(rbase), P<const uint32_t>(rnum),
                     cap, nsrc, Pd, m, me, P<uint32_t>(cnt), P<uint32_t>(bstart), P<uint32_t>(pj),
                     P<uint32_t>(luid), P<uint64_t>(bkeys), P<uint32_t>(ubase), P<uint32_t>(unum),
                     P<unsigned long long>(ucount), P<uint32_t>(err), S(st),
                     P<const uint32_t>(roff));
  }, py::arg("rkeys"), py::arg("rbase"), py::arg("rnum"), py::arg("cap"), py::arg("nsrc"),
     py::arg("Pd"), py::arg("m"), py::arg("me"), py::arg("cnt"), py::arg("bstart"), py::arg("pj"),
     py::arg("luid"), py::arg("bkeys"), py::arg("ubase"), py::arg("unum"), py::arg("ucount"),
     py::arg("err"), py::arg("st"), py::arg("roff") = 0);
  m.def("srv_fill", [](int Pn, uintptr_t bstart, uintptr_t ubase, uintptr_t unum, uintptr_t pj,
                       uintptr_t luid, uintptr_t rows, uintptr_t out, int D, uintptr_t st) {
    if (D == 1)
      launch_bd_fill_occ_p(Pn, P<const uint32_t>(bstart), P<const uint32_t>(ubase),
                           P<const uint32_t>(unum), P<const uint32_t>(luid),
                           P<const float>(rows), P<float>(out), P<const uint32_t>(pj), S(st));
    else
      launch_srv_fill_rows(Pn, P<const uint32_t>(bstart), P<const uint32_t>(ubase),
                           P<const uint32_t>(pj), P<const uint32_t>(luid), P<const float>(rows),
                           P<float>(out), D, S(st));
  });
  // merged gradients per distinct key; with a table the update is fused
  // (scalar rows: from the snapshot (blind store) or read from the row)
  m.def("srv_merge", [](int Pn, uintptr_t bstart, uintptr_t ubase, uintptr_t unum, uintptr_t pj,
                        uintptr_t luid, uintptr_t grads, uintptr_t merged, int D,
                        std::optional<DevTable> t, uintptr_t slots, uintptr_t snap,
                        std::optional<OptParams> op, uintptr_t st) {
    if (D == 1)
      launch_bd_reduce_p(Pn, P<const uint32_t>(bstart), P<const uint32_t>(ubase),
                         P<const uint32_t>(unum), P<const uint32_t>(pj), P<const uint32_t>(luid),
                         P<const float>(grads), 1, P<float>(merged), t ? &*t : nullptr,
                         P<const long long>(slots), P<const float>(snap), op ? &*op : nullptr,
                         S(st));
    else
      launch_srv_merge_rows(Pn, P<const uint32_t>(bstart), P<const uint32_t>(ubase),
                            P<const uint32_t>(unum), P<const uint32_t>(pj),
                            P<const uint32_t>(luid), P<const float>(grads), P<float>(merged), D,
                            S(st), t ? &*t : nullptr, P<const long long>(slots),
                            op ? &*op : nullptr);
  }, py::arg("P"), py::arg("bstart"), py::arg("ubase"), py::arg("unum"), py::arg("pj"),
     py::arg("luid"), py::arg("grads"), py::arg("merged"), py::arg("D"),
     py::arg("t") = std::nullopt, py::arg("slots") = 0, py::arg("snap") = 0,
     py::arg("op") = std::nullopt, py::arg("st") = 0);
  m.def("fm_fwd_g", [](uintptr_t inv, std::vector<uintptr_t> ix, uintptr_t labels, int B,
                       int F, int dim, uintptr_t uvals, uintptr_t gs, uintptr_t gss,
                       uintptr_t loss, uintptr_t pred, uintptr_t st) {
    launch_fm_fwd_g(P<const uint32_t>(inv), make_bdindex(ix), P<const float>(labels), B, F, dim,
                    P<const float>(uvals), P<float>(gs), P<float>(gss), P<float>(loss),
                    P<float>(pred), S(st));
  });
  m.def("bd_reduce_fm", [](long long n, int nranks, uintptr_t scratch, uintptr_t pj,
                           uintptr_t luid, uintptr_t gs, uintptr_t gss, int F, int dim,
                           uintptr_t uvals, uintptr_t ugrad, uintptr_t st, uintptr_t ovf,
                           std::optional<DevTable> t, uintptr_t slots, std::optional<OptParams> op,
                           int ndest) {
    launch_bd_reduce_fm(n, nranks, P<const uint32_t>(scratch), P<const uint32_t>(pj),
                        P<const uint32_t>(luid), P<const float>(gs), P<const float>(gss), F, dim,
                        P<const float>(uvals), P<float>(ugrad), S(st), P<uint32_t>(ovf),
                        t ? &*t : nullptr, P<const long long>(slots), op ? &*op : nullptr, ndest);
  }, py::arg("n"), py::arg("nranks"), py::arg("scratch"), py::arg("pj"), py::arg("luid"),
     py::arg("gs"), py::arg("gss"), py::arg("F"), py::arg("dim"), py::arg("uvals"),
     py::arg("ugrad"), py::arg("st"), py::arg("ovf") = 0, py::arg("t") = py::none(),
     py::arg("slots") = 0, py::arg("op") = py::none(), py::arg("ndest") = 0);
  m.def("bd_fm_ovf_words", &bd_fm_ovf_words);
  // ---- native worker API (worker.h): pull / push with async handles
  py::class_<Handle>(m, "Handle")
      .def("wait", &Handle::wait, py::call_guard<py::gil_scoped_release>())
      .def("done", &Handle::done);
  py::class_<GpuWorker>(m, "GpuWorker")
      .def(py::init([](const DevTable& t, uintptr_t size_ctr, uintptr_t err, const InitParams& ip,
                       const OptParams& op, int G, long long max_keys) {
             return new GpuWorker(t, P<unsigned long long>(size_ctr), P<int>(err), ip, op, G,
                                  max_keys);
           }),
           py::arg("t"), py::arg("size_ctr"), py::arg("err"), py::arg("init"), py::arg("opt"),
           py::arg("G"), py::arg("max_keys"))
      .def("pull", [](GpuWorker& w, uintptr_t keys, long long n, uintptr_t vals, uintptr_t st) {
        return w.pull(P<const uint64_t>(keys), n, P<float>(vals), S(st));
      })
      .def("push", [](GpuWorker& w, uintptr_t keys, long long n, uintptr_t grads, uintptr_t st) {
        return w.push(P<const uint64_t>(keys), n, P<const float>(grads), S(st));
      })
      .def("unique_count_ptr",
           [](const GpuWorker& w) { return reinterpret_cast<uintptr_t>(w.unique_count()); })
      .def_property_readonly("max_keys", &GpuWorker::max_keys);
  // A stream whose kernels may only occupy `keep` of the device's CUs, spread
  // evenly over the CU index space (hipExtStreamCreateWithCUMask): limits how
  // much of the memory system a side stream's kernels can claim.
  m.def("cu_mask_stream", [](int device, int keep) {
    check_hip(hipSetDevice(device), "hipSetDevice");
    hipDeviceProp_t prop;
    check_hip(hipGetDeviceProperties(&prop, device), "hipGetDeviceProperties");
    const int n = prop.multiProcessorCount;
    if (keep < 1 || keep > n) throw std::invalid_argument("cu_mask_stream: keep out of range");
    std::vector<uint32_t> mask((n + 31) / 32, 0u);
    for (int i = 0; i < n; ++i)
      if ((long long)(i + 1) * keep / n > (long long)i * keep / n) mask[i / 32] |= 1u << (i % 32);
    hipStream_t s;
    check_hip(hipExtStreamCreateWithCUMask(&s, (uint32_t)mask.size(), mask.data()),
              "hipExtStreamCreateWithCUMask");
    return reinterpret_cast<uintptr_t>(s);
  });
  m.def("fm_fwd_bwd", [](uintptr_t inv, uintptr_t labels, int B, int F, int dim, uintptr_t uvals,
                         uintptr_t ugrad, uintptr_t loss, uintptr_t pred, uintptr_t st) {
    launch_fm_fwd_bwd(P<const uint32_t>(inv), P<const float>(labels), B, F, dim,
                      P<const float>(uvals), P<float>(ugrad), P<float>(loss), P<float>(pred),
                      S(st));
  });
  m.def("w2v_sgns", [](uintptr_t inv_c, uintptr_t inv_x, uintptr_t inv_n, int B, int C, int D,
                       float neg_scale, uintptr_t uvals, uintptr_t ugrad, uintptr_t loss,
                       uintptr_t st, int bf16) {
    launch_w2v_sgns(P<const uint32_t>(inv_c), P<const uint32_t>(inv_x), P<const uint32_t>(inv_n), B,
                    C, D, neg_scale, P<const float>(uvals), P<float>(ugrad), P<float>(loss), S(st),
                    bf16);
  }, py::arg("inv_c"), py::arg("inv_x"), py::arg("inv_n"), py::arg("B"), py::arg("C"),
     py::arg("D"), py::arg("neg_scale"), py::arg("uvals"), py::arg("ugrad"), py::arg("loss"),
     py::arg("st"), py::arg("bf16") = 0);
  m.def("w2v_win", [](uintptr_t inv_c, uintptr_t inv_w, uintptr_t inv_n, uintptr_t meta, int B,
                      int W, int D, float neg_per_pair, uintptr_t uvals, uintptr_t ugrad,
                      uintptr_t loss, uintptr_t pairs, uintptr_t st, uintptr_t ograd,
                      uintptr_t otail) {
    launch_w2v_win(P<const uint32_t>(inv_c), P<const uint32_t>(inv_w), P<const uint32_t>(inv_n),
                   P<const int32_t>(meta), B, W, D, neg_per_pair, P<const float>(uvals),
                   P<float>(ugrad), P<float>(loss), P<float>(pairs), S(st), P<float>(ograd),
                   P<float>(otail));
  }, py::arg("inv_c"), py::arg("inv_w"), py::arg("inv_n"), py::arg("meta"), py::arg("B"),
     py::arg("W"), py::arg("D"), py::arg("neg_per_pair"), py::arg("uvals"), py::arg("ugrad"),
     py::arg("loss"), py::arg("pairs"), py::arg("st"), py::arg("ograd") = 0,
     py::arg("otail") = 0);
  m.def("w2v_pp", [](uintptr_t inv_c, uintptr_t inv_w, uintptr_t inv_n, uintptr_t meta, int B,
                     int W, int K, int D, uintptr_t uvals, uintptr_t ograd, uintptr_t gpair,
                     uintptr_t loss, uintptr_t pairs, uintptr_t st, uintptr_t gnc) {
    launch_w2v_pp(P<const uint32_t>(inv_c), P<const uint32_t>(inv_w), P<const uint32_t>(inv_n),
                  P<const int32_t>(meta), B, W, K, D, P<const float>(uvals), P<float>(ograd),
                  P<float>(gpair), P<float>(loss), P<float>(pairs), S(st), P<float>(gnc));
  });
  m.def("w2v_osort", [](int P_, uintptr_t bstart, uintptr_t unum, uintptr_t ubase, uintptr_t pj,
                        uintptr_t luid, uintptr_t ord, uintptr_t items, uintptr_t st,
                        uintptr_t uhot) {
    launch_w2v_osort(P_, P<const uint32_t>(bstart), P<const uint32_t>(unum),
                     P<const uint32_t>(ubase), P<const uint32_t>(pj), P<const uint32_t>(luid),
                     P<uint32_t>(ord), P<uint32_t>(items), S(st), P<uint8_t>(uhot));
  }, py::arg("P"), py::arg("bstart"), py::arg("unum"), py::arg("ubase"), py::arg("pj"),
     py::arg("luid"), py::arg("ord"), py::arg("items"), py::arg("st"), py::arg("uhot") = 0);
  m.def("w2v_oreduce", [](uintptr_t items, long long n, uintptr_t ord, uintptr_t ograd,
                          uintptr_t otail, int B, int W, int D, uintptr_t ugrad, uintptr_t st,
                          uintptr_t gnc, long long negbase, uintptr_t uvals, uintptr_t acc,
                          uintptr_t acc_out, int acc_n, std::optional<DevTable> t,
                          uintptr_t slots, std::optional<OptParams> op) {
    launch_w2v_oreduce(P<const uint32_t>(items), n, P<const uint32_t>(ord), P<const float>(ograd),
                       P<const float>(otail), B, W, D, P<float>(ugrad), S(st),
                       P<const float>(gnc), negbase, P<const float>(uvals), P<float>(acc),
                       P<float>(acc_out), acc_n, t ? &*t : nullptr, P<const long long>(slots),
                       op ? &*op : nullptr);
  }, py::arg("items"), py::arg("n"), py::arg("ord"), py::arg("ograd"), py::arg("otail"),
     py::arg("B"), py::arg("W"), py::arg("D"), py::arg("ugrad"), py::arg("st"),
     py::arg("gnc") = 0, py::arg("negbase") = 0, py::arg("uvals") = 0, py::arg("acc") = 0,
     py::arg("acc_out") = 0, py::arg("acc_n") = 0, py::arg("t") = py::none(),
     py::arg("slots") = 0, py::arg("op") = py::none());
  m.def("w2v_stream_gen", [](uint64_t seed, long long base, int B, int W, int L, long long nneg,
                             long long V, float noise, uintptr_t keys, uintptr_t meta, uintptr_t st,
                             uintptr_t step_dev, long long step_mul, long long step_add) {
    launch_w2v_stream_gen(seed, base, B, W, L, nneg, V, noise, P<uint64_t>(keys),
                          P<int32_t>(meta), S(st), P<const long long>(step_dev), step_mul,
                          step_add);
  }, py::arg("seed"), py::arg("base"), py::arg("B"), py::arg("W"), py::arg("L"),
     py::arg("nneg"), py::arg("V"), py::arg("noise"), py::arg("keys"), py::arg("meta"),
     py::arg("st"), py::arg("step_dev") = 0, py::arg("step_mul") = 0, py::arg("step_add") = 0);
  m.def("w2v_gen", [](uint64_t seed, long long base, int B, int C, int W, long long nneg,
                      long long V, float noise, uintptr_t keys, uintptr_t st, uintptr_t step_dev,
                      long long step_mul, long long step_add) {
    launch_w2v_gen(seed, base, B, C, W, nneg, V, noise, P<uint64_t>(keys), S(st),
                   P<const long long>(step_dev), step_mul, step_add);
  }, py::arg("seed"), py::arg("base"), py::arg("B"), py::arg("C"), py::arg("W"),
     py::arg("nneg"), py::arg("V"), py::arg("noise"), py::arg("keys"), py::arg("st"),
     py::arg("step_dev") = 0, py::arg("step_mul") = 0, py::arg("step_add") = 0);
  m.def("w2v_smem_bytes", &w2v_smem_bytes);

  // ---- RCCL
  py::class_<RcclComm>(m, "RcclComm", py::module_local())
      .def(py::init([](int rank, int nranks, py::bytes uid, int device) {
             return new RcclComm(rank, nranks, std::string(uid), device);
           }),
           py::arg("rank"), py::arg("nranks"), py::arg("uid"), py::arg("device"))
      .def_static("unique_id", []() { return py::bytes(RcclComm::unique_id()); })
      .def_property_readonly("rank", &RcclComm::rank)
      .def_property_readonly("nranks", &RcclComm::nranks)
      .def("alltoallv", &RcclComm::alltoallv, py::arg("send"), py::arg("scounts"),
           py::arg("sdispls"), py::arg("recv"), py::arg("rcounts"), py::arg("rdispls"),
           py::arg("elem_bytes"), py::arg("stream"), py::arg("send_cap") = -1,
           py::arg("recv_cap") = -1, py::call_guard<py::gil_scoped_release>())
      .def("comm_count", &RcclComm::comm_count)
      .def("alltoall", &RcclComm::alltoall, py::call_guard<py::gil_scoped_release>())
      .def("allreduce", &RcclComm::allreduce, py::call_guard<py::gil_scoped_release>())
      .def("broadcast", &RcclComm::broadcast, py::call_guard<py::gil_scoped_release>())
      .def("allgather", &RcclComm::allgather, py::call_guard<py::gil_scoped_release>())
      .def("abort", &RcclComm::abort);
}
