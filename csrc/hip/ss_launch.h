// ss_launch.h — host-side launch helpers and the launcher declarations that the
// pybind11 module (bindings.cpp) calls.  Kernels never allocate or synchronise:
// every launcher only enqueues on the caller's stream (hipGraph-capturable).
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>
#include <stdexcept>
#include <string>
#include <vector>
#include "bdindex.h"
#include "ss_device.h"

namespace ss {

[[noreturn]] inline void throw_error(const std::string& msg) { throw std::runtime_error(msg); }

inline void check_hip(hipError_t e, const char* what) {
  if (e != hipSuccess) throw_error(std::string(what) + ": " + hipGetErrorString(e));
}

inline void check_launch(const char* what) { check_hip(hipGetLastError(), what); }

// --- table.hip
void launch_probe(const DevTable& t, const uint64_t* keys, const SegList& sl, long long max_n,
                  long long* slots, const InitParams& ip, int insert,
                  unsigned long long* size_ctr, int* err, int G, hipStream_t st);
void launch_gather(const DevTable& t, const long long* slots, const SegList& sl, long long max_n,
                   float* out, int G, hipStream_t st);
void launch_pull_unique(const DevTable& t, const uint64_t* keys, const SegList& sl,
                        long long max_n, long long* slots, float* out, const InitParams& ip,
                        unsigned long long* size_ctr, int* err, int G, hipStream_t st);
void launch_pull_unique_bk(const DevTable& t, const uint64_t* bkeys, const uint32_t* bstart,
                           const uint32_t* unum, const uint32_t* ubase, int P, long long* slots,
                           float* out, const InitParams& ip, unsigned long long* size_ctr,
                           int* err, int G, hipStream_t st, float* snap = nullptr,
                           int slot32 = 0);
// region tables, region-aligned buckets (launch_bd_dedup returned rbits):
// one workgroup per bucket claims new keys' slots in LDS (no device atomic,
// nothing written to the table); the fused merge stores [w | h | key]
// (launch_bd_reduce with bkeys) or launch_commit_claims writes them
void launch_pull_claim_bk(const DevTable& t, const uint64_t* bkeys, const uint32_t* bstart,
                          const uint32_t* unum, const uint32_t* ubase, int P, int* slots32,
                          float* out, float* snap, const InitParams& ip,
                          unsigned long long* size_ctr, int* err, hipStream_t st,
                          const uint32_t* luid = nullptr, float* occ = nullptr,
                          const uint32_t* pj = nullptr, SelfSeg self = SelfSeg{});
// read-only lookup of a bucket view's unique keys (no insert; zeros if absent)
void launch_lookup_bk(const DevTable& t, const uint64_t* bkeys, const uint32_t* bstart,
                      const uint32_t* unum, const uint32_t* ubase, int P, float* out, int G,
                      hipStream_t st);
bool apply_masked_ok(const DevTable& t, const OptParams& op);
void launch_commit_claims(const DevTable& t, const uint64_t* bkeys, const uint32_t* bstart,
                          const uint32_t* unum, const uint32_t* ubase, int P, const int* slots32,
                          const float* snap, hipStream_t st, int* err = nullptr);
// only (optional): apply only at positions with only[pos] != 0 (wide rows);
// slot32: `slots` holds 4-byte slot indices (a snapshot pull of scalar rows)
void launch_apply(const DevTable& t, const long long* slots, const float* grads,
                  const SegList& sl, long long max_n, const OptParams& op, int G, hipStream_t st,
                  const float* snap = nullptr, const uint8_t* only = nullptr, int slot32 = 0);
void launch_assign(const DevTable& t, const uint64_t* keys, const float* rows, long long n,
                   unsigned long long* size_ctr, int* err, int G, hipStream_t st);
void launch_export(const DevTable& t, unsigned long long s0, long long n, uint64_t* keys_out,
                   float* rows_out, unsigned long long* cursor, hipStream_t st);
void launch_probe_hist(const DevTable& t, unsigned long long* hist, int nbins, hipStream_t st);

// --- dedup.hip
struct RouteSpec {
  const int* frag_map;  // frag -> destination rank (device)
  int frag_num;
  int nranks;
  // > 0: the bucketed dedup buckets whole regions of a region table with
  // 2^rbits regions (ss_device.h), so a bucket's pull owns its regions'
  // inserts (k_pull_claim_bk); 0: buckets by dedup_hash
  int rbits = 0;
  // fragment of a key = fmix64(key) % frag_num (reference hashfrag.h:48-53);
  // a 64-bit modulo is a long software sequence on the GPU, so power-of-two
  // fragment counts (the default 1024) take the mask instead — same result
  __host__ __device__ __forceinline__ uint32_t frag_of(uint64_t h) const {
    return (frag_num & (frag_num - 1)) == 0 ? (uint32_t)(h & (uint64_t)(frag_num - 1))
                                            : (uint32_t)(h % (uint64_t)frag_num);
  }
  __device__ __forceinline__ uint32_t dest_of(uint64_t key) const {
    return nranks == 1 ? 0u : (uint32_t)frag_map[frag_of(fmix64(key))];
  }
};
int dedup_blocks(long long n);
void launch_dedup_route(const uint64_t* keys, long long n, uint64_t* scratch_keys,
                        uint32_t* scratch_tag, unsigned long long scratch_cap, uint32_t* slot_of,
                        RouteSpec rs, long long ucap, unsigned long long* ucount, uint64_t* ukeys,
                        float* ugrad, int gdim, uint32_t* blk_cnt, uint32_t* inv,
                        hipStream_t st);
void launch_route_keys(const uint64_t* keys, long long n, RouteSpec rs, int* dest,
                       hipStream_t st);
void launch_gather_rows(const float* src, const uint32_t* idx, long long n, int dim, float* out,
                        hipStream_t st);
void launch_scatter_add_rows(const float* src, const uint32_t* idx, long long n, int dim,
                             float* out, hipStream_t st);

// --- models.hip
// --- data.hip: batch B x F cut out of an HBM-resident CSR dataset
void launch_csr_batch(const uint64_t* offs, const uint64_t* keys, const float* vals,
                      const float* labels, long long rows, long long cursor, int B, int F,
                      const long long* step_dev, long long step_add, uint64_t* out_keys,
                      float* out_vals, float* out_labels, hipStream_t st);
void launch_w2v_corpus_window(const uint64_t* tokens, const uint32_t* sent_of, long long nsent,
                              const uint64_t* table, long long table_size, const float* keep,
                              long long N, uint64_t seed, long long step,
                              const long long* step_dev, long long step_add, int B, int W,
                              long long nneg, uint64_t out_bit, uint64_t* keys, int32_t* meta,
                              hipStream_t st);
void launch_w2v_win(const uint32_t* inv_c, const uint32_t* inv_w, const uint32_t* inv_n,
                    const int32_t* meta, int B, int W, int D, float neg_per_pair,
                    const float* uvals, float* ugrad, float* loss_sum, float* pair_sum,
                    hipStream_t st, float* ograd = nullptr, float* otail = nullptr);
void launch_w2v_osort(int P, const uint32_t* bstart, const uint32_t* unum, const uint32_t* ubase,
                      const uint32_t* pj, const uint32_t* luid, uint32_t* ord, uint32_t* items,
                      hipStream_t st, uint8_t* uhot = nullptr);
void launch_w2v_pp(const uint32_t* inv_c, const uint32_t* inv_w, const uint32_t* inv_n,
                   const int32_t* meta, int B, int W, int K, int D, const float* uvals,
                   float* ograd, float* gpair, float* loss_sum, float* pair_sum, hipStream_t st,
                   float* gnc);
void launch_w2v_oreduce(const uint32_t* items, long long n, const uint32_t* ord, const float* ograd,
                        const float* otail, int B, int W, int D, float* ugrad, hipStream_t st,
                        const float* gnc = nullptr, long long negbase = 0,
                        const float* uvals = nullptr, float* acc = nullptr,
                        float* acc_out = nullptr, int acc_n = 0, const DevTable* tab = nullptr,
                        const long long* slots = nullptr, const OptParams* op = nullptr);
void launch_w2v_stream_gen(uint64_t seed, long long base, int B, int W, int L, long long nneg,
                           long long V, float noise, uint64_t* keys, int32_t* meta,
                           hipStream_t st, const long long* step_dev, long long step_mul,
                           long long step_add);
void launch_w2v_corpus_batch(const uint64_t* tokens, const uint64_t* sent_offs,
                             const uint32_t* sent_of, const uint64_t* table, long long table_size,
                             const float* keep, long long N, uint64_t seed, long long step,
                             const long long* step_dev, long long step_add, int B, int C, int W,
                             long long nneg, uint64_t out_bit, uint64_t* keys, hipStream_t st);
void launch_gen_ctr(uint64_t seed, long long sample_base, int B, int F, long long vocab_per_field,
                    float tail_frac, float truth_scale, float truth_bias, uint64_t* keys,
                    float* labels, hipStream_t st, const long long* step_dev = nullptr,
                    long long step_mul = 0, long long step_add = 0);
void launch_lr_fwd_bwd(const uint32_t* inv, const float* xval, const float* labels, int B, int F,
                       const float* uvals, float* ugrad, float* loss_sum, float* pred,
                       hipStream_t st);

void launch_fm_fwd_g(const uint32_t* inv, const BdIndex& ix, const float* labels, int B, int F, int dim, const float* uvals, float* gs,
                     float* gss, float* loss_sum, float* pred, hipStream_t st);
void launch_fm_fwd_bwd(const uint32_t* inv, const float* labels, int B, int F, int dim,
                       const float* uvals, float* ugrad, float* loss_sum, float* pred,
                       hipStream_t st);

// --- segreduce.hip
int sr_nbins(long long max_unique);
int sr_nchunks(long long n);
int sr_max_items(long long n);
long long sr_hist_words(long long n);
long long dedup_cnt_words(long long n, int nranks);
void launch_sr_plan(const uint32_t* inv, long long n, const unsigned long long* ucount,
                    int nranks, long long ucap, uint32_t* hist, int nbins, void* plan,
                    void* items, uint32_t* nitems, hipStream_t st);
void launch_sr_reduce(const void* plan, const float* gocc, const void* items,
                      const uint32_t* nitems, long long n, const unsigned long long* ucount,
                      int nranks, long long ucap, float* ugrad, hipStream_t st);
void launch_lr_fwd_g(const uint32_t* inv, const BdIndex& ix, const float* xval, const float* labels, int B, int F, const float* uvals,
                     float* g, int per_sample, float* loss_sum, float* pred, hipStream_t st,
                     const float* occ = nullptr, SelfSeg occ_self = SelfSeg{});

// --- bdedup.hip (bucketed dedup: partition by hash, LDS dedup per bucket)
// ndest: destinations that receive keys (effective server count, <= nranks;
// 0 = nranks) — sizes the buckets per destination (bdedup.hip bd_layout)
long long bd_max_keys();
long long bd_scratch_words(long long n, int nranks, int ndest = 0);
long long bd_ubase_offset(long long n, int nranks, int ndest = 0);
std::vector<long long> bd_offsets(long long n, int nranks, int ndest = 0);
int bd_buckets(long long n, int nranks, int ndest = 0);
// returns the region bits the call's buckets follow (rs.rbits if the layout
// allows region buckets — one rank, >= 4 regions per bucket — else 0)
int launch_bd_dedup(const uint64_t* keys, long long n, RouteSpec rs, long long ucap,
                    uint32_t* scratch, uint32_t* pj, uint32_t* pos_of, uint32_t* bkt,
                    uint32_t* luid, uint64_t* bkeys, unsigned long long* ucount, uint64_t* ukeys,
                    float* ugrad, int gdim, uint32_t* inv, int place, hipStream_t st,
                    unsigned long long* dbg = nullptr, uint32_t* rec = nullptr,
                    uint8_t* usingle = nullptr, int ndest = 0, long long lay_n = 0,
                    int msub = 1, uint32_t* usub = nullptr, uint32_t* spj = nullptr,
                    uint64_t* gkeys = nullptr, uint32_t* gspj = nullptr);
int bd_record_layout_bit();
int bd_record_group_bit();
int bd_target_dist();
int bd_target_for(int nranks, bool records);
void launch_rec_grad(const unsigned long long* ucount, int nd, long long gap, const uint32_t* spj,
                     const float* gs, const float* xval, int F, float* grec, hipStream_t st,
                     float* lacc = nullptr, float* lacc_out = nullptr, int lacc_n = 0,
                     int skip = -1);
void launch_bd_reduce(long long n, int nranks, const uint32_t* scratch, const uint32_t* pj,
                      const uint32_t* luid, const float* gs, const float* xval, int F,
                      float* ugrad, hipStream_t st, int osi = 0,
                      const uint8_t* usingle = nullptr, const DevTable* t = nullptr,
                      const long long* slots = nullptr, const float* snap = nullptr,
                      const OptParams* op = nullptr, int ndest = 0, int slot32 = 0,
                      float* lacc = nullptr, float* lacc_out = nullptr, int lacc_n = 0,
                      const uint64_t* bkeys = nullptr);
// occ[p] = uvals[uid of occurrence position p] (scalar rows; 0 where none):
// one workgroup per dedup bucket, for the LR forward's one-gather mode
void launch_bd_fill_occ(long long n, int nranks, const uint32_t* scratch, const uint32_t* luid,
                        const float* uvals, float* occ, int osi, hipStream_t st, int ndest, const uint32_t* pj = nullptr);
void launch_bd_unplace(long long n, int nranks, const uint32_t* scratch, const float* src,
                       float* dst, int dim, hipStream_t st, int ndest = 0);

void launch_bd_reduce_fm(long long n, int nranks, const uint32_t* scratch, const uint32_t* pj,
                         const uint32_t* luid, const float* gs, const float* gss, int F, int dim,
                         const float* uvals, float* ugrad, hipStream_t st,
                         uint32_t* ovf = nullptr, const DevTable* t = nullptr,
                         const long long* slots = nullptr, const OptParams* op = nullptr,
                         int ndest = 0);
long long bd_fm_ovf_words(long long n);

// explicit-layout forms of the bucket kernels (server-side merge)
void launch_bd_reduce_p(int P, const uint32_t* bstart, const uint32_t* ubase, const uint32_t* unum,
                        const uint32_t* pj, const uint32_t* luid, const float* gs, int F,
                        float* ugrad, const DevTable* t, const long long* slots,
                        const float* snap, const OptParams* op, hipStream_t st,
                        SelfSeg self = {}, int slot32 = 0, const uint64_t* bkeys = nullptr);
void launch_bd_fill_occ_p(int P, const uint32_t* bstart, const uint32_t* ubase,
                          const uint32_t* unum, const uint32_t* luid, const float* uvals,
                          float* occ, const uint32_t* pj, hipStream_t st, SelfSeg self = {});

// --- server.hip (N>1: merge of the keys a round receives from all sources)
int srv_sub_buckets(int nsrc, long long lay_n = 0, int ndest = 0);
void launch_srv_dedup(const uint64_t* rkeys, const uint32_t* rbase, const uint32_t* rnum,
                      long long cap, int nsrc, int Pd, int m, int me, uint32_t* cnt,
                      uint32_t* bstart, uint32_t* pj, uint32_t* luid, uint64_t* bkeys,
                      uint32_t* ubase, uint32_t* unum, unsigned long long* ucount, uint32_t* err,
                      hipStream_t st, const uint32_t* roff = nullptr, SelfSeg self = {});
void launch_srv_fill_rows(int P, const uint32_t* bstart, const uint32_t* ubase,
                          const uint32_t* pj, const uint32_t* luid, const float* rows, float* out,
                          int D, hipStream_t st, SelfSeg self = {});
void launch_srv_merge_rows(int P, const uint32_t* bstart, const uint32_t* ubase,
                           const uint32_t* unum, const uint32_t* pj, const uint32_t* luid,
                           const float* grads, float* merged, int D, hipStream_t st,
                           const DevTable* t = nullptr, const long long* slots = nullptr,
                           const OptParams* op = nullptr, SelfSeg self = {});

// --- w2v.hip
size_t w2v_smem_bytes(int D);
void launch_w2v_sgns(const uint32_t* inv_c, const uint32_t* inv_x, const uint32_t* inv_n, int B,
                     int C, int D, float neg_scale, const float* uvals, float* ugrad,
                     float* loss_sum, hipStream_t st, int bf16 = 0);
void launch_w2v_gen(uint64_t seed, long long base, int B, int C, int W, long long nneg,
                    long long V, float noise, uint64_t* keys, hipStream_t st,
                    const long long* step_dev = nullptr, long long step_mul = 0,
                    long long step_add = 0);

}  // namespace ss
