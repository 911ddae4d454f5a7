// data.hip — HBM-resident training data: batch assembly on the device.
//
// The reference's apps parse text on the worker's CPU for every pass
// (BaseAlgorithm::parse_record over scan_file_by_line, /root/reference/src/
// core/framework/SwiftWorker.h:19-30, utils/file.h:14-33).  Here a file is
// parsed ONCE by the native loader (csrc/host/dataio.h, CSR: row offsets,
// keys, values, labels) and the whole shard is uploaded to HBM3E (288 GB per
// GPU holds e.g. 45M rows x 39 fields of u64 keys in 14 GB); each step's
// padded B x F batch is then cut out of it by one streaming kernel instead of
// a host fill + 82 MB PCIe copy per step (batch 262144 x 39).
#include "ss_device.h"
#include "ss_launch.h"

namespace ss {

// One lane per (sample, field) of the batch: sample b is dataset row
// (cursor + b) mod rows; its first min(len, F) keys are copied, the rest of
// the F slots get the EMPTY key (the dedup skips it) and value 0 — the same
// layout SparseDataset::fill produces on the host.  Keys of a row are
// contiguous, so consecutive lanes read consecutive words.  With step_dev
// (hipGraph replays) the cursor is ((*step_dev + step_add) * B) mod rows.
__global__ __launch_bounds__(256) void k_csr_batch(const uint64_t* __restrict__ offs,
                                                   const uint64_t* __restrict__ keys,
                                                   const float* __restrict__ vals,
                                                   const float* __restrict__ labels,
                                                   unsigned long long rows,
                                                   unsigned long long cursor, int B, int F,
                                                   const long long* __restrict__ step_dev,
                                                   long long step_add,
                                                   uint64_t* __restrict__ out_keys,
                                                   float* __restrict__ out_vals,
                                                   float* __restrict__ out_labels) {
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i >= (long long)B * F) return;
  const int b = (int)(i / F), f = (int)(i - (long long)b * F);
  unsigned long long c0 = cursor;
  if (step_dev)
    c0 = ((unsigned long long)(*step_dev + step_add) * (unsigned long long)B) % rows;
  const unsigned long long r = (c0 + (unsigned long long)b) % rows;
  const uint64_t o = offs[r];
  const uint64_t len = offs[r + 1] - o;
  const bool have = (uint64_t)f < len;
  out_keys[i] = have ? keys[o + f] : kEmptyKey;
  if (out_vals) out_vals[i] = have ? (vals ? vals[o + f] : 1.f) : 0.f;
  if (f == 0) out_labels[b] = labels[r];
}

void launch_csr_batch(const uint64_t* offs, const uint64_t* keys, const float* vals,
                      const float* labels, long long rows, long long cursor, int B, int F,
                      const long long* step_dev, long long step_add, uint64_t* out_keys,
                      float* out_vals, float* out_labels, hipStream_t st) {
  if (rows <= 0) throw_error("csr_batch: empty dataset");
  if (B <= 0 || F <= 0) return;
  const long long n = (long long)B * F;
  hipLaunchKernelGGL(k_csr_batch, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, offs, keys,
                     vals, labels, (unsigned long long)rows,
                     (unsigned long long)(((cursor % rows) + rows) % rows), B, F, step_dev,
                     step_add, out_keys, out_vals, out_labels);
  check_launch("k_csr_batch");
}

}  // namespace ss
