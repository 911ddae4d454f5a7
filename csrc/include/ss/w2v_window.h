// ss/w2v_window.h — the windowed skip-gram batch layout, shared by the host
// corpus batcher (csrc/host/dataio.h), the device batchers (csrc/hip/data.hip,
// csrc/hip/w2v.hip) and the tile kernel that consumes it (k_w2v_win_bf16).
//
// A batch is a RUN of B + 2W consecutive token positions of the stream; the B
// middle positions are the centers and every position within a center's
// (reduced) window in the same sentence is one of its contexts — word2vec's
// sliding window, so a center's contexts are not stored per pair: they are
// the run's neighbouring positions.  Per position one 32-bit meta word:
//
//     meta = (sentence tag mod 2^27) << 4 | b      b = reduced window, 1..W
//     meta = -1                                    masked (sub-sampled / padding)
//
// Pair (center c, position q) is a positive pair iff both are unmasked, in the
// same sentence and 0 < |q - c| <= b(c)  (word2vec's "b = rand() % window"
// shrink of the window, here 1 + hash % W).  Sub-sampled tokens are masked in
// place: they neither train nor count as context (word2vec removes them
// before windowing, which widens the window over them; here it does not).
#pragma once
#include <cstdint>

#include "ss/hash.h"

namespace ss {

static constexpr int kW2vMaxWindow = 15;  // b fits the meta word's low 4 bits

SS_HD int32_t w2v_meta(uint64_t sent_tag, int b) {
  return (int32_t)((((uint32_t)sent_tag & 0x7FFFFFFu) << 4) | (uint32_t)b);
}

// reduced window of the token at (global, per-rank) stream position gpos
SS_HD int w2v_reduced_window(uint64_t seed, uint64_t gpos, int W) {
  return 1 + (int)fastrange64(splitmix64(seed ^ 0x5EEDB0A7ull ^ (gpos * 0x9E3779B97F4A7C15ull)),
                              (uint64_t)W);
}

// frequent-word sub-sampling decision for stream position gpos at `step`
SS_HD bool w2v_keep(uint64_t seed, uint64_t step, uint64_t gpos, float keep_prob) {
  return u01(splitmix64(seed ^ 0x4B33F00Dull ^ (step * 0xD1B54A32D192ED03ull) ^
                        (gpos * 0x9E3779B97F4A7C15ull))) < keep_prob;
}

SS_HD bool w2v_pair_ok(int32_t mc, int32_t mq, int dist) {
  const int ad = dist < 0 ? -dist : dist;
  return mc >= 0 && mq >= 0 && (mc >> 4) == (mq >> 4) && ad != 0 && ad <= (mc & 15);
}

}  // namespace ss
