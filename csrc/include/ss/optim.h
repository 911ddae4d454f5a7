// ss/optim.h — parameter initialisers and per-coordinate update rules shared
// bit-for-bit (modulo libm rounding) by the gfx950 table kernels and the host
// CPU table, so a CPU server and an MI355X server apply identical semantics.
//
// These replace the user-subclassed PullAccessMethod::init_param and
// PushAccessMethod::apply_push_value of the reference
// (/root/reference/src/core/parameter/sparse_access_method.h:10-48) with a
// fixed, compiled menu.
#pragma once
#include <cmath>
#include <cstdint>
#include <cstring>

#include "ss/hash.h"

namespace ss {

// kInitConst: every parameter = scale.  kInitMarker: parameters get the
// kInitMarkerBits NaN payload, so the host can find the keys a pull just
// created and run a user's tensor-code initialiser on them
// (HbmTable.set_init_method; the reference's PullAccessMethod::init_param,
// sparse_access_method.h:10-28).
enum InitKind : int { kInitZero = 0, kInitUniform = 1, kInitNormal = 2, kInitConst = 3,
                      kInitMarker = 4 };
static constexpr uint32_t kInitMarkerBits = 0x7FBADBADu;
enum OptKind : int { kOptSGD = 0, kOptAdaGrad = 1, kOptFTRL = 2, kOptAdam = 3 };

struct InitParams {
  int kind;
  float scale;       // uniform: (u - 0.5) * scale ; normal: N(0,1) * scale
  float state_init;  // initial value of every optimizer-state float
  uint64_t seed;
  int zero_bit;      // keys with this bit set start at zero (-1: none) — e.g. the
                     // word2vec output-embedding namespace (syn1neg starts at 0)
};

struct OptParams {
  int kind;
  float lr;
  float l1, l2;
  float eps;
  float beta1, beta2;  // Adam
  float bc1, bc2;      // Adam bias corrections 1/(1-b^t), host-computed per round
  float ftrl_alpha, ftrl_beta;
  float grad_scale;    // multiplies incoming gradients
  float clip;          // |g| clip, 0 = off
};

SS_HD int opt_state_width(int kind, int dim) {
  return kind == kOptAdaGrad ? dim : ((kind == kOptFTRL || kind == kOptAdam) ? 2 * dim : 0);
}

#if defined(__HIP_DEVICE_COMPILE__)
#define SS_RSQRT(x) __frsqrt_rn(x)
#define SS_LOGF(x) __logf(x)
#define SS_COSF(x) __cosf(x)
#else
#define SS_RSQRT(x) (1.0f / std::sqrt(x))
#define SS_LOGF(x) std::log(x)
#define SS_COSF(x) std::cos(x)
#endif

// Deterministic per-(key, j) initial value: independent of the inserting lane,
// the shard layout and the world size, so checkpoints are reproducible.
SS_HD float init_value(const InitParams& ip, uint64_t key, uint32_t j, uint32_t dim) {
  (void)dim;
  if (ip.kind == kInitZero) return 0.0f;
  if (ip.kind == kInitMarker) {
    const uint32_t b = kInitMarkerBits;
    float f;
    std::memcpy(&f, &b, 4);
    return f;
  }
  if (ip.zero_bit >= 0 && ((key >> ip.zero_bit) & 1ull)) return 0.0f;
  if (ip.kind == kInitConst) return ip.scale;
  const uint64_t r =
      splitmix64(ip.seed ^ (key * 0x9E3779B97F4A7C15ull) ^ ((uint64_t)j << 48) ^ (uint64_t)j);
  if (ip.kind == kInitUniform) {
    // reference word2vec convention: (rand/RAND_MAX - 0.5) / size  (vec1.h:223-226)
    return (u01(r) - 0.5f) * ip.scale;
  }
  float u1 = u01(r);
  u1 = u1 < 1e-7f ? 1e-7f : u1;
  const float u2 = u01(splitmix64(r));
  return std::sqrt(-2.0f * SS_LOGF(u1)) * SS_COSF(6.2831853f * u2) * ip.scale;
}

// One coordinate of an optimizer step. `row` = params, `st` = state base.
// Register form: w = parameter, s1/s2 = the optimizer state slots of this
// coordinate (AdaGrad: s1 = sum g^2; FTRL: s1 = z, s2 = n; Adam: s1 = m,
// s2 = v).  Kernels load a row's coordinates first, update in registers and
// store after (no load behind a store of the same row).
SS_HD void opt_update(const OptParams& op, float& w, float& s1, float& s2, float g) {
  g *= op.grad_scale;
  if (op.clip > 0.f) g = g < -op.clip ? -op.clip : (g > op.clip ? op.clip : g);
  switch (op.kind) {
    case kOptSGD: {
      g += op.l2 * w;
      w = w - op.lr * g;
    } break;
    case kOptAdaGrad: {
      g += op.l2 * w;
      s1 = s1 + g * g;
      w = w - op.lr * g * SS_RSQRT(s1 + op.eps);
    } break;
    case kOptFTRL: {
      // FTRL-Proximal (per-coordinate); w is kept materialised in the row.
      const float n2 = s2 + g * g;
      const float sigma = (std::sqrt(n2) - std::sqrt(s2)) / op.ftrl_alpha;
      s1 += g - sigma * w;
      s2 = n2;
      const float az = std::fabs(s1);
      w = az <= op.l1 ? 0.0f
                      : -(s1 - std::copysign(op.l1, s1)) /
                            ((op.ftrl_beta + std::sqrt(n2)) / op.ftrl_alpha + op.l2);
    } break;
    case kOptAdam: {
      g += op.l2 * w;
      s1 = op.beta1 * s1 + (1.f - op.beta1) * g;
      s2 = op.beta2 * s2 + (1.f - op.beta2) * g * g;
      w = w - op.lr * (s1 * op.bc1) / (std::sqrt(s2 * op.bc2) + op.eps);
    } break;
  }
}

// number of state floats per coordinate
SS_HD int opt_state_per_coord(int kind) {
  return kind == kOptSGD ? 0 : (kind == kOptAdaGrad ? 1 : 2);
}

SS_HD void opt_apply(const OptParams& op, float* row, float* st, uint32_t dim, uint32_t j,
                     float g) {
  const int ns = opt_state_per_coord(op.kind);
  float w = row[j], s1 = ns > 0 ? st[j] : 0.f, s2 = ns > 1 ? st[dim + j] : 0.f;
  opt_update(op, w, s1, s2, g);
  row[j] = w;
  if (ns > 0) st[j] = s1;
  if (ns > 1) st[dim + j] = s2;
}

}  // namespace ss
