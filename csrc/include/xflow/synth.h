// xflow-amd: synthetic Criteo-shaped sample recipe shared by both backends.
//
// Field f draws a rank from a truncated power law over its vocabulary
// (inverse CDF of p(x) ~ x^-s on [1, V+1)), hashes (field, rank) into the
// model's hashed feature space, and the label is drawn from a planted logistic
// model over the same hashed keys so that logloss is meaningful.  Counter
// based: (seed, step, row, field) fully determine a sample.
//
// The per-element math uses IEEE basic float operations only (no libm; both
// builds compile without FMA contraction), so the host and gfx950 produce
// bit-identical batches.  The inverse CDF x = (A*u + 1)^(1/e) is evaluated as
// exp2(log2(A*u + 1) / e) with the short log2/exp2 below: ~40 VALU ops per
// element instead of a double-precision pow, which made the generator
// VALU-bound (PMC: ~356 VALU instructions per element).
#pragma once

#include <string.h>

#include "xflow/common.h"

namespace xflow {

constexpr int kSynthMaxFields = 64;

XF_HD u64 mulhi64(u64 a, u64 b) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __umul64hi(a, b);
#else
  return (u64)(((unsigned __int128)a * b) >> 64);
#endif
}

XF_HD u32 synth_f2u(float f) {
  u32 u;
  memcpy(&u, &f, 4);
  return u;
}

XF_HD float synth_u2f(u32 u) {
  float f;
  memcpy(&f, &u, 4);
  return f;
}

XF_HD double synth_unit(u64 h) {  // (0,1)
  return ((double)(h >> 11) + 0.5) * (1.0 / 9007199254740992.0);
}

XF_HD float synth_unit_f(u64 h) {  // (0,1), exact in float
  return ((float)(u32)(h >> 41) + 0.5f) * (1.0f / 8388608.0f);
}

// log2(x) of a positive normal float: exponent + atanh series of the mantissa
// reduced to [sqrt(1/2), sqrt(2)) (|t| <= 0.172, truncation error < 2e-8).
XF_HD float synth_log2(float x) {
  const u32 b = synth_f2u(x);
  int e = (int)((b >> 23) & 0xFFu) - 127;
  float m = synth_u2f((b & 0x7FFFFFu) | 0x3F800000u);  // [1, 2)
  if (m > 1.41421356f) {
    m = m * 0.5f;
    e += 1;
  }
  const float t = (m - 1.0f) / (m + 1.0f);
  const float t2 = t * t;
  // 2/ln2 * (t + t^3/3 + t^5/5 + t^7/7 + t^9/9)
  float p = 0.11111111f;
  p = p * t2 + 0.14285714f;
  p = p * t2 + 0.2f;
  p = p * t2 + 0.33333333f;
  p = p * t2 + 1.0f;
  return (float)e + (p * t) * 2.88539008f;
}

// 2^y for y in [-126, 126]: the integer part goes into the exponent bits, 2^f
// for f in [-0.5, 0.5] is a degree-6 Taylor polynomial (error < 2e-7).
XF_HD float synth_exp2(float y) {
  const float r = y + 0.5f;
  int n = (int)r;
  if ((float)n > r) n -= 1;  // floor
  const float f = (y - (float)n) * 0.69314718f;
  float p = 0.0013888889f;
  p = p * f + 0.0083333333f;
  p = p * f + 0.041666667f;
  p = p * f + 0.16666667f;
  p = p * f + 0.5f;
  p = p * f + 1.0f;
  p = p * f + 1.0f;
  return synth_u2f(synth_f2u(p) + ((u32)n << 23));
}

XF_HD u64 synth_step_mix(u64 step) { return fmix64(step + 0x51ed27); }

XF_HD u64 synth_row_seed_mixed(u64 seed, u64 step_mix, int64_t r) {
  return fmix64(seed * 0x9e3779b97f4a7c15ull ^ step_mix ^ ((u64)r * 0xd1b54a32d192ed03ull));
}

XF_HD u64 synth_row_seed(u64 seed, u64 step, int64_t r) {
  return synth_row_seed_mixed(seed, synth_step_mix(step), r);
}

// Per-field constants of the truncated power law, computed once per batch in
// double on the host and rounded to float for the per-element recipe.
struct SynthField {
  u64 vocab;
  u64 fseed;     // (f + 1) * 0x94d049bb133111eb: the field's term of the element hash
  float A;       // (V+1)^(1-s) - 1
  float inv_e;   // 1/(1-s)
  float log2v1;  // log2(V+1), for s == 1
  int unit_s;
};

inline SynthField synth_field(u64 vocab, double s, int f) {
  SynthField F;
  F.vocab = vocab ? vocab : 1;
  F.fseed = (u64)(f + 1) * 0x94d049bb133111ebull;
  const double V = (double)F.vocab;
  F.unit_s = fabs(s - 1.0) < 1e-9;
  F.log2v1 = (float)log2(V + 1.0);
  const double e = 1.0 - s;
  F.A = F.unit_s ? 0.0f : (float)(pow(V + 1.0, e) - 1.0);
  F.inv_e = F.unit_s ? 0.0f : (float)(1.0 / e);
  return F;
}

// High 64 bits of a * b for b < 2^32: a*b = ah*b*2^32 + al*b, and
// floor((ah*b + floor(al*b / 2^32)) / 2^32) is exact (the sum < 2^64).  Three
// 32-bit multiplies on gfx950 instead of the general form's seven.
XF_HD u64 mulhi64_u32(u64 a, u32 b) {
  const u64 lo_hi = ((u64)(u32)a * b) >> 32;
  return ((a >> 32) * (u64)b + lo_hi) >> 32;
}

// Key of field f for the row, and its planted weight.  Both come from one
// hash of (field, rank): the key from its high bits (multiply-high into
// [0, hash_space), no 64-bit division), the weight from its low bits, so
// every occurrence of a key carries the same planted weight.
// kSmall: hash_space < 2^32 and every vocab < 2^31 (synth_small_ok, checked
// once per batch): the same bits through 32-bit rank conversion and the
// 32-bit multiply-high -- the generator is VALU-bound on 64-bit multiplies.
template <bool kSmall = false>
XF_HD u64 synth_sample(u64 rowseed, int f, const SynthField& F, u64 hash_space, float scale,
                       float& weight) {
  const u64 h = fmix64(rowseed + F.fseed);  // (a 64-bit multiply per element saved)
  const float u = synth_unit_f(h);
  const float y = F.unit_s ? u * F.log2v1 : synth_log2(F.A * u + 1.0f) * F.inv_e;
  u64 rank;
  if constexpr (kSmall) {
    // exp2(y) <= ~(V+1)(1 + 2^-20) < 2^32 for V < 2^31: the u32 conversion
    // truncates exactly as the u64 one does
    u32 r32 = (u32)synth_exp2(y);
    if (r32 < 1u) r32 = 1u;
    if (r32 > (u32)F.vocab) r32 = (u32)F.vocab;
    rank = r32;
  } else {
    rank = (u64)synth_exp2(y);
    if (rank < 1) rank = 1;
    if (rank > F.vocab) rank = F.vocab;
  }
  const u64 hk = fmix64(((u64)(f + 1) << 40) ^ (rank - 1) ^ 0x3c6ef372fe94f82bull);
  weight = scale * ((float)((u32)hk >> 8) * (2.0f / 16777216.0f) - 1.0f);
  if constexpr (kSmall) return mulhi64_u32(hk, (u32)hash_space);
  return mulhi64(hk, hash_space);
}

inline bool synth_small_ok(const u64* vocab, int fields, u64 hash_space) {
  if (hash_space >> 32) return false;
  for (int f = 0; f < fields; ++f)
    if ((vocab[f] ? vocab[f] : 1) >= (1ull << 31)) return false;
  return true;
}

XF_HD float synth_label(u64 rowseed, float logit) {
  double ul = synth_unit(fmix64(rowseed ^ 0xa54ff53a5f1d36f1ull));
  double p = 1.0 / (1.0 + exp(-(double)logit));
  return ul < p ? 1.0f : 0.0f;
}

}  // namespace xflow
