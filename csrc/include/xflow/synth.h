// xflow-amd: synthetic Criteo-shaped sample recipe shared by both backends.
//
// Field f draws a rank from a truncated power law over its vocabulary
// (inverse CDF of p(x) ~ x^-s on [1, V+1)), hashes (field, rank) into the
// model's hashed feature space, and the label is drawn from a planted logistic
// model over the same hashed keys so that logloss is meaningful.  Counter
// based: (seed, step, row, field) fully determine a sample.
#pragma once

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

XF_HD double synth_unit(u64 h) {  // (0,1)
  return ((double)(h >> 11) + 0.5) * (1.0 / 9007199254740992.0);
}

XF_HD float synth_planted_weight(u64 key, float scale) {
  u64 h = fmix64(key ^ 0x6a09e667f3bcc909ull);
  return scale * (float)(2.0 * synth_unit(h) - 1.0);
}

XF_HD u64 synth_row_seed(u64 seed, u64 step, int64_t r) {
  return fmix64(seed * 0x9e3779b97f4a7c15ull ^ fmix64(step + 0x51ed27) ^
                ((u64)r * 0xd1b54a32d192ed03ull));
}

// Per-field constants of the truncated power law, computed once per batch.
struct SynthField {
  u64 vocab;
  double A;      // (V+1)^(1-s) - 1
  double inv_e;  // 1/(1-s)
  double logv1;  // ln(V+1), for s == 1
  int unit_s;
};

XF_HD SynthField synth_field(u64 vocab, double s) {
  SynthField F;
  F.vocab = vocab ? vocab : 1;
  double V = (double)F.vocab;
  F.unit_s = fabs(s - 1.0) < 1e-9;
  F.logv1 = log(V + 1.0);
  double e = 1.0 - s;
  F.A = F.unit_s ? 0.0 : pow(V + 1.0, e) - 1.0;
  F.inv_e = F.unit_s ? 0.0 : 1.0 / e;
  return F;
}

XF_HD u64 synth_key(u64 rowseed, int f, const SynthField& F, u64 hash_space) {
  u64 h = fmix64(rowseed + (u64)(f + 1) * 0x94d049bb133111ebull);
  double u = synth_unit(h);
  double x = F.unit_s ? exp(u * F.logv1) : pow(F.A * u + 1.0, F.inv_e);
  u64 rank = (u64)x;
  if (rank < 1) rank = 1;
  if (rank > F.vocab) rank = F.vocab;
  // hash into [0, hash_space) by multiply-high (no 64-bit division)
  return mulhi64(fmix64(((u64)(f + 1) << 40) ^ (rank - 1) ^ 0x3c6ef372fe94f82bull), hash_space);
}

XF_HD float synth_label(u64 rowseed, float logit) {
  double ul = synth_unit(fmix64(rowseed ^ 0xa54ff53a5f1d36f1ull));
  double p = 1.0 / (1.0 + exp(-(double)logit));
  return ul < p ? 1.0f : 0.0f;
}

}  // namespace xflow
