// xflow-amd: shared host/device definitions.
//
// Everything in this header is usable from both the C++ CPU backend and the
// gfx950 HIP kernels.  It holds the per-element math that defines reference
// behaviour (sigmoid clamps, FTRL-Proximal closed form, SGD) so that both
// backends execute bit-for-bit the same scalar recipe.
//
// Reference semantics:
//   sigmoid            /root/reference/src/base/base.h:54-63
//   FTRL-Proximal      /root/reference/src/optimizer/ftrl.h:58-74 (w), :125-141 (v)
//   SGD                /root/reference/src/optimizer/sgd.h:50-52, :94-96
//   v lazy init        /root/reference/src/optimizer/ftrl.h:114-120 (N(0,1)*1e-2)
#pragma once

#include <stdint.h>
#include <math.h>

#if defined(__HIPCC__)
#define XF_HD __host__ __device__ __forceinline__
#else
#define XF_HD inline
#endif

namespace xflow {

using u64 = uint64_t;
using u32 = uint32_t;

// Slot sentinel for every open-addressing table.  A user key equal to the
// sentinel is remapped to kEmptyKey-1 (documented in docs/DESIGN.md).
constexpr u64 kEmptyKey = ~0ull;

XF_HD u64 sanitize_key(u64 k) { return k == kEmptyKey ? kEmptyKey - 1 : k; }

// 64-bit finaliser (murmur3 fmix64).  Low bits index table slots, the high
// 32 bits choose the owning rank, so the two are independent.
XF_HD u64 fmix64(u64 h) {
  h ^= h >> 33;
  h *= 0xff51afd7ed558ccdull;
  h ^= h >> 33;
  h *= 0xc4ceb9fe1a85ec53ull;
  h ^= h >> 33;
  return h;
}

// Synthetic "historic" key i of a prefilled table (Backend::table_prefill):
// bit 62 set, so it never equals a hashed feature below 2^62.
XF_HD u64 prefill_key(u64 seed, u64 i) {
  return (1ull << 62) | (fmix64(seed * 0x9E3779B97F4A7C15ull + i) >> 2);
}

XF_HD u32 owner_of(u64 key, u32 world) {
  return world <= 1 ? 0u : (u32)((fmix64(key) >> 32) % world);
}

// Reference sigmoid: clamp at |x|>30, otherwise e^x/(1+e^x) evaluated in
// double with the literal base 2.718281828 (base.h:54-63).
XF_HD float sigmoid_ref(float x) {
  if (x < -30.0f) return 1e-6f;
  if (x > 30.0f) return 1.0f;
  // pow(2.718281828, x) == exp(x * ln(2.718281828))
  const double kLnBase = 0.9999999998311266;  // ln(2.718281828)
  double ex = exp((double)x * kLnBase);
  return (float)(ex / (1.0 + ex));
}

// ---------------------------------------------------------------------------
// Optimizers.  The table stores per parameter either (n, z) [FTRL] or w [SGD].
// FTRL's weight is a pure function of (z, n) after the first push, so it is
// never stored: pull recomputes it with exactly the reference float recipe.
// ---------------------------------------------------------------------------
struct FtrlParams {
  float alpha = 5e-2f;    // ftrl.h:17
  float beta = 1.0f;      // ftrl.h:18
  float lambda1 = 5e-5f;  // ftrl.h:19
  float lambda2 = 10.0f;  // ftrl.h:20
};

// (sn = sqrtf(n): a chain of pushes onto one parameter carries it, so each
// push takes one square root instead of three -- the same floats)
// The reference divides by alpha twice per push (ftrl.h:62,69); here both
// are products with float(1 / alpha): a push's dependency chain (a hot key's
// slice-long chain of pushes is sequential by definition) keeps one IEEE
// division instead of three, within an ulp of the quotients.
XF_HD float ftrl_inv_alpha(const FtrlParams& p) { return 1.0f / p.alpha; }
XF_HD float ftrl_weight_sn(float z, float sn, const FtrlParams& p) {
  if (fabsf(z) <= p.lambda1) return 0.0f;
  float tmpr = 0.0f;
  if (z > 0.0f) tmpr = z - p.lambda1;
  if (z < 0.0f) tmpr = z + p.lambda1;
  float tmpl = -1.0f * ((p.beta + sn) * ftrl_inv_alpha(p) + p.lambda2);
  return tmpr / tmpl;
}

XF_HD float ftrl_weight(float z, float n, const FtrlParams& p) {
  return ftrl_weight_sn(z, sqrtf(n), p);
}

// One FTRL-Proximal push of gradient g onto (n, z) whose current weight is w.
XF_HD void ftrl_push_sn(float& n, float& z, float& sn, float w, float g, const FtrlParams& p) {
  float nn = n + g * g;
  float snn = sqrtf(nn);
  z += g - (snn - sn) * ftrl_inv_alpha(p) * w;
  n = nn;
  sn = snn;
}

XF_HD void ftrl_push(float& n, float& z, float w, float g, const FtrlParams& p) {
  float sn = sqrtf(n);
  ftrl_push_sn(n, z, sn, w, g, p);
}

struct SgdParams {
  float lr = 0.001f;      // sgd.h:16
  float v_init = 0.001f;  // sgd.h:69
};

// ---------------------------------------------------------------------------
// Deterministic lazy initialisation of latent (v) parameters: N(0,1)*scale,
// derived from (seed, key, dim) by a counter-based hash + Box-Muller.  The
// reference draws from a time-seeded default_random_engine (base.h:33-44), so
// any N(0,1) source is behaviour-equivalent; ours is reproducible and needs no
// RNG state, which lets any reader of an un-pushed slot materialise the value.
// ---------------------------------------------------------------------------
XF_HD float normal_init(u64 key, u32 dim, u64 seed) {
  u64 a = fmix64(key ^ (seed * 0x9e3779b97f4a7c15ull) ^ ((u64)dim << 48) ^ 0x243f6a8885a308d3ull);
  u64 b = fmix64(a ^ 0x13198a2e03707344ull);
  // 24-bit uniforms in (0,1]
  float u1 = ((float)(a >> 40) + 1.0f) * (1.0f / 16777216.0f);
  float u2 = ((float)(b >> 40)) * (1.0f / 16777216.0f);
  float r = sqrtf(-2.0f * logf(u1));
  return r * cosf(6.283185307179586f * u2);
}

}  // namespace xflow
