// xflow-amd: on-device synthetic Criteo-shaped batch generator (gfx950).
// One lane per row; the per-sample recipe is xflow/synth.h (shared with the
// CPU backend).  Field constants travel by value in the kernel arguments.
#include "kernels.h"
#include "hip_util.h"
#include "xflow/synth.h"

namespace xflow {
namespace hip {

struct SynthConsts {
  SynthField f[kSynthMaxFields];
};

// A workgroup owns kSynthRows rows.  The row seeds (two fmix64 rounds each, a
// large share of an element's 64-bit multiplies if recomputed per element)
// and the field constants are staged in LDS once.  Lanes then walk the tile's
// (row, field) elements in memory order, so key/fgid stores are coalesced;
// each element's planted weight is parked in LDS and one lane per row sums
// them in field order (deterministic, the same order as the CPU backend).
constexpr int kSynthRows = 64;

template <bool kSmall>
__global__ void __launch_bounds__(kBlock) k_synth(SynthArgs a, SynthConsts c) {
  __shared__ float pw[kSynthRows * kSynthMaxFields];
  __shared__ u64 rseed[kSynthRows];
  __shared__ SynthField fc[kSynthMaxFields];
  __shared__ int64_t fofs[kSynthMaxFields];  // field-major: f * col_stride (no 64-bit multiply per key)
  const int F = a.fields;
  const int64_t r0 = (int64_t)blockIdx.x * kSynthRows;
  const int rows = (int)min((int64_t)kSynthRows, a.rows - r0);
  const int n = rows * F;
  const bool field_major = a.col_stride > 0;
  if ((int)threadIdx.x < rows)
    rseed[threadIdx.x] = synth_row_seed_mixed(a.seed, synth_step_mix(a.step), r0 + threadIdx.x);
  if ((int)threadIdx.x < F) {
    fc[threadIdx.x] = c.f[threadIdx.x];
    fofs[threadIdx.x] = (int64_t)threadIdx.x * a.col_stride;
  }
  __syncthreads();
  for (int e = threadIdx.x; e < n; e += blockDim.x) {
    int rl, f;
    if (field_major) {  // consecutive lanes take consecutive rows of one field
      f = rows == kSynthRows ? e / kSynthRows : e / rows;
      rl = e - f * rows;
    } else {
      rl = e / F;
      f = e - rl * F;
    }
    float w;
    const u64 key = synth_sample<kSmall>(rseed[rl], f, fc[f], a.hash_space, a.planted_scale, w);
    const int64_t o = field_major ? fofs[f] + r0 + rl : r0 * F + e;
    a.keys[o] = key;
    if (a.fgid) a.fgid[o] = f;
    pw[rl * F + f] = w;
  }
  __syncthreads();
  if ((int)threadIdx.x < rows) {
    float logit = a.planted_bias;
    for (int f = 0; f < F; ++f) logit += pw[threadIdx.x * F + f];
    a.labels[r0 + threadIdx.x] = synth_label(rseed[threadIdx.x], logit);
  }
}

void launch_synth(const SynthArgs& a, hipStream_t st) {
  if (a.rows <= 0) return;
  if (a.fields > kSynthMaxFields) throw std::runtime_error("synth: at most 64 fields");
  SynthConsts c;
  for (int f = 0; f < a.fields; ++f) c.f[f] = synth_field(a.vocab[f], (double)a.zipf_s[f], f);
  const dim3 grid((int)((a.rows + kSynthRows - 1) / kSynthRows));
  if (synth_small_ok(a.vocab, a.fields, a.hash_space))
    hipLaunchKernelGGL(k_synth<true>, grid, dim3(kBlock), 0, st, a, c);
  else
    hipLaunchKernelGGL(k_synth<false>, grid, dim3(kBlock), 0, st, a, c);
  XF_HIP_CHECK(hipGetLastError());
}

}  // namespace hip
}  // namespace xflow
