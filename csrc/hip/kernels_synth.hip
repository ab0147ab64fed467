// xflow-amd: on-device synthetic Criteo-shaped batch generator (gfx950).
// One lane per row; the per-sample recipe is xflow/synth.h (shared with the
// CPU backend).  Field constants travel by value in the kernel arguments.
#include "kernels.h"
#include "hip_util.h"
#include "xflow/synth.h"

namespace xflow {
namespace hip {

struct SynthConsts {
  u64 vocab[kSynthMaxFields];
  float s[kSynthMaxFields];
};

__global__ void __launch_bounds__(kBlock) k_synth(SynthArgs a, SynthConsts c) {
  int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= a.rows) return;
  const u64 rs = synth_row_seed(a.seed, a.step, r);
  float logit = a.planted_bias;
  for (int f = 0; f < a.fields; ++f) {
    u64 key = synth_key(rs, f, c.vocab[f], (double)c.s[f], a.hash_space);
    a.keys[r * a.fields + f] = key;
    if (a.fgid) a.fgid[r * a.fields + f] = f;
    logit += synth_planted_weight(key, a.planted_scale);
  }
  a.labels[r] = synth_label(rs, logit);
}

void launch_synth(const SynthArgs& a, hipStream_t st) {
  if (a.rows <= 0) return;
  if (a.fields > kSynthMaxFields) throw std::runtime_error("synth: at most 64 fields");
  SynthConsts c;
  for (int f = 0; f < a.fields; ++f) {
    c.vocab[f] = a.vocab[f] ? a.vocab[f] : 1;
    c.s[f] = a.zipf_s[f];
  }
  hipLaunchKernelGGL(k_synth, dim3((int)((a.rows + kBlock - 1) / kBlock)), dim3(kBlock), 0, st, a,
                     c);
  XF_HIP_CHECK(hipGetLastError());
}

}  // namespace hip
}  // namespace xflow
