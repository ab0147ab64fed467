// Kernel experiment harness (gfx950): times the dedup and LR forward/backward
// launchers and a few memory-pattern probes on the bench's synthetic
// Criteo-shaped batch with hipEvents.  Built by scripts/gpu.sh kbench:
//   hipcc --offload-arch=gfx950 -O3 tools/kbench.hip csrc/hip/kernels_*.hip
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "hip_util.h"
#include "kernels.h"

using namespace xflow;
using namespace xflow::hip;

static std::vector<uint64_t> criteo_vocab() {
  const uint64_t cat[26] = {39884406, 39043, 17289, 7420, 20263, 3, 7120, 1543, 63,
                            38532951, 2953546, 403346, 10, 2208, 11938, 155, 4, 976,
                            14, 39979771, 25641295, 39664984, 585935, 12972, 108, 36};
  double big = 0, small = 13 * 64;
  for (uint64_t v : cat) (v > 1000000 ? big : small) += (double)v;
  double scale = std::max(1.0, (1e9 - small) / big);
  std::vector<uint64_t> v(13, 64);
  for (uint64_t c : cat) v.push_back(c > 1000000 ? (uint64_t)(c * scale) : c);
  return v;
}

struct Ev {
  hipEvent_t a, b;
  Ev() {
    XF_HIP_CHECK(hipEventCreate(&a));
    XF_HIP_CHECK(hipEventCreate(&b));
  }
  void start() { XF_HIP_CHECK(hipEventRecord(a, 0)); }
  float stop() {
    XF_HIP_CHECK(hipEventRecord(b, 0));
    XF_HIP_CHECK(hipEventSynchronize(b));
    float ms = 0;
    XF_HIP_CHECK(hipEventElapsedTime(&ms, a, b));
    return ms;
  }
};

template <typename T>
static T* dalloc(size_t n) {
  T* p = nullptr;
  XF_HIP_CHECK(hipMalloc(&p, n * sizeof(T) + 64));
  return p;
}

__global__ void k_rand_idx(u32* idx, int64_t n, u64 range, u64 seed) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    idx[i] = (u32)(fmix64((u64)i ^ seed) % range);
}
__global__ void k_scatter_atomic(float* dst, const u32* idx, int64_t n) {
  int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i < n) atomicAdd(&dst[idx[i]], 1.0f);
}
__global__ void k_scatter_store(float* dst, const u32* idx, int64_t n) {
  int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i < n) dst[idx[i]] = 1.0f;
}
__global__ void k_contig_atomic(float* dst, int64_t n) {
  int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i < n) atomicAdd(&dst[i], 1.0f);
}
// Per-XCD partial buffers with workgroup-scope atomics: do they execute in
// the XCD's L2 instead of at the memory side?
__device__ __forceinline__ u32 xcc_id() {
  u32 v;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(v));
  return v & 7u;
}
template <int SCOPE>
__global__ void k_scatter_atomic_xcd(float* dst, size_t stride, const u32* idx, int64_t n) {
  int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  float* d = dst + xcc_id() * stride;
  if (i < n) __hip_atomic_fetch_add(&d[idx[i]], 1.0f, __ATOMIC_RELAXED, SCOPE);
}
__global__ void k_sum_xcd(const float* src, size_t stride, float* out, int64_t n) {
  int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i >= n) return;
  float s = 0;
  for (int x = 0; x < 8; ++x) s += src[x * stride + i];
  out[i] = s;
}
__global__ void k_gather(const float* src, const u32* idx, float* out, int64_t n) {
  int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i < n) out[i] = src[idx[i]];
}

// Decomposition of k_dedup_insert (kernels_table.hip): kGlobal=false stops
// after the LDS level (slot = LDS index), kStamp=false skips the stamp stores;
// `leaders` counts global probes.
template <bool kGlobal, bool kStamp>
__global__ void __launch_bounds__(kBlock) k_dedup_var(const u64* __restrict__ keys, int64_t nnz,
                                                      ScratchView sv, u32* __restrict__ pos,
                                                      unsigned long long* leaders) {
  constexpr int IT = 8, L2N = 12;
  constexpr u32 kL = 1u << L2N;
  __shared__ u64 t_key[kL];
  __shared__ u32 t_slot[kL];
  u64* __restrict__ skeys = sv.keys;
  const u64 cap = sv.cap, mask = cap - 1;
  const int64_t base = (int64_t)blockIdx.x * (kBlock * IT) + threadIdx.x;
  for (u32 i = threadIdx.x; i < kL; i += kBlock) t_key[i] = kEmptyKey;
  u64 k[IT], s[IT];
  u32 h[IT];
#pragma unroll
  for (int j = 0; j < IT; ++j) {
    int64_t i = base + (int64_t)j * kBlock;
    k[j] = i < nnz ? sanitize_key(keys[i]) : 0ull;
    const u64 f = fmix64(k[j]);
    s[j] = f & mask;
    h[j] = (u32)(f >> (64 - L2N));
  }
  __syncthreads();
  u32 lead = 0;
#pragma unroll
  for (int j = 0; j < IT; ++j) {
    if (base + (int64_t)j * kBlock >= nnz) continue;
    u32 x = h[j];
    while (true) {
      const u64 c = t_key[x];
      if (c == k[j]) break;
      if (c == kEmptyKey) {
        const u64 prev = atomicCAS((unsigned long long*)&t_key[x], (unsigned long long)kEmptyKey,
                                   (unsigned long long)k[j]);
        if (prev == kEmptyKey) {
          lead |= 1u << j;
          break;
        }
        if (prev == k[j]) break;
      }
      x = (x + 1) & (kL - 1);
    }
    h[j] = x;
  }
  if (kGlobal) {
    u64 cur[IT];
#pragma unroll
    for (int j = 0; j < IT; ++j) cur[j] = (lead >> j) & 1u ? skeys[s[j]] : k[j];
#pragma unroll
    for (int j = 0; j < IT; ++j) {
      if (!((lead >> j) & 1u)) continue;
      u64 sj = s[j], c = cur[j];
      while (c != k[j]) {
        if (c == kEmptyKey) {
          u64 prev = atomicCAS((unsigned long long*)&skeys[sj], (unsigned long long)kEmptyKey,
                               (unsigned long long)k[j]);
          if (prev == kEmptyKey || prev == k[j]) break;
        }
        sj = (sj + 1) & mask;
        c = skeys[sj];
      }
      t_slot[h[j]] = (u32)sj;
      if (kStamp) sv.stamps[sj] = sv.epoch;
    }
  } else {
#pragma unroll
    for (int j = 0; j < IT; ++j)
      if ((lead >> j) & 1u) t_slot[h[j]] = h[j];
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < IT; ++j) {
    int64_t i = base + (int64_t)j * kBlock;
    if (i < nnz) pos[i] = t_slot[h[j]];
  }
  block_count_add<kBlock>(leaders, __popc(lead));
}

// Floors of the LDS level: MODE 0 = key load + fmix + pos store only;
// MODE 1 = + LDS table init, barrier and one read-only probe per item.
template <int MODE>
__global__ void __launch_bounds__(kBlock) k_stream_var(const u64* __restrict__ keys, int64_t nnz,
                                                       u32* __restrict__ pos) {
  constexpr int IT = 8, L2N = 12;
  constexpr u32 kL = 1u << L2N;
  __shared__ u64 t_key[MODE ? kL : 1];
  const int64_t base = (int64_t)blockIdx.x * (kBlock * IT) + threadIdx.x;
  if (MODE)
    for (u32 i = threadIdx.x; i < kL; i += kBlock) t_key[i] = kEmptyKey;
  u64 k[IT];
  u32 h[IT];
#pragma unroll
  for (int j = 0; j < IT; ++j) {
    int64_t i = base + (int64_t)j * kBlock;
    k[j] = i < nnz ? sanitize_key(keys[i]) : 0ull;
    h[j] = (u32)(fmix64(k[j]) >> (64 - L2N));
  }
  if (MODE) {
    __syncthreads();
#pragma unroll
    for (int j = 0; j < IT; ++j) h[j] += t_key[h[j]] == k[j] ? 1u : 0u;
  }
#pragma unroll
  for (int j = 0; j < IT; ++j) {
    int64_t i = base + (int64_t)j * kBlock;
    if (i < nnz) pos[i] = h[j];
  }
}

int main(int argc, char** argv) {
  const int64_t rows = argc > 1 ? atoll(argv[1]) : 262144;
  const int F = 39;
  const int64_t nnz = rows * F;
  const int iters = 10;
  auto vocab = criteo_vocab();
  std::vector<float> zipf(F, 1.05f);
  for (int f = 0; f < 13; ++f) zipf[f] = 0.8f;
  u64* keys = dalloc<u64>(nnz);
  float* labels = dalloc<float>(rows);
  SynthArgs sa;
  sa.keys = keys;
  sa.labels = labels;
  sa.rows = rows;
  sa.fields = F;
  sa.vocab = vocab.data();
  sa.zipf_s = zipf.data();
  sa.seed = 1234;
  const bool field_major = getenv("KB_FIELD") && atoi(getenv("KB_FIELD"));
  sa.col_stride = field_major ? rows : 0;
  printf("layout: %s\n", field_major ? "field-major" : "row-major");
  Ev ev;

  // ---- memory-pattern probes ------------------------------------------------
  {
    const int64_t n = 2950000;
    u32* idx = dalloc<u32>(n);
    float* dst = dalloc<float>((size_t)1 << 25);
    float* out = dalloc<float>(n);
    XF_HIP_CHECK(hipMemset(dst, 0, sizeof(float) << 25));
    for (u64 range : {(u64)2000000, (u64)1 << 25}) {
      hipLaunchKernelGGL(k_rand_idx, dim3(2048), dim3(256), 0, 0, idx, n, range, 7ull);
      float t[4] = {0, 0, 0, 0};
      for (int it = 0; it < iters + 1; ++it) {
        ev.start();
        hipLaunchKernelGGL(k_scatter_atomic, dim3((n + 255) / 256), dim3(256), 0, 0, dst, idx, n);
        float a = ev.stop();
        ev.start();
        hipLaunchKernelGGL(k_scatter_store, dim3((n + 255) / 256), dim3(256), 0, 0, dst, idx, n);
        float b = ev.stop();
        ev.start();
        hipLaunchKernelGGL(k_contig_atomic, dim3((n + 255) / 256), dim3(256), 0, 0, dst, n);
        float c = ev.stop();
        ev.start();
        hipLaunchKernelGGL(k_gather, dim3((n + 255) / 256), dim3(256), 0, 0, dst, idx, out, n);
        float d = ev.stop();
        if (it) {
          t[0] += a;
          t[1] += b;
          t[2] += c;
          t[3] += d;
        }
      }
      printf("probe n=%ld range=%llu: scattered atomic %.1f us, scattered store %.1f us, "
             "contiguous atomic %.1f us, scattered gather %.1f us\n",
             (long)n, (unsigned long long)range, 1e3 * t[0] / iters, 1e3 * t[1] / iters,
             1e3 * t[2] / iters, 1e3 * t[3] / iters);
      // per-XCD copies, workgroup / agent scope; check no add was lost
      const size_t stride = range;
      float* xb = dalloc<float>(stride * 8);
      float* sum = dalloc<float>(range);
      for (int scope = 0; scope < 2; ++scope) {
        XF_HIP_CHECK(hipMemset(xb, 0, stride * 8 * 4));
        float tt = 0;
        for (int it = 0; it < iters; ++it) {
          ev.start();
          if (scope == 0)
            hipLaunchKernelGGL((k_scatter_atomic_xcd<__HIP_MEMORY_SCOPE_WORKGROUP>),
                               dim3((n + 255) / 256), dim3(256), 0, 0, xb, stride, idx, n);
          else
            hipLaunchKernelGGL((k_scatter_atomic_xcd<__HIP_MEMORY_SCOPE_AGENT>),
                               dim3((n + 255) / 256), dim3(256), 0, 0, xb, stride, idx, n);
          tt += ev.stop();
        }
        hipLaunchKernelGGL(k_sum_xcd, dim3((range + 255) / 256), dim3(256), 0, 0, xb, stride,
                           sum, (int64_t)range);
        std::vector<float> h(range);
        XF_HIP_CHECK(hipMemcpy(h.data(), sum, range * 4, hipMemcpyDeviceToHost));
        double tot = 0;
        for (float v : h) tot += v;
        printf("  per-XCD %s-scope atomics: %.1f us, total %.0f (expect %.0f)\n",
               scope == 0 ? "workgroup" : "agent", 1e3 * tt / iters, tot, (double)n * iters);
      }
      XF_HIP_CHECK(hipFree(xb));
      XF_HIP_CHECK(hipFree(sum));
    }
  }

  // ---- dedup at several scratch capacities ----------------------------------
  for (int log2cap : {25, 24, 23, 22}) {
    const u64 cap = (u64)1 << log2cap;
    ScratchView sv;
    sv.keys = dalloc<u64>(cap);
    sv.stamps = dalloc<u32>(cap);
    sv.cap = cap;
    sv.claims = dalloc<unsigned long long>(1);
    sv.rebuild_at = cap / 2;
    if (getenv("KB_ADAPT") && atoi(getenv("KB_ADAPT"))) {
      sv.ctl = dalloc<unsigned long long>(4);
      unsigned long long c0[4] = {cap, 0, 0, 0};
      XF_HIP_CHECK(hipMemcpy(sv.ctl, c0, sizeof(c0), hipMemcpyHostToDevice));
    }
    DedupOut o;
    o.pos = dalloc<u32>(nnz);
    o.uniq_keys = dalloc<u64>(nnz);
    o.uniq_pos = dalloc<u32>(nnz);
    o.n_uniq = dalloc<int64_t>(1);
    o.overflow = dalloc<u32>(1);
    o.block_counts = dalloc<u32>(cap / 4096 + 1);
    launch_fill_u64(sv.keys, kEmptyKey, cap, 0);
    XF_HIP_CHECK(hipMemset(sv.stamps, 0, cap * 4));
    XF_HIP_CHECK(hipMemset(sv.claims, 0, 8));
    XF_HIP_CHECK(hipMemset(o.overflow, 0, 4));
    float tsyn = 0, tded = 0;
    int64_t nu = 0;
    const int warm = 5, steps = getenv("KB_STEPS") ? atoi(getenv("KB_STEPS")) : iters;
    for (int step = 0; step < warm + steps; ++step) {
      sa.step = step;
      ev.start();
      launch_synth(sa, 0);
      float a = ev.stop();
      sv.epoch = step + 1;
      ev.start();
      launch_dedup(keys, nnz, sv, o, 0);
      float b = ev.stop();
      if (step >= warm) {
        tsyn += a;
        tded += b;
      }
    }
    XF_HIP_CHECK(hipMemcpy(&nu, o.n_uniq, 8, hipMemcpyDeviceToHost));
    printf("dedup cap=2^%d: synth %.1f us, dedup %.1f us, n_uniq %ld\n", log2cap,
           1e3 * tsyn / steps, 1e3 * tded / steps, (long)nu);
    if (sv.ctl) {
      unsigned long long c[4];
      XF_HIP_CHECK(hipMemcpy(c, sv.ctl, sizeof(c), hipMemcpyDeviceToHost));
      printf("  adaptive: active cap %llu, max unique %llu, pending %llu\n", c[0], c[1], c[2]);
      sv.ctl = nullptr;  // decomposition below runs at the full capacity
    }
    {
      unsigned long long* lc = dalloc<unsigned long long>(1);
      const int g = (int)((nnz + kBlock * 8 - 1) / (kBlock * 8));
      float tv[3] = {0, 0, 0}, ts[2] = {0, 0};
      for (int it = 0; it < iters + 1; ++it) {
        ev.start();
        hipLaunchKernelGGL(k_stream_var<0>, dim3(g), dim3(kBlock), 0, 0, keys, nnz, o.pos);
        float s0 = ev.stop();
        ev.start();
        hipLaunchKernelGGL(k_stream_var<1>, dim3(g), dim3(kBlock), 0, 0, keys, nnz, o.pos);
        float s1 = ev.stop();
        if (it) {
          ts[0] += s0;
          ts[1] += s1;
        }
        XF_HIP_CHECK(hipMemset(lc, 0, 8));
        ev.start();
        hipLaunchKernelGGL((k_dedup_var<false, false>), dim3(g), dim3(kBlock), 0, 0, keys, nnz, sv,
                           o.pos, lc);
        float a = ev.stop();
        ev.start();
        hipLaunchKernelGGL((k_dedup_var<true, false>), dim3(g), dim3(kBlock), 0, 0, keys, nnz, sv,
                           o.pos, lc);
        float b = ev.stop();
        ev.start();
        hipLaunchKernelGGL((k_dedup_var<true, true>), dim3(g), dim3(kBlock), 0, 0, keys, nnz, sv,
                           o.pos, lc);
        float c = ev.stop();
        if (it) {
          tv[0] += a;
          tv[1] += b;
          tv[2] += c;
        }
      }
      unsigned long long nl = 0;
      XF_HIP_CHECK(hipMemcpy(&nl, lc, 8, hipMemcpyDeviceToHost));
      printf("  floors: stream %.1f us, +lds init/read %.1f us\n", 1e3 * ts[0] / iters,
             1e3 * ts[1] / iters);
      printf("  insert decomposition: lds-only %.1f us, +global probe %.1f us, +stamps %.1f us, "
             "leaders/step %llu\n",
             1e3 * tv[0] / iters, 1e3 * tv[1] / iters, 1e3 * tv[2] / iters, nl / 3);
    }

    if (log2cap == 25) {
      // LR forward (+backward) on the last batch: wpull/grad indexed by slot
      float* wp = dalloc<float>(cap);
      float* grad = dalloc<float>(cap);
      LossStats* st = dalloc<LossStats>(1);
      XF_HIP_CHECK(hipMemset(wp, 0, cap * 4));
      XF_HIP_CHECK(hipMemset(grad, 0, cap * 4));
      FwdArgs fa;
      fa.batch.keys = keys;
      fa.batch.labels = labels;
      fa.batch.rows = rows;
      fa.batch.nnz = nnz;
      fa.batch.nnz_per_row = F;
      fa.batch.col_stride = sa.col_stride;
      fa.pos = o.pos;
      fa.wpull = wp;
      fa.stats = st;
      fa.model.kind = kLR;
      fa.S = 1;
      fa.agg_ok = true;
      float tf = 0, tb = 0;
      for (int it = 0; it < iters + 1; ++it) {
        fa.grad = nullptr;
        ev.start();
        launch_forward_backward(fa, 0);
        float a = ev.stop();
        fa.grad = grad;
        ev.start();
        launch_forward_backward(fa, 0);
        float b = ev.stop();
        if (it) {
          tf += a;
          tb += b;
        }
      }
      printf("lr: forward %.1f us, forward+backward %.1f us\n", 1e3 * tf / iters,
             1e3 * tb / iters);
    }
  }
  return 0;
}
