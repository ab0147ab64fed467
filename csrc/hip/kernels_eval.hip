// xflow-amd: device-side evaluation metrics (gfx950).
//
// Reference: Base::calculate_auc (/root/reference/src/base/base.h:84-110) --
// rank 0 sorts every test prediction by pctr (descending) with std::sort and
// walks them once: area += (#positives ranked above) for each negative,
// logloss += y*log2(p) + (1-y)*log2(1-p).  Here the test shard's predictions
// stay in HBM:
//
//   1. stable LSD radix sort of (key = ~bits(pctr), label) pairs, 4 passes of
//      8 bits (pctr > 0, so the float bits order like the values; ~ makes it
//      descending; ties keep prediction order), each pass
//        k_rs_hist     per-tile digit histograms (LDS)
//        k_rs_scan     per-digit exclusive scan over tiles (one workgroup per digit)
//        k_rs_scatter  stable scatter: per-wave digit match (8 ballots), wave
//                      counts combined in wave order through LDS
//   2. k_auc_pos / k_auc_area  positives per tile, then for every negative the
//      positives before it -- an exact int64 area (the reference accumulates it
//      in float, exact below 2^24)
//   3. k_logloss  log2 / ln likelihood terms in prediction order, fixed-order
//      double reductions (deterministic), no sort needed.
//
// Only the final scalars travel to the host (EvalMetrics).
#include <algorithm>
#include <cstring>

#include "kernels.h"
#include "hip_util.h"

namespace xflow {
namespace hip {

constexpr int kRsBlock = 1024;
constexpr int kRsItems = 4;
constexpr int kRsTile = kRsBlock * kRsItems;  // elements per tile (workgroup)
constexpr int kRsWaves = kRsBlock / kWave;
constexpr int kRsDigits = 256;

__global__ void __launch_bounds__(kRsBlock) k_rs_hist(const u32* __restrict__ keys, int64_t n,
                                                      int shift, u32* __restrict__ ghist,
                                                      int tiles) {
  __shared__ u32 h[kRsDigits];
  for (int d = threadIdx.x; d < kRsDigits; d += kRsBlock) h[d] = 0u;
  __syncthreads();
  const int64_t base = (int64_t)blockIdx.x * kRsTile;
#pragma unroll
  for (int t = 0; t < kRsItems; ++t) {
    const int64_t e = base + (int64_t)t * kRsBlock + threadIdx.x;
    if (e < n) atomicAdd(&h[(keys[e] >> shift) & 0xFFu], 1u);
  }
  __syncthreads();
  for (int d = threadIdx.x; d < kRsDigits; d += kRsBlock)
    ghist[(size_t)d * tiles + blockIdx.x] = h[d];
}

// one workgroup per digit: exclusive scan of the tiles' counts (in place), total
__global__ void __launch_bounds__(kBlock) k_rs_scan(u32* __restrict__ ghist, int tiles,
                                                    u32* __restrict__ tot) {
  const size_t row = (size_t)blockIdx.x * tiles;
  u32 carry = 0;
  for (int c0 = 0; c0 < tiles; c0 += kBlock) {
    const int i = c0 + (int)threadIdx.x;
    const u32 v = i < tiles ? ghist[row + i] : 0u;
    u32 t;
    const u32 ex = block_exclusive_scan<kBlock>(v, &t);
    if (i < tiles) ghist[row + i] = carry + ex;
    carry += t;
  }
  if (threadIdx.x == 0) tot[blockIdx.x] = carry;
}

__global__ void __launch_bounds__(kRsBlock) k_rs_scatter(const u32* __restrict__ keys,
                                                         const u32* __restrict__ vals, int64_t n,
                                                         int shift, const u32* __restrict__ ghist,
                                                         const u32* __restrict__ tot, int tiles,
                                                         u32* __restrict__ okeys,
                                                         u32* __restrict__ ovals) {
  __shared__ u32 base[kRsDigits];     // digit start + this tile's offset in the digit
  __shared__ u32 run[kRsDigits];      // elements of the digit placed by earlier rounds
  __shared__ u32 wcnt[kRsWaves][kRsDigits];
  const int lane = lane_id(), w = threadIdx.x / kWave;
  if (threadIdx.x < kRsDigits) {
    // exclusive scan of the 256 digit totals (sequential: 256 adds)
    u32 s = 0;
    for (int d = 0; d < (int)threadIdx.x; ++d) s += tot[d];
    base[threadIdx.x] = s + ghist[(size_t)threadIdx.x * tiles + blockIdx.x];
    run[threadIdx.x] = 0u;
  }
  const int64_t tb = (int64_t)blockIdx.x * kRsTile;
  for (int t = 0; t < kRsItems; ++t) {
    for (int i = threadIdx.x; i < kRsWaves * kRsDigits; i += kRsBlock) (&wcnt[0][0])[i] = 0u;
    __syncthreads();
    const int64_t e = tb + (int64_t)t * kRsBlock + threadIdx.x;
    const bool valid = e < n;
    const u32 k = valid ? keys[e] : 0u;
    const u32 dg = (k >> shift) & 0xFFu;
    // lanes of this wave with the same digit (match over the 8 digit bits)
    unsigned long long m = __ballot(valid);
#pragma unroll
    for (int bit = 0; bit < 8; ++bit) {
      const unsigned long long b = __ballot(valid && ((dg >> bit) & 1u));
      m &= ((dg >> bit) & 1u) ? b : ~b;
    }
    const u32 rank = (u32)__popcll(m & ((1ull << lane) - 1ull));
    if (valid && rank == 0) wcnt[w][dg] = (u32)__popcll(m);
    __syncthreads();
    if (threadIdx.x < kRsDigits) {  // wave-order prefix per digit
      u32 r = run[threadIdx.x];
      for (int ww = 0; ww < kRsWaves; ++ww) {
        const u32 c = wcnt[ww][threadIdx.x];
        wcnt[ww][threadIdx.x] = r;
        r += c;
      }
      run[threadIdx.x] = r;
    }
    __syncthreads();
    if (valid) {
      const u32 pos = base[dg] + wcnt[w][dg] + rank;
      okeys[pos] = k;
      ovals[pos] = vals[e];
    }
    __syncthreads();
  }
}

__global__ void __launch_bounds__(kBlock) k_auc_keys(const float* __restrict__ pctr,
                                                     const float* __restrict__ labels, int64_t n,
                                                     u32* __restrict__ keys, u32* __restrict__ vals) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    keys[i] = ~__float_as_uint(fmaxf(pctr[i], 0.0f));  // descending pctr
    vals[i] = labels[i] > 0.5f ? 1u : 0u;
  }
}

// positives per tile of the sorted labels
__global__ void __launch_bounds__(kBlock) k_auc_pos(const u32* __restrict__ lab, int64_t n,
                                                    u32* __restrict__ bpos) {
  const int64_t base = (int64_t)blockIdx.x * kRsTile;
  u32 c = 0;
  for (int i = threadIdx.x; i < kRsTile; i += kBlock) {
    const int64_t e = base + i;
    if (e < n) c += lab[e];
  }
  u32 t;
  block_exclusive_scan<kBlock>(c, &t);
  if (threadIdx.x == 0) bpos[blockIdx.x] = t;
}

// exclusive scan of the tiles' positives (one workgroup), total in *tp
__global__ void __launch_bounds__(kBlock) k_auc_scan(u32* __restrict__ bpos, int tiles,
                                                     unsigned long long* __restrict__ tp) {
  unsigned long long carry = 0;
  for (int c0 = 0; c0 < tiles; c0 += kBlock) {
    const int i = c0 + (int)threadIdx.x;
    const u32 v = i < tiles ? bpos[i] : 0u;
    u32 t;
    const u32 ex = block_exclusive_scan<kBlock>(v, &t);
    if (i < tiles) bpos[i] = (u32)(carry + ex);
    carry += t;
  }
  if (threadIdx.x == 0) *tp = carry;
}

// per tile: sum over its negatives of the positives ranked above them (the
// tile's items in order: thread-contiguous runs of kRsItems)
__global__ void __launch_bounds__(kBlock) k_auc_area(const u32* __restrict__ lab, int64_t n,
                                                     const u32* __restrict__ bpos,
                                                     unsigned long long* __restrict__ part) {
  constexpr int kPer = kRsTile / kBlock;
  const int64_t base = (int64_t)blockIdx.x * kRsTile + (int64_t)threadIdx.x * kPer;
  u32 l[kPer];
  u32 c = 0;
#pragma unroll
  for (int j = 0; j < kPer; ++j) {
    l[j] = base + j < n ? lab[base + j] : 2u;  // 2: past the end
    c += l[j] == 1u;
  }
  u32 t;
  u32 before = bpos[blockIdx.x] + block_exclusive_scan<kBlock>(c, &t);
  unsigned long long area = 0;
#pragma unroll
  for (int j = 0; j < kPer; ++j) {
    if (l[j] == 1u) ++before;
    else if (l[j] == 0u) area += before;
  }
  __shared__ unsigned long long s[kBlock / kWave];
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) area += __shfl_xor(area, o);
  if (threadIdx.x % kWave == 0) s[threadIdx.x / kWave] = area;
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned long long a = 0;
    for (int i = 0; i < kBlock / kWave; ++i) a += s[i];
    part[blockIdx.x] = a;
  }
}

// log-likelihood terms in prediction order; per-workgroup double partials in a
// fixed order (deterministic)
constexpr int kLlGrid = 1024;

__global__ void __launch_bounds__(kBlock) k_logloss(const float* __restrict__ pctr,
                                                    const float* __restrict__ labels, int64_t n,
                                                    double* __restrict__ part) {
  double l2 = 0.0, ln = 0.0;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const float p = pctr[i];
    const int y = labels[i] > 0.5f ? 1 : 0;
    // base.h:98-99: y * log2(float p) + (1.0 - y) * log2(double 1 - p)
    l2 += (double)((float)y * log2f(p)) + (1.0 - y) * log2(1.0 - (double)p);
    const float pc = fminf(fmaxf(p, 1e-7f), 1.0f - 1e-7f);
    ln += y ? -log((double)pc) : -log(1.0 - (double)pc);
  }
  __shared__ double s2[kBlock / kWave], sl[kBlock / kWave];
  l2 = wave_sum(l2);
  ln = wave_sum(ln);
  if (threadIdx.x % kWave == 0) {
    s2[threadIdx.x / kWave] = l2;
    sl[threadIdx.x / kWave] = ln;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    double a = 0.0, b = 0.0;
    for (int i = 0; i < kBlock / kWave; ++i) {
      a += s2[i];
      b += sl[i];
    }
    part[2 * blockIdx.x] = a;
    part[2 * blockIdx.x + 1] = b;
  }
}

// fixed-order final sums: out = {area (u64), log2 sum, ln sum}
__global__ void k_eval_final(const unsigned long long* __restrict__ apart, int tiles,
                             const double* __restrict__ lpart, int lblocks,
                             unsigned long long* __restrict__ area, double* __restrict__ sums) {
  if (threadIdx.x == 0) {
    unsigned long long a = 0;
    for (int i = 0; i < tiles; ++i) a += apart[i];
    *area = a;
  } else if (threadIdx.x == 1) {
    double l2 = 0.0, ln = 0.0;
    for (int i = 0; i < lblocks; ++i) {
      l2 += lpart[2 * i];
      ln += lpart[2 * i + 1];
    }
    sums[0] = l2;
    sums[1] = ln;
  }
}

void launch_eval_metrics(const float* pctr, const float* labels, int64_t n, EvalMetrics* out,
                         hipStream_t st) {
  *out = EvalMetrics();
  out->n = n;
  if (n <= 0) return;
  if (n >= (1ll << 31)) throw std::runtime_error("eval_metrics: at most 2^31-1 predictions");
  const int tiles = (int)((n + kRsTile - 1) / kRsTile);
  const int lblocks = (int)std::min<int64_t>(kLlGrid, (n + kBlock - 1) / kBlock);
  // workspace: 2 x (keys, vals) ping-pong, digit histograms, tile partials, results
  size_t off = 0;
  auto take = [&](size_t bytes) {
    const size_t o = off;
    off += (bytes + 255) & ~(size_t)255;
    return o;
  };
  const size_t o_k0 = take(4 * (size_t)n), o_v0 = take(4 * (size_t)n), o_k1 = take(4 * (size_t)n),
               o_v1 = take(4 * (size_t)n), o_h = take(4 * (size_t)kRsDigits * tiles),
               o_tot = take(4 * kRsDigits), o_bp = take(4 * (size_t)tiles),
               o_ap = take(8 * (size_t)tiles), o_lp = take(16 * (size_t)lblocks),
               o_res = take(8 * 4);
  char* ws = nullptr;
  XF_HIP_CHECK(hipMallocAsync(reinterpret_cast<void**>(&ws), off, st));
  u32* k0 = reinterpret_cast<u32*>(ws + o_k0);
  u32* v0 = reinterpret_cast<u32*>(ws + o_v0);
  u32* k1 = reinterpret_cast<u32*>(ws + o_k1);
  u32* v1 = reinterpret_cast<u32*>(ws + o_v1);
  u32* gh = reinterpret_cast<u32*>(ws + o_h);
  u32* tot = reinterpret_cast<u32*>(ws + o_tot);
  u32* bp = reinterpret_cast<u32*>(ws + o_bp);
  auto* ap = reinterpret_cast<unsigned long long*>(ws + o_ap);
  auto* lp = reinterpret_cast<double*>(ws + o_lp);
  auto* res = reinterpret_cast<unsigned long long*>(ws + o_res);  // area, tp, sums x2
  hipLaunchKernelGGL(k_auc_keys, dim3(grid_for(n)), dim3(kBlock), 0, st, pctr, labels, n, k0, v0);
  for (int pass = 0; pass < 4; ++pass) {
    const int shift = 8 * pass;
    hipLaunchKernelGGL(k_rs_hist, dim3(tiles), dim3(kRsBlock), 0, st, k0, n, shift, gh, tiles);
    hipLaunchKernelGGL(k_rs_scan, dim3(kRsDigits), dim3(kBlock), 0, st, gh, tiles, tot);
    hipLaunchKernelGGL(k_rs_scatter, dim3(tiles), dim3(kRsBlock), 0, st, k0, v0, n, shift, gh, tot,
                       tiles, k1, v1);
    std::swap(k0, k1);
    std::swap(v0, v1);
  }
  hipLaunchKernelGGL(k_auc_pos, dim3(tiles), dim3(kBlock), 0, st, v0, n, bp);
  hipLaunchKernelGGL(k_auc_scan, dim3(1), dim3(kBlock), 0, st, bp, tiles, res + 1);
  hipLaunchKernelGGL(k_auc_area, dim3(tiles), dim3(kBlock), 0, st, v0, n, bp, ap);
  hipLaunchKernelGGL(k_logloss, dim3(lblocks), dim3(kBlock), 0, st, pctr, labels, n, lp);
  hipLaunchKernelGGL(k_eval_final, dim3(1), dim3(64), 0, st, ap, tiles, lp, lblocks, res,
                     reinterpret_cast<double*>(res + 2));
  XF_HIP_CHECK(hipGetLastError());
  unsigned long long h[4];
  XF_HIP_CHECK(hipMemcpyAsync(h, res, sizeof(h), hipMemcpyDeviceToHost, st));
  XF_HIP_CHECK(hipFreeAsync(ws, st));
  XF_HIP_CHECK(hipStreamSynchronize(st));
  out->area = h[0];
  out->tp = (int64_t)h[1];
  double d[2];
  std::memcpy(d, h + 2, sizeof(d));
  out->log2_sum = d[0];
  out->ln_sum = d[1];
}

}  // namespace hip
}  // namespace xflow
