// xflow-amd: gfx950 HIP helpers (wave64 primitives, launch sizing, errors).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <stdexcept>
#include <string>

#include "xflow/backend.h"
#include "xflow/common.h"

#define XF_HIP_CHECK(expr)                                                        \
  do {                                                                            \
    hipError_t _e = (expr);                                                       \
    if (_e != hipSuccess) {                                                       \
      throw std::runtime_error(std::string("HIP error: ") + hipGetErrorString(_e) + \
                               " at " __FILE__ ":" + std::to_string(__LINE__) +   \
                               " (" #expr ")");                                   \
    }                                                                             \
  } while (0)

// Device-side bounds asserts, compiled in only by a debug build
// (XFLOW_DEVICE_ASSERT=1 python -m xflow_amd._build): a failing check prints
// the condition and traps the wave.  GPU sanitizers are not available on the
// MI355X pool; these asserts plus AMD_SERIALIZE_KERNEL=3 localise a fault.
#if defined(XFLOW_DEVICE_ASSERT) && XFLOW_DEVICE_ASSERT
#define XF_DASSERT(cond)                                                           \
  do {                                                                             \
    if (!(cond)) {                                                                 \
      printf("xflow device assert failed: %s at %s:%d\n", #cond, __FILE__, __LINE__); \
      __builtin_trap();                                                            \
    }                                                                              \
  } while (0)
#else
#define XF_DASSERT(cond) \
  do {                   \
  } while (0)
#endif

namespace xflow {
namespace hip {

constexpr int kWave = 64;        // CDNA wavefront width
constexpr int kBlock = 256;      // 4 waves per workgroup
// Memory-bound grid cap: 256 CUs x 8 resident 256-thread blocks.
constexpr int kMaxGrid = 2048;

inline int grid_for(int64_t n, int block = kBlock, int cap = kMaxGrid) {
  if (n <= 0) return 1;
  int64_t g = (n + block - 1) / block;
  return (int)(g < cap ? g : cap);
}

// Compute units of the current device (cached per device id).
inline int device_cus() {
  static int cached[64] = {};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
  if (!cached[dev]) {
    int v = 0;
    if (hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || v <= 0)
      v = 256;
    cached[dev] = v;
  }
  return cached[dev];
}

__device__ __forceinline__ int lane_id() { return __lane_id(); }

// Wave-aggregated append: every lane with `pred` gets a unique index from one
// atomicAdd per wave on `counter`.  Lanes without pred receive -1.
template <typename T>
__device__ __forceinline__ T wave_append(T* counter, bool pred) {
  unsigned long long m = __ballot(pred);
  if (m == 0ull) return (T)-1;
  int lane = lane_id();
  int leader = __ffsll((long long)m) - 1;
  T base = 0;
  if (lane == leader) base = atomicAdd(counter, (T)__popcll(m));
  base = __shfl(base, leader);
  unsigned long long below = (lane == 0) ? 0ull : (m & ((~0ull) >> (64 - lane)));
  return pred ? base + (T)__popcll(below) : (T)-1;
}

// Workgroup barrier that waits only for this wave's LDS operations.  A
// __syncthreads() fence also drains vmcnt, i.e. every outstanding no-return
// global atomic, which turns a column loop of fire-and-forget gradient flushes
// into one L2 round trip per column.  Use only where no global memory written
// before the barrier is read by another wave after it.
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// Capacity snapshot (HostSnap): one 64-bit vector store (size, flags and
// sequence number packed) to coherent host memory by lane 0 of the first
// wave.  The apply kernels call it first: the step's pulls -- the only
// inserts -- have completed, so the size and flags are final.
__device__ __forceinline__ void store_snapshot(HostSnap* dst, const u32* mon,
                                               unsigned long long seq) {
  if (blockIdx.x != 0 || threadIdx.x != 0) return;
  const unsigned long long size = *reinterpret_cast<const unsigned long long*>(mon);
  __hip_atomic_store(&dst->word, pack_snapshot(size, mon[2], mon[3], seq), __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_SYSTEM);
}


__device__ __forceinline__ int wave_max(int v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = max(v, __shfl_xor(v, o));
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = kWave / 2; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o));
  return v;
}

// Block-wide exclusive scan of one value per lane; returns the exclusive
// prefix and writes the block total to *total.
template <int BLOCK>
__device__ __forceinline__ unsigned int block_exclusive_scan(unsigned int v, unsigned int* total) {
  __shared__ unsigned int wsum[BLOCK / kWave];
  const int lane = threadIdx.x % kWave, w = threadIdx.x / kWave;
  unsigned int incl = v;
#pragma unroll
  for (int o = 1; o < kWave; o <<= 1) {
    unsigned int t = __shfl_up(incl, o);
    if (lane >= o) incl += t;
  }
  if (lane == kWave - 1) wsum[w] = incl;
  __syncthreads();
  unsigned int off = 0, tot = 0;
#pragma unroll
  for (int i = 0; i < BLOCK / kWave; ++i) {
    off += (i < w) ? wsum[i] : 0u;
    tot += wsum[i];
  }
  __syncthreads();
  *total = tot;
  return off + incl - v;
}

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

__device__ __forceinline__ unsigned int wave_sum_u32(unsigned int v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

// Workgroup-wide sum of a per-lane count, then ONE no-return atomic by lane 0
// of wave 0.  Bookkeeping counters (table size, dedup claims) are single
// addresses: per-wave atomics on them serialise at one L2 channel.
template <int BLOCK>
__device__ __forceinline__ void block_count_add(unsigned long long* counter, unsigned int v) {
  __shared__ unsigned int part[BLOCK / kWave];
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  if (threadIdx.x % kWave == 0) part[threadIdx.x / kWave] = v;
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned int t = 0;
#pragma unroll
    for (int i = 0; i < BLOCK / kWave; ++i) t += part[i];
    if (t) atomicAdd(counter, (unsigned long long)t);
  }
}

// Deterministic gradient sums.  Float atomics add in whatever order the
// hardware serves them, so a sum's rounding changes run to run.  The LR and
// reference-FM reductions therefore accumulate fixed-point integers
// (v * 2^FX, int64 LDS atomics): integer addition is associative, so every
// partial and final sum is bitwise independent of the order.  2^36 for LR
// (|loss| <= 1: totals < 2^27 rows fit, resolution 1.5e-11) and 2^32 for FM's
// loss*vsum.  The value of a partial sum passed between kernels is the float
// of the exact integer sum, itself order independent.
template <int FX>
__device__ __forceinline__ long long fx_from(float v) {
  return (long long)__builtin_rint((double)v * (double)(1ull << FX));
}
// Largest |v| a fixed-point input may have: 2^(62-FX-16), i.e. 2^16 such
// inputs still sum inside int64 (LR: |loss| <= 1 << 2^10; FM: loss*vsum).
// Out-of-range or non-finite inputs (a diverged model) are clamped -- NaN to
// 0 -- so the conversion stays defined, and the caller flags them.
template <int FX>
__device__ __forceinline__ float fx_clamp(float v, u32& bad) {
  constexpr float kLim = (float)(1ull << (62 - FX - 16));
  if (fabsf(v) <= kLim) return v;
  bad = 1u;
  return v == v ? copysignf(kLim, v) : 0.0f;
}
template <int FX>
__device__ __forceinline__ double fx_to_double(long long a) {
  return (double)a * (1.0 / (double)(1ull << FX));
}
// Fixed point with a per-step scale (MVM's T = loss*M: a product over
// fields, no static range fits): the step's largest |input| (vmax, float
// bits, found by the forward) sets 2^fx so that 2^head inputs of that size
// still sum inside int64 -- head = log2 of the batch's rows (at least 18:
// one dup-free row contributes one input per (key, slice)), resolution
// vmax * 2^-(62 - head), i.e. float's relative precision on the largest
// values and deterministic, order-free sums.
__host__ __device__ inline int fx_head_bits(int64_t rows) {
  int h = 0;
  while (h < 62 && (1ll << h) < rows) ++h;
  return h < 18 ? 18 : h;
}
__device__ __forceinline__ int fx_scale_bits(const u32* vmax, int head) {
  int e = 0;
  const float m = vmax ? __uint_as_float(*vmax) : 0.0f;
  if (m > 0.0f && m == m && m <= 3.0e38f) frexpf(m, &e);
  const int fx = 62 - head - e;
  return fx < 0 ? 0 : (fx > 60 ? 60 : fx);
}
__device__ __forceinline__ long long fx_from_rt(float v, int fx) {
  const double d = ldexp((double)v, fx);
  // (a non-finite or out-of-range input -- a diverged step, flagged by the
  // forward -- converts to 0 instead of an undefined int64 conversion)
  return (d == d && fabs(d) < 4.6e18) ? (long long)__builtin_rint(d) : 0ll;
}
__device__ __forceinline__ double fx_to_double_rt(long long a, int fx) {
  return ldexp((double)a, -fx);
}

template <int NV>
struct FxBits {
  static constexpr int kFx = NV == 1 ? 36 : 32;
};

// Read a device-side element count, clamped to the launch's upper bound.
__device__ __forceinline__ int64_t dev_count(const int64_t* n_dev, int64_t n_host,
                                             int64_t n_max) {
  int64_t n = n_dev ? *n_dev : n_host;
  return n < n_max ? n : n_max;
}

}  // namespace hip
}  // namespace xflow
