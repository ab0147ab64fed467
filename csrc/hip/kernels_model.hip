// xflow-amd: fused forward + backward kernels for LR / FM / MVM (gfx950).
//
// One lane per row.  The pulled parameters of the batch's unique keys live in
// a dense buffer indexed by the key's dedup-scratch slot (`wpull[pos]`), so a
// row gathers its features with one dependent load each and never touches the
// persistent table.  The loss-weighted gradient contributions are added
// (un-normalised, like the reference's running sums) into `grad[pos][slice]`;
// the per-slice division by row count happens when the gradients are pushed.
//
// Reference math:
//   LR   lr_worker.cc:121-143 (loss), :100-119 (gradient)
//   FM   fm_worker.cc:159-202 (loss), :126-157 (gradient)      [kFmReference]
//   MVM  mvm_worker.cc:172-218 (loss), :137-170 (gradient)
#include <cstdio>
#include <cstdlib>
#include <type_traits>
#include "kernels.h"
#include "hip_util.h"

namespace xflow {
namespace hip {

// Diagnostic build only (-DXFLOW_KTIMING): per-phase shader-clock cycles of
// the column-walk producers (k_fm_std_red, k_lr), summed over waves (each
// wave accumulates in registers, lane 0 adds them once), printed every 25
// launches (ktime_dump).
#ifdef XFLOW_KTIMING
__device__ unsigned long long g_ktime[16];
#define XF_KT_DECL                  \
  unsigned long long kt_acc_[8] = {}; \
  unsigned long long kt_ = clock64()
#define XF_KT(p)                                  \
  do {                                            \
    const unsigned long long n_ = clock64();      \
    kt_acc_[p] += n_ - kt_;                       \
    kt_ = n_;                                     \
  } while (0)
#define XF_KT_FLUSH()                                                    \
  do {                                                                   \
    if (lane_id() == 0) {                                                \
      for (int p_ = 0; p_ < 8; ++p_) atomicAdd(&g_ktime[p_], kt_acc_[p_]); \
      atomicAdd(&g_ktime[15], 1ull);                                     \
    }                                                                    \
  } while (0)
#else
#define XF_KT_DECL (void)0
#define XF_KT(p) (void)0
#define XF_KT_FLUSH() (void)0
#endif
#ifdef XFLOW_KTIMING
static void ktime_dump(const char* what, int nphase, hipStream_t st) {
  static int calls = 0;
  if (++calls % 25) return;
  unsigned long long t[16];
  XF_HIP_CHECK(hipStreamSynchronize(st));
  XF_HIP_CHECK(hipMemcpyFromSymbol(t, HIP_SYMBOL(g_ktime), sizeof(t)));
  const double w = (double)(t[15] ? t[15] : 1);
  std::fprintf(stderr, "[ktime] %s waves %llu  cycles/wave:", what, t[15]);
  for (int p = 0; p < nphase; ++p) std::fprintf(stderr, " p%d %.0f", p, t[p] / w);
  std::fprintf(stderr, "\n");
}
#endif

// unique index of a gradient row: through the slot -> unique map, or the row
// itself when the positions already are unique indices (inv == null)
__device__ __forceinline__ u32 uix(const u32* inv, u64 x) { return inv ? inv[x] : (u32)x; }

__device__ __forceinline__ int slice_of(const BatchView& b, int64_t r, int S) {
  if (b.slice_rows <= 0) return 0;
  int64_t s = r / b.slice_rows;
  return (int)(s < S ? s : S - 1);
}

// Bucket geometry of this step's gradient reduction (FwdArgs::red_bcap):
// the smallest shift >= base that keeps ceil(dests / 2^shift) within
// kRedMaxBuckets, dests = (batch scratch capacity) * S.
constexpr int kCsrVecMinShift = 14;
struct RedGeom {
  const unsigned long long* bcap;
  u64 cap;
  int S;
  // unique-index positions (FwdArgs::red_nuq): dests = unique * S + s lie
  // below the batch's unique count times S
  const int64_t* nuq;
  int maxb;  // bucket cap (FwdArgs::red_maxb)
  int fx_head;  // scaled fixed point (MVM): fx_head_bits of the batch's rows
  // smallest bucket shift: the CSR vector reduction (k_red_csr_vec) takes
  // buckets of 2^kCsrVecMinShift dests -- fewer, fuller buckets amortise its
  // per-bucket phases, and the producer writes fewer per-bucket counts
  int min_shift;
  __device__ __forceinline__ u64 rows() const {
    return nuq ? (u64)*nuq : (bcap ? (u64)*bcap : cap);
  }
  __device__ __forceinline__ int shift(int base) const {
    const u64 dests = rows() * (u64)S;
    int sh = base;
    while (((dests + (1ull << sh) - 1) >> sh) > (u64)kRedMaxBuckets) ++sh;
    // a larger cap (vector records) only where a bucket would otherwise span
    // four or more LDS units: at two, the extra buckets' per-(bucket,
    // workgroup) counts and offsets cost more than the records' second read
    // (FM-8 std --slices 8 -1.2 %, --slices 64 +5.5 %: profiles/r4_negative_ab.txt)
    if (maxb > kRedMaxBuckets && sh - base >= 2)
      while (sh > base && ((dests + (1ull << (sh - 1)) - 1) >> (sh - 1)) <= (u64)maxb) --sh;
    return sh < min_shift ? min_shift : sh;
  }
  // buckets this step's dests reach (of the nb allocated for the full
  // capacity): producers, scans and sums skip the rest
  __device__ __forceinline__ int active(int shift, int nb) const {
    const u64 dests = rows() * (u64)S;
    const u64 n = (dests + (1ull << shift) - 1) >> shift;
    return n < (u64)nb ? (int)n : nb;
  }
};

__host__ __device__ inline RedGeom red_geom(const FwdArgs& a) {
  const int S = a.S;
  return RedGeom{a.red_bcap, a.red_cap, S, a.red_nuq, a.red_maxb > 0 ? a.red_maxb : kRedMaxBuckets,
                 fx_head_bits(a.batch.rows), a.red_csr.cnt && a.red_csr.ew > 0 ? kCsrVecMinShift : 0};
}

__device__ __forceinline__ int red_active(const FwdArgs& a, int base) {
  const RedGeom g = red_geom(a);
  return g.active(g.shift(base), a.red_nb);
}

// Per-row loss statistics, reduced per workgroup then one f64 atomic each.
struct StatAcc {
  double ln = 0, l2 = 0, rows = 0, pos = 0;
  u32 bad = 0;  // a non-finite / out-of-range prediction or gradient input (FwdArgs::fx_bad)
  __device__ void add(float p, float y) {
    bad |= !(p >= 0.0f && p <= 1.0f) ? 1u : 0u;
    float pc = fminf(fmaxf(p, 1e-7f), 1.0f - 1e-7f);
    ln += (y > 0.5f) ? -(double)logf(pc) : -(double)logf(1.0f - pc);
    l2 += (y > 0.5f) ? (double)log2f(p) : (double)log2f(1.0f - p);
    rows += 1.0;
    pos += (y > 0.5f) ? 1.0 : 0.0;
  }
};

template <int BLOCK>
__device__ void flush_stats(StatAcc a, LossStats* out, u32* bad_flag = nullptr) {
  if (bad_flag && __ballot(a.bad != 0u) && threadIdx.x % kWave == 0) atomicOr(bad_flag, 2u);
  if (!out) return;
  __shared__ double red[4][BLOCK / kWave];
  a.ln = wave_sum(a.ln);
  a.l2 = wave_sum(a.l2);
  a.rows = wave_sum(a.rows);
  a.pos = wave_sum(a.pos);
  int w = threadIdx.x / kWave, l = threadIdx.x % kWave;
  if (l == 0) {
    red[0][w] = a.ln;
    red[1][w] = a.l2;
    red[2][w] = a.rows;
    red[3][w] = a.pos;
  }
  __syncthreads();
  if (threadIdx.x < 4) {
    double s = 0;
    for (int i = 0; i < BLOCK / kWave; ++i) s += red[threadIdx.x][i];
    double* dst = threadIdx.x == 0 ? &out->ln_loss
                  : threadIdx.x == 1 ? &out->log2_lik
                  : threadIdx.x == 2 ? &out->rows
                                     : &out->positives;
    if (s != 0.0) atomicAdd(dst, s);
  }
}

// ---------------------------------------------------------------------------
// LR
// ---------------------------------------------------------------------------
// Exact per-column gradient aggregation in LDS.
//
// CTR keys are heavily skewed: in the Criteo-shaped batch the top 1000 keys
// carry ~60% of all occurrences, so per-occurrence global float atomics
// serialise on a few hot addresses.  The backward therefore walks a workgroup's
// rows column by column (occurrence j of every row = field j for fixed-width
// CTR rows and for field-ordered libffm lines): a column has at most kBlock
// occurrences, which are summed exactly in an LDS open-addressing table of
// 2*kBlock slots (load <= 0.5, never overflows), then flushed with one global
// atomic per distinct key.  Two tables alternate so one barrier per column
// suffices: column j inserts into table j&1 while the flush of table (j-1)&1
// by other waves completes before the next barrier.
constexpr u32 kColEmpty = 0xFFFFFFFFu;

// LOG2 = log2(table slots) = log2(2 * workgroup size)
template <int PS, int LOG2>
struct ColumnAgg {
  static constexpr int kSlots = 1 << LOG2;
  u32 (*tag)[kSlots];
  float (*acc)[kSlots * PS];

  __device__ __forceinline__ void init() {
    for (int i = threadIdx.x; i < kSlots; i += blockDim.x) {
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        tag[t][i] = kColEmpty;
#pragma unroll
        for (int c = 0; c < PS; ++c) acc[t][i * PS + c] = 0.0f;
      }
    }
  }
  // slot of `dest` in table t (claimed on first use); a column inserts at most
  // kSlots/2 keys, so the probe always terminates
  __device__ __forceinline__ int insert(int t, u32 dest) {
    u32 h = (dest * 0x9E3779B1u) >> (32 - LOG2);
    while (true) {  // (one CAS against an empty slot per probe step, no read first)
      const u32 old = atomicCAS(&tag[t][h], kColEmpty, dest);
      if (old == kColEmpty || old == dest) return (int)h;
      h = (h + 1) & (kSlots - 1);
    }
  }
  __device__ __forceinline__ void add(int t, int h, int c, float g) {
    atomicAdd(&acc[t][h * PS + c], g);
  }
  // one global atomic per (distinct key, non-zero component); resets the
  // table.  Consecutive lanes take consecutive components of a key's gradient
  // row, so a wave's atomics land on a few contiguous PS*4-byte segments
  // instead of 64 scattered rows.
  __device__ __forceinline__ void flush(int t, float* __restrict__ grad) {
    if constexpr (PS == 1) {
      for (int i = threadIdx.x; i < kSlots; i += blockDim.x) {
        u32 d = tag[t][i];
        if (d == kColEmpty) continue;
        float v = acc[t][i];
        if (v != 0.0f) atomicAdd(&grad[d], v);
        acc[t][i] = 0.0f;
        tag[t][i] = kColEmpty;
      }
    } else {
      for (int e = threadIdx.x; e < kSlots * PS; e += blockDim.x) {
        const int i = e / PS, c = e - i * PS;
        u32 d = tag[t][i];
        if (d == kColEmpty) continue;
        float v = acc[t][e];
        if (v != 0.0f) atomicAdd(&grad[(size_t)d * PS + c], v);
        acc[t][e] = 0.0f;
      }
      __syncthreads();  // every lane has read the tags before they are reset
      for (int i = threadIdx.x; i < kSlots; i += blockDim.x) tag[t][i] = kColEmpty;
    }
  }
};

// Column aggregation for the atomic-free LR backward (PS == 1), double
// buffered (column j uses table j & 1, one barrier per column).  Per column:
// every occurrence inserts its dest -- one CAS against kFree per probe step --
// and so claims a slot or finds it claimed; one that found it claimed adds
// its values to the slot and marks it joined; a claimer takes its record's
// index from the workgroup's running count and counts it in the LDS histogram
// of dest >> kRedShift that drives the reduction kernels below.  After the
// barrier each claimer frees its slot and writes its record -- its own
// values, plus the slot's sums if joined (then zeroed) -- so the table is
// empty again when column j + 2 reuses it.  A key alone in its column (most
// of the long-tail occurrences) costs one CAS, one flag read and one tag
// write: no accumulator traffic, no slot list.
// NV = values aggregated per key: 1 (LR: Σ loss) or 2 (reference-math FM:
// Σ loss and Σ loss*vsum, expanded to the 1+D gradient in k_red_sum).
// Records: NV == 1 -> u64 (dest | value << 32), NV == 2 -> uint3 (dest, v0, v1):
// 12 bytes, dwordx3 accesses (a quarter less traffic than padded uint4 records).
// kTabs = 1: one table, freed before the next column inserts (a second
// barrier per column) -- twice the slots in the same LDS.
template <int LOG2, int NV = 1, int kTabs = 2>
struct ListAgg {
  static constexpr int kSlots = 1 << LOG2;
  static constexpr int kShift = red_shift(NV);
  static constexpr int kFx = FxBits<NV>::kFx;
  static constexpr u32 kFree = 0xffffffffu;  // (no dest: dest < trash_pos * S)
  u32 (*tag)[kSlots];
  long long (*acc)[kSlots * NV];  // fixed-point sums (deterministic, see fx_from)
  unsigned short (*list)[kSlots / 2];  // (storage of the joined flags: kSlots bytes per table)
  u32* nlist;   // [0]: the workgroup's records so far
  u32* hist;    // [red_nb]
  u64* region;  // this workgroup's pair region
  u32 written;  // (unused: total() after the last barrier)
  int shift = kShift;  // bucket = dest >> shift (RedGeom: runtime, >= kShift)
  u32 bad = 0;   // a clamped fixed-point input (see fx_clamp), OR-ed into the stats flag
#ifdef XFLOW_KTIMING
  unsigned long long* kt_acc_ = nullptr;  // (the kernel's phase counters: 4 insert, 5 barrier, 6 flush)
  unsigned long long* kt_cur_ = nullptr;
#define XF_KTL(p)                                  \
  do {                                             \
    if (kt_acc_) {                                 \
      const unsigned long long n_ = clock64();     \
      kt_acc_[p] += n_ - *kt_cur_;                 \
      *kt_cur_ = n_;                               \
    }                                              \
  } while (0)
#else
#define XF_KTL(p) (void)0
#endif

  __device__ __forceinline__ unsigned char* joined(int t) {
    return reinterpret_cast<unsigned char*>(&list[t][0]);
  }
  __device__ __forceinline__ void init(int nb) {
    for (int i = threadIdx.x; i < kSlots; i += blockDim.x) {
#pragma unroll
      for (int tt = 0; tt < kTabs; ++tt) {
        tag[tt][i] = kFree;
        joined(tt)[i] = 0;
#pragma unroll
        for (int v = 0; v < NV; ++v) acc[tt][i * NV + v] = 0ll;
      }
    }
    for (int i = threadIdx.x; i < nb; i += blockDim.x) hist[i] = 0u;
    if (threadIdx.x == 0) nlist[0] = 0u;
    written = 0;
  }
  // records written by the workgroup (after its last column and a barrier)
  __device__ __forceinline__ u32 total() const { return nlist[0]; }
  // at most kSlots/2 keys per column in an empty table: the probe terminates
  __device__ __forceinline__ int insert(int t, u32 dest, bool& claimed) {
    u32 h = (dest * 0x9E3779B1u) >> (32 - LOG2);
    while (true) {
      const u32 old = atomicCAS(&tag[t][h], kFree, dest);
      if (old == kFree) {
        claimed = true;
        return (int)h;
      }
      if (old == dest) return (int)h;
      h = (h + 1) & (kSlots - 1);
    }
  }
  // called by every lane of the workgroup (wave-uniform control flow)
  __device__ __forceinline__ void column(int j, bool has, u32 dest, float loss,
                                         float loss2 = 0.0f) {
    const int t = kTabs == 2 ? (j & 1) : 0;
    bool claimed = false;
    int h = 0;
    long long v[NV];
    v[0] = 0ll;
    if constexpr (NV > 1) v[1] = 0ll;
    if (has) {
      h = insert(t, dest, claimed);
      v[0] = fx_from<kFx>(fx_clamp<kFx>(loss, bad));
      if constexpr (NV > 1) v[1] = fx_from<kFx>(fx_clamp<kFx>(loss2, bad));
    }
    if (has && !claimed) {
#pragma unroll
      for (int c = 0; c < NV; ++c)
        atomicAdd(reinterpret_cast<unsigned long long*>(&acc[t][h * NV + c]), (unsigned long long)v[c]);
      joined(t)[h] = 1;
    }
    const unsigned long long m = __ballot(claimed);
    u32 idx = 0;
    if (m) {
      const int lane = lane_id();
      const int leader = __ffsll((long long)m) - 1;
      u32 base = 0;
      if (lane == leader) base = atomicAdd(&nlist[0], (u32)__popcll(m));
      idx = __shfl(base, leader) + (u32)__popcll(m & ((1ull << lane) - 1ull));
    }
    if (claimed) {
      XF_DASSERT((int)(dest >> shift) < kRedMaxBuckets);
      atomicAdd(&hist[dest >> shift], 1u);
    }
    XF_KTL(4);
    lds_barrier();
    XF_KTL(5);
    if (claimed) {
      tag[t][h] = kFree;
      if (joined(t)[h]) {
        joined(t)[h] = 0;
#pragma unroll
        for (int c = 0; c < NV; ++c) {
          v[c] += acc[t][h * NV + c];
          acc[t][h * NV + c] = 0ll;
        }
      }
      const float v0 = (float)fx_to_double<kFx>(v[0]);
      if constexpr (NV == 1) {
        region[idx] = (u64)dest | ((u64)__float_as_uint(v0) << 32);
      } else {
        const float v1 = (float)fx_to_double<kFx>(v[1]);
        reinterpret_cast<uint3*>(region)[idx] =
            make_uint3(dest, __float_as_uint(v0), __float_as_uint(v1));
      }
    }
    XF_KTL(6);
    if constexpr (kTabs == 1) lds_barrier();  // (freed before the next column inserts)
  }
};

constexpr int ilog2c(int v) { return v <= 1 ? 0 : 1 + ilog2c(v / 2); }

// A row's dedup positions, column by column, kPosChunk columns per load
// batch: a chunk's loads are issued together (one memory latency per chunk)
// and the next chunk's are issued before this chunk's columns run, so the
// column walks below -- a chain of LDS round trips and barriers per column --
// never wait on a global load.  (A load issued and consumed inside the walk
// costs a full memory latency per column: the barriers' memory clobber keeps
// the compiler from hoisting it, and the records' conditional stores make its
// vmcnt wait a vmcnt(0).)  Every lane loads from a valid address (pos[0]
// outside its row) and the row bounds select trash_pos at the use.
constexpr int kPosChunk = 8;
struct PosStream {
  const u32* __restrict__ pos;
  RowSpan rs;
  int len;
  u32 trash;
  u32 cur[kPosChunk], nxt[kPosChunk];
  u32 okc = 0, okn = 0;
  __device__ __forceinline__ PosStream(const u32* p, const RowSpan& r, int n, u32 tr,
                                       bool prime = true)
      : pos(p), rs(r), len(n), trash(tr) {
    if (prime) fetch(cur, okc, 0);
  }
  __device__ __forceinline__ void fetch(u32 (&dst)[kPosChunk], u32& ok, int j0) const {
    ok = 0u;
#pragma unroll
    for (int q = 0; q < kPosChunk; ++q) {
      const bool v = j0 + q < len;
      dst[q] = pos[v ? rs.at(j0 + q) : 0];
      ok |= (u32)v << q;
    }
  }
  __device__ __forceinline__ void prefetch(int j0) { fetch(nxt, okn, j0); }
  __device__ __forceinline__ u32 get(int q) const { return (okc >> q) & 1u ? cur[q] : trash; }
  __device__ __forceinline__ void advance() {
#pragma unroll
    for (int q = 0; q < kPosChunk; ++q) cur[q] = nxt[q];
    okc = okn;
  }
};

// Rows of at most kLrRegCols features keep their dedup positions in registers:
// every pos load of a row is issued before the first use (one memory latency
// instead of one per 4 features), and the backward column walk reuses them
// instead of re-reading pos.  Longer rows take the streaming path.
constexpr int kLrRegCols = 40;

// Backward of one column: exact LDS aggregation, then the LDS-only barrier
// and the flush of the table (global atomics left in flight, or pairs).
template <int LOG2>
__device__ __forceinline__ void lr_column(ColumnAgg<1, LOG2>& agg, int j, bool has, u32 dest,
                                          float loss, float* __restrict__ grad) {
  const int t = j & 1;
  if (has) agg.add(t, agg.insert(t, dest), 0, loss);
  lds_barrier();
  agg.flush(t, grad);
}

// LR: one lane per row, the sum order is the row's feature order (bitwise
// equal to the CPU backend).  BLOCK rows per workgroup: larger workgroups
// aggregate mid-frequency keys better (Criteo-shaped batch: 4.29 M global
// atomics at 256 rows, 2.95 M at 1024 rows, for 10.2 M occurrences).
template <bool kGrad, bool kAgg, int BLOCK, bool kRed = false>
__global__ void __launch_bounds__(BLOCK) k_lr(FwdArgs a) {
  XF_KT_DECL;
  constexpr int LOG2 = ilog2c(2 * BLOCK);
  // the reduction's column tables: 4 x BLOCK slots (a column's load <= 1/4:
  // short probe chains -- the insert is a chain of dependent LDS CASes, and
  // the barrier waits for the longest); the workgroup owns its CU anyway
  constexpr int LOG2R = ilog2c(4 * BLOCK);
  constexpr int C = kLrRegCols;
  constexpr bool kCol = kAgg && !kRed;  // column tables with global atomics
  __shared__ u32 s_tag[kCol ? 2 : 1][kCol ? (1 << LOG2) : 1];
  __shared__ float s_acc[kCol ? 2 : 1][kCol ? (1 << LOG2) : 1];
  __shared__ long long s_fx[kRed ? 2 : 1][kRed ? (1 << LOG2R) : 1];
  __shared__ int s_wmax[BLOCK / kWave];
  __shared__ u32 s_tag32[kRed ? 2 : 1][kRed ? (1 << LOG2R) : 1];
  __shared__ unsigned short s_list[kRed ? 2 : 1][kRed ? (1 << LOG2R) / 2 : 1];
  __shared__ u32 s_hist[kRed ? kRedMaxBuckets : 1];
  __shared__ u32 s_nlist[3];
  const BatchView& b = a.batch;
  const u32* __restrict__ pos = a.pos;
  const float* __restrict__ wp = a.wpull;
  int64_t r = (int64_t)blockIdx.x * BLOCK + threadIdx.x;
  const bool active = r < b.rows;
  RowSpan rs;
  if (active) rs = row_span(b, r);
  const int len = rs.len;
  // (the unused aggregator of an instantiation points at a 1-element array)
  ColumnAgg<1, LOG2> agg{reinterpret_cast<u32(*)[1 << LOG2]>(&s_tag[0][0]),
                         reinterpret_cast<float(*)[1 << LOG2]>(&s_acc[0][0])};
  if constexpr (kCol) agg.init();
  ListAgg<LOG2R> lagg{reinterpret_cast<u32(*)[1 << LOG2R]>(&s_tag32[0][0]),
                      reinterpret_cast<long long(*)[1 << LOG2R]>(&s_fx[0][0]),
                      reinterpret_cast<unsigned short(*)[(1 << LOG2R) / 2]>(&s_list[0][0]),
                     s_nlist, s_hist, nullptr, 0u};
  if constexpr (kRed) {
    // the workgroup's pair region starts at its first row's first occurrence
    // (published to the other waves by the barrier below)
    const int64_t r0 = (int64_t)blockIdx.x * BLOCK;
    lagg.region = a.red_pairs + (b.row_ptr ? (int64_t)b.row_ptr[r0] : r0 * b.nnz_per_row);
    lagg.init(red_active(a, red_shift(1)));
    lagg.shift = red_geom(a).shift(red_shift(1));
#ifdef XFLOW_KTIMING
    lagg.kt_acc_ = kt_acc_;
    lagg.kt_cur_ = &kt_;
#endif
  }
  // block-uniform longest row: selects the register path and bounds the
  // backward column walk
  int maxlen;
  if (!b.row_ptr) {
    maxlen = (int)b.nnz_per_row;
    if constexpr (kAgg) __syncthreads();
  } else {
    int m = wave_max(len);
    if (threadIdx.x % kWave == 0) s_wmax[threadIdx.x / kWave] = m;
    __syncthreads();
    maxlen = 0;
#pragma unroll
    for (int w = 0; w < BLOCK / kWave; ++w) maxlen = max(maxlen, s_wmax[w]);
  }
  StatAcc st;
  float loss = 0.0f;
  const u32 s = active ? (u32)slice_of(b, r, a.S) : 0u;
  const u32 S = (u32)a.S;
  XF_KT(0);
  if (maxlen <= C) {
    u32 pv[C];
#pragma unroll
    for (int j = 0; j < C; ++j) pv[j] = j < len ? pos[rs.at(j)] : 0u;
    float wv[C];
#pragma unroll
    for (int j = 0; j < C; ++j) wv[j] = j < len ? wp[pv[j]] : 0.0f;
    if (active) {
      float wx = 0.0f;
#pragma unroll
      for (int j = 0; j < C; ++j)
        if (j < len) wx += wv[j];
      float p = sigmoid_ref(wx);
      float y = b.labels[r];
      loss = p - y;
      if (a.pctr) a.pctr[r] = p;
      st.add(p, y);
    }
    XF_KT(1);
    if constexpr (kGrad) {
      if constexpr (!kAgg) {
#pragma unroll
        for (int j = 0; j < C; ++j)
          if (j < len) atomicAdd(&a.grad[pv[j] * S + s], loss);
      } else {
#pragma unroll
        for (int j = 0; j < C; ++j) {
          if (j >= maxlen) continue;
          if constexpr (kRed) lagg.column(j, j < len && pv[j] != a.trash_pos, pv[j] * S + s, loss);
          else lr_column<LOG2>(agg, j, j < len, pv[j] * S + s, loss, a.grad);
        }
      }
    }
    XF_KT(2);
  } else {
    if (active) {
      float wx = 0.0f;
      int j = 0;
      for (; j + 4 <= len; j += 4) {
        u32 p0 = pos[rs.at(j)], p1 = pos[rs.at(j + 1)], p2 = pos[rs.at(j + 2)],
            p3 = pos[rs.at(j + 3)];
        float w0 = wp[p0], w1 = wp[p1], w2 = wp[p2], w3 = wp[p3];
        wx += w0;
        wx += w1;
        wx += w2;
        wx += w3;
      }
      for (; j < len; ++j) wx += wp[pos[rs.at(j)]];
      float p = sigmoid_ref(wx);
      float y = b.labels[r];
      loss = p - y;
      if (a.pctr) a.pctr[r] = p;
      st.add(p, y);
    }
    if constexpr (kGrad) {
      if constexpr (!kAgg) {
        for (int j = 0; j < len; ++j) atomicAdd(&a.grad[pos[rs.at(j)] * S + s], loss);
      } else {
        PosStream ps(pos, rs, len, a.trash_pos);
        for (int j0 = 0; j0 < maxlen; j0 += kPosChunk) {
          ps.prefetch(j0 + kPosChunk);
#pragma unroll
          for (int q = 0; q < kPosChunk; ++q) {
            const int j = j0 + q;
            if (j >= maxlen) break;
            const u32 pj = ps.get(q);
            const u32 dest = pj * S + s;
            if constexpr (kRed) lagg.column(j, pj != a.trash_pos, dest, loss);
            else lr_column<LOG2>(agg, j, j < len, dest, loss, a.grad);
          }
          ps.advance();
        }
      }
    }
  }
  if constexpr (kRed) {
    __syncthreads();
    if (threadIdx.x == 0) {
      a.red_count[blockIdx.x] = lagg.total();
      if (a.red_records) atomicAdd(a.red_records, (unsigned long long)lagg.total());
    }
    for (int i = threadIdx.x, n = red_active(a, red_shift(1)); i < n; i += BLOCK)
      a.red_hist[(size_t)i * gridDim.x + blockIdx.x] = s_hist[i];
  }
  st.bad |= lagg.bad;
  flush_stats<BLOCK>(st, a.stats, a.fx_bad);
  XF_KT(3);
  XF_KT_FLUSH();
}

// ---------------------------------------------------------------------------
// FM: pulled row = [w, v_0 .. v_{D-1}, pad] (pstride floats)
// ---------------------------------------------------------------------------
constexpr int fm_ps(int D) { return ((1 + D) + 3) & ~3; }
constexpr int fm_block(int D) { return fm_ps(D) <= 12 ? 256 : (fm_ps(D) <= 20 ? 128 : 64); }

// FM: one lane per row; the pulled row [w, v_0..v_{D-1}, pad] is read as
// PS/4 dwordx4 loads.  Backward: the P = 1+D gradient components of every
// occurrence are summed per (key, slice) exactly in the per-column LDS tables
// (vector accumulators), then flushed with one global atomic per non-zero
// component -- hot keys cost one atomic per workgroup instead of one per row.
template <int D, bool kGrad, bool kAgg>
__global__ void __launch_bounds__(fm_block(D)) k_fm(FwdArgs a) {
  constexpr int PS = fm_ps(D);
  constexpr int BLOCK = fm_block(D);
  constexpr int LOG2 = ilog2c(2 * BLOCK);
  __shared__ u32 s_tag[kAgg ? 2 : 1][kAgg ? (1 << LOG2) : 1];
  __shared__ float s_acc[kAgg ? 2 : 1][kAgg ? (1 << LOG2) * PS : 1];
  __shared__ int s_maxlen;
  const BatchView& b = a.batch;
  const bool standard = a.model.fm_math == kFmStandard;
  const u32* __restrict__ pos = a.pos;
  const float4* __restrict__ wp4 = reinterpret_cast<const float4*>(a.wpull);
  int64_t r = (int64_t)blockIdx.x * BLOCK + threadIdx.x;
  const bool active = r < b.rows;
  RowSpan rs;
  StatAcc st;
  float loss = 0.0f, vsum = 0.0f;
  float vs[D];
#pragma unroll
  for (int k = 0; k < D; ++k) vs[k] = 0.0f;
  if (active) {
    rs = row_span(b, r);
    float wx = 0.0f, vp = 0.0f;
    for (int j = 0; j < rs.len; ++j) {
      float w[PS];
      const float4* src = wp4 + (size_t)pos[rs.at(j)] * (PS / 4);
#pragma unroll
      for (int q = 0; q < PS / 4; ++q) {
        float4 v4 = src[q];
        w[4 * q] = v4.x;
        w[4 * q + 1] = v4.y;
        w[4 * q + 2] = v4.z;
        w[4 * q + 3] = v4.w;
      }
      wx += w[0];
#pragma unroll
      for (int k = 0; k < D; ++k) {
        vs[k] += w[1 + k];
        vp += w[1 + k] * w[1 + k];
      }
    }
    float y;
    if (standard) {
      float sq = 0.0f;
#pragma unroll
      for (int k = 0; k < D; ++k) sq += vs[k] * vs[k];
      y = wx + 0.5f * (sq - vp);
    } else {
#pragma unroll
      for (int k = 0; k < D; ++k) vsum += vs[k];
      y = wx + (vsum * vsum - vp);
    }
    float p = sigmoid_ref(y);
    float lab = b.labels[r];
    loss = p - lab;
    if (a.pctr) a.pctr[r] = p;
    st.add(p, lab);
  }
  if (kGrad) {
    const u32 s = active ? (u32)slice_of(b, r, a.S) : 0u;
    const u32 S = (u32)a.S;
    const float gw = standard ? loss : loss * (float)a.model.v_dim;  // (real D: padded dims are inert)
    auto contrib = [&](u32 p, float* c) {
      const float4* src = wp4 + (size_t)p * (PS / 4);
      float w[PS];
#pragma unroll
      for (int q = 0; q < PS / 4; ++q) {
        float4 v4 = src[q];
        w[4 * q] = v4.x;
        w[4 * q + 1] = v4.y;
        w[4 * q + 2] = v4.z;
        w[4 * q + 3] = v4.w;
      }
      c[0] = gw;
#pragma unroll
      for (int k = 0; k < D; ++k) c[1 + k] = loss * ((standard ? vs[k] : vsum) - w[1 + k]);
    };
    if constexpr (!kAgg) {
      for (int j = 0; j < rs.len; ++j) {
        const u32 p = pos[rs.at(j)];
        float c[1 + D];
        contrib(p, c);
        float* g = a.grad + ((size_t)p * S + s) * PS;
#pragma unroll
        for (int k = 0; k < 1 + D; ++k) atomicAdd(&g[k], c[k]);
      }
    } else {
      ColumnAgg<PS, LOG2> agg{s_tag, s_acc};
      if (threadIdx.x == 0) s_maxlen = 0;
      agg.init();
      __syncthreads();
      const int len = rs.len;
      if (len > 0) atomicMax(&s_maxlen, len);
      __syncthreads();
      const int maxlen = s_maxlen;
      for (int j = 0; j < maxlen; ++j) {
        const int t = j & 1;
        if (j < len) {
          const u32 p = pos[rs.at(j)];
          float c[1 + D];
          contrib(p, c);
          const int h = agg.insert(t, p * S + s);
#pragma unroll
          for (int k = 0; k < 1 + D; ++k) agg.add(t, h, k, c[k]);
        }
        __syncthreads();
        agg.flush(t, a.grad);
      }
    }
  }
  flush_stats<BLOCK>(st, a.stats, a.fx_bad);
}


// ---------------------------------------------------------------------------
// LR gradient reduction without global atomics (FwdArgs::red_*).
// Scattered float atomics execute at the memory side at ~20 G adds/s on
// gfx950 (one 4-byte add per lane, 64 rows per wave instruction), which made
// the ~3 M per-column partial sums of a Criteo-shaped batch cost ~145 us.
// Here they are partitioned by destination bucket (dest >> kRedShift) with
// plain stores and summed per bucket in a 64 KB LDS accumulator.
//   1. k_red_scan     per bucket: exclusive scan of the workgroups' counts
//   2. k_red_scatter  per producing workgroup: bucket starts (scan of the
//                     bucket totals), then its pairs to their bucket ranges
//   3. k_red_sum      per bucket: LDS sums, one plain store per non-zero dest
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(kBlock) k_red_scan(u32* __restrict__ hist, int groups,
                                                     u32* __restrict__ tot, RedGeom geom,
                                                     int base) {
  if ((int)blockIdx.x >= geom.active(geom.shift(base), (int)gridDim.x)) return;
  const size_t row = (size_t)blockIdx.x * groups;
  u32 carry = 0;
  for (int c0 = 0; c0 < groups; c0 += kBlock) {
    const int i = c0 + (int)threadIdx.x;
    const u32 v = i < groups ? hist[row + i] : 0u;
    u32 t;
    const u32 ex = block_exclusive_scan<kBlock>(v, &t);
    if (i < groups) hist[row + i] = carry + ex;
    carry += t;
  }
  if (threadIdx.x == 0) tot[blockIdx.x] = carry;
}

constexpr int kRedBlock = 1024;
constexpr int kRedUnroll = 4;

// record of one (dest, NV values) partial sum; NV >= 3: standard-FM vector
// records (dest, v_0 .. v_{NV-1}, pad) of vec_rec_words(NV) words
template <int W>
struct VecRec {
  uint4 q[W / 4];
};
template <int NV> struct VecRedRec {
  using T = VecRec<vec_rec_words(NV)>;
  __device__ static u32 dest(const T& r) { return r.q[0].x; }
};
template <int NV> struct RedRec;
template <> struct RedRec<1> {
  using T = u64;
  __device__ static u32 dest(T r) { return (u32)r; }
};
template <> struct RedRec<2> {
  using T = uint3;
  __device__ static u32 dest(T r) { return r.x; }
};

template <int NV, typename R = RedRec<NV>>
__global__ void __launch_bounds__(kRedBlock) k_red_scatter(BatchView b, int rows_per_group,
                                                           const void* __restrict__ pairs,
                                                           const u32* __restrict__ count,
                                                           const u32* __restrict__ hist,
                                                           const u32* __restrict__ tot,
                                                           u32* __restrict__ start, int nb,
                                                           void* __restrict__ sorted,
                                                           RedGeom geom) {
  using T = typename R::T;
  const int kShift = geom.shift(red_shift(NV));
  __shared__ u32 cur[kRedMaxBuckets];
  const int g = blockIdx.x, groups = gridDim.x;
  nb = geom.active(kShift, nb);
  u32 carry = 0;
  for (int c0 = 0; c0 < nb; c0 += kRedBlock) {
    const int i = c0 + (int)threadIdx.x;
    const u32 v = i < nb ? tot[i] : 0u;
    u32 t;
    const u32 ex = block_exclusive_scan<kRedBlock>(v, &t);
    if (i < nb) {
      cur[i] = carry + ex + hist[(size_t)i * groups + g];
      if (g == 0) start[i] = carry + ex;
    }
    carry += t;
  }
  if (g == 0 && threadIdx.x == 0) start[nb] = carry;
  __syncthreads();
  const int64_t r0 = (int64_t)g * rows_per_group;
  const T* src = static_cast<const T*>(pairs) +
                 (b.row_ptr ? (int64_t)b.row_ptr[r0] : r0 * b.nnz_per_row);
  T* dst = static_cast<T*>(sorted);
  const u32 n = count[g];
  // kRedUnroll independent load -> LDS rank -> store chains per lane
  for (u32 i0 = threadIdx.x; i0 < n; i0 += kRedUnroll * kRedBlock) {
    T pr[kRedUnroll];
#pragma unroll
    for (int q = 0; q < kRedUnroll; ++q) {
      const u32 i = i0 + (u32)q * kRedBlock;
      if (i < n) pr[q] = src[i];
    }
    u32 p[kRedUnroll];
#pragma unroll
    for (int q = 0; q < kRedUnroll; ++q)
      if (i0 + (u32)q * kRedBlock < n) {
        XF_DASSERT((int)(R::dest(pr[q]) >> kShift) < nb);
        p[q] = atomicAdd(&cur[R::dest(pr[q]) >> kShift], 1u);
      }
#pragma unroll
    for (int q = 0; q < kRedUnroll; ++q)
      if (i0 + (u32)q * kRedBlock < n) dst[p[q]] = pr[q];
  }
}

// Final gradient rows.  NV == 1: grad[dest] = Σ (LR).  NV == 2: reference-math
// FM (fm_worker.cc:126-157), per (key, slice) dest = slot*S + s with B = Σ loss
// and C = Σ loss*vsum: g_w = D*B, g_v[k] = Σ loss*(vsum - v_k) = C - v_k*B.
struct RedFinal {
  float* grad;
  const float* wpull;  // [slot][ps] pulled rows (NV == 2)
  int S, ps, D;
  float* out;          // NV == 1 send-order output (FwdArgs::red_out), or null
  const u32* inv;
  const int32_t* rows;
  bool compact;        // NV == 2: store (B, C) only (FwdArgs::fm_compact)
  u32* masks;          // slice-presence bits (FwdArgs::red_masks; unique order with out), or null
};

// Slice bits of one slot from the presence bitmap: its dests slot*S + s that
// fall in [lo, lo + kR).
template <u32 kR>
__device__ __forceinline__ u32 slot_bits(const u32* pbits, u64 slot, u64 S, u64 lo) {
  u32 bits = 0;
  for (u64 s = 0; s < S; ++s) {
    const u64 d = slot * S + s;
    if (d >= lo && d < lo + kR && ((pbits[(d - lo) >> 5] >> ((d - lo) & 31)) & 1u))
      bits |= 1u << s;
  }
  return bits;
}

// Slice bits of every slot whose dests slot*S + s meet the unit [lo, lo + kR),
// from the unit's presence bitmap (bit l: dest lo + l has records): one plain
// store per slot inside the unit, an atomic OR for a slot straddling its edge
// (S not dividing kR; the masks start zeroed).  masks are indexed by slot, or
// by the slot's unique index (inv != null: unique-order outputs).
template <u32 kR>
__device__ __forceinline__ void unit_masks(const u32* pbits, u64 lo, u64 S, u32* __restrict__ masks,
                                           const u32* __restrict__ inv) {
  const u64 s0 = lo / S, s1 = (lo + kR + S - 1) / S;
  for (u64 slot = s0 + threadIdx.x; slot < s1; slot += blockDim.x) {
    const u32 bits = slot_bits<kR>(pbits, slot, S, lo);
    if (!bits) continue;
    u64 m = slot;
    if (inv) {
      m = inv[slot];
      if (m == 0xFFFFFFFFu) continue;  // (the trash slot)
    }
    if (slot * S >= lo && slot * S + S <= lo + kR) masks[m] = bits;
    else atomicOr(&masks[m], bits);
  }
}

// A bucket's sums are either initialised and written densely (all kR dests)
// or per record: with the 4x-headroom dedup scratch and S slices, a bucket's
// dests are mostly untouched (S = 8 at bench shape: ~1500 records over 16384
// dests), and the dense passes cost more than the per-record phases on
// register-held records.
//
// One (bucket, sub) unit of k_red_sum: records [beg, end) of bucket b, dests
// [lo, lo + kR).  Barriers are LDS-only: a unit's global stores need not land
// before the next unit starts.
template <int NV>
__device__ __forceinline__ void red_sum_unit(u64 lo, u32 beg, u32 end,
                                             const void* __restrict__ sorted, const RedFinal& f,
                                             long long* acc, u32* pbits, u32* cbits) {
  using T = typename RedRec<NV>::T;
  constexpr int kShift = red_shift(NV);
  constexpr u32 kR = 1u << kShift;
  constexpr int kFx = FxBits<NV>::kFx;
  if (beg == end) return;
  // sparse units hold their records in registers across the three phases
  constexpr int kSp = 2 * kRedUnroll;
  const bool dense = end - beg > (u32)(kSp * kRedBlock);  // (block-uniform)
  const T* src = static_cast<const T*>(sorted);
  const u64 S = (u64)f.S;
  auto add = [&](const T& r, u32 l) {
    if (f.masks) atomicOr(&pbits[l >> 5], 1u << (l & 31));
    if constexpr (NV == 1) {
      atomicAdd(reinterpret_cast<unsigned long long*>(&acc[l]),
                (unsigned long long)fx_from<kFx>(__uint_as_float((u32)(r >> 32))));
    } else {
      atomicAdd(reinterpret_cast<unsigned long long*>(&acc[l * 2]),
                (unsigned long long)fx_from<kFx>(__uint_as_float(r.y)));
      atomicAdd(reinterpret_cast<unsigned long long*>(&acc[l * 2 + 1]),
                (unsigned long long)fx_from<kFx>(__uint_as_float(r.z)));
    }
  };
  T pr[kSp];
  u32 lr[kSp];  // (sparse) the record's local dest, kR: none
  if (dense) {
    for (u32 i = threadIdx.x; i < kR * NV; i += kRedBlock) acc[i] = 0ll;
    if (f.masks)
      for (u32 i = threadIdx.x; i < kR / 32; i += kRedBlock) pbits[i] = 0u;
    lds_barrier();
    for (u32 i0 = beg + threadIdx.x; i0 < end; i0 += kRedUnroll * kRedBlock) {
#pragma unroll
      for (int q = 0; q < kRedUnroll; ++q) {
        const u32 i = i0 + (u32)q * kRedBlock;
        if (i < end) pr[q] = src[i];
      }
#pragma unroll
      for (int q = 0; q < kRedUnroll; ++q) {
        if (i0 + (u32)q * kRedBlock >= end) continue;
        const u64 d = (u64)RedRec<NV>::dest(pr[q]), l = d - lo;
        if (l < kR) add(pr[q], (u32)l);  // (else another unit's dest)
      }
    }
  } else {
#pragma unroll
    for (int q = 0; q < kSp; ++q) {
      const u32 i = beg + threadIdx.x + (u32)q * kRedBlock;
      lr[q] = kR;
      if (i < end) {
        pr[q] = src[i];
        const u64 d = (u64)RedRec<NV>::dest(pr[q]), l = d - lo;
        if (l < kR) lr[q] = (u32)l;
      }
    }
    // zero what the records touch (same-value plain stores), and for the
    // masks every bitmap word their slots' dests cover
#pragma unroll
    for (int q = 0; q < kSp; ++q) {
      const u32 l = lr[q];
      if (l >= kR) continue;
#pragma unroll
      for (int v = 0; v < NV; ++v) acc[(u64)l * NV + v] = 0ll;
      cbits[l >> 5] = 0u;
      if (f.masks) {
        const u64 d0 = ((lo + l) / S) * S;
        const u64 a0 = d0 > lo ? d0 - lo : 0, a1 = d0 + S - 1 - lo;
        pbits[a0 >> 5] = 0u;
        if (a1 < kR) pbits[a1 >> 5] = 0u;
      }
    }
    lds_barrier();
#pragma unroll
    for (int q = 0; q < kSp; ++q)
      if (lr[q] < kR) add(pr[q], lr[q]);
  }
  lds_barrier();
  // slice bits of a slot: one plain store per slot inside [lo, lo + kR), an
  // atomic OR for a slot that straddles its edge (S not dividing kR)
  auto put_mask = [&](u64 slot, u32 bits) {
    u64 m = slot;
    if (f.out) {  // (NV == 1, S > 1) unique order
      m = uix(f.inv, slot);
      if (m == 0xFFFFFFFFu) return;
    }
    if (slot * S >= lo && slot * S + S <= lo + kR) f.masks[m] = bits;
    else atomicOr(&f.masks[m], bits);
  };
  // the sum of dest lo + l (skipped when zero: grad is zero outside this
  // step's keys -- except a present slice of the unique-order S > 1 output,
  // which the apply reads by its slice bit)
  auto emit = [&](u32 l, bool present) {
    const u64 dest = lo + l;
    if constexpr (NV == 1) {
      const long long a = acc[l];
      if (a == 0 && !(present && f.out && S > 1)) return;
      if (f.out) {
        // normalised like the gather would (lr_worker.cc:116-118, in double);
        // S > 1: [unique][slice], per-slice rows
        const u64 slot = dest / S, sl = dest - slot * S;
        const u32 o = uix(f.inv, slot);
        if (o != 0xFFFFFFFFu)  // (not the trash slot)
          f.out[(u64)o * S + sl] = (float)(fx_to_double<kFx>(a) / (double)f.rows[sl]);
      } else {
        f.grad[dest] = (float)fx_to_double<kFx>(a);
      }
    } else {
      // (a present slice of the S > 1 unique-order output is written even
      // when zero: the apply reads it by its slice bit)
      if (acc[2 * l] == 0 && acc[2 * l + 1] == 0 && !(present && f.out && S > 1)) return;
      const float B = (float)fx_to_double<kFx>(acc[2 * l]);
      const float C = (float)fx_to_double<kFx>(acc[2 * l + 1]);
      if (f.compact) {  // expanded by the apply (k_apply_group)
        if (f.out) {    // unique (send) order; S > 1: [unique][slice]
          const u64 slot = dest / S, sl = dest - slot * S;
          const u32 o0 = uix(f.inv, slot);
          if (o0 == 0xFFFFFFFFu) return;
          const u64 o = (u64)o0 * S + sl;
          if (f.rows) {  // normalised before the expansion (the send buffer, the fused step)
            const double rows = (double)f.rows[sl];  // (one rounding, as k_red_csr)
            reinterpret_cast<float2*>(f.out)[o] =
                make_float2((float)(fx_to_double<kFx>(acc[2 * l]) / rows),
                            (float)(fx_to_double<kFx>(acc[2 * l + 1]) / rows));
          } else {  // normalised by the apply
            reinterpret_cast<float2*>(f.out)[o] = make_float2(B, C);
          }
        } else {
          *reinterpret_cast<float2*>(f.grad + dest * f.ps) = make_float2(B, C);
        }
        return;
      }
      // rows are padded to 16 B: dwordx4 loads of v and stores of the row
      const float4* v4 = reinterpret_cast<const float4*>(f.wpull + (dest / S) * f.ps);
      float4* g4 = reinterpret_cast<float4*>(f.grad + dest * f.ps);
      for (int q = 0; q < f.ps / 4; ++q) {
        const float4 v = v4[q];
        float o[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int c = 4 * q + e;  // component: 0 = w, 1..D = v, above = pad
          o[e] = c == 0 ? (float)f.D * B : (c <= f.D ? C - o[e] * B : 0.0f);
        }
        g4[q] = make_float4(o[0], o[1], o[2], o[3]);
      }
    }
  };
  if (dense) {
    for (u32 l = threadIdx.x; l < kR; l += kRedBlock)
      emit(l, f.masks && ((pbits[l >> 5] >> (l & 31)) & 1u));
    if (f.masks) {
      const u64 s0 = lo / S, s1 = (lo + kR + S - 1) / S;
      for (u64 slot = s0 + threadIdx.x; slot < s1; slot += kRedBlock) {
        const u32 bits = slot_bits<kR>(pbits, slot, S, lo);
        if (bits) put_mask(slot, bits);
      }
    }
  } else {
    // one writer per dest (the record that claims its bit), and per slot the
    // writer of its lowest present dest
#pragma unroll
    for (int q = 0; q < kSp; ++q) {
      const u32 l = lr[q];
      if (l >= kR) continue;
      const u32 bit = 1u << (l & 31);
      if (atomicOr(&cbits[l >> 5], bit) & bit) continue;
      emit(l, true);
      if (f.masks) {
        const u64 slot = (lo + l) / S;
        const u32 bits = slot_bits<kR>(pbits, slot, S, lo);
        if (slot * S + (u64)__ffs(bits) - 1 == lo + l) put_mask(slot, bits);
      }
    }
  }
}

// A persistent grid (one workgroup per CU: the accumulator fills the LDS)
// walks this step's (bucket, sub) units -- a bucket of 2^shift dests is
// summed in 2^(shift - kShift) units of kR dests (one in the common case) --
// so the sparse units of a many-slice step do not each pay a workgroup
// launch; the next unit's record range is loaded during the current one.
template <int NV>
__global__ void __launch_bounds__(kRedBlock) k_red_sum(const void* __restrict__ sorted,
                                                       const u32* __restrict__ start, RedFinal f,
                                                       RedGeom geom, int nb) {
  constexpr int kShift = red_shift(NV);
  constexpr u32 kR = 1u << kShift;
  // fixed-point accumulators: the bucket's sums do not depend on record order
  __shared__ long long acc[kR * NV];
  __shared__ u32 pbits[kR / 32];  // (f.masks) dests some record reached
  __shared__ u32 cbits[kR / 32];  // (sparse) dests whose sum is being stored
  const int shift = geom.shift(kShift);
  const u32 act = (u32)geom.active(shift, nb);
  const u32 units = act << (shift - kShift);
  u32 id = blockIdx.x, nbeg = 0, nend = 0;
  if (id < units) {
    nbeg = start[id % act];
    nend = start[id % act + 1];
  }
  for (; id < units; id += gridDim.x) {
    const u32 beg = nbeg, end = nend, b = id % act, sub = id / act;
    const u32 nid = id + gridDim.x;
    if (nid < units) {
      nbeg = start[nid % act];
      nend = start[nid % act + 1];
    }
    const u64 lo = ((u64)b << shift) + ((u64)sub << kShift);
    red_sum_unit<NV>(lo, beg, end, sorted, f, acc, pbits, cbits);
    lds_barrier();  // the next unit reinitialises what this one read
  }
}

// ---------------------------------------------------------------------------
// CSR reduction (FwdArgs::red_csr): every slice of the step in one pass.
// Dests are key * 2^slog2 + slice, so a bucket's dests are whole keys and
// the bucket's distinct dests in dest order ARE its keys' entries in (key,
// slice) order.  Per bucket (one workgroup), per window of 2^16 dests:
//   1. a presence bitmap of the window's dests (one bit per dest: 8 KB) and
//      its prefix popcounts -> the rank of every present dest;
//   2. per key of the window: cnt = its present slices, off = rank of the
//      first (entries start at the bucket's first record index: a bucket
//      has at most as many distinct dests as records);
//   3. the sums: an LDS hash table keyed by dest when the window holds at
//      most kCsrHash / 2 records (the common case: a bucket's records are a
//      sparse sample of its dests), else direct-indexed sub-windows of
//      kCsrHash dests; fixed-point int64 (order-free, deterministic), each
//      distinct dest written once at its rank.
// A bucket of at most kCsrReg * kCsrBlock records keeps them in registers
// across the passes.
// ---------------------------------------------------------------------------
constexpr int kCsrBlock = 512;
constexpr int kCsrWinLog2 = 16;
constexpr int kCsrWords = 1 << (kCsrWinLog2 - 5);
constexpr int kCsrHash = 4096;
constexpr int kCsrReg = 4;

template <int NV>
__global__ void __launch_bounds__(kCsrBlock) k_red_csr(const void* __restrict__ sorted,
                                                       const u32* __restrict__ start, CsrOut c,
                                                       RedGeom geom, int nb) {
  using T = typename RedRec<NV>::T;
  constexpr int kFx = FxBits<NV>::kFx;
  constexpr int kWaves = kCsrBlock / kWave;
  __shared__ u32 bits[kCsrWords];
  __shared__ u32 wscan[kCsrWords];
  __shared__ u32 tag[kCsrHash];
  __shared__ long long acc[kCsrHash * NV];
  __shared__ u32 s_part[kWaves];
  const int shift = geom.shift(red_shift(NV));
  const int b = (int)blockIdx.x;
  if (b >= geom.active(shift, nb)) return;
  const u32 beg = start[b], end = start[b + 1];
  if (beg == end) return;  // (no records: no key of the batch has a dest here)
  const u64 nuq = *geom.nuq;
  const T* src = static_cast<const T*>(sorted);
  const u64 blo = (u64)b << shift, bhi = blo + (1ull << shift);
  const int wl2 = shift < kCsrWinLog2 ? shift : kCsrWinLog2;
  const u32 wn = 1u << wl2;
  const int sl = c.slog2;
  const u32 smask = (1u << sl) - 1u;
  const u32 nrec = end - beg;
  const int tid = (int)threadIdx.x;
  const bool reg = nrec <= (u32)(kCsrReg * kCsrBlock) && shift <= kCsrWinLog2;
  T pr[kCsrReg];
  u32 pd[kCsrReg];  // (reg) the record's dest - blo, ~0: none
#pragma unroll
  for (int q = 0; q < kCsrReg; ++q) {
    pd[q] = ~0u;
    const u32 i = beg + (u32)tid + (u32)q * kCsrBlock;
    if (reg && i < end) {
      pr[q] = src[i];
      pd[q] = (u32)((u64)RedRec<NV>::dest(pr[q]) - blo);
    }
  }
  auto rank = [&](u32 d) -> u32 {
    return wscan[d >> 5] + (u32)__popc(bits[d >> 5] & ((1u << (d & 31)) - 1u));
  };
  auto emit = [&](u32 o, u32 d, const long long* a) {
    const u32 slice = d & smask;
    const double rows = c.rows ? (double)c.rows[slice] : 1.0;
    if constexpr (NV == 1) {
      const float v = (float)(fx_to_double<kFx>(a[0]) / rows);
      static_cast<u64*>(c.ent)[o] = (u64)slice | ((u64)__float_as_uint(v) << 32);
    } else {
      const float B = (float)(fx_to_double<kFx>(a[0]) / rows);
      const float C = (float)(fx_to_double<kFx>(a[1]) / rows);
      static_cast<uint3*>(c.ent)[o] = make_uint3(slice, __float_as_uint(B), __float_as_uint(C));
    }
  };
  auto add = [&](u32 h, const T& r) {
    if constexpr (NV == 1) {
      atomicAdd(reinterpret_cast<unsigned long long*>(&acc[h]),
                (unsigned long long)fx_from<kFx>(__uint_as_float((u32)(r >> 32))));
    } else {
      atomicAdd(reinterpret_cast<unsigned long long*>(&acc[2 * h]),
                (unsigned long long)fx_from<kFx>(__uint_as_float(r.y)));
      atomicAdd(reinterpret_cast<unsigned long long*>(&acc[2 * h + 1]),
                (unsigned long long)fx_from<kFx>(__uint_as_float(r.z)));
    }
  };
  u32 out = beg;
  for (u64 wlo = blo; wlo < bhi; wlo += wn) {
    const u32 woff = (u32)(wlo - blo);
    // 1. presence bitmap of the window
    for (u32 i = (u32)tid; i < (wn >> 5); i += kCsrBlock) bits[i] = 0u;
    lds_barrier();
    u32 mine = 0;
    if (reg) {
#pragma unroll
      for (int q = 0; q < kCsrReg; ++q) {
        const u32 d = pd[q] - woff;
        if (pd[q] != ~0u && d < wn) {
          atomicOr(&bits[d >> 5], 1u << (d & 31));
          ++mine;
        }
      }
    } else {
      for (u32 i = beg + (u32)tid; i < end; i += kCsrBlock) {
        const u64 d = (u64)RedRec<NV>::dest(src[i]) - wlo;
        if (d < wn) {
          atomicOr(&bits[d >> 5], 1u << (d & 31));
          ++mine;
        }
      }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) mine += __shfl_xor(mine, o);
    if (tid % kWave == 0) s_part[tid / kWave] = mine;
    lds_barrier();
    u32 nwin = 0;
#pragma unroll
    for (int w = 0; w < kWaves; ++w) nwin += s_part[w];
    if (nwin == 0) continue;  // (block-uniform)
    // prefix popcounts: each lane scans wn / 32 / kCsrBlock consecutive words
    constexpr int kPer = kCsrWords / kCsrBlock;
    const u32 nwords = wn >> 5;
    u32 loc[kPer], tl = 0;
#pragma unroll
    for (int q = 0; q < kPer; ++q) {
      const u32 w = (u32)tid * kPer + (u32)q;
      loc[q] = w < nwords ? (u32)__popc(bits[w]) : 0u;
      tl += loc[q];
    }
    u32 total;
    u32 ex = block_exclusive_scan<kCsrBlock>(tl, &total);
#pragma unroll
    for (int q = 0; q < kPer; ++q) {
      const u32 w = (u32)tid * kPer + (u32)q;
      if (w < nwords) wscan[w] = ex;
      ex += loc[q];
    }
    lds_barrier();
    // 2. per key: entry count and first entry
    {
      const u64 k0 = wlo >> sl;
      const u32 nk = wn >> sl;
      for (u32 kk = (u32)tid; kk < nk; kk += kCsrBlock) {
        const u64 k = k0 + kk;
        if (k >= nuq) break;
        const u32 o = kk << sl;
        u32 cnt = 0, first = ~0u;
        if (sl < 5) {  // (the key's 2^sl presence bits inside one word)
          const u32 m = (bits[o >> 5] >> (o & 31)) & ((1u << (1u << sl)) - 1u);
          cnt = (u32)__popc(m);
          if (m) first = o + (u32)__ffs(m) - 1u;
        } else {
          for (u32 w = 0; w < (1u << (sl - 5)); ++w) {
            const u32 x = bits[(o >> 5) + w];
            cnt += (u32)__popc(x);
            if (x && first == ~0u) first = o + 32u * w + (u32)__ffs(x) - 1u;
          }
        }
        c.cnt[k] = cnt;
        c.off[k] = out + (cnt ? rank(first) : 0u);
      }
    }
    // 3. sums, each distinct dest written once at its rank
    if (nwin <= (u32)(kCsrHash / 2)) {
      for (u32 i = (u32)tid; i < (u32)kCsrHash; i += kCsrBlock) {
        tag[i] = ~0u;
#pragma unroll
        for (int v = 0; v < NV; ++v) acc[i * NV + v] = 0ll;
      }
      lds_barrier();
      auto insert = [&](u32 d, const T& r) {
        u32 h = (d * 0x9E3779B1u) >> (32 - ilog2c(kCsrHash));
        while (true) {  // (one CAS against an empty slot per probe step)
          const u32 old = atomicCAS(&tag[h], ~0u, d);
          if (old == ~0u || old == d) break;
          h = (h + 1) & (kCsrHash - 1);
        }
        add(h, r);
      };
      if (reg) {
#pragma unroll
        for (int q = 0; q < kCsrReg; ++q) {
          const u32 d = pd[q] - woff;
          if (pd[q] != ~0u && d < wn) insert(d, pr[q]);
        }
      } else {
        for (u32 i = beg + (u32)tid; i < end; i += kCsrBlock) {
          const T r = src[i];
          const u64 d = (u64)RedRec<NV>::dest(r) - wlo;
          if (d < wn) insert((u32)d, r);
        }
      }
      lds_barrier();
      for (u32 i = (u32)tid; i < (u32)kCsrHash; i += kCsrBlock) {
        const u32 d = tag[i];
        if (d != ~0u) emit(out + rank(d), d, &acc[i * NV]);
      }
      lds_barrier();
    } else {
      for (u32 sub = 0; sub < wn; sub += kCsrHash) {
        for (u32 i = (u32)tid; i < (u32)(kCsrHash * NV); i += kCsrBlock) acc[i] = 0ll;
        lds_barrier();
        if (reg) {
#pragma unroll
          for (int q = 0; q < kCsrReg; ++q) {
            const u32 d = pd[q] - woff - sub;
            if (pd[q] != ~0u && d < (u32)kCsrHash && pd[q] - woff < wn) add(d, pr[q]);
          }
        } else {
          for (u32 i = beg + (u32)tid; i < end; i += kCsrBlock) {
            const T r = src[i];
            const u64 d = (u64)RedRec<NV>::dest(r) - wlo - sub;
            if (d < (u64)kCsrHash) add((u32)d, r);
          }
        }
        lds_barrier();
        for (u32 l = (u32)tid; l < (u32)kCsrHash; l += kCsrBlock) {
          const u32 d = sub + l;
          if ((bits[d >> 5] >> (d & 31)) & 1u) emit(out + rank(d), d, &acc[l * NV]);
        }
        lds_barrier();
      }
    }
    out += total;
  }
}

template <int NV>
static void launch_reduction(const FwdArgs& a, int groups, int rows_per_group, hipStream_t st) {
  u32* start = a.red_tot + a.red_nb + 1;
  hipLaunchKernelGGL(k_red_scan, dim3(a.red_nb), dim3(kBlock), 0, st, a.red_hist, groups,
                     a.red_tot, red_geom(a), red_shift(NV));
  hipLaunchKernelGGL(k_red_scatter<NV>, dim3(groups), dim3(kRedBlock), 0, st, a.batch,
                     rows_per_group, static_cast<const void*>(a.red_pairs), a.red_count,
                     a.red_hist, a.red_tot, start, a.red_nb, static_cast<void*>(a.red_sorted),
                     red_geom(a));
  if (a.red_csr.cnt) {
    if (!a.red_nuq || a.red_out || a.S != (1 << a.red_csr.slog2) ||
        a.red_csr.slog2 > red_shift(NV) || (NV == 2 && !a.fm_compact))
      throw std::runtime_error("CSR reduction: unique positions, S = 2^slog2 <= 2^shift, no other outputs");
    hipLaunchKernelGGL(k_red_csr<NV>, dim3(a.red_nb), dim3(kCsrBlock), 0, st,
                       static_cast<const void*>(a.red_sorted), start, a.red_csr, red_geom(a), a.red_nb);
    return;
  }
  if (a.red_out && (NV == 2 ? !a.fm_compact : false))
    throw std::runtime_error("red_out: compact rows (reference FM)");
  if (a.red_out && a.S != 1 && !a.red_masks)
    throw std::runtime_error("red_out with several slices needs the slice bits (red_masks)");
  RedFinal f{a.grad, a.wpull, a.S, a.model.pstride(), a.model.v_dim,
             a.red_out, a.red_inv, a.red_rows, NV == 2 && a.fm_compact,
             a.S > 1 ? a.red_masks : nullptr};
  const u32 grid = std::min<u32>((u32)(a.red_nb * a.red_nsub), (u32)device_cus());
  hipLaunchKernelGGL(k_red_sum<NV>, dim3(grid), dim3(kRedBlock), 0, st,
                     static_cast<const void*>(a.red_sorted), start, f, red_geom(a), a.red_nb);
}

// Reference-math FM on the atomic-free reduction path.  The gradient of key i
// in row r is loss_r*D for w and loss_r*(vsum_r - v_ik) for v (fm_worker.cc:
// 126-157), so per (key, slice) only B = Σ loss and C = Σ loss*vsum need
// summing -- two LDS atomics per occurrence instead of 1+D -- and k_red_sum
// expands them with the pulled v: g_w = D*B, g_v[k] = C - v_k*B.
template <int D, int BLOCK>
__global__ void __launch_bounds__(BLOCK) k_fm_red(FwdArgs a) {
  constexpr int PS = fm_ps(D);
  constexpr int LOG2 = ilog2c(2 * BLOCK);
  __shared__ u32 s_tag32[2][1 << LOG2];
  __shared__ long long s_acc[2][(1 << LOG2) * 2];
  __shared__ unsigned short s_list[2][BLOCK];
  __shared__ u32 s_hist[kRedMaxBuckets];
  __shared__ u32 s_nlist[3];
  __shared__ int s_wmax[BLOCK / kWave];
  const BatchView& b = a.batch;
  const u32* __restrict__ pos = a.pos;
  const float4* __restrict__ wp4 = reinterpret_cast<const float4*>(a.wpull);
  const int64_t r = (int64_t)blockIdx.x * BLOCK + threadIdx.x;
  const bool active = r < b.rows;
  RowSpan rs;
  if (active) rs = row_span(b, r);
  const int len = rs.len;
  const int64_t r0 = (int64_t)blockIdx.x * BLOCK;
  u64* region = reinterpret_cast<u64*>(reinterpret_cast<uint3*>(a.red_pairs) +
                                       (b.row_ptr ? (int64_t)b.row_ptr[r0]
                                                  : r0 * b.nnz_per_row));
  ListAgg<LOG2, 2> lagg{s_tag32, s_acc, s_list, s_nlist, s_hist, region, 0u};
  lagg.init(red_active(a, red_shift(2)));
  lagg.shift = red_geom(a).shift(red_shift(2));
  int maxlen;
  if (!b.row_ptr) {
    maxlen = b.nnz_per_row;
    __syncthreads();
  } else {
    const int m = wave_max(len);
    if (threadIdx.x % kWave == 0) s_wmax[threadIdx.x / kWave] = m;
    __syncthreads();
    maxlen = 0;
#pragma unroll
    for (int w = 0; w < BLOCK / kWave; ++w) maxlen = max(maxlen, s_wmax[w]);
  }
  StatAcc st;
  float loss = 0.0f, vsum = 0.0f;
  if (active) {
    float vs[D];
#pragma unroll
    for (int k = 0; k < D; ++k) vs[k] = 0.0f;
    float wx = 0.0f, vp = 0.0f;
    for (int j = 0; j < len; ++j) {
      const float4* src = wp4 + (size_t)pos[rs.at(j)] * (PS / 4);
      float w[PS];
#pragma unroll
      for (int q = 0; q < PS / 4; ++q) {
        const float4 v4 = src[q];
        w[4 * q] = v4.x;
        w[4 * q + 1] = v4.y;
        w[4 * q + 2] = v4.z;
        w[4 * q + 3] = v4.w;
      }
      wx += w[0];
#pragma unroll
      for (int k = 0; k < D; ++k) {
        vs[k] += w[1 + k];
        vp += w[1 + k] * w[1 + k];
      }
    }
#pragma unroll
    for (int k = 0; k < D; ++k) vsum += vs[k];
    const float p = sigmoid_ref(wx + (vsum * vsum - vp));
    const float lab = b.labels[r];
    loss = p - lab;
    if (a.pctr) a.pctr[r] = p;
    st.add(p, lab);
  }
  const u32 s = active ? (u32)slice_of(b, r, a.S) : 0u;
  const u32 S = (u32)a.S;
  const float lv = loss * vsum;
  PosStream ps(pos, rs, len, a.trash_pos);
  for (int j0 = 0; j0 < maxlen; j0 += kPosChunk) {
    ps.prefetch(j0 + kPosChunk);
#pragma unroll
    for (int q = 0; q < kPosChunk; ++q) {
      if (j0 + q >= maxlen) break;
      const u32 pj = ps.get(q);
      lagg.column(j0 + q, pj != a.trash_pos, pj * S + s, loss, lv);
    }
    ps.advance();
  }
  __syncthreads();
  if (threadIdx.x == 0) {
      a.red_count[blockIdx.x] = lagg.total();
      if (a.red_records) atomicAdd(a.red_records, (unsigned long long)lagg.total());
    }
  for (int i = threadIdx.x, n = red_active(a, red_shift(2)); i < n; i += BLOCK)
    a.red_hist[(size_t)i * gridDim.x + blockIdx.x] = s_hist[i];
  st.bad |= lagg.bad;
  flush_stats<BLOCK>(st, a.stats, a.fx_bad);
}

// Standard-math FM (Rendle) on the atomic-free reduction.  The occurrence
// gradient has 1+D components (loss; loss*(vs_k - v_k)), all of them needed
// per key.  Each column's contributions are summed per (key, slice) in an LDS
// table with 1+D fixed-point accumulators per slot (one insert per
// occurrence; 1+D integer atomics for every occurrence after the slot's
// first; deterministic), and the flush emits one vector
// record (dest, 1+D sums) per (key, slice, column) -- 48 bytes at D = 8 --
// which k_red_scan / k_red_scatter partition by dest bucket and
// k_red_sum_vec sums into the slot-indexed gradient rows.  Before: LDS column
// tables flushed with (1+D) global float atomics per (key, column,
// workgroup), 1.15 ms of a 1.6 ms FM-8 step.
// One LDS table (flushed, then a barrier, per column): 2x the rows of a
// double-buffered table for the same LDS -- larger workgroups aggregate hot
// keys over more rows (A/B: 128 rows per workgroup -21 %, 256 -> 512 below)
// (fmstd_block: backend.h)

// kSeg (the scatter-free form, launch_fmstd_reduction): a pre-pass counts the
// workgroup's occurrences per bucket -- an upper bound of its records there --
// and the flush writes each record into its bucket's sub-range of the
// workgroup region (LDS cursor), so the region leaves the kernel already
// partitioned by bucket; the sub-range starts go to red_sorted (as u32
// [bucket][workgroup]) and k_red_sum_vec<D, true> reads a bucket's records
// straight from the producers' regions -- no k_red_scatter pass over the
// (48-byte) records.
// kSplit: the forward ran in k_fm_std_fwd (its own high-occupancy launch: this
// kernel's LDS tables leave a CU two waves per SIMD for the row gathers), which
// left (loss, loss*vs_k) per row in red_rowv -- the same floats the fused form
// computes here, so both forms sum identical fixed-point values.
// kScaled (MVM): T = loss*M spans many orders of magnitude (a product over
// fields), beyond any one static fixed-point scale: the int64 sums use the
// step's scale (fx_scale_bits of FwdArgs::red_vmax, set by the forward).

template <int D, int BLOCK, bool kSeg = false, bool kSplit = false, bool kScaled = false>
__global__ void __launch_bounds__(BLOCK) k_fm_std_red(FwdArgs a) {
  XF_KT_DECL;
  constexpr int PS = fm_ps(D);
  constexpr int NV = 1 + D;
  static_assert(BLOCK == fmstd_block(D), "producer block");
  // (not a power of two: 2.75 x BLOCK at D = 8 with int32 sums)
  constexpr u32 kSlots = (u32)(kScaled ? fmstd_slots(D) : fmstd_slots32(D));
  constexpr u32 kFree = 0xffffffffu;  // (no dest: dest < trash_pos * S)
  constexpr int kFx = FxBits<1>::kFx;
  // Column accumulators.  kScaled (MVM): int64 at the step's scale.  Else
  // int32 at a per-workgroup, per-component scale: a column adds at most one
  // value per row (BLOCK of them), each below 2^31 / BLOCK once scaled by the
  // workgroup's largest |value| of that component, so no sum overflows -- and
  // an int32 LDS atomic touches one bank where an int64 one touched two (the
  // random-slot atomics were 64 % bank-conflict cycles, profiles/r5_fmstd_pmc.txt).
  // Order-free integer sums either way: deterministic.
  using Acc = typename std::conditional<kScaled, long long, int>::type;
  // slot tags: the claiming dest, kFree once its claimer has flushed it
  __shared__ u32 s_tag[kSlots];
  __shared__ Acc s_acc[1][kSlots * NV];
  __shared__ int s_fxc[NV];
  __shared__ float s_cmax[NV][BLOCK / kWave];
  const int fxs = kScaled ? fx_scale_bits(a.red_vmax, fx_head_bits(a.batch.rows)) : kFx;
  // a slot some occurrence joined (added to) this column; its claimer flushes it
  __shared__ unsigned char s_join[kSlots];
  constexpr int kMaxB = vec_red_max_buckets(D);
  // per-bucket counts, then (kSeg) each bucket's record cursor in the region
  __shared__ u32 s_hist[kMaxB];
  __shared__ u32 s_total;
  __shared__ int s_wmax[BLOCK / kWave];
  const BatchView& b = a.batch;
  const u32* __restrict__ pos = a.pos;
  const float4* __restrict__ wp4 = reinterpret_cast<const float4*>(a.wpull);
  const int64_t r = (int64_t)blockIdx.x * BLOCK + threadIdx.x;
  const bool active = r < b.rows;
  RowSpan rs;
  if (active) rs = row_span(b, r);
  const int len = rs.len;
  const int64_t r0 = (int64_t)blockIdx.x * BLOCK;
  using Rec = typename VecRedRec<NV>::T;
  constexpr int W = vec_rec_words(NV);
  Rec* region = reinterpret_cast<Rec*>(a.red_pairs) +
                (b.row_ptr ? (int64_t)b.row_ptr[r0] : r0 * b.nnz_per_row);
  const RedGeom geom = red_geom(a);
  const int shift = geom.shift(red_shift(NV));
  for (int i = threadIdx.x; i < kSlots; i += BLOCK) {
    s_tag[i] = kFree;
    s_join[i] = 0;
#pragma unroll
    for (int c = 0; c < NV; ++c) s_acc[0][i * NV + c] = (Acc)0;
  }
  for (int i = threadIdx.x, n = geom.active(shift, a.red_nb); i < n; i += BLOCK) s_hist[i] = 0u;
  if (threadIdx.x == 0) s_total = 0u;
  int maxlen;
  if (!b.row_ptr) {
    maxlen = b.nnz_per_row;
    __syncthreads();
  } else {
    const int m = wave_max(len);
    if (threadIdx.x % kWave == 0) s_wmax[threadIdx.x / kWave] = m;
    __syncthreads();
    maxlen = 0;
#pragma unroll
    for (int w = 0; w < BLOCK / kWave; ++w) maxlen = max(maxlen, s_wmax[w]);
  }
  XF_KT(0);
  const u32 S = (u32)a.S;
  const u32 sl = active ? (u32)slice_of(b, r, a.S) : 0u;
  // kSplit: the row's vector (FM: loss, loss*vs_k; MVM: T_k = loss*M_k); a
  // one-slice MVM step emits nothing for an all-zero one (a zero contribution
  // -- every unique key is pushed anyway), several slices need every
  // occurrence (the records' presence gives the slice bits), and so does
  // standard FM: every unique key then has a record and the reduction writes
  // every unique-order row (the pull does not zero them, Engine::train_step)
  float t[PS];
  bool live = active;
  if (kSplit && active) {
    const float4* rv = reinterpret_cast<const float4*>(a.red_rowv + (size_t)r * PS);
#pragma unroll
    for (int q = 0; q < PS / 4; ++q) {
      const float4 v4 = rv[q];
      t[4 * q] = v4.x;
      t[4 * q + 1] = v4.y;
      t[4 * q + 2] = v4.z;
      t[4 * q + 3] = v4.w;
    }
    bool nz = false;
#pragma unroll
    for (int c = 0; c < NV; ++c) nz |= t[c] != 0.0f;
    live = nz || S > 1u || !kScaled;
  }
  constexpr int kPer = kMaxB / BLOCK;
  // kSeg: this thread's buckets' sub-range starts kept for the tail (when
  // they fit a few registers; else re-read from red_sorted)
  constexpr bool kRegStart = kSeg && kPer <= 8;
  u32 sstart[kRegStart ? kPer : 1];
  if constexpr (kSeg) {
    // occurrences per bucket (s_hist, zeroed above) -> sub-range starts (the cursors)
    const PosStream pp(pos, rs, live ? len : 0, a.trash_pos, false);
    for (int j0 = 0; j0 < maxlen; j0 += kPosChunk) {
      u32 pv[kPosChunk], ok;
      pp.fetch(pv, ok, j0);
#pragma unroll
      for (int q = 0; q < kPosChunk; ++q)
        if (((ok >> q) & 1u) && pv[q] != a.trash_pos)
          atomicAdd(&s_hist[(pv[q] * S + sl) >> shift], 1u);
    }
    __syncthreads();
    const int nb = geom.active(shift, a.red_nb);
    u32 c[kPer], sum = 0;
#pragma unroll
    for (int q = 0; q < kPer; ++q) {
      const int i = (int)threadIdx.x * kPer + q;
      c[q] = i < nb ? s_hist[i] : 0u;
      sum += c[q];
    }
    u32 tot;
    u32 ex = block_exclusive_scan<BLOCK>(sum, &tot);
    u32* sub_out = reinterpret_cast<u32*>(a.red_sorted);
#pragma unroll
    for (int q = 0; q < kPer; ++q) {
      const int i = (int)threadIdx.x * kPer + q;
      if (i < nb) {
        sub_out[(size_t)i * gridDim.x + blockIdx.x] = ex;
        s_hist[i] = ex;  // now the record cursor
      }
      if constexpr (kRegStart) sstart[q] = ex;
      ex += c[q];
    }
    __syncthreads();
  }
  XF_KT(1);
  StatAcc st;
  float loss = 0.0f;
  float vs[D];  // (kSplit: loss*vs_k)
#pragma unroll
  for (int k = 0; k < D; ++k) vs[k] = 0.0f;
  if (kSplit && active) {
    loss = t[0];
#pragma unroll
    for (int k = 0; k < D; ++k) vs[k] = t[1 + k];
  } else if (active) {
    float wx = 0.0f, vp = 0.0f;
    for (int j = 0; j < len; ++j) {
      const float4* src = wp4 + (size_t)pos[rs.at(j)] * (PS / 4);
      float w[PS];
#pragma unroll
      for (int q = 0; q < PS / 4; ++q) {
        const float4 v4 = src[q];
        w[4 * q] = v4.x;
        w[4 * q + 1] = v4.y;
        w[4 * q + 2] = v4.z;
        w[4 * q + 3] = v4.w;
      }
      wx += w[0];
#pragma unroll
      for (int k = 0; k < D; ++k) {
        vs[k] += w[1 + k];
        vp += w[1 + k] * w[1 + k];
      }
    }
    float sq = 0.0f;
#pragma unroll
    for (int k = 0; k < D; ++k) sq += vs[k] * vs[k];
    const float p = sigmoid_ref(wx + 0.5f * (sq - vp));
    const float lab = b.labels[r];
    loss = p - lab;
    if (a.pctr) a.pctr[r] = p;
    st.add(p, lab);
  }
  const int lane = lane_id();
  u32 written = 0, bad = 0;
  // the column walk's positions arrive a chunk ahead (PosStream)
  PosStream ps(pos, rs, live ? len : 0, a.trash_pos);
  // the row's fixed-point values, the same for every column: converted once
  // (factorised: Σ loss*(vs_k - v_k) = C_k - v_k*B with B = Σ loss and C_k =
  // Σ loss*vs_k -- v_k is the key's pulled value, one per step -- so the
  // column walk needs no second gather of the pulled row; k_red_sum_vec
  // expands C - v*B once per dest)
  Acc rowv[NV];
  if constexpr (kScaled) {  // (kSplit: the row's vector, |.| <= the step's vmax)
    rowv[0] = fx_from_rt(loss, fxs);
#pragma unroll
    for (int k = 0; k < D; ++k) rowv[1 + k] = fx_from_rt(vs[k], fxs);
  } else {
    // per-component scale from the workgroup's largest |value| (see s_acc)
    float f[NV];
    f[0] = loss;
#pragma unroll
    for (int k = 0; k < D; ++k) f[1 + k] = kSplit ? vs[k] : loss * vs[k];
#pragma unroll
    for (int c = 0; c < NV; ++c) {
      float m = f[c] == f[c] ? fabsf(f[c]) : INFINITY;
      if (!(m <= 3.0e38f)) bad = 1u;  // non-finite: a diverged model (flagged, read as 0)
      m = wave_max(m <= 3.0e38f ? m : 0.0f);
      if (lane_id() == 0) s_cmax[c][threadIdx.x / kWave] = m;
    }
    __syncthreads();
    if (threadIdx.x < NV) {
      float m = 0.0f;
#pragma unroll
      for (int w = 0; w < BLOCK / kWave; ++w) m = fmaxf(m, s_cmax[threadIdx.x][w]);
      int e = 0;
      if (m > 0.0f) frexpf(m, &e);  // m < 2^e
      constexpr int kHead = ilog2c(BLOCK) + 1;  // (BLOCK terms, plus rounding slack)
      const int fx = 31 - kHead - e;
      s_fxc[threadIdx.x] = fx < -100 ? -100 : (fx > 100 ? 100 : fx);
    }
    __syncthreads();
#pragma unroll
    for (int c = 0; c < NV; ++c) {
      const double d = ldexp((double)f[c], s_fxc[c]);
      rowv[c] = (d == d && fabs(d) < 2.1e9) ? (int)__builtin_rint(d) : 0;
    }
  }
  // Per column: insert (claim a free slot, or find the dest's); an occurrence
  // that found its (key, slice) already claimed adds its NV values to the slot
  // and marks it joined; a claimer reserves its record's place right away.
  // After a barrier each claimer frees its slot and writes the record -- its
  // own values plus, if joined, the slot's sums (then zeroed) -- so the next
  // column starts on an empty table: the insert is one CAS against kFree per
  // probe step (no read first, no stale tags), and a key alone in its column
  // (25-35 % of the occurrences at the Criteo shape) costs one CAS, one flag
  // read and one tag write -- no accumulator traffic.
  int fxc[NV];  // (the workgroup's scales, out of LDS once)
#pragma unroll
  for (int c = 0; c < NV; ++c) fxc[c] = kScaled ? 0 : s_fxc[c];
  XF_KT(2);
  for (int j0 = 0; j0 < maxlen; j0 += kPosChunk) {
    ps.prefetch(j0 + kPosChunk);
#pragma unroll
    for (int q = 0; q < kPosChunk; ++q) {
      if (j0 + q >= maxlen) break;
      const u32 pj = ps.get(q);
      const bool has = pj != a.trash_pos;
      const u32 dest = pj * S + sl;
      bool claimed = false;
      u32 h = 0;
      if (has) {
        h = (u32)(((u64)(dest * 0x9E3779B1u) * kSlots) >> 32);
        while (true) {  // <= BLOCK keys per column in > BLOCK free slots: terminates
          const u32 old = atomicCAS(&s_tag[h], kFree, dest);
          if (old == kFree) {
            claimed = true;
            break;
          }
          if (old == dest) break;
          h = h + 1 == kSlots ? 0u : h + 1;
        }
      }
      if (has && !claimed) {
        Acc* acc = &s_acc[0][h * NV];
#pragma unroll
        for (int c = 0; c < NV; ++c) {
          if constexpr (kScaled)
            atomicAdd(reinterpret_cast<unsigned long long*>(&acc[c]), (unsigned long long)rowv[c]);
          else
            atomicAdd(&acc[c], rowv[c]);
        }
        s_join[h] = 1;
      }
      u32 idx = 0;
      if constexpr (kSeg) {  // the record's place in its bucket's sub-range
        if (claimed) idx = atomicAdd(&s_hist[dest >> shift], 1u);
      } else {  // the record's index in the workgroup region
        const unsigned long long m = __ballot(claimed);
        if (m) {
          const int leader = __ffsll((long long)m) - 1;
          u32 base = 0;
          if (lane == leader) base = atomicAdd(&s_total, (u32)__popcll(m));
          idx = __shfl(base, leader) + (u32)__popcll(m & ((1ull << lane) - 1ull));
        }
        if (claimed) atomicAdd(&s_hist[dest >> shift], 1u);
      }
      XF_KT(3);
      lds_barrier();
      XF_KT(4);
      if (claimed) {
        s_tag[h] = kFree;
        Acc* acc = &s_acc[0][h * NV];
        Acc sum[NV];
#pragma unroll
        for (int c = 0; c < NV; ++c) sum[c] = rowv[c];
        if (s_join[h]) {
          s_join[h] = 0;
#pragma unroll
          for (int c = 0; c < NV; ++c) {
            sum[c] += acc[c];
            acc[c] = (Acc)0;
          }
        }
        u32 wv[W];
        wv[0] = dest;
#pragma unroll
        for (int c = 0; c < NV; ++c)
          wv[1 + c] = __float_as_uint(kScaled ? (float)fx_to_double_rt((long long)sum[c], fxs)
                                              : (float)ldexp((double)sum[c], -fxc[c]));
#pragma unroll
        for (int c = 1 + NV; c < W; ++c) wv[c] = 0u;
        Rec rec;
#pragma unroll
        for (int u = 0; u < W / 4; ++u)
          rec.q[u] = make_uint4(wv[4 * u], wv[4 * u + 1], wv[4 * u + 2], wv[4 * u + 3]);
        region[idx] = rec;
        if constexpr (kSeg) ++written;
      }
      XF_KT(5);
      lds_barrier();  // (one table: freed before the next column inserts)
      XF_KT(6);
    }
    ps.advance();
  }
  if constexpr (kSeg) {  // (the non-kSeg count is s_total already)
    const u32 wsum = wave_sum_u32(written);
    if (lane == 0 && wsum) atomicAdd(&s_total, wsum);
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    written = s_total;
    a.red_count[blockIdx.x] = written;
    if (a.red_records) atomicAdd(a.red_records, (unsigned long long)written);
  }
  // (kSeg: the cursor ends at the bucket's start in the region + its records;
  // the starts are still in the registers of the pre-pass's bucket mapping)
  if constexpr (kRegStart) {
    const int nb = geom.active(shift, a.red_nb);
#pragma unroll
    for (int q = 0; q < kPer; ++q) {
      const int i = (int)threadIdx.x * kPer + q;
      if (i < nb) a.red_hist[(size_t)i * gridDim.x + blockIdx.x] = s_hist[i] - sstart[q];
    }
  } else {
    const u32* sub_start = reinterpret_cast<const u32*>(a.red_sorted);
    for (int i = threadIdx.x, n = geom.active(shift, a.red_nb); i < n; i += BLOCK) {
      const size_t at = (size_t)i * gridDim.x + blockIdx.x;
      a.red_hist[at] = kSeg ? s_hist[i] - sub_start[at] : s_hist[i];
    }
  }
  st.bad |= bad;
  flush_stats<BLOCK>(st, a.stats, a.fx_bad);
  XF_KT(7);
  XF_KT_FLUSH();
}

// Sums of a bucket's vector records: units of kR dests (as k_red_sum) with
// (1+D) int64 accumulators per dest in LDS; every dest a record reached gets
// its whole gradient row (pad components 0) -- the rows are the step's
// (slot, slice) gradients the apply reads.
// kSeg: no scatter pass -- bucket bk's records are the producers' sub-ranges
// (k_fm_std_red<.., true>): segment g holds hist[bk][g+1] - hist[bk][g]
// records (hist: k_red_scan's exclusive prefix over the workgroups, tot[bk]
// the total) at region(g) + subs[bk][g]; record i of the bucket is found by a
// binary search of the LDS-staged prefix.
// (kSegMaxGroups: backend.h)
struct SegSrc {
  const u32* hist;   // [nb][groups] exclusive prefix (k_red_scan)
  const u32* tot;    // [nb]
  const u32* subs;   // [nb][groups] sub-range start in the workgroup region
  BatchView b;
  int rows_per_group, groups;
};

// G: segment-table capacity (groups); 512 keeps the rank-8 form at 76 KB of
// LDS, two workgroups per CU (the per-unit phases are latency chains)
// kMvm: the records are MVM's per-row T = loss*M sums (NV = 1 + D = the MVM
// latent dim) and the final gradient is g_k += Σ T_k / (1 + v_k), none where
// v_k == 0 (mvm_worker.cc:137-170: the occurrence's field sum S is the key's
// own v in a row without repeated fields); added to the rows (a repeated-field
// row's gradients arrive there by atomics first).
template <int D, bool kSeg = false, int G = kSegMaxGroups, bool kMvm = false>
__global__ void __launch_bounds__(kRedBlock) k_red_sum_vec(const void* __restrict__ sorted,
                                                           const u32* __restrict__ start,
                                                           float* __restrict__ grad,
                                                           RedGeom geom, int nb,
                                                           float* __restrict__ out,
                                                           const u32* __restrict__ inv,
                                                           const float* __restrict__ wpull,
                                                           int S, SegSrc sg,
                                                           u32* __restrict__ masks,
                                                           const u32* __restrict__ vmax,
                                                           const u32* __restrict__ dup = nullptr) {
  constexpr int NV = 1 + D;
  constexpr int PS = fm_ps(D);
  constexpr int kShift = red_shift(NV);
  constexpr u32 kR = 1u << kShift;
  constexpr int kFx = FxBits<1>::kFx;
  constexpr int W = vec_rec_words(NV);
  using Rec = typename VecRedRec<NV>::T;
  __shared__ long long acc[kR * NV];
  // MVM: the step's fixed-point scale (k_fm_std_red kScaled)
  const int fxs = kMvm ? fx_scale_bits(vmax, geom.fx_head) : kFx;
  // MVM: no repeated-field row added to the rows this step -- they hold the
  // pull's zeros, so the epilogue stores without reading them
  const bool rows_zero = kMvm && dup && *dup == 0u;
  __shared__ u32 seen[kR / 32];
  __shared__ u32 s_pre[kSeg ? G : 1];
  __shared__ u32 s_seg[kSeg ? G : 1];
  const Rec* src = static_cast<const Rec*>(sorted);
  const int shift = geom.shift(kShift);
  const u32 act = (u32)geom.active(shift, nb);
  // A workgroup takes whole buckets: a bucket wider than a unit (several
  // slices' dests) is summed unit after unit by the same workgroup, so its
  // segment table is staged once (per unit, the staging -- two loads per
  // producer workgroup -- cost more than the records at 32 slices)
  const u32 nsubs = 1u << (shift - kShift);
  for (u32 bk = blockIdx.x; bk < act; bk += gridDim.x) {
    u32 beg, end;
    if constexpr (kSeg) {
      beg = 0;
      end = sg.tot[bk];
    } else {
      beg = start[bk];
      end = start[bk + 1];
    }
    if (beg == end) continue;  // (block-uniform)
    if constexpr (kSeg) {
      // segment g: records [s_pre[g], s_pre[g+1]) of the bucket, at s_seg[g] + i
      const size_t row0 = (size_t)bk * sg.groups;
      for (int g = threadIdx.x; g < sg.groups; g += kRedBlock) {
        const int64_t r0 = (int64_t)g * sg.rows_per_group;
        const u32 base = (u32)(sg.b.row_ptr ? sg.b.row_ptr[r0] : r0 * sg.b.nnz_per_row);
        const u32 p = sg.hist[row0 + g];
        s_pre[g] = p;
        s_seg[g] = base + sg.subs[row0 + g] - p;
      }
    }
  for (u32 sub = 0; sub < nsubs; ++sub) {
    const u64 lo = ((u64)bk << shift) + ((u64)sub << kShift);
    for (u32 i = threadIdx.x; i < kR * NV; i += kRedBlock) acc[i] = 0ll;
    for (u32 i = threadIdx.x; i < kR / 32; i += kRedBlock) seen[i] = 0u;
    lds_barrier();
    for (u32 i = beg + threadIdx.x; i < end; i += kRedBlock) {
      u32 ri = i;
      if constexpr (kSeg) {
        int l0 = 0, l1 = sg.groups;  // first g with s_pre[g] > i
        while (l0 < l1) {
          const int m = (l0 + l1) >> 1;
          if (s_pre[m] <= i) l0 = m + 1;
          else l1 = m;
        }
        ri = s_seg[l0 - 1] + i;
      }
      const Rec r = src[ri];
      const u64 l = (u64)r.q[0].x - lo;
      if (l >= kR) continue;  // (another sub-unit's dest)
      u32 wv[W];
#pragma unroll
      for (int q = 0; q < W / 4; ++q) {
        wv[4 * q] = r.q[q].x;
        wv[4 * q + 1] = r.q[q].y;
        wv[4 * q + 2] = r.q[q].z;
        wv[4 * q + 3] = r.q[q].w;
      }
      long long* ap = acc + l * NV;
#pragma unroll
      for (int c = 0; c < NV; ++c)
        atomicAdd(reinterpret_cast<unsigned long long*>(&ap[c]),
                  (unsigned long long)fx_from_rt(__uint_as_float(wv[1 + c]), fxs));
      atomicOr(&seen[l >> 5], 1u << (l & 31));
    }
    lds_barrier();
    for (u32 l = threadIdx.x; l < kR; l += kRedBlock) {
      if (!((seen[l >> 5] >> (l & 31)) & 1u)) continue;
      if constexpr (kMvm) {
        const u64 slot = (lo + l) / (u64)S;
        float* row = grad + (lo + l) * PS;
        if (out) {
          const u32 u = uix(inv, slot);
          if (u == 0xFFFFFFFFu) continue;
          row = out + ((u64)u * (u64)S + (lo + l - slot * (u64)S)) * PS;
        }
        // (whole rows as dwordx4: the pulled v, the row's earlier atomics)
        const float4* w4 = reinterpret_cast<const float4*>(wpull + slot * PS);
        float4* r4 = reinterpret_cast<float4*>(row);
        float w[PS], o[PS];
#pragma unroll
        for (int q = 0; q < PS / 4; ++q) {
          const float4 a4 = w4[q], b4 = rows_zero ? make_float4(0.f, 0.f, 0.f, 0.f) : r4[q];
          w[4 * q] = a4.x, w[4 * q + 1] = a4.y, w[4 * q + 2] = a4.z, w[4 * q + 3] = a4.w;
          o[4 * q] = b4.x, o[4 * q + 1] = b4.y, o[4 * q + 2] = b4.z, o[4 * q + 3] = b4.w;
        }
#pragma unroll
        for (int c = 0; c < NV; ++c) {
          const long long t = acc[l * NV + c];
          if (t != 0 && w[c] != 0.0f) o[c] += (float)(fx_to_double_rt(t, fxs) / (1.0 + (double)w[c]));
        }
#pragma unroll
        for (int q = 0; q < PS / 4; ++q) r4[q] = make_float4(o[4 * q], o[4 * q + 1], o[4 * q + 2], o[4 * q + 3]);
        continue;
      }
      // (B, C_0..C_{D-1}) -> g_w = B, g_v[k] = C_k - v_k*B (k_fm_std_red)
      const double B = fx_to_double_rt(acc[l * NV], fxs);
      const float4* v4 = reinterpret_cast<const float4*>(wpull + ((lo + l) / (u64)S) * PS);
      float o[PS];
#pragma unroll
      for (int q = 0; q < PS / 4; ++q) {
        const float4 v = v4[q];
        o[4 * q] = v.x;
        o[4 * q + 1] = v.y;
        o[4 * q + 2] = v.z;
        o[4 * q + 3] = v.w;
      }
      o[0] = (float)B;
#pragma unroll
      for (int c = 1; c < PS; ++c)
        o[c] = c < NV ? (float)(fx_to_double_rt(acc[l * NV + c], fxs) - (double)o[c] * B) : 0.0f;
      float* row = grad + (lo + l) * PS;
      if (out) {  // the unique-order row (FwdArgs::red_out); S > 1: [unique][slice]
        const u64 slot = (lo + l) / (u64)S;
        const u32 u = uix(inv, slot);
        if (u == 0xFFFFFFFFu) continue;
        row = out + ((u64)u * (u64)S + (lo + l - slot * (u64)S)) * PS;
      }
      float4* g4 = reinterpret_cast<float4*>(row);
#pragma unroll
      for (int q = 0; q < PS / 4; ++q) g4[q] = make_float4(o[4 * q], o[4 * q + 1], o[4 * q + 2], o[4 * q + 3]);
    }
    // S > 1: each slot's slice bits from the records' presence (every
    // occurrence leaves a record, so a slice that touched the key is present
    // even with a zero gradient -- it still pushes, like the reference's slice)
    if (masks) unit_masks<kR>(seen, lo, (u64)S, masks, out ? inv : nullptr);
    lds_barrier();  // (the next unit reinitialises what this one read)
  }
  }
}


// One-workgroup exclusive scan of n u32 counts (n + 1 outputs, the last the
// total): the CSR entries' base of every bucket from its record total.
__global__ void __launch_bounds__(kRedBlock) k_scan_small(const u32* __restrict__ in, int nb,
                                                        u32* __restrict__ out, RedGeom geom,
                                                        int base) {
  const int n = geom.active(geom.shift(base), nb);  // (k_red_scan's buckets)
  u32 carry = 0;
  for (int c0 = 0; c0 < n; c0 += kRedBlock) {
    const int i = c0 + (int)threadIdx.x;
    const u32 v = i < n ? in[i] : 0u;
    u32 t;
    const u32 ex = block_exclusive_scan<kRedBlock>(v, &t);
    if (i < n) out[i] = carry + ex;
    carry += t;
  }
  if (threadIdx.x == 0) out[n] = carry;
}

// CSR form of the standard-FM vector reduction (several slices, dests =
// unique * 2^slog2 + slice): only the touched (key, slice) pairs become
// entries (slice, g_w, g_v_0 .. g_v_{D-1}) -- expanded with the pulled v
// (g_w = B, g_v = C - v*B, fm_worker.cc:159-202 in Rendle's form) and divided
// by the slice's rows -- in (key, slice) order, with each key's (off, cnt):
// the per-key push chains of the reference's per-slice pushes
// (fm_worker.cc:241-242) in one apply.  Per bucket and window of 2^15 dests:
// (1) a presence bitmap of the records' dests, (2) its prefix popcounts --
// the rank of a present dest is its entry index, (3) the keys' (off, cnt)
// from the bitmap, (4) the records' fixed-point sums accumulated at their
// rank (1024 ranks at a time, NV int64 each in LDS), then expanded and
// written.  Only distinct present dests take LDS, so the many-slice dest
// space (2^slog2 per key) costs one pass over the records, not one per
// 2^10-dest unit as the dense rows did.
constexpr int kCsrVecWin = 15;
// kMvm: the records are MVM's per-row T = loss*M sums (scaled fixed point,
// k_red_sum_vec<.., kMvm>) and an entry is g_k = Σ T_k / (1 + v_k), 0 where
// v_k == 0 (mvm_worker.cc:137-170); rows with a repeated field are added
// after, by the MvmDup passes (k_mdup_*).
template <int D, int G, bool kMvm = false>
__global__ void __launch_bounds__(kRedBlock) k_red_csr_vec(const void* __restrict__ recs, RedGeom geom,
                                                         int nb, SegSrc sg,
                                                         const u32* __restrict__ estart,
                                                         CsrOut co, const float* __restrict__ wpull,
                                                         const u32* __restrict__ vmax) {
  constexpr int NV = 1 + D;
  constexpr int PS = fm_ps(D);
  constexpr int kShift = red_shift(NV);
  // ranks per accumulation chunk: NV int64 each in <= 120 KB of LDS (one
  // workgroup per CU; a bucket holds ~500-1000 distinct dests, so at 1024
  // ranks one chunk -- one second pass over the records -- covers it: 512
  // at MVM-10's NV = 10 took a third pass, 332 vs 213 us for FM-8)
  constexpr u32 kR = (120 * 1024 / (8 * NV) < 2048 ? 120 * 1024 / (8 * NV) : 2048) & ~63u;
  constexpr u32 kWords = 1u << (kCsrVecWin - 5);
  static_assert(kWords == kRedBlock, "one bitmap word per thread");
  constexpr int kFx = FxBits<1>::kFx;
  using Rec = typename VecRedRec<NV>::T;
  __shared__ long long acc[kR * NV];
  __shared__ u32 bits[kWords];
  __shared__ u32 wscan[kWords];
  __shared__ u32 rdest[kR];
  __shared__ u32 s_pre[G];
  __shared__ u32 s_seg[G];
  __shared__ u32 s_tot;
  const Rec* src = static_cast<const Rec*>(recs);
  const int shift = geom.shift(kShift);
  const u32 act = (u32)geom.active(shift, nb);
  const int sl = co.slog2;
  const u32 smask = (1u << sl) - 1u;
  const int ew = co.ew, P = co.P;
  float* ent = static_cast<float*>(co.ent);
  const int tid = (int)threadIdx.x;
  const int fxs = kMvm ? fx_scale_bits(vmax, geom.fx_head) : kFx;
  for (u32 bk = blockIdx.x; bk < act; bk += gridDim.x) {
    const u32 nrec = sg.tot[bk];
    if (nrec == 0) continue;  // (block-uniform)
    const size_t row0 = (size_t)bk * sg.groups;
    for (int g = tid; g < sg.groups; g += kRedBlock) {
      const int64_t r0 = (int64_t)g * sg.rows_per_group;
      const u32 base = (u32)(sg.b.row_ptr ? sg.b.row_ptr[r0] : r0 * sg.b.nnz_per_row);
      const u32 pf = sg.hist[row0 + g];
      s_pre[g] = pf;
      s_seg[g] = base + sg.subs[row0 + g] - pf;
    }
    auto rec_at = [&](u32 i) -> const Rec& {
      int l0 = 0, l1 = sg.groups;  // first g with s_pre[g] > i
      while (l0 < l1) {
        const int m = (l0 + l1) >> 1;
        if (s_pre[m] <= i) l0 = m + 1;
        else l1 = m;
      }
      return src[s_seg[l0 - 1] + i];
    };
    u32 ebase = estart[bk];
    const u64 blo = (u64)bk << shift;
    const u64 bhi = blo + (1ull << shift);
    for (u64 lo = blo; lo < bhi; lo += 1ull << kCsrVecWin) {
      // (1) presence
      bits[tid] = 0u;
      lds_barrier();
      for (u32 i = tid; i < nrec; i += kRedBlock) {
        const u64 l = (u64)rec_at(i).q[0].x - lo;
        if (l < (1ull << kCsrVecWin)) atomicOr(&bits[l >> 5], 1u << (l & 31));
      }
      lds_barrier();
      // (2) ranks
      u32 tot;
      const u32 ex = block_exclusive_scan<kRedBlock>((u32)__popc(bits[tid]), &tot);
      wscan[tid] = ex;
      if (tid == 0) s_tot = tot;
      lds_barrier();
      const u32 ndist = s_tot;
      if (ndist == 0) continue;  // (block-uniform)
      auto rank = [&](u32 l) {
        return wscan[l >> 5] + (u32)__popc(bits[l >> 5] & ((1u << (l & 31)) - 1u));
      };
      // (3) the keys' (off, cnt): the window holds 2^(15 - slog2) keys whole
      for (u32 k = tid; k < (1u << (kCsrVecWin - sl)); k += kRedBlock) {
        const u32 l0 = k << sl;
        u32 cnt;
        if (sl >= 5) {
          cnt = 0;
          for (u32 w = l0 >> 5; w < (l0 + (1u << sl)) >> 5; ++w) cnt += (u32)__popc(bits[w]);
        } else {
          cnt = (u32)__popc((bits[l0 >> 5] >> (l0 & 31)) & ((1u << (1u << sl)) - 1u));
        }
        if (cnt) {
          const u32 u = (u32)((lo + l0) >> sl);
          co.off[u] = ebase + rank(l0);
          co.cnt[u] = cnt;
        }
      }
      // (4) sums at the ranks, kR ranks at a time
      for (u32 c0 = 0; c0 < ndist; c0 += kR) {
        for (u32 i = tid; i < kR * NV; i += kRedBlock) acc[i] = 0ll;
        lds_barrier();
        for (u32 i = tid; i < nrec; i += kRedBlock) {
          const Rec& rr = rec_at(i);
          const u64 l = (u64)rr.q[0].x - lo;
          if (l >= (1ull << kCsrVecWin)) continue;
          const u32 r = rank((u32)l) - c0;
          if (r >= kR) continue;
          const Rec r4 = rr;
          u32 wv[vec_rec_words(NV)];
#pragma unroll
          for (int q = 0; q < vec_rec_words(NV) / 4; ++q) {
            wv[4 * q] = r4.q[q].x;
            wv[4 * q + 1] = r4.q[q].y;
            wv[4 * q + 2] = r4.q[q].z;
            wv[4 * q + 3] = r4.q[q].w;
          }
          rdest[r] = wv[0];  // (every record of the rank writes the same dest)
          long long* ap = acc + r * NV;
#pragma unroll
          for (int c = 0; c < NV; ++c)
            atomicAdd(reinterpret_cast<unsigned long long*>(&ap[c]),
                      (unsigned long long)fx_from_rt(__uint_as_float(wv[1 + c]), fxs));
        }
        lds_barrier();
        const u32 nr = min(kR, ndist - c0);
        for (u32 t = tid; t < nr; t += kRedBlock) {
          const u32 d = rdest[t];
          const u32 u = d >> sl, s = d & smask;
          const double rows = co.rows ? (double)co.rows[s] : 1.0;
          const float* v = wpull + (u64)u * PS;
          float* e = ent + (u64)(ebase + c0 + t) * (u32)ew;
          e[0] = __uint_as_float(s);
          if constexpr (kMvm) {
#pragma unroll
            for (int c = 0; c < NV; ++c) {
              const long long tc = acc[t * NV + c];
              if (c < P)
                e[1 + c] = tc != 0 && v[c] != 0.0f
                               ? (float)(fx_to_double_rt(tc, fxs) / (1.0 + (double)v[c]) / rows)
                               : 0.0f;
            }
          } else {
            const double B = fx_to_double_rt(acc[t * NV], fxs);
            e[1] = (float)(B / rows);
#pragma unroll
            for (int c = 1; c < NV; ++c)
              if (c < P) e[1 + c] = (float)((fx_to_double_rt(acc[t * NV + c], fxs) - (double)v[c] * B) / rows);
          }
        }
        lds_barrier();  // (the next chunk reinitialises what this one read)
      }
      ebase += ndist;
    }
  }
}

// MVM rows with a repeated field (MvmDup): three order-free passes after the
// reduction.  (1) resolve each record's target -- CSR: its (key, slice)
// entry, found among the key's entries (every occurrence left a record, so
// it exists) -- and zero the target's accumulators and claim; (2) add the
// records' components in fixed point at the step's scale (the forward's
// largest |c|; 2^head of them fit int64); (3) the first record of a target
// adds the sums to the row / entry once (entries divided by the slice's rows,
// as the entry itself is).  Integer sums: deterministic in any order.
__global__ void __launch_bounds__(kBlock) k_mdup_prep(MvmDup m, CsrOut co, int D, int max_n) {
  const u32 n = min(*m.n, (u32)min<int64_t>(max_n, m.cap));
  const bool csr = co.cnt != nullptr;
  const int sl = co.slog2;
  const u32 smask = (1u << sl) - 1u;
  const float* ent = static_cast<const float*>(co.ent);
  for (u32 i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    float* r = m.rec + (size_t)i * m.ew;
    u32 t = __float_as_uint(r[0]);
    if (csr) {
      const u32 u = t >> sl, s = t & smask;
      const u32 o = co.off[u], c = co.cnt[u];
      u32 e = o;
      while (e < o + c && __float_as_uint(ent[(size_t)e * co.ew]) != s) ++e;
      t = e < o + c ? e : 0xFFFFFFFFu;
      r[0] = __uint_as_float(t);
    }
    if (t == 0xFFFFFFFFu || (int64_t)t >= m.cap) continue;
    for (int k = 0; k < D; ++k) m.acc[(size_t)t * D + k] = 0ll;
    m.claim[t] = 0u;
  }
}

__global__ void __launch_bounds__(kBlock) k_mdup_acc(MvmDup m, int D, int head, int max_n) {
  const u32 n = min(*m.n, (u32)min<int64_t>(max_n, m.cap));
  const int fxs = fx_scale_bits(m.vmax, head);
  for (u32 i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const float* r = m.rec + (size_t)i * m.ew;
    const u32 t = __float_as_uint(r[0]);
    if (t == 0xFFFFFFFFu || (int64_t)t >= m.cap) continue;
    for (int k = 0; k < D; ++k)
      atomicAdd(reinterpret_cast<unsigned long long*>(&m.acc[(size_t)t * D + k]),
                (unsigned long long)fx_from_rt(r[1 + k], fxs));
  }
}

__global__ void __launch_bounds__(kBlock) k_mdup_fin(MvmDup m, CsrOut co, float* __restrict__ out,
                                                     int PS, int D, int head, int max_n) {
  const u32 n = min(*m.n, (u32)min<int64_t>(max_n, m.cap));
  const int fxs = fx_scale_bits(m.vmax, head);
  const bool csr = co.cnt != nullptr;
  for (u32 i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const u32 t = __float_as_uint(m.rec[(size_t)i * m.ew]);
    if (t == 0xFFFFFFFFu || (int64_t)t >= m.cap) continue;
    if (atomicExch(&m.claim[t], 1u) != 0u) continue;  // (one adder per target)
    const long long* ac = m.acc + (size_t)t * D;
    if (csr) {
      float* e = static_cast<float*>(co.ent) + (size_t)t * co.ew;
      const u32 s = __float_as_uint(e[0]);
      const double rows = co.rows ? (double)co.rows[s] : 1.0;
      for (int k = 0; k < co.P && k + 1 < co.ew && k < D; ++k)
        e[1 + k] += (float)(fx_to_double_rt(ac[k], fxs) / rows);
    } else {
      float* row = out + (size_t)t * PS;
      for (int k = 0; k < D; ++k) row[k] += (float)fx_to_double_rt(ac[k], fxs);
    }
  }
}

// the step's record count and scale back to 0 once the passes read them (a
// step without a forward -- 0 rows -- must find them 0, whatever the parity)
__global__ void k_mdup_done(u32* n, u32* vmax) {
  *n = 0u;
  *vmax = 0u;
}

static void launch_mdup(const FwdArgs& a, int D, hipStream_t st) {
  const int64_t nmax = a.batch.nnz < a.mdup.cap ? a.batch.nnz : a.mdup.cap;
  const int g = (int)std::min<int64_t>(2048, (nmax + kBlock - 1) / kBlock + 1);
  const int head = fx_head_bits(a.batch.nnz);
  CsrOut co = a.red_csr.cnt ? a.red_csr : CsrOut();
  hipLaunchKernelGGL(k_mdup_prep, dim3(g), dim3(kBlock), 0, st, a.mdup, co, D, (int)nmax);
  hipLaunchKernelGGL(k_mdup_acc, dim3(g), dim3(kBlock), 0, st, a.mdup, D, head, (int)nmax);
  hipLaunchKernelGGL(k_mdup_fin, dim3(g), dim3(kBlock), 0, st, a.mdup, co, a.red_out,
                     D == 1 ? 1 : (D + 3) & ~3, D, head, (int)nmax);  // (mvm_ps)
  hipLaunchKernelGGL(k_mdup_done, dim3(1), dim3(1), 0, st, a.mdup.n, a.mdup.vmax);
}

// Standard-math FM forward of the split form (k_fm_std_red<.., kSplit>): one
// lane per row, the same sums in the same order as the fused kernel; writes
// (loss, loss*vs_0 .. loss*vs_{D-1}, pad) per row to red_rowv.
template <int D>
__global__ void __launch_bounds__(kBlock) k_fm_std_fwd(FwdArgs a) {
  constexpr int PS = fm_ps(D);
  const BatchView& b = a.batch;
  const u32* __restrict__ pos = a.pos;
  const float4* __restrict__ wp4 = reinterpret_cast<const float4*>(a.wpull);
  const int64_t r = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  StatAcc st;
  if (r < b.rows) {
    const RowSpan rs = row_span(b, r);
    float vs[D];
#pragma unroll
    for (int k = 0; k < D; ++k) vs[k] = 0.0f;
    float wx = 0.0f, vp = 0.0f;
    for (int j = 0; j < rs.len; ++j) {
      const float4* src = wp4 + (size_t)pos[rs.at(j)] * (PS / 4);
      float w[PS];
#pragma unroll
      for (int q = 0; q < PS / 4; ++q) {
        const float4 v4 = src[q];
        w[4 * q] = v4.x;
        w[4 * q + 1] = v4.y;
        w[4 * q + 2] = v4.z;
        w[4 * q + 3] = v4.w;
      }
      wx += w[0];
#pragma unroll
      for (int k = 0; k < D; ++k) {
        vs[k] += w[1 + k];
        vp += w[1 + k] * w[1 + k];
      }
    }
    float sq = 0.0f;
#pragma unroll
    for (int k = 0; k < D; ++k) sq += vs[k] * vs[k];
    const float p = sigmoid_ref(wx + 0.5f * (sq - vp));
    const float lab = b.labels[r];
    const float loss = p - lab;
    if (a.pctr) a.pctr[r] = p;
    st.add(p, lab);
    float o[PS];
    o[0] = loss;
#pragma unroll
    for (int c = 1; c < PS; ++c) o[c] = c <= D ? loss * vs[c - 1] : 0.0f;
    float4* t4 = reinterpret_cast<float4*>(a.red_rowv + (size_t)r * PS);
#pragma unroll
    for (int q = 0; q < PS / 4; ++q) t4[q] = make_float4(o[4 * q], o[4 * q + 1], o[4 * q + 2], o[4 * q + 3]);
  }
  flush_stats<kBlock>(st, a.stats, a.fx_bad);
}



// Vector-record reduction of NV = 1 + D sums per (key, slice): standard FM
// (rows (loss, loss*vs_k) from k_fm_std_fwd, expanded with the pulled v) or,
// kMvm, MVM (rows T_k = loss*M_k from k_mvm2<.., kRed>, divided by 1 + v_k).
template <int D, bool kMvm = false>
static void launch_vec_reduction(const FwdArgs& a, hipStream_t st) {
  constexpr int BLOCK = fmstd_block(D);
  constexpr int NV = 1 + D;
  if (kMvm && (!a.red_rowv || !a.red_vmax))
    throw std::runtime_error("MVM vector reduction needs red_rowv and red_vmax");
  const int groups = (int)((a.batch.rows + BLOCK - 1) / BLOCK);
  const RedGeom geom = red_geom(a);
  const u32 grid = std::min<u32>((u32)(a.red_nb * a.red_nsub), (u32)device_cus());
  if (a.red_out && a.S != 1 && !a.red_masks)
    throw std::runtime_error("vector-record red_out with several slices needs the slice bits");
  u32* masks = a.S > 1 ? a.red_masks : nullptr;
  // scatter-free form: the sub-range starts ([nb][groups] u32) live in red_sorted
  // (XFLOW_FMSTD_SEG=0: the dense producer region + k_red_scatter instead, an A/B switch)
  static const bool seg_on = [] {
    const char* e = std::getenv("XFLOW_FMSTD_SEG");
    return !(e && e[0] == '0');
  }();
  const bool seg = seg_on && groups <= kSegMaxGroups &&
                   (int64_t)a.red_nb * groups <= 2 * a.red_sorted_words &&
                   a.red_sorted_words * 8 / (vec_rec_words(NV) * 4) < (1ll << 32);
  if (a.red_maxb > vec_red_max_buckets(D) || (!seg && a.red_maxb > kRedMaxBuckets))
    throw std::runtime_error("vector reduction: bucket cap beyond the producer's");
  const bool split = a.red_rowv != nullptr;
  // (one slice: the rows' only other writer is k_mvm2's repeated-field atomics)
  const u32* dup = kMvm && a.S == 1 ? a.red_dup : nullptr;
  if (a.red_csr.cnt) {  // several slices as CSR entries (Engine::train_step_csr)
    if (!seg || !split || a.red_out || !a.red_nuq || a.S != (1 << a.red_csr.slog2) ||
        (kMvm && !a.mdup.rec) ||
        a.red_csr.slog2 > red_shift(NV) || a.red_csr.P > NV || a.red_csr.P < 1 ||
        a.red_csr.ew < csr_row_words(a.red_csr.P))
      throw std::runtime_error("CSR vector reduction: split scatter-free form, unique positions, "
                               "S = 2^slog2 <= 2^shift, full-row entries (MVM: dup records)");
  }
#ifdef XFLOW_KTIMING
  ktime_dump("fmstd (init prepass rowv insert bar1 flush bar2 tail)", 8, st);
#endif
  if (split && !kMvm)
    hipLaunchKernelGGL(k_fm_std_fwd<D>, dim3((int)((a.batch.rows + kBlock - 1) / kBlock)),
                       dim3(kBlock), 0, st, a);
  if (a.red_csr.cnt) {
    hipLaunchKernelGGL((k_fm_std_red<D, BLOCK, true, true, kMvm>), dim3(groups), dim3(BLOCK), 0, st, a);
    hipLaunchKernelGGL(k_red_scan, dim3(a.red_nb), dim3(kBlock), 0, st, a.red_hist, groups,
                       a.red_tot, geom, red_shift(NV));
    u32* estart = a.red_tot + a.red_nb + 1;  // (nb + 1 words: the scatter's starts, unused here)
    hipLaunchKernelGGL(k_scan_small, dim3(1), dim3(kRedBlock), 0, st, a.red_tot, a.red_nb, estart,
                       geom, red_shift(NV));
    const SegSrc sg{a.red_hist, a.red_tot, reinterpret_cast<const u32*>(a.red_sorted), a.batch,
                    BLOCK, groups};
    const u32 g2 = std::min<u32>((u32)a.red_nb, (u32)device_cus());
    if (groups <= 512)
      hipLaunchKernelGGL((k_red_csr_vec<D, 512, kMvm>), dim3(g2), dim3(kRedBlock), 0, st,
                         static_cast<const void*>(a.red_pairs), geom, a.red_nb, sg, estart,
                         a.red_csr, a.wpull, a.red_vmax);
    else
      hipLaunchKernelGGL((k_red_csr_vec<D, kSegMaxGroups, kMvm>), dim3(g2), dim3(kRedBlock), 0, st,
                         static_cast<const void*>(a.red_pairs), geom, a.red_nb, sg, estart,
                         a.red_csr, a.wpull, a.red_vmax);
    if (kMvm && a.mdup.rec) launch_mdup(a, NV, st);  // (rows with a repeated field)
    return;
  }
  if (seg) {
    if (split) hipLaunchKernelGGL((k_fm_std_red<D, BLOCK, true, true, kMvm>), dim3(groups), dim3(BLOCK), 0, st, a);
    else hipLaunchKernelGGL((k_fm_std_red<D, BLOCK, true>), dim3(groups), dim3(BLOCK), 0, st, a);
    hipLaunchKernelGGL(k_red_scan, dim3(a.red_nb), dim3(kBlock), 0, st, a.red_hist, groups,
                       a.red_tot, geom, red_shift(NV));
    const SegSrc sg{a.red_hist, a.red_tot, reinterpret_cast<const u32*>(a.red_sorted), a.batch,
                    BLOCK, groups};
    if (groups <= 512) {
      const u32 grid2 = std::min<u32>((u32)(a.red_nb * a.red_nsub), 2u * (u32)device_cus());
      hipLaunchKernelGGL((k_red_sum_vec<D, true, 512, kMvm>), dim3(grid2), dim3(kRedBlock), 0, st,
                         static_cast<const void*>(a.red_pairs), nullptr, a.grad, geom, a.red_nb,
                         a.red_out, a.red_inv, a.wpull, a.S, sg, masks, a.red_vmax, dup);
    } else {
      hipLaunchKernelGGL((k_red_sum_vec<D, true, kSegMaxGroups, kMvm>), dim3(grid), dim3(kRedBlock), 0, st,
                         static_cast<const void*>(a.red_pairs), nullptr, a.grad, geom, a.red_nb,
                         a.red_out, a.red_inv, a.wpull, a.S, sg, masks, a.red_vmax, dup);
    }
    if (kMvm && a.mdup.rec && a.red_out) launch_mdup(a, NV, st);  // (rows with a repeated field)
    return;
  }
  if (split) hipLaunchKernelGGL((k_fm_std_red<D, BLOCK, false, true, kMvm>), dim3(groups), dim3(BLOCK), 0, st, a);
  else hipLaunchKernelGGL((k_fm_std_red<D, BLOCK>), dim3(groups), dim3(BLOCK), 0, st, a);
  hipLaunchKernelGGL(k_red_scan, dim3(a.red_nb), dim3(kBlock), 0, st, a.red_hist, groups,
                     a.red_tot, geom, red_shift(NV));
  u32* start = a.red_tot + a.red_nb + 1;
  hipLaunchKernelGGL((k_red_scatter<NV, VecRedRec<NV>>), dim3(groups), dim3(kRedBlock), 0, st,
                     a.batch, BLOCK, static_cast<const void*>(a.red_pairs), a.red_count,
                     a.red_hist, a.red_tot, start, a.red_nb, static_cast<void*>(a.red_sorted),
                     geom);
  hipLaunchKernelGGL((k_red_sum_vec<D, false, kSegMaxGroups, kMvm>), dim3(grid), dim3(kRedBlock), 0, st,
                     static_cast<const void*>(a.red_sorted), start, a.grad, geom, a.red_nb,
                     a.red_out, a.red_inv, a.wpull, a.S, SegSrc{}, masks, a.red_vmax, dup);
  if (kMvm && a.mdup.rec && a.red_out) launch_mdup(a, NV, st);  // (rows with a repeated field)
}

// Reference-math FM on compact value rows (FwdArgs::fm_vals): each feature's
// pulled row is (w, Σ_k v_k, Σ_k v_k^2, 0), one dwordx4 -- the reference's
// y = Σ w + (Σ_f Σ_k v)^2 - Σ_f Σ_k v^2 (fm_worker.cc:159-202) needs nothing
// else, and its backward only Σ loss and Σ loss*vsum per key (k_fm_red).
// A third of the gather traffic of the full-row kernel, independent of D.
template <int BLOCK, bool kGrad>
__global__ void __launch_bounds__(BLOCK) k_fm_vals(FwdArgs a) {
  // one column table of 4 x BLOCK slots (load <= 1/4: short probe chains) in
  // the LDS of two alternating 2 x BLOCK ones, at one more barrier per column
  constexpr int LOG2 = ilog2c(4 * BLOCK);
  __shared__ u32 s_tag32[1][kGrad ? (1 << LOG2) : 1];
  __shared__ long long s_acc[1][kGrad ? (1 << LOG2) * 2 : 1];
  __shared__ unsigned short s_list[1][kGrad ? (1 << LOG2) / 2 : 1];
  __shared__ u32 s_hist[kGrad ? kRedMaxBuckets : 1];
  __shared__ u32 s_nlist[3];
  __shared__ int s_wmax[BLOCK / kWave];
  const BatchView& b = a.batch;
  const u32* __restrict__ pos = a.pos;
  const float4* __restrict__ wp4 = reinterpret_cast<const float4*>(a.wpull);
  const int64_t r = (int64_t)blockIdx.x * BLOCK + threadIdx.x;
  const bool active = r < b.rows;
  RowSpan rs;
  if (active) rs = row_span(b, r);
  const int len = rs.len;
  const int64_t r0 = (int64_t)blockIdx.x * BLOCK;
  ListAgg<LOG2, 2, 1> lagg{reinterpret_cast<u32(*)[1 << LOG2]>(&s_tag32[0][0]),
                           reinterpret_cast<long long(*)[(1 << LOG2) * 2]>(&s_acc[0][0]),
                           reinterpret_cast<unsigned short(*)[(1 << LOG2) / 2]>(&s_list[0][0]),
                           s_nlist, s_hist, nullptr, 0u};
  int maxlen = 0;
  if constexpr (kGrad) {
    lagg.region = reinterpret_cast<u64*>(reinterpret_cast<uint3*>(a.red_pairs) +
                                         (b.row_ptr ? (int64_t)b.row_ptr[r0] : r0 * b.nnz_per_row));
    lagg.init(red_active(a, red_shift(2)));
    lagg.shift = red_geom(a).shift(red_shift(2));
    if (!b.row_ptr) {
      maxlen = b.nnz_per_row;
      __syncthreads();
    } else {
      const int m = wave_max(len);
      if (threadIdx.x % kWave == 0) s_wmax[threadIdx.x / kWave] = m;
      __syncthreads();
#pragma unroll
      for (int w = 0; w < BLOCK / kWave; ++w) maxlen = max(maxlen, s_wmax[w]);
    }
  }
  StatAcc st;
  float loss = 0.0f, vsum = 0.0f;
  if (active) {
    float wx = 0.0f, vp = 0.0f;
    int j = 0;
    for (; j + 4 <= len; j += 4) {  // four independent row loads in flight
      float4 q[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) q[u] = wp4[pos[rs.at(j + u)]];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        wx += q[u].x;
        vsum += q[u].y;
        vp += q[u].z;
      }
    }
    for (; j < len; ++j) {
      const float4 q = wp4[pos[rs.at(j)]];
      wx += q.x;
      vsum += q.y;
      vp += q.z;
    }
    const float p = sigmoid_ref(wx + (vsum * vsum - vp));
    const float lab = b.labels[r];
    loss = p - lab;
    if (a.pctr) a.pctr[r] = p;
    st.add(p, lab);
  }
  if constexpr (kGrad) {
    const u32 s = active ? (u32)slice_of(b, r, a.S) : 0u;
    const u32 S = (u32)a.S;
    const float lv = loss * vsum;
    PosStream ps(pos, rs, len, a.trash_pos);
    for (int j0 = 0; j0 < maxlen; j0 += kPosChunk) {
      ps.prefetch(j0 + kPosChunk);
#pragma unroll
      for (int q = 0; q < kPosChunk; ++q) {
        if (j0 + q >= maxlen) break;
        const u32 pj = ps.get(q);
        lagg.column(j0 + q, pj != a.trash_pos, pj * S + s, loss, lv);
      }
      ps.advance();
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      a.red_count[blockIdx.x] = lagg.total();
      if (a.red_records) atomicAdd(a.red_records, (unsigned long long)lagg.total());
    }
    for (int i = threadIdx.x, n = red_active(a, red_shift(2)); i < n; i += BLOCK)
      a.red_hist[(size_t)i * gridDim.x + blockIdx.x] = s_hist[i];
  }
  st.bad |= lagg.bad;
  flush_stats<BLOCK>(st, a.stats, a.fx_bad);
}

// ---------------------------------------------------------------------------
// Standard-math FM forward on the matrix cores (v_mfma_f32_16x16x4_f32), the
// row-indicator form of DESIGN.md section 6: a wave owns 16 rows; for every
// (row quad m, field f) one MFMA adds, for the 4 rows of the quad, the
// field's latent row v (columns 0..D-1) and its squares (columns D..2D-1) to
// the 16 x 16 accumulator tile D[row][column]:
//   A[i][q] = (i == 4m + q)       (one-hot: 4 of the 64 A entries are 1)
//   B[q][c] = v[row 4m+q, f][c], v^2[..][c - D]
// so D[i][k] = sum_f v_ik = vs_k and D[i][D+k] = sum_f v_ik^2, exact f32 adds
// in field order (fmaf chain).  y = sum_f w + 0.5 sum_k (vs_k^2 - sum_f v^2)
// (Rendle's sum trick; fm_math = standard).  An honest A/B against the VALU
// forward (one lane per row) -- see profiles/r2_fm_mfma_ab.txt: 15/16 of each
// MFMA's work multiplies by the zero entries of A, so the matrix-core form
// needs 4*F instructions per 16 rows where the VALU form spends F*D FMAs per
// row; both are bound by the gather of the pulled rows.
// Selected for forward-only standard FM with ModelSpec::fm_mfma.
using f32x4 = __attribute__((ext_vector_type(4))) float;

template <int D>
__global__ void __launch_bounds__(256) k_fm_fwd_mfma(FwdArgs a) {
  static_assert(2 * D <= 16, "one 16-column tile: D <= 8");
  constexpr int PS = fm_ps(D);
  const BatchView& b = a.batch;
  const int lane = lane_id();
  const int q = lane >> 4, c = lane & 15;
  const int64_t r0 = ((int64_t)blockIdx.x * (blockDim.x / kWave) + threadIdx.x / kWave) * 16;
  int F = b.nnz_per_row;
  if (b.row_ptr) {  // longest row of the wave's 16
    int len = 0;
    const int64_t r = r0 + (lane & 15);
    if (lane < 16 && r < b.rows) len = (int)(b.row_ptr[r + 1] - b.row_ptr[r]);
    F = wave_max(len);
  }
  f32x4 acc = {0.0f, 0.0f, 0.0f, 0.0f};
  float wx[4] = {0.0f, 0.0f, 0.0f, 0.0f};  // lanes with c == 0: w sums of rows 4m+q
#pragma unroll
  for (int m = 0; m < 4; ++m) {
    const int64_t row = r0 + 4 * m + q;
    RowSpan rs;
    if (row < b.rows) rs = row_span(b, row);
    const float av = (c == 4 * m + q) ? 1.0f : 0.0f;  // A[i = c][k = q]
    for (int f = 0; f < F; ++f) {
      float bv = 0.0f, w = 0.0f;
      if (f < rs.len) {
        const float* src = a.wpull + (size_t)a.pos[rs.at(f)] * PS;
        w = src[0];
        const float v = c < D ? src[1 + c] : (c < 2 * D ? src[1 + c - D] : 0.0f);
        bv = c < D ? v : v * v;
      }
      wx[m] += w;
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bv, acc, 0, 0, 0);
    }
  }
  // D[row = 4*(lane>>4) + reg][col = lane & 15]: per row, sum over the 16 columns
  float t[4];
#pragma unroll
  for (int reg = 0; reg < 4; ++reg) {
    const float x = acc[reg];
    t[reg] = c < D ? x * x : (c < 2 * D ? -x : 0.0f);
  }
  // (vs_k^2 terms first, then the squares: same association on every lane)
#pragma unroll
  for (int o = 1; o < 16; o <<= 1)
#pragma unroll
    for (int reg = 0; reg < 4; ++reg) t[reg] += __shfl_xor(t[reg], o);
  // lane 16*g + 0 holds rows 4g .. 4g+3; their w sums sit in lanes (q = reg, c = 0), index m = g
  StatAcc st;
#pragma unroll
  for (int reg = 0; reg < 4; ++reg) {
    const int g = lane >> 4;
    float wxs = 0.0f;
#pragma unroll
    for (int m = 0; m < 4; ++m) {
      const float x = __shfl(wx[m], 16 * reg);  // lane (q = reg, c = 0)
      if (m == g) wxs = x;
    }
    const int64_t row = r0 + 4 * g + reg;
    if (c == 0 && row < b.rows) {
      const float p = sigmoid_ref(wxs + 0.5f * t[reg]);
      const float lab = b.labels[row];
      if (a.pctr) a.pctr[row] = p;
      st.add(p, lab);
    }
  }
  flush_stats<256>(st, a.stats, a.fx_bad);
}

// XFLOW_FMSTD_ATOMICS=1 keeps standard-math FM on the column-table + global
// Rows per producer workgroup on the reduction path: the model's R, or --
// when the batch fills at most an eighth of the CUs (a slice group of a step
// of 256 slices or more) -- halved (down to 128) until it fills them, within
// the workgroups the reduction's buffers hold.  A producer's time is its
// column walk, nearly independent of its rows; narrower workgroups aggregate
// less, so the records' sums cost more (A/B, profiles/r4_negative_ab.txt 13:
// LR --slices 256 +5.5 %, --slices 64 -1.5 % when narrowed to fill the CUs).
static int narrow_rows(const FwdArgs& a, int R) {
  const int64_t rows = a.batch.rows;
  auto groups = [&](int r) { return (rows + r - 1) / r; };
  if (a.red_groups <= 0 || groups(R) * 8 > device_cus()) return R;
  while (R > 128 && groups(R) < device_cus() && groups(R / 2) <= a.red_groups) R /= 2;
  return R;
}

template <bool kGrad>
static void dispatch_fm(const FwdArgs& a, hipStream_t st) {
  const bool agg = kGrad && a.agg_ok;
  const bool red = agg && a.model.fm_math == kFmReference && a.red_pairs && a.red_nb > 0 &&
                   a.red_nb <= kRedMaxBuckets;
  if (a.fm_compact && !red) throw std::runtime_error("fm_compact needs the FM reduction path");
  if (a.red_masks && a.S > 1 && a.model.fm_math == kFmReference && !red)
    throw std::runtime_error("red_masks need the FM reduction path");
  if (!kGrad && a.model.fm_math == kFmStandard && a.model.fm_mfma) {
    const int g = (int)((a.batch.rows + 63) / 64);  // 4 waves x 16 rows
    switch (a.model.kernel_dim()) {
      case 1: hipLaunchKernelGGL(k_fm_fwd_mfma<1>, dim3(g), dim3(256), 0, st, a); break;
      case 2: hipLaunchKernelGGL(k_fm_fwd_mfma<2>, dim3(g), dim3(256), 0, st, a); break;
      case 4: hipLaunchKernelGGL(k_fm_fwd_mfma<4>, dim3(g), dim3(256), 0, st, a); break;
      case 8: hipLaunchKernelGGL(k_fm_fwd_mfma<8>, dim3(g), dim3(256), 0, st, a); break;
      default: throw std::runtime_error("FM MFMA forward: v_dim 1, 2, 4 or 8");
    }
    return;
  }
  if (a.fm_vals) {
    if (a.model.fm_math != kFmReference) throw std::runtime_error("fm_vals: reference math only");
    constexpr int R = kFmGroupRows;
    const int gr = (int)((a.batch.rows + R - 1) / R);
    if (kGrad) {
      if (!red || !a.fm_compact) throw std::runtime_error("fm_vals: needs the compact reduction");
      const int Rn = narrow_rows(a, R);
      const int gn = (int)((a.batch.rows + Rn - 1) / Rn);
      switch (Rn) {
        case 1024: hipLaunchKernelGGL((k_fm_vals<1024, true>), dim3(gn), dim3(Rn), 0, st, a); break;
        case 512: hipLaunchKernelGGL((k_fm_vals<512, true>), dim3(gn), dim3(Rn), 0, st, a); break;
        case 256: hipLaunchKernelGGL((k_fm_vals<256, true>), dim3(gn), dim3(Rn), 0, st, a); break;
        default: hipLaunchKernelGGL((k_fm_vals<128, true>), dim3(gn), dim3(Rn), 0, st, a); break;
      }
      launch_reduction<2>(a, gn, Rn, st);
    } else {
      hipLaunchKernelGGL((k_fm_vals<R, false>), dim3(gr), dim3(R), 0, st, a);
    }
    return;
  }
  // standard math: per-component records through the LR reduction pipeline
  const bool red_std = agg && a.model.fm_math == kFmStandard && a.red_pairs && a.red_nb > 0 &&
                       a.red_nb <= (a.red_maxb > 0 ? a.red_maxb : kRedMaxBuckets);
  if (a.red_masks && a.S > 1 && a.model.fm_math == kFmStandard && !red_std)
    throw std::runtime_error("red_masks need the standard-FM reduction path");
  if (a.red_out && a.model.fm_math == kFmStandard && !red_std)
    throw std::runtime_error("standard FM red_out needs the vector-record reduction");
  switch (a.model.kernel_dim()) {
#define XF_FM_CASE(DD)                                                                   \
  case DD: {                                                                             \
    constexpr int B = fm_block(DD);                                                      \
    int g = (int)((a.batch.rows + B - 1) / B);                                           \
    if (red_std) {                                                                       \
      launch_vec_reduction<DD>(a, st);                                                 \
    } else if (red) {                                                                    \
      constexpr int R = kFmGroupRows;                                                    \
      const int gr = (int)((a.batch.rows + R - 1) / R);                                  \
      hipLaunchKernelGGL((k_fm_red<DD, R>), dim3(gr), dim3(R), 0, st, a);                \
      launch_reduction<2>(a, gr, R, st);                                                 \
    } else if (agg) {                                                                    \
      hipLaunchKernelGGL((k_fm<DD, kGrad, true>), dim3(g), dim3(B), 0, st, a);           \
    } else {                                                                             \
      hipLaunchKernelGGL((k_fm<DD, kGrad, false>), dim3(g), dim3(B), 0, st, a);          \
    }                                                                                    \
    break;                                                                               \
  }
    XF_FM_CASE(1) XF_FM_CASE(2) XF_FM_CASE(4) XF_FM_CASE(8) XF_FM_CASE(10) XF_FM_CASE(16)
    XF_FM_CASE(32)
#undef XF_FM_CASE
    default:
      throw std::runtime_error("FM: unsupported v_dim (1,2,4,8,10,16,32)");
  }
}

// ---------------------------------------------------------------------------
// MVM, one lane per row with register-resident latent sums.  Each occurrence's
// pulled row [v_0..v_{D-1}, pad] is read with dwordx4 loads once per pass; the
// per-field sums S[g][k] are the occurrence's own v when every field occurs at
// most once in the row (CTR rows; checked per row with a 64-bit field mask),
// otherwise they are summed over the row's occurrences of that field.  The
// backward aggregates each occurrence's D-vector per (key, slice) in the LDS
// column tables (vector flush) instead of D global atomics per occurrence.
// Reference math: mvm_worker.cc:137-218 (product over fields [0, G), G = maxf
// (compat) or maxf + 1 (fixed); gradient loss*M_k/(1+S) when S != 0).
constexpr int mvm_ps(int D) { return D == 1 ? 1 : (D + 3) & ~3; }
constexpr int mvm_block(int D) { return mvm_ps(D) <= 12 ? 256 : (mvm_ps(D) <= 20 ? 128 : 64); }

template <int PS>
__device__ __forceinline__ void load_row(const float* __restrict__ wp, u32 p, float (&w)[PS]) {
  if constexpr (PS % 4 == 0) {
    const float4* src = reinterpret_cast<const float4*>(wp) + (size_t)p * (PS / 4);
#pragma unroll
    for (int q = 0; q < PS / 4; ++q) {
      const float4 v4 = src[q];
      w[4 * q] = v4.x;
      w[4 * q + 1] = v4.y;
      w[4 * q + 2] = v4.z;
      w[4 * q + 3] = v4.w;
    }
  } else {
#pragma unroll
    for (int c = 0; c < PS; ++c) w[c] = wp[(size_t)p * PS + c];
  }
}

constexpr int mvm_block_for(int D, bool red) { return red ? kMvmGroupRows : mvm_block(D); }

template <int D, bool kGrad, bool kAgg, bool kRed = false>
__global__ void __launch_bounds__(mvm_block_for(D, kRed)) k_mvm2(FwdArgs a) {
  constexpr int PS = mvm_ps(D);
  constexpr int BLOCK = mvm_block_for(D, kRed);
  constexpr int LOG2 = ilog2c(2 * BLOCK);
  __shared__ u32 s_tag[kAgg ? 2 : 1][kAgg ? (1 << LOG2) : 1];
  __shared__ float s_acc[kAgg ? 2 : 1][kAgg ? (1 << LOG2) * PS : 1];
  __shared__ int s_wmax[BLOCK / kWave];
  const BatchView& b = a.batch;
  const bool compat = a.model.mvm_math == kMvmCompat;
  const u32* __restrict__ pos = a.pos;
  const float* __restrict__ wp = a.wpull;
  const int64_t r = (int64_t)blockIdx.x * BLOCK + threadIdx.x;
  const bool active = r < b.rows;
  RowSpan rs;
  if (active) rs = row_span(b, r);
  const int len = rs.len;
  // fields of the row: mask of those < 64, duplicate / out-of-mask flags
  unsigned long long mask = 0ull;
  bool dup = false, sorted = true;
  int maxf = 0;
  for (int j = 0; j < len; ++j) {
    const int f = b.fgid[rs.at(j)];
    if (j > 0 && f <= maxf) sorted = false;
    maxf = max(maxf, f);
    if (f < 0 || f >= 64) {
      dup = true;
    } else {
      if ((mask >> f) & 1ull) dup = true;
      mask |= 1ull << f;
    }
  }
  const int G = compat ? maxf : maxf + 1;
  // sum of the row's latent rows of field f, component-wise (slow path)
  auto field_sum = [&](int f, float (&S)[D]) {
#pragma unroll
    for (int k = 0; k < D; ++k) S[k] = 0.0f;
    for (int j = 0; j < len; ++j) {
      if (b.fgid[rs.at(j)] != f) continue;
      float w[PS];
      load_row<PS>(wp, pos[rs.at(j)], w);
#pragma unroll
      for (int k = 0; k < D; ++k) S[k] += w[k];
    }
  };
  float M[D];
  float y = 0.0f;
  StatAcc st;
  float loss = 0.0f;
  if (active) {
    bool complete;  // every field g < G occurs (else some S[g] = 0 and M = 0)
    if (dup || G > 64) {
      complete = true;
      for (int g = 0; g < G && complete; ++g) {
        bool found = false;
        for (int j = 0; j < len && !found; ++j) found = b.fgid[rs.at(j)] == g;
        complete = found;
      }
    } else {
      const unsigned long long need = G >= 64 ? ~0ull : ((1ull << G) - 1ull);
      complete = (mask & need) == need;
    }
#pragma unroll
    for (int k = 0; k < D; ++k) M[k] = complete ? 1.0f : 0.0f;
    if (complete) {
      if (!dup && sorted) {
        // occurrence order = field order g = 0..G-1 (the reference's product order)
        for (int j = 0; j < len; ++j) {
          if (b.fgid[rs.at(j)] >= G) break;
          float w[PS];
          load_row<PS>(wp, pos[rs.at(j)], w);
#pragma unroll
          for (int k = 0; k < D; ++k) M[k] *= w[k];
        }
      } else if (!dup) {
        for (int g = 0; g < G; ++g) {
          int jj = 0;
          while (b.fgid[rs.at(jj)] != g) ++jj;
          float w[PS];
          load_row<PS>(wp, pos[rs.at(jj)], w);
#pragma unroll
          for (int k = 0; k < D; ++k) M[k] *= w[k];
        }
      } else {
        for (int g = 0; g < G; ++g) {
          float S[D];
          field_sum(g, S);
#pragma unroll
          for (int k = 0; k < D; ++k) M[k] *= S[k];
        }
      }
    }
#pragma unroll
    for (int k = 0; k < D; ++k) y += M[k];
    const float p = sigmoid_ref(y);
    const float lab = b.labels[r];
    loss = p - lab;
    if (a.pctr) a.pctr[r] = p;
    st.add(p, lab);
  }
  if constexpr (kGrad) {
    const u32 s = active ? (u32)slice_of(b, r, a.S) : 0u;
    const u32 S = (u32)a.S;
    // gradient of the row's j-th occurrence
    auto contrib = [&](int j, float (&c)[D]) {
      float Sf[D];
      if (!dup) {
        float w[PS];
        load_row<PS>(wp, pos[rs.at(j)], w);
#pragma unroll
        for (int k = 0; k < D; ++k) Sf[k] = w[k];
      } else {
        field_sum(b.fgid[rs.at(j)], Sf);
      }
#pragma unroll
      for (int k = 0; k < D; ++k)
        c[k] = (Sf[k] == 0.0f) ? 0.0f
                               : (float)((double)loss * ((double)M[k] / (1.0 + (double)Sf[k])));
    };
    if constexpr (kRed) {
      // Dup-free rows: S of an occurrence is the key's own v, so the gradient
      // factorises as T_k/(1+v_k) with T = loss*M per row: the row's T goes
      // to red_rowv and the vector-record reduction (k_fm_std_red<D-1, ..,
      // kSplit> + k_red_sum_vec<.., kMvm>) sums T per (key, slice) and
      // divides once.  Rows with a repeated field (S = field sum): global
      // atomics, and T = 0 (their occurrences still leave records, for the
      // slice bits of a multi-slice step).
      float tmax = 0.0f;  // |T| of the row (the step's fixed-point scale)
      if (active) {
        float* t = a.red_rowv + (size_t)r * PS;
#pragma unroll
        for (int k = 0; k < PS; ++k) {
          const float v = (!dup && k < D) ? loss * M[k] : 0.0f;
          t[k] = v;
          // (a non-finite T maxes to inf: fx_scale_bits then keeps the
          // static 2^44 scale and the clamp flags the step)
          tmax = fmaxf(tmax, v == v ? fabsf(v) : INFINITY);
        }
      }
      {
        __shared__ float s_tmax[BLOCK / kWave];
        tmax = wave_max(tmax);
        if (threadIdx.x % kWave == 0) s_tmax[threadIdx.x / kWave] = tmax;
        __syncthreads();
        if (threadIdx.x == 0) {
          float m = 0.0f;
#pragma unroll
          for (int w = 0; w < BLOCK / kWave; ++w) m = fmaxf(m, s_tmax[w]);
          if (m > 0.0f) atomicMax(a.red_vmax, __float_as_uint(m));  // (>= 0: bits order as values)
          if (!(m <= 3.0e38f)) atomicOr(a.fx_bad, 2u);  // non-finite T: a diverged model
          if (blockIdx.x == 0) *a.red_vmax_next = 0u;  // (the next step's word)
          if (blockIdx.x == 0 && a.red_dup_next) *a.red_dup_next = 0u;

        }
      }
      // repeated-field rows on the unique-row / CSR outputs: fixed-point
      // records for the order-free passes after the reduction (MvmDup)
      const bool md = a.mdup.rec && (a.red_out || a.red_csr.cnt);
      // (one flag write per wave with a repeated-field row added by atomics: FwdArgs::red_dup)
      if (a.red_dup && !md && __ballot(active && dup) && lane_id() == 0) atomicOr(a.red_dup, 1u);
      float cmax = 0.0f;
      if (active && dup && md) {
        const int ew = a.mdup.ew;
        for (int j = 0; j < len; ++j) {
          float c[D];
          contrib(j, c);
          const u32 pj = pos[rs.at(j)];
          if (pj == a.trash_pos) continue;
          // target: the (key, slice) dest (CSR; resolved to its entry later)
          // or the key's unique-order row
          const u32 tgt = a.red_csr.cnt ? pj * S + s : uix(a.red_inv, pj);
          if (tgt == 0xFFFFFFFFu) continue;
          const u32 at = atomicAdd(a.mdup.n, 1u);
          if (at >= (u32)a.mdup.cap) continue;  // (cannot happen: <= one per occurrence)
          float* rec = a.mdup.rec + (size_t)at * ew;
          rec[0] = __uint_as_float(tgt);
#pragma unroll
          for (int k = 0; k < D; ++k) {
            rec[1 + k] = c[k];
            cmax = fmaxf(cmax, c[k] == c[k] ? fabsf(c[k]) : INFINITY);
          }
        }
      } else if (active && dup) {
        for (int j = 0; j < len; ++j) {
          float c[D];
          contrib(j, c);
          const u32 pj = pos[rs.at(j)];
          float* g = a.grad + ((size_t)pj * S + s) * PS;
          if (a.red_out) {  // (one slice: the unique-order rows the reduction adds to)
            const u32 o = uix(a.red_inv, pj);
            if (o == 0xFFFFFFFFu) continue;
            g = a.red_out + (size_t)o * PS;
          }
#pragma unroll
          for (int k = 0; k < D; ++k) atomicAdd(&g[k], c[k]);
        }
      }
      if (md) {  // (every lane: the wave's largest |c| sets the step's scale)
        cmax = wave_max(cmax);
        if (lane_id() == 0 && cmax > 0.0f) {
          atomicMax(a.mdup.vmax, __float_as_uint(fminf(cmax, 3.4e38f)));
          if (!(cmax <= 3.0e38f)) atomicOr(a.fx_bad, 2u);  // non-finite: a diverged model
        }
      }
    } else if constexpr (!kAgg) {
      for (int j = 0; j < len; ++j) {
        float c[D];
        contrib(j, c);
        float* g = a.grad + ((size_t)pos[rs.at(j)] * S + s) * PS;
#pragma unroll
        for (int k = 0; k < D; ++k) atomicAdd(&g[k], c[k]);
      }
    } else {
      ColumnAgg<PS, LOG2> agg{s_tag, s_acc};
      agg.init();
      const int m = wave_max(len);
      if (threadIdx.x % kWave == 0) s_wmax[threadIdx.x / kWave] = m;
      __syncthreads();
      int maxlen = 0;
#pragma unroll
      for (int w = 0; w < BLOCK / kWave; ++w) maxlen = max(maxlen, s_wmax[w]);
      for (int j = 0; j < maxlen; ++j) {
        const int t = j & 1;
        if (j < len) {
          float c[D];
          contrib(j, c);
          const int h = agg.insert(t, pos[rs.at(j)] * S + s);
#pragma unroll
          for (int k = 0; k < D; ++k) agg.add(t, h, k, c[k]);
        }
        __syncthreads();
        agg.flush(t, a.grad);
      }
    }
  }
  flush_stats<BLOCK>(st, a.stats, a.fx_bad);
}

template <bool kGrad>
static void dispatch_mvm(const FwdArgs& a, hipStream_t st) {
  const bool agg = kGrad && a.agg_ok;
  const bool red = agg && a.red_pairs && a.red_rowv && a.red_nb > 0 &&
                   a.red_nb <= (a.red_maxb > 0 ? a.red_maxb : kRedMaxBuckets);
  if (a.red_masks && a.S > 1 && !(red && a.model.kernel_dim() >= 2))
    throw std::runtime_error("red_masks need the MVM reduction path");
  switch (a.model.kernel_dim()) {
#define XF_MVM_CASE(DD)                                                                  \
  case DD: {                                                                             \
    constexpr int B = mvm_block(DD);                                                     \
    const int g = (int)((a.batch.rows + B - 1) / B);                                     \
    if (a.red_out && !(red && DD >= 2))                                                  \
      throw std::runtime_error("MVM red_out needs the bucket reduction");                \
    if (red && DD >= 2) {                                                                \
      constexpr int R = kMvmGroupRows;                                                   \
      const int gr = (int)((a.batch.rows + R - 1) / R);                                  \
      hipLaunchKernelGGL((k_mvm2<DD, kGrad, false, true>), dim3(gr), dim3(R), 0, st, a); \
      launch_vec_reduction<(DD >= 2 ? DD - 1 : 1), true>(a, st);                          \
    } else if (agg) {                                                                    \
      hipLaunchKernelGGL((k_mvm2<DD, kGrad, true>), dim3(g), dim3(B), 0, st, a);         \
    } else {                                                                             \
      hipLaunchKernelGGL((k_mvm2<DD, kGrad, false>), dim3(g), dim3(B), 0, st, a);        \
    }                                                                                    \
    break;                                                                               \
  }
    XF_MVM_CASE(1) XF_MVM_CASE(2) XF_MVM_CASE(4) XF_MVM_CASE(8) XF_MVM_CASE(10) XF_MVM_CASE(16)
    XF_MVM_CASE(32)
#undef XF_MVM_CASE
    default:
      throw std::runtime_error("MVM: unsupported v_dim (1,2,4,8,10,16,32)");
  }
}

void launch_forward_backward(const FwdArgs& a, hipStream_t st) {
  if (a.batch.rows <= 0) return;
  const bool grad = a.grad != nullptr;
  int grid = (int)((a.batch.rows + kBlock - 1) / kBlock);
  switch (a.model.kind) {
    case kLR: {
      // LDS aggregation needs every destination index to fit a u32 tag
      constexpr int kLrBlock = 1024;
      int g = (int)((a.batch.rows + kLrBlock - 1) / kLrBlock);
      const bool red = grad && a.agg_ok && a.red_pairs && a.red_nb > 0 &&
                       a.red_nb <= kRedMaxBuckets;
      if (a.red_out && !(red && (a.S == 1 || a.red_masks)))
        throw std::runtime_error("red_out needs the LR bucket reduction (S > 1: with slice bits)");
      if (a.red_masks && a.S > 1 && !red)
        throw std::runtime_error("red_masks need the LR bucket reduction");
      if (red) {
        const int R = narrow_rows(a, kLrGroupRows);
        const int gr = (int)((a.batch.rows + R - 1) / R);
        switch (R) {
          case 1024: hipLaunchKernelGGL((k_lr<true, true, 1024, true>), dim3(gr), dim3(R), 0, st, a); break;
          case 512: hipLaunchKernelGGL((k_lr<true, true, 512, true>), dim3(gr), dim3(R), 0, st, a); break;
          case 256: hipLaunchKernelGGL((k_lr<true, true, 256, true>), dim3(gr), dim3(R), 0, st, a); break;
          default: hipLaunchKernelGGL((k_lr<true, true, 128, true>), dim3(gr), dim3(R), 0, st, a); break;
        }
#ifdef XFLOW_KTIMING
        ktime_dump("lr (init forward walk-other tail insert barrier flush)", 7, st);
#endif
        launch_reduction<1>(a, gr, R, st);
      } else if (grad && a.agg_ok)
        hipLaunchKernelGGL((k_lr<true, true, kLrBlock>), dim3(g), dim3(kLrBlock), 0, st, a);
      else if (grad)
        hipLaunchKernelGGL((k_lr<true, false, kBlock>), dim3(grid), dim3(kBlock), 0, st, a);
      else
        hipLaunchKernelGGL((k_lr<false, false, kBlock>), dim3(grid), dim3(kBlock), 0, st, a);
      break;
    }
    case kFM:
      if (grad) dispatch_fm<true>(a, st);
      else dispatch_fm<false>(a, st);
      break;
    case kMVM:
      if (!a.batch.fgid) throw std::runtime_error("MVM needs field ids (fgid)");
      if (grad) dispatch_mvm<true>(a, st);
      else dispatch_mvm<false>(a, st);
      break;
    default:
      throw std::runtime_error("unknown model kind");
  }
  XF_HIP_CHECK(hipGetLastError());
}

__global__ void k_slice_masks(BatchView b, const u32* __restrict__ pos, u32* __restrict__ tmask,
                              int S) {
  int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= b.rows) return;
  const RowSpan rs = row_span(b, r);
  u32 bit = 1u << slice_of(b, r, S);
  for (int j = 0; j < rs.len; ++j) atomicOr(&tmask[pos[rs.at(j)]], bit);
}

void launch_slice_masks(const BatchView& b, const u32* pos, u32* tmask, hipStream_t st) {
  if (b.rows <= 0) return;
  int S = b.slice_rows > 0 ? (int)((b.rows + b.slice_rows - 1) / b.slice_rows) : 1;
  hipLaunchKernelGGL(k_slice_masks, dim3((int)((b.rows + kBlock - 1) / kBlock)), dim3(kBlock), 0,
                     st, b, pos, tmask, S);
  XF_HIP_CHECK(hipGetLastError());
}

}  // namespace hip
}  // namespace xflow
