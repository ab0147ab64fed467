// xflow-amd: gfx950 kernels for the HBM-resident sparse parameter store.
//
// Replaces the ps-lite KVServer + unordered_map store of the reference
// (/root/reference/src/optimizer/ftrl.h:38-152, server.h:20-35) and the
// worker-side sort/unique key preparation (lr_worker.cc:146-166):
//
//   dedup        persistent, epoch-stamped open-addressing scratch table: each
//                occurrence finds (or CAS-claims, for keys new to the table)
//                its key's slot and stamps it; the unique list is compacted
//                from the stamps without global atomics.  No sort at all.
//   table_pull   probe/insert of unique keys into the persistent table and
//                evaluation of the reference pull value (FTRL weight closed form
//                from (n,z), lazy N(0,1)*1e-2 latent init).
//   table_apply  per-coordinate FTRL-Proximal / SGD push (one lane per key for
//                LR, one lane group per key for multi-parameter models),
//                contributions applied in (slice) order -> deterministic.
//
// All kernels are memory-latency bound (random 16-64 B accesses): they keep
// several independent probes in flight per lane, count bookkeeping with one
// atomic per workgroup (single-address atomics serialise), and read
// device-side element counts so a whole step runs without host syncs.
#include <cstdlib>
#include <cstring>
#include <type_traits>

#include "kernels.h"
#include "hip_util.h"

namespace xflow {
namespace hip {

constexpr u32 kNoSlot = 0xFFFFFFFFu;
// grid cap of the lane-group pull/apply kernels (8 K workgroups of 256: four
// resident rounds; their grid-stride loops pipeline the random row accesses,
// see RowPipe -- 16 K measured 2 % slower on FM-8, 64 K 6 %)
constexpr int kGroupGridCap = 8192;

// ---------------------------------------------------------------------------
// dedup
// ---------------------------------------------------------------------------
// The worker dedup table is persistent across steps (see ScratchView): hot
// keys keep their slot, so after warm-up almost every occurrence is a plain
// hit.  CTR keys are extremely skewed (top-1000 keys ~60% of occurrences); a
// table cleared every step made each hot key a same-address CAS storm.
//
// Device-side rebuilds.  With ctl (adaptive capacity, the HIP engine) the
// compaction decides them: k_compact_scan switches the active capacity for
// the next batch (ctl[0]) while keeping this batch's in ctl[3], and
// k_compact_write frees the new capacity's slots right after reading its own
// (each thread owns 16 slots) -- no extra launches per step.  Without ctl the
// table is rebuilt by the two kernels below once `claims` exceeds rebuild_at.
__device__ __forceinline__ u64 active_cap(const ScratchView& sv) {
  return sv.ctl ? (u64)sv.ctl[0] : sv.cap;
}

// capacity this batch was deduplicated with (valid after k_compact_scan)
__device__ __forceinline__ u64 batch_cap(const ScratchView& sv) {
  return sv.ctl ? (u64)sv.ctl[3] : sv.cap;
}

// this batch spilled past the active capacity (ScratchView::ctl[4])
__device__ __forceinline__ bool batch_spilled(const ScratchView& sv) {
  return sv.ctl && sv.ctl[4] == (unsigned long long)sv.epoch;
}

__global__ void k_scratch_maybe_clear(u64* __restrict__ skeys, u64 cap,
                                      const unsigned long long* __restrict__ claims,
                                      u64 rebuild_at, const unsigned long long* __restrict__ ctl) {
  u64 n = cap;
  if (ctl) {
    n = ctl[2];
    if (n == 0) return;
  } else if (*claims <= rebuild_at) {
    return;
  }
  const u64 stride = (u64)gridDim.x * blockDim.x;
  for (u64 s = (u64)blockIdx.x * blockDim.x + threadIdx.x; s < n; s += stride)
    skeys[s] = kEmptyKey;
}

__global__ void k_scratch_claims_reset(unsigned long long* claims, u64 rebuild_at,
                                       unsigned long long* ctl) {
  if (ctl) {
    if (ctl[2]) {
      ctl[0] = ctl[2];
      ctl[2] = 0ull;
      *claims = 0ull;
    }
  } else if (*claims > rebuild_at) {
    *claims = 0ull;
  }
}

// ScratchView::grow: rebuild at the grown capacity before the insert
// (k_scratch_maybe_clear and k_scratch_claims_reset apply ctl[2]).
__global__ void k_scratch_grow(unsigned long long* __restrict__ ctl, u64 cap_alloc, float grow) {
  const double need = (double)kScratchHeadroom * (double)ctl[1] * (double)grow;
  u64 want = kScratchMinCap;
  while ((double)want < need && want < cap_alloc) want <<= 1;
  if (want > cap_alloc) want = cap_alloc;
  ctl[2] = want > ctl[0] ? want : 0ull;
}

// Step 1 -- insert / stamp, two levels.
//   (a) workgroup level: the block's kDedupChunk occurrences (1024: measured
//       137 us per 10.2 M-key batch vs 154 at 2048, 158 at 512, 196 at 4096)
//       are deduplicated in an LDS hash table (2x oversized, 64-bit ds CAS);
//       the first occurrence of each key becomes its leader.
//   (b) global level: only leaders probe the persistent table -- all of their
//       first-probe loads in flight before any is resolved -- CAS new keys,
//       write the epoch stamp and publish the slot in LDS; every occurrence
//       then reads its slot from LDS.
// Hot keys (an int-field value can occur in half the rows) otherwise send one
// read and one stamp store per occurrence to the same L2 channel; with (a)
// they cost one per workgroup.
constexpr int kDedupItems = 4;
constexpr int kDedupChunk = kBlock * kDedupItems;
constexpr int kDedupLog2 = 11;  // LDS slots = 2 * kDedupChunk
static_assert((1 << kDedupLog2) == 2 * kDedupChunk, "LDS dedup table sizing");

__global__ void __launch_bounds__(kBlock) k_dedup_insert(const u64* __restrict__ keys, int64_t nnz,
                                                         ScratchView sv, u32* __restrict__ pos,
                                                         u32* __restrict__ overflow) {
  constexpr u32 kL = 1u << kDedupLog2;
  __shared__ u64 t_key[kL];  // keys during the LDS level, then leaders' slots
  u64* __restrict__ skeys = sv.keys;
  const u64 cap = active_cap(sv), mask = cap - 1;
  const u32 parts = (u32)sv.parts;
  const u64 R = parts > 1 ? cap / parts : cap;  // probe range per owner
  // (ScratchView::home_bits: the top bits of the table home's hash bits)
  const int clog = 63 - __clzll((long long)cap);
  const int hshift = sv.home_bits > clog ? sv.home_bits - clog : 0;
  const int64_t base = (int64_t)blockIdx.x * kDedupChunk + threadIdx.x;
  for (u32 i = threadIdx.x; i < kL; i += kBlock) t_key[i] = kEmptyKey;
  u64 k[kDedupItems], s[kDedupItems];
  u32 h[kDedupItems];
#pragma unroll
  for (int j = 0; j < kDedupItems; ++j) {
    int64_t i = base + (int64_t)j * kBlock;
    k[j] = i < nnz ? sanitize_key(keys[i]) : 0ull;
    const u64 f = fmix64(k[j]);
    s[j] = parts > 1 ? (u64)((u32)(f >> 32) % parts) * R + (((f & 0xffffffffull) * R) >> 32)
                     : (f >> hshift) & mask;
    h[j] = (u32)(f >> (64 - kDedupLog2));
  }
  __syncthreads();
  u32 lead = 0;
#pragma unroll
  for (int j = 0; j < kDedupItems; ++j) {
    if (base + (int64_t)j * kBlock >= nnz) continue;
    u32 x = h[j];
    while (true) {  // (one CAS against an empty slot per probe step, no read first)
      const u64 prev = atomicCAS((unsigned long long*)&t_key[x], (unsigned long long)kEmptyKey,
                                 (unsigned long long)k[j]);
      if (prev == kEmptyKey) {
        lead |= 1u << j;
        break;
      }
      if (prev == k[j]) break;
      x = (x + 1) & (kL - 1);  // <= kDedupChunk keys in kL slots: terminates
    }
    h[j] = x;
  }
  // every LDS lookup is done: the leaders' table entries can now carry slots
  __syncthreads();
  // global level, leaders only: all first-probe loads in flight, then each
  // leader resolves (CAS only for keys new to the table)
  u64 cur[kDedupItems];
#pragma unroll
  for (int j = 0; j < kDedupItems; ++j) cur[j] = (lead >> j) & 1u ? skeys[s[j]] : k[j];
  unsigned int claimed = 0;
#pragma unroll
  for (int j = 0; j < kDedupItems; ++j) {
    if (!((lead >> j) & 1u)) continue;
    u64 sj = s[j], c = cur[j];
    u64 n = 0;
    while (c != k[j]) {
      if (c == kEmptyKey) {
        u64 prev = atomicCAS((unsigned long long*)&skeys[sj], (unsigned long long)kEmptyKey,
                             (unsigned long long)k[j]);
        if (prev == kEmptyKey) {
          ++claimed;
          break;
        }
        if (prev == k[j]) break;
      }
      if (++n >= R) {
        // the active table is full (a surge of distinct keys): probe on in
        // the rest of the allocation, which this batch's compaction then
        // covers (ScratchView::ctl[4])
        if (sv.ctl && parts == 1 && cap < sv.cap && n == R) {
          sv.ctl[4] = sv.epoch;
          const u64 Z = sv.cap - cap;
          sj = cap + fmix64(k[j]) % Z;
          c = skeys[sj];
          for (u64 m = 0; c != k[j]; ) {
            if (c == kEmptyKey) {
              u64 prev = atomicCAS((unsigned long long*)&skeys[sj], (unsigned long long)kEmptyKey,
                                   (unsigned long long)k[j]);
              if (prev == kEmptyKey) {
                ++claimed;
                break;
              }
              if (prev == k[j]) break;
            }
            if (++m >= Z) {
              sj = sv.cap;
              break;
            }
            if (++sj == sv.cap) sj = cap;
            c = skeys[sj];
          }
          if (sj < sv.cap) break;
        }
        // no free slot: the key's occurrences go to the trash slot (index
        // cap: never stamped, so never in the unique list; its pulled row is
        // zero and its gradients are dropped) and the step is flagged --
        // never merged into another key's slot
        *overflow = 1u;
        sj = sv.cap;
        break;
      }
      if (parts > 1) {
        ++sj;
        if (sj % R == 0) sj -= R;  // wrap inside the owner's range
      } else {
        sj = (sj + 1) & mask;
      }
      c = skeys[sj];
    }
    XF_DASSERT(sj <= sv.cap);
    t_key[h[j]] = sj;
    if (sj < sv.cap) sv.stamps[sj] = (unsigned char)sv.epoch;
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < kDedupItems; ++j) {
    int64_t i = base + (int64_t)j * kBlock;
    if (i < nnz) pos[i] = (u32)t_key[h[j]];
  }
  // one no-return atomic per workgroup for the rebuild counter
  block_count_add<kBlock>(sv.claims, claimed);
}

// Step 2 -- compaction of the slots stamped with this epoch into the unique
// list, without a single global atomic: (a) each workgroup counts its 4096
// slots (coalesced stamp reads), (b) one workgroup scans the counts, (c) each
// workgroup re-reads its stamps (L3/L2 resident) and writes (key, slot) at
// its offset.  Output order = slot order: deterministic.
constexpr int kCompactItems = 16;
constexpr int kCompactChunk = kBlock * kCompactItems;
constexpr int kScanBlock = 1024;

// 16 consecutive byte stamps as one dwordx4 load (cap is a power of two >=
// 16, so a 16-slot group is either fully inside the table or fully outside).
__device__ __forceinline__ unsigned int compact_hits(const ScratchView& sv, u64 base, u64 cap,
                                                     unsigned int& cnt) {
  unsigned int hit = 0;
  cnt = 0;
  if (base >= cap) return 0;
  const uint4 q = *reinterpret_cast<const uint4*>(sv.stamps + base);
  const u32 w[4] = {q.x, q.y, q.z, q.w};
  const u32 e = sv.epoch & 0xFFu;
#pragma unroll
  for (int j = 0; j < 16; ++j) hit |= (unsigned int)(((w[j >> 2] >> (8 * (j & 3))) & 0xFFu) == e) << j;
  cnt = __popc(hit);
  return hit;
}

// lane t owns the 16 consecutive slots [base + 16t, base + 16t + 16): the
// stamp loads are dwordx4-able and the output stays in slot order
__global__ void __launch_bounds__(kBlock) k_compact_count(ScratchView sv,
                                                          unsigned int* __restrict__ counts) {
  const u64 base = (u64)blockIdx.x * kCompactChunk + (u64)threadIdx.x * kCompactItems;
  unsigned int cnt;
  compact_hits(sv, base, batch_spilled(sv) ? sv.cap : active_cap(sv), cnt);
  unsigned int tot;
  block_exclusive_scan<kBlock>(cnt, &tot);
  if (threadIdx.x == 0) counts[blockIdx.x] = tot;
}

// Also sizes the scratch for the next batch (ctl): active cap = the power of
// two >= kScratchHeadroom x the largest batch seen, rebuilt when it should
// grow, when it is 4x too large, or when the keys claimed since the last
// rebuild fill half of it.  A rebuild takes effect here: ctl[3] keeps this
// batch's capacity for k_compact_write / k_partition_counts, ctl[0] becomes
// the new one, ctl[2] tells k_compact_write how many slots to free.
__global__ void __launch_bounds__(kScanBlock) k_compact_scan(
    unsigned int* __restrict__ counts, int nb, unsigned long long* __restrict__ n_out,
    unsigned long long* __restrict__ claims, unsigned long long* __restrict__ ctl,
    u64 cap_alloc, unsigned long long* __restrict__ n_copy,
    unsigned long long* __restrict__ cap_out, u32 epoch) {
  // only the blocks of this batch's capacity hold stamps (the rest count 0):
  // at 4x headroom that is 1/8 of the allocation's blocks
  if (ctl) {
    const u64 lim = ctl[4] == epoch ? cap_alloc : (u64)ctl[0];  // (read before thread 0 updates ctl)
    const u64 nbl = (lim + kCompactChunk - 1) / kCompactChunk;
    if (nbl < (u64)nb) nb = (int)nbl;
  }
  unsigned long long carry = 0;
  for (int c0 = 0; c0 < nb; c0 += kScanBlock) {
    int i = c0 + (int)threadIdx.x;
    unsigned int v = i < nb ? counts[i] : 0u;
    unsigned int tot;
    unsigned int ex = block_exclusive_scan<kScanBlock>(v, &tot);
    if (i < nb) counts[i] = (unsigned int)(carry + ex);  // exclusive offsets (< 2^32 slots)
    carry += tot;
  }
  if (threadIdx.x == 0) {
    *n_out = carry;
    if (n_copy) *n_copy = carry;  // e.g. the one-owner counts of a world-1 sharded step
    if (ctl) {
      const u64 mx = ctl[1] > carry ? ctl[1] : carry;
      ctl[1] = mx;
      u64 want = kScratchMinCap;
      while (want < kScratchHeadroom * mx && want < cap_alloc) want <<= 1;
      if (want > cap_alloc) want = cap_alloc;
      const u64 cur = ctl[0];
      // (stale claims <= cur / 2 at a batch start: 2x the most unique keys
      // seen fit in the active table; a larger surge spills, see ctl[4])
      const bool rebuild = *claims > cur / 2 || want > cur || want * 4 <= cur;
      ctl[3] = cur;
      ctl[2] = rebuild ? want : 0ull;
      if (rebuild) {
        ctl[0] = want;
        *claims = 0ull;
      }
    }
    // (the reduction's bucket geometry: a spilled batch's slots reach cap_alloc)
    if (cap_out) *cap_out = ctl && ctl[4] != epoch ? ctl[3] : cap_alloc;
  }
}

__global__ void __launch_bounds__(kBlock) k_compact_write(ScratchView sv,
                                                          const unsigned int* __restrict__ offs,
                                                          u64* __restrict__ uk,
                                                          u32* __restrict__ up,
                                                          u32* __restrict__ inv) {
  const u64 base = (u64)blockIdx.x * kCompactChunk + (u64)threadIdx.x * kCompactItems;
  unsigned int cnt;
  unsigned int hit = compact_hits(sv, base, batch_spilled(sv) ? sv.cap : batch_cap(sv), cnt);
  unsigned int tot;
  unsigned int ex = block_exclusive_scan<kBlock>(cnt, &tot);
  unsigned long long dst = (unsigned long long)offs[blockIdx.x] + ex;
  u32 iv[kCompactItems];
  // the thread's 16 keys (one 128-byte line) loaded before any store: the
  // stores to uk may alias sv.keys for the compiler, which would otherwise
  // serialise one load round trip per hit
  u64 kv[kCompactItems];
  if (hit) {
    const ulonglong2* kp = reinterpret_cast<const ulonglong2*>(sv.keys + base);
#pragma unroll
    for (int q = 0; q < kCompactItems / 2; ++q) {
      const ulonglong2 v = kp[q];
      kv[2 * q] = v.x;
      kv[2 * q + 1] = v.y;
    }
  }
#pragma unroll
  for (int j = 0; j < kCompactItems; ++j) {
    iv[j] = 0xFFFFFFFFu;
    if (!(hit & (1u << j))) continue;
    u64 s = base + (u64)j;
    uk[dst] = kv[j];
    up[dst] = (u32)s;
    iv[j] = (u32)dst;
    ++dst;
  }
  // inv for all of the thread's slots as four dwordx4 stores (whole lines
  // instead of ~10 % scattered dword stores); non-hit slots get a sentinel
  if (inv && hit) {
    uint4* ip = reinterpret_cast<uint4*>(inv + base);
#pragma unroll
    for (int j = 0; j < kCompactItems / 4; ++j)
      ip[j] = make_uint4(iv[4 * j], iv[4 * j + 1], iv[4 * j + 2], iv[4 * j + 3]);
  }
  // rebuild decided by k_compact_scan: free this thread's slots of the new
  // capacity (its own slots, already read above)
  const u64 fresh = sv.ctl ? (u64)sv.ctl[2] : 0ull;
  if (base < fresh) {
    ulonglong2* kp = reinterpret_cast<ulonglong2*>(sv.keys + base);
#pragma unroll
    for (int j = 0; j < kCompactItems / 2; ++j) kp[j] = make_ulonglong2(kEmptyKey, kEmptyKey);
  }
}

// Unique-index positions (the fused single-rank step): each occurrence's
// scratch slot becomes its index in the batch's unique list (inv, written by
// the compaction), the trash slot's occurrences get `none`.  Pulled rows,
// gradient destinations (unique * S + s) and the unique-order outputs then
// share one dense index space: the reductions span the batch's unique keys
// instead of the 4x-headroom scratch capacity, the pulled rows are 4x denser
// in the caches, and no slot -> unique map is read at the output.  Four
// occurrences per lane (dwordx4 in and out, four independent gathers: 39.7 us
// per 10.2 M occurrences; sixteen per lane measured 44.7 us).
constexpr int kRemapPer = 4;

__global__ void __launch_bounds__(kBlock) k_remap_pos(u32* __restrict__ pos, int64_t nnz,
                                                      const u32* __restrict__ inv, u32 none) {
  const int64_t i = ((int64_t)blockIdx.x * kBlock + threadIdx.x) * kRemapPer;
  auto map = [&](u32 u) { return u == 0xFFFFFFFFu ? none : u; };
  if (i + kRemapPer <= nnz) {
    uint4 p[kRemapPer / 4];
#pragma unroll
    for (int q = 0; q < kRemapPer / 4; ++q) p[q] = reinterpret_cast<const uint4*>(pos + i)[q];
    u32 u[kRemapPer];
#pragma unroll
    for (int q = 0; q < kRemapPer / 4; ++q) {
      u[4 * q] = inv[p[q].x];
      u[4 * q + 1] = inv[p[q].y];
      u[4 * q + 2] = inv[p[q].z];
      u[4 * q + 3] = inv[p[q].w];
    }
#pragma unroll
    for (int q = 0; q < kRemapPer / 4; ++q)
      reinterpret_cast<uint4*>(pos + i)[q] =
          make_uint4(map(u[4 * q]), map(u[4 * q + 1]), map(u[4 * q + 2]), map(u[4 * q + 3]));
  } else {
    for (int64_t j = i; j < nnz; ++j) pos[j] = map(inv[pos[j]]);
  }
}

void launch_remap_pos(u32* pos, int64_t nnz, const u32* inv, u32 none, hipStream_t st) {
  if (nnz <= 0) return;
  if (reinterpret_cast<uintptr_t>(pos) & 15) throw std::runtime_error("remap_pos: pos must be 16-byte aligned");
  const int64_t lanes = (nnz + kRemapPer - 1) / kRemapPer;
  hipLaunchKernelGGL(k_remap_pos, dim3((unsigned)((lanes + kBlock - 1) / kBlock)), dim3(kBlock), 0,
                     st, pos, nnz, inv, none);
  XF_HIP_CHECK(hipGetLastError());
}

// Owner-partitioned dedup: the unique list is in slot order, so owner o's
// keys start at the number of stamped slots below o*R = the compaction offset
// of the chunk holding o*R plus the hits in that chunk below it (one wave per
// boundary, 64 slots per lane).  counts[o] = start[o+1] - start[o].
constexpr int kPartBlock = 1024;

__global__ void __launch_bounds__(kPartBlock) k_partition_counts(
    ScratchView sv, const unsigned int* __restrict__ offs, const int64_t* __restrict__ n_uniq,
    int64_t* __restrict__ counts, int64_t seq) {
  __shared__ int64_t start[kMaxParts + 1];
  const u32 parts = (u32)sv.parts;
  const u64 R = batch_cap(sv) / parts;
  const int lane = threadIdx.x % kWave, w = threadIdx.x / kWave;
  for (u32 o = w; o <= parts; o += kPartBlock / kWave) {
    if (o == 0 || o == parts) {
      if (lane == 0) start[o] = o == 0 ? 0 : *n_uniq;
      continue;
    }
    const u64 b = (u64)o * R, c = b / kCompactChunk, c0 = c * kCompactChunk;
    unsigned int hits = 0;
    for (u64 q = c0 + (u64)lane * 64; q < c0 + (u64)lane * 64 + 64; ++q)
      hits += (q < b && sv.stamps[q] == (unsigned char)sv.epoch) ? 1u : 0u;
#pragma unroll
    for (int d = 32; d > 0; d >>= 1) hits += __shfl_xor(hits, d);
    if (lane == 0) start[o] = (int64_t)offs[c] + hits;
  }
  __syncthreads();
  for (u32 o = threadIdx.x; o < parts; o += kPartBlock) {
    XF_DASSERT(start[o + 1] >= start[o]);
    const int64_t c = start[o + 1] - start[o];
    counts[o] = seq >= 0 ? encode_count(c, seq) : c;
  }
}

void launch_partition_counts(const ScratchView& s, const u32* chunk_offsets,
                             const int64_t* n_uniq, int64_t* counts, int64_t seq, hipStream_t st) {
  if (s.parts < 2 || s.parts > kMaxParts) throw std::runtime_error("partition_counts: bad parts");
  hipLaunchKernelGGL(k_partition_counts, dim3(1), dim3(kPartBlock), 0, st, s, chunk_offsets,
                     n_uniq, counts, seq);
  XF_HIP_CHECK(hipGetLastError());
}

void launch_dedup(const u64* keys, int64_t nnz, ScratchView s, DedupOut o, hipStream_t st) {
  if (nnz <= 0) return;
  if (!s.ctl || s.grow > 0.0f) {
    // fixed capacity: threshold rebuild before the batch; adaptive: growth
    if (s.ctl) hipLaunchKernelGGL(k_scratch_grow, dim3(1), dim3(1), 0, st, s.ctl, s.cap, s.grow);
    hipLaunchKernelGGL(k_scratch_maybe_clear, dim3(grid_for((int64_t)s.cap)), dim3(kBlock), 0, st,
                       s.keys, s.cap, s.claims, s.rebuild_at, s.ctl);
    hipLaunchKernelGGL(k_scratch_claims_reset, dim3(1), dim3(1), 0, st, s.claims, s.rebuild_at,
                       s.ctl);
  }
  int g1 = (int)((nnz + kDedupChunk - 1) / kDedupChunk);
  hipLaunchKernelGGL(k_dedup_insert, dim3(g1), dim3(kBlock), 0, st, keys, nnz, s, o.pos,
                     o.overflow);
  if (!o.block_counts) throw std::runtime_error("dedup: block_counts workspace missing");
  // sized for the allocated capacity; blocks past the active one count zero
  int g2 = (int)((s.cap + kCompactChunk - 1) / kCompactChunk);
  hipLaunchKernelGGL(k_compact_count, dim3(g2), dim3(kBlock), 0, st, s, o.block_counts);
  hipLaunchKernelGGL(k_compact_scan, dim3(1), dim3(kScanBlock), 0, st, o.block_counts, g2,
                     reinterpret_cast<unsigned long long*>(o.n_uniq), s.claims, s.ctl, s.cap,
                     reinterpret_cast<unsigned long long*>(o.n_uniq_copy), o.cap_out, s.epoch);
  hipLaunchKernelGGL(k_compact_write, dim3(g2), dim3(kBlock), 0, st, s, o.block_counts,
                     o.uniq_keys, o.uniq_pos, o.inv);
  XF_HIP_CHECK(hipGetLastError());
}

// The persistent scratch needs no per-step reset (stamps expire with the
// epoch); kept as an explicit full clear for callers that want a cold table.
__global__ void k_scratch_reset(u64* __restrict__ skeys, const u32* __restrict__ pos,
                                const int64_t* n_dev, int64_t n_max) {
  int64_t n = dev_count(n_dev, n_max, n_max);
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
    skeys[pos[i]] = kEmptyKey;
}

void launch_scratch_reset(ScratchView s, const u32* pos, const int64_t* n_dev, int64_t n_max,
                          hipStream_t st) {
  if (n_max <= 0) return;
  hipLaunchKernelGGL(k_scratch_reset, dim3(grid_for(n_max)), dim3(kBlock), 0, st, s.keys, pos,
                     n_dev, n_max);
  XF_HIP_CHECK(hipGetLastError());
}

__global__ void k_fill_u64(u64* p, u64 v, size_t n) {
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) p[i] = v;
}

struct SmallBytes {
  unsigned char b[256];
};

__global__ void k_upload_small(unsigned char* __restrict__ dst, SmallBytes v, int n) {
  for (int i = threadIdx.x; i < n; i += blockDim.x) dst[i] = v.b[i];
}

void launch_upload_small(void* dst, const void* src, size_t bytes, hipStream_t st) {
  if (bytes == 0) return;
  if (bytes > sizeof(SmallBytes)) throw std::runtime_error("upload_small: at most 256 bytes");
  SmallBytes v;
  std::memcpy(v.b, src, bytes);
  hipLaunchKernelGGL(k_upload_small, dim3(1), dim3(64), 0, st, static_cast<unsigned char*>(dst),
                     v, (int)bytes);
  XF_HIP_CHECK(hipGetLastError());
}

// (e.g. the sharded step's split sizes into pinned memory: a copy-engine D2H
// left ~6 us of idle GPU behind it per step)
__global__ void k_download_small(unsigned char* __restrict__ dst,
                                 const unsigned char* __restrict__ src, int n) {
  for (int i = threadIdx.x; i < n; i += blockDim.x) dst[i] = src[i];
}

void launch_download_small(void* host_dst, const void* src, size_t bytes, hipStream_t st) {
  if (bytes == 0) return;
  if (bytes > (1u << 16)) throw std::runtime_error("download_small: at most 64 KB");
  hipLaunchKernelGGL(k_download_small, dim3(1), dim3(256), 0, st,
                     static_cast<unsigned char*>(host_dst), static_cast<const unsigned char*>(src),
                     (int)bytes);
  XF_HIP_CHECK(hipGetLastError());
}

__global__ void k_snapshot(HostSnap* dst, const u32* mon, unsigned long long seq) {
  store_snapshot(dst, mon, seq);
}

void launch_snapshot(HostSnap* dst, const u32* mon, unsigned long long seq, hipStream_t st) {
  hipLaunchKernelGGL(k_snapshot, dim3(1), dim3(64), 0, st, dst, mon, seq);
  XF_HIP_CHECK(hipGetLastError());
}

#define XF_APPLY_SNAPSHOT(a) \
  if ((a).snap) store_snapshot((a).snap, (a).snap_mon, (a).snap_seq)

void launch_fill_u64(u64* p, u64 v, size_t n, hipStream_t st) {
  if (n == 0) return;
  hipLaunchKernelGGL(k_fill_u64, dim3(grid_for((int64_t)n)), dim3(kBlock), 0, st, p, v, n);
  XF_HIP_CHECK(hipGetLastError());
}

__global__ void k_table_clear(TableView t) {
  const u64 stride = (u64)gridDim.x * blockDim.x;
  const int W = t.L.stride;
  for (u64 s = (u64)blockIdx.x * blockDim.x + threadIdx.x; s < t.cap; s += stride) {
    u32* sp = t.words + s * (u64)W;
    sp[0] = 0xFFFFFFFFu;
    sp[1] = 0xFFFFFFFFu;
    for (int w = 2; w < W; ++w) sp[w] = 0u;
  }
}

void launch_table_clear(const TableView& t, hipStream_t st) {
  hipLaunchKernelGGL(k_table_clear, dim3(grid_for((int64_t)t.cap)), dim3(kBlock), 0, st, t);
  XF_HIP_CHECK(hipGetLastError());
}

// ---------------------------------------------------------------------------
// persistent table probe
// ---------------------------------------------------------------------------
__device__ __forceinline__ u32 probe(const TableView& t, u64 key, bool insert, bool& claimed) {
  u64 s = table_home(t, fmix64(key));
  const int stride = t.L.stride;
  for (u64 n = 0; n < t.probe_limit; ++n) {
    u64* kp = reinterpret_cast<u64*>(t.words + s * (u64)stride);
    u64 cur = *kp;
    if (cur == key) return (u32)s;
    if (cur == kEmptyKey) {
      if (!insert) return kNoSlot;
      u64 prev = atomicCAS((unsigned long long*)kp, (unsigned long long)kEmptyKey,
                           (unsigned long long)key);
      if (prev == kEmptyKey) { claimed = true; return (u32)s; }
      if (prev == key) return (u32)s;
    }
    s = table_next(t, s);
  }
  // bounded chain (TableView::probe_limit): a key is never stored further out
  if (insert) *t.overflow = 1u;
  return kNoSlot;
}

// LR-FTRL fast path: 16-byte slots {key, n, z}; one dwordx4 load yields the
// key and the optimizer state together.  Each lane owns kPullItems keys spaced
// one block apart and issues all first-probe loads before resolving any (the
// table is tens of GB: every probe is an HBM miss, so memory-level parallelism
// is what matters).
//
// Line-at-a-time probing: the first round loads only the key's home slot (at
// low load it answers almost every probe); a chain that continues loads the
// REST of the aligned 64-byte line (up to 3 slots, independent dwordx4
// loads) in one round trip and resolves those probe positions from
// registers, then whole lines.  Same table layout and probe order as
// one-slot linear probing, but at a realistic load (0.47: a 1e9-key model in
// 2^31 slots) a chain costs one extra round trip per line, not per slot.
constexpr int kPullItems = 2;
constexpr int kPullChunk = kBlock * kPullItems;
constexpr int kLineSlots = 4;  // 16-byte slots per 64-byte line

__global__ void __launch_bounds__(kBlock) k_pull_lr16(TableView t, FtrlParams fp,
                                                      const u64* __restrict__ keys,
                                                      const int64_t* n_dev, int64_t n_host,
                                                      int64_t n_max, bool insert,
                                                      u32* __restrict__ out_slot,
                                                      float* __restrict__ out_vals,
                                                      const u32* __restrict__ out_map,
                                                      float2* __restrict__ out_nz,
                                                      float* __restrict__ zero_out) {
  const int64_t n = dev_count(n_dev, n_host, n_max);
  if ((int64_t)blockIdx.x * kPullChunk >= n) return;  // (grid sized by capacity)
  const u64 segm = (1ull << t.seg_log2) - 1;  // (chains wrap inside a segment)
  uint4* slots = reinterpret_cast<uint4*>(t.words);
  const int64_t base = (int64_t)blockIdx.x * kPullChunk + threadIdx.x;
  u64 key[kPullItems], s[kPullItems];
  uint4 v[kPullItems];
#pragma unroll
  for (int j = 0; j < kPullItems; ++j) {
    int64_t i = base + (int64_t)j * kBlock;
    key[j] = i < n ? sanitize_key(keys[i]) : 0ull;
    s[j] = table_home(t, fmix64(key[j]));
  }
#pragma unroll
  for (int j = 0; j < kPullItems; ++j) {
    int64_t i = base + (int64_t)j * kBlock;
    if (i < n) v[j] = slots[s[j]];
  }
  // output rows loaded up front too: after the first key's stores the
  // compiler could not hoist them (possible aliasing), one round trip each
  u32 orow[kPullItems];
#pragma unroll
  for (int j = 0; j < kPullItems; ++j) {
    int64_t i = base + (int64_t)j * kBlock;
    orow[j] = (out_map && i < n) ? out_map[i] : (u32)i;
  }
  unsigned int claims = 0;
#pragma unroll
  for (int j = 0; j < kPullItems; ++j) {
    int64_t i = base + (int64_t)j * kBlock;
    if (i >= n) continue;
    u32 slot = kNoSlot;
    float w = 0.0f;
    float2 nz = make_float2(0.0f, 0.0f);  // fresh slot: zero state
    u64 sj = s[j];
    int q0 = (int)(sj & (kLineSlots - 1)), q1 = q0 + 1;  // registers hold [q0, q1) of the line
    uint4 ln[kLineSlots];
#pragma unroll
    for (int q = 0; q < kLineSlots; ++q) ln[q] = v[j];  // (only ln[q0] is read in round one)
    bool done = false;
    // c = slots examined so far = probe distance of the round's first slot;
    // slots at distance >= probe_limit are never examined (bounded chains)
    for (u64 c = 0; c < t.probe_limit && !done;) {
#pragma unroll
      for (int q = 0; q < kLineSlots; ++q) {
        if (q < q0 || q >= q1 || done || c + (u64)(q - q0) >= t.probe_limit) continue;
        const u64 cur = (u64)ln[q].x | ((u64)ln[q].y << 32);
        const u64 sq = (sj & ~(u64)(kLineSlots - 1)) + (u64)q;
        if (cur == key[j]) {
          slot = (u32)sq;
          nz = make_float2(__uint_as_float(ln[q].z), __uint_as_float(ln[q].w));
          w = ftrl_weight(nz.y, nz.x, fp);
          done = true;
        } else if (cur == kEmptyKey) {
          if (!insert) {
            done = true;
          } else {
            const u64 prev = atomicCAS(reinterpret_cast<unsigned long long*>(&slots[sq]),
                                       (unsigned long long)kEmptyKey, (unsigned long long)key[j]);
            if (prev == kEmptyKey) {  // fresh slot: state is zero -> w = 0
              ++claims;
              slot = (u32)sq;
              done = true;
            } else if (prev == key[j]) {  // claimed by another lane this launch
              slot = (u32)sq;
              done = true;
            }
            // else: taken by another key meanwhile -- keep probing
          }
        }
      }
      if (done) break;
      c += (u64)(q1 - q0);
      // next: the rest of this line after the home slot, then whole lines --
      // every slot of a round is loaded at once (one dependent round trip)
      if (q1 < kLineSlots) {
        q0 = q1;
      } else {
        sj = (sj & ~segm) | (((sj | (u64)(kLineSlots - 1)) + 1) & segm);
        q0 = 0;
      }
      q1 = kLineSlots;
      const uint4* line = slots + (sj & ~(u64)(kLineSlots - 1));
#pragma unroll
      for (int q = 0; q < kLineSlots; ++q)
        if (q >= q0) ln[q] = line[q];
    }
    if (insert && slot == kNoSlot) *t.overflow = 1u;
    if (out_slot) out_slot[i] = slot;
    if (out_vals) out_vals[out_map ? (int64_t)orow[j] : i] = w;
    if (out_nz) out_nz[i] = nz;
    if (zero_out) zero_out[i] = 0.0f;  // (width 1: LR)
  }
  block_count_add<kBlock>(t.size, claims);
}

__global__ void __launch_bounds__(kBlock) k_pull_generic(PullArgs a) {
  int64_t n = dev_count(a.n_dev, a.n_host, a.n_max);
  const TableView& t = a.table;
  const TableLayout& L = t.L;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  unsigned int claims = 0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    u64 key = sanitize_key(a.keys[i]);
    bool claimed = false;
    u32 slot = probe(t, key, a.insert, claimed);
    claims += claimed;
    if (a.out_slot) a.out_slot[i] = slot;
    if (a.out_vals) {
      float* dst = a.out_vals + (size_t)(a.out_map ? a.out_map[i] : i) * a.pstride;
      if (slot == kNoSlot) {
        for (int p = 0; p < L.P; ++p) dst[p] = absent_weight(key, p, L, a.opt);
      } else {
        const u32* sp = t.words + (u64)slot * L.stride;
        for (int p = 0; p < L.P; ++p) dst[p] = slot_weight(sp, key, p, L, a.opt);
      }
    }
  }
  block_count_add<kBlock>(t.size, claims);
}

// Multi-parameter layouts (FM / MVM / SGD): phase 1 probes one key per lane
// (kPullItems keys in flight) and records the slot; phase 2 evaluates the
// pull values with a group of G lanes per key (G = pow2 >= pstride), so the
// slot's state words and the output row are read/written contiguously.
// Keys per lane (sequential chains): 2 measured +0.6 % over 4 and 1 on FM-8
// at table load 0.47; probing slot pairs per round trip -1.2 %
// (profiles/r2_s3_fm_pull_apply_pipeline.txt).  The grid is sized by the
// capacity, so blocks past the device count return at once.
constexpr int kProbeItems = 2;
__global__ void __launch_bounds__(kBlock) k_pull_probe(TableView t, const u64* __restrict__ keys,
                                                       const int64_t* n_dev, int64_t n_host,
                                                       int64_t n_max, bool insert,
                                                       u32* __restrict__ out_slot) {
  const int64_t n = dev_count(n_dev, n_host, n_max);
  const int64_t base = (int64_t)blockIdx.x * (kBlock * kProbeItems) + threadIdx.x;
  if ((int64_t)blockIdx.x * (kBlock * kProbeItems) >= n) return;  // (grid sized by capacity)
  unsigned int claims = 0;
#pragma unroll
  for (int j = 0; j < kProbeItems; ++j) {
    int64_t i = base + (int64_t)j * kBlock;
    if (i >= n) continue;
    bool claimed = false;
    out_slot[i] = probe(t, sanitize_key(keys[i]), insert, claimed);
    claims += claimed;
  }
  block_count_add<kBlock>(t.size, claims);
}

// Packed lane groups for the multi-parameter pull/apply: P lanes per key
// (lane p owns parameter p), floor(64/P) keys per wave, never straddling a
// wave.  In pow2 groups of 16 lanes these kernels were VALU-issue bound (FTRL
// closed form with IEEE division/sqrt, lazy N(0,1) init; PMC of the FM-8
// apply: 1626 VALU instructions per wave for 16 keys, 50 % of wave cycles
// waiting): packing 7 FM-8 keys (P = 9) into a wave is 1.75x fewer
// instructions per key.  Packed, they are bound by the dependent random row
// accesses instead (an apply fed the pull's weights, skipping the closed
// form, was slower), which RowPipe overlaps with the previous key's math.
struct PackedLane {
  int P, K, g, p;        // lanes per key, keys per wave, key in wave, param
  bool on;               // lane belongs to a key group (64 % P lanes idle)
  int64_t first, stride;  // key index of this lane's group, grid stride in keys
};

__device__ __forceinline__ PackedLane packed_lane(int P) {
  PackedLane r;
  r.P = P;
  r.K = kWave / P;
  const int lane = threadIdx.x % kWave;
  r.g = lane / P;
  r.p = lane - r.g * P;
  r.on = r.g < r.K;
  const int64_t waves = (int64_t)(blockDim.x / kWave);
  r.first = ((int64_t)blockIdx.x * waves + threadIdx.x / kWave) * r.K + r.g;
  r.stride = (int64_t)gridDim.x * waves * r.K;
  return r;
}

// One key's slot words a lane of its packed group needs (key, pushed flag,
// the lane's param state), loaded one grid-stride iteration ahead of use by
// the multi-parameter pull/apply: with the slot index loaded two ahead, the
// random row access of iteration t+1 is in flight while iteration t computes.
struct RowPre {
  u64 key = 0;
  u32 flag = 1;
  float s0 = 0.0f, s1 = 0.0f;  // FTRL (n, z); SGD w
};

__device__ __forceinline__ RowPre row_pre(const u32* __restrict__ words, u32 slot, int p,
                                          const TableLayout& L) {
  RowPre r;
  if (slot == kNoSlot) return r;
  const u32* sp = words + (u64)slot * L.stride;
  r.key = *reinterpret_cast<const u64*>(sp);
  if (L.has_flag) r.flag = sp[L.flag_word];
  if (L.opt == kFTRL) {
    const float2 nz = *reinterpret_cast<const float2*>(sp + 2 + 2 * p);
    r.s0 = nz.x;
    r.s1 = nz.y;
  } else {
    r.s0 = __uint_as_float(sp[2 + p]);
  }
  return r;
}

// The same words from the pull's stash (PullArgs::out_nz, FTRL): entry i's
// (n, z) of param p at [i * P + p], n < 0 marking a key never pushed; the
// key from the unique list.  Coalesced, unlike the slot's row.
__device__ __forceinline__ RowPre row_stash(const float2* __restrict__ stash,
                                            const u64* __restrict__ keys, int64_t i, int p,
                                            int P) {
  RowPre r;
  const float2 nz = stash[(size_t)i * P + p];
  r.key = keys[i];
  r.flag = nz.x >= 0.0f ? 1u : 0u;
  r.s0 = nz.x >= 0.0f ? nz.x : 0.0f;
  r.s1 = nz.y;
  return r;
}

// Grid-stride pipeline over a packed group's keys: slots two iterations
// ahead, row words one ahead (RowPre) -- from the slot's row, or from the
// pull's stash when the caller sets `stash` (and `keys`).
struct RowPipe {
  int64_t stride, n;
  u32 s_cur, s_nx;
  RowPre r_nx;
  const float2* stash = nullptr;
  const u64* keys = nullptr;
  __device__ __forceinline__ RowPre row(const u32* words, u32 slot, int64_t i, int p,
                                        const TableLayout& L) const {
    return stash ? row_stash(stash, keys, i, p, L.P) : row_pre(words, slot, p, L);
  }
  __device__ __forceinline__ void start(const u32* __restrict__ slots, const u32* words,
                                        int64_t i, int p, const TableLayout& L) {
    s_cur = i < n ? slots[i] : kNoSlot;
    s_nx = i + stride < n ? slots[i + stride] : kNoSlot;
    if (i < n) r_nx = row(words, s_cur, i, p, L);
  }
  // at the top of iteration i: returns (slot, row) of i, issues i + stride's
  // row loads and i + 2 * stride's slot load
  __device__ __forceinline__ u32 next(const u32* __restrict__ slots, const u32* words, int64_t i,
                                      int p, const TableLayout& L, RowPre& r) {
    const u32 slot = s_cur;
    r = r_nx;
    s_cur = s_nx;
    if (i + stride < n) r_nx = row(words, s_cur, i + stride, p, L);
    if (i + 2 * stride < n) s_nx = slots[i + 2 * stride];
    return slot;
  }
};

__global__ void __launch_bounds__(kBlock) k_pull_values(PullArgs a) {
  const int64_t n = dev_count(a.n_dev, a.n_host, a.n_max);
  const TableLayout& L = a.table.L;
  const PackedLane pl = packed_lane(L.P);
  const int p = pl.p;
  const int gbase = (threadIdx.x % kWave) - p;  // lane of the group's param 0
  // (a key group's lanes share i: the group-uniform loop keeps them together
  // through the shuffles; idle lanes run no iteration)
  int64_t i = pl.on ? pl.first : n;
  RowPipe pipe;
  pipe.stride = pl.stride;
  pipe.n = n;
  pipe.start(a.out_slot, a.table.words, i, p, L);
  // the output row index one iteration ahead as well: loaded after this
  // iteration's stores it would wait for them (gfx9 vmcnt counts stores)
  u32 om_nx = (a.out_map && i < n) ? a.out_map[i] : 0u;
  for (; i < n; i += pl.stride) {
    RowPre rp;
    const u32 slot = pipe.next(a.out_slot, a.table.words, i, p, L, rp);
    const u32 om = om_nx;
    if (a.out_map && i + pl.stride < n) om_nx = a.out_map[i + pl.stride];
    float v;
    if (slot == kNoSlot) {
      v = absent_weight(sanitize_key(a.keys[i]), p, L, a.opt);
    } else {
      v = state_weight(rp.key, rp.flag != 0u, rp.s0, rp.s1, p, L, a.opt);
    }
    if (a.out_nz)  // the apply's stash (FTRL): (n, z), n = -1 for a key never pushed
      reinterpret_cast<float2*>(a.out_nz)[(size_t)i * L.P + p] =
          make_float2(slot != kNoSlot && rp.flag ? rp.s0 : -1.0f, slot != kNoSlot ? rp.s1 : 0.0f);
    if (a.out_w) {
      a.out_w[(size_t)i * a.pstride + p] = v;
      for (int c = L.P + p; c < a.pstride; c += L.P) a.out_w[(size_t)i * a.pstride + c] = 0.0f;
    }
    if (a.zero_out)
      for (int c = p; c < a.zero_width; c += L.P) a.zero_out[(size_t)i * a.zero_width + c] = 0.0f;
    if (!a.out_vals) continue;
    const size_t row = a.out_map ? (size_t)om : (size_t)i;
    if (a.fm_vals) {
      // (w, Σ_k v_k, Σ_k v_k^2) of the key, summed in param order by lane 0
      float sv = 0.0f, qv = 0.0f;
      for (int j = L.p_w; j < L.P; ++j) {
        const float x = __shfl(v, gbase + j);
        sv += x;
        qv += x * x;
      }
      if (p == 0) reinterpret_cast<float4*>(a.out_vals)[row] = make_float4(v, sv, qv, 0.0f);
    } else {
      a.out_vals[row * a.pstride + p] = v;
      for (int c = L.P + p; c < a.pstride; c += L.P) a.out_vals[row * a.pstride + c] = 0.0f;
    }
  }
}

// grid for packed groups: one key per group up to the cap
static int packed_grid(int64_t n, int P) {
  const int64_t keys_per_block = (int64_t)(kBlock / kWave) * (kWave / P);
  const int64_t g = (n + keys_per_block - 1) / keys_per_block;
  return (int)(g < 1 ? 1 : (g < kGroupGridCap ? g : kGroupGridCap));
}


void launch_table_pull(const PullArgs& a, hipStream_t st) {
  if (a.n_max <= 0) return;
  const TableLayout& L = a.table.L;
  int grid = grid_for(a.n_dev ? a.n_max : a.n_host);
  if (L.stride == 4 && L.P == 1 && L.opt == kFTRL && !L.has_flag) {
    if (a.zero_out && a.zero_width != 1) throw std::runtime_error("table_pull: zero_width");
    int64_t nm = a.n_dev ? a.n_max : a.n_host;
    int g = (int)((nm + kPullChunk - 1) / kPullChunk);
    hipLaunchKernelGGL(k_pull_lr16, dim3(g > 0 ? g : 1), dim3(kBlock), 0, st, a.table, a.opt.ftrl, a.keys,
                       a.n_dev, a.n_host, a.n_max, a.insert, a.out_slot, a.out_vals, a.out_map,
                       reinterpret_cast<float2*>(a.out_nz), a.zero_out);
  } else if (a.out_slot && a.pstride >= 2 && L.P <= kWave) {
    if (a.fm_vals && L.P < 2) throw std::runtime_error("fm_vals: bad layout");
    const int64_t nm = a.n_dev ? a.n_max : a.n_host;
    const int g1 = (int)((nm + kBlock * kProbeItems - 1) / (kBlock * kProbeItems));
    hipLaunchKernelGGL(k_pull_probe, dim3(g1 > 0 ? g1 : 1), dim3(kBlock), 0, st, a.table, a.keys,
                       a.n_dev, a.n_host, a.n_max, a.insert, a.out_slot);
    if (a.out_vals || a.out_w || a.zero_out) {
      // one key per lane group where possible: the grid-stride iterations of
      // a group are dependent random-access chains (latency bound)
      hipLaunchKernelGGL(k_pull_values, dim3(packed_grid(nm, L.P)), dim3(kBlock), 0, st, a);
    }
  } else {
    if (a.fm_vals || a.out_w) throw std::runtime_error("table_pull: fm_vals/out_w need the group path");
    hipLaunchKernelGGL(k_pull_generic, dim3(grid), dim3(kBlock), 0, st, a);
  }
  XF_HIP_CHECK(hipGetLastError());
}

// ---------------------------------------------------------------------------
// apply (push)
// ---------------------------------------------------------------------------
// The reference divides a float sum by the row count in double and rounds to
// float (lr_worker.cc:116-118).  For a float x and an integer n < 2^24 (exact
// in float) that equals the correctly rounded float quotient x / n: double
// rounding is innocuous for division when the wide format has >= 2p+2 bits
// (53 >= 2*24+2), so the f64 division sequence is replaced by the f32 one.
__device__ __forceinline__ float norm_grad(float raw, const int32_t* slice_rows, int s) {
  if (!slice_rows) return raw;
  const int32_t r = slice_rows[s];
  return r < (1 << 24) ? raw / (float)r : (float)((double)raw / (double)r);
}

// LR-FTRL, one slice, 16-byte slots: read (n,z) as one dwordx2, write it back.
// One key per lane, grid-stride: measured faster than issuing four keys per
// lane up front (54 vs 49 us for 850 K keys) -- twice the waves in flight hide
// the dependent slot -> state chain better than per-lane ILP.
template <bool kSlices>
__global__ void __launch_bounds__(kBlock) k_apply_lr16(ApplyArgs a) {
  XF_APPLY_SNAPSHOT(a);
  int64_t n = dev_count(a.n_dev, a.n_host, a.n_max);
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const FtrlParams fp = a.opt.ftrl;
  if constexpr (kSlices) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
      // unique-order [key][slice] normalised sums: the present slices' pushes
      // in slice order (the CPU backend's Hogwild order); a key no slice of
      // this group touched is skipped before any table access
      const u32 m0 = a.masks[i];
      if (!m0) continue;
      if (a.masks_clear) const_cast<u32*>(a.masks)[i] = 0u;
      u32 slot = a.slots[i];
      if (slot == kNoSlot) continue;
      float2* st = reinterpret_cast<float2*>(a.table.words + (u64)slot * 4 + 2);
      // (the pull's stash for the step's first group; later groups read the
      // state the earlier ones wrote)
      float2 nz = a.nz_stash ? reinterpret_cast<const float2*>(a.nz_stash)[i] : *st;
      const float* g = a.grads + (size_t)i * a.S;
      float sn = sqrtf(nz.x);
      for (u32 m = m0; m; m &= m - 1) {
        const float w = ftrl_weight_sn(nz.y, sn, fp);
        ftrl_push_sn(nz.x, nz.y, sn, w, g[__ffs(m) - 1], fp);
      }
      *st = nz;
    }
  } else {
    // the next key's loads are issued before this key's stores: on gfx9
    // vmcnt also counts stores, so a load issued after them would wait for
    // their completion as well
    struct In {
      u32 slot, row;
      float raw;
      float2 nz;
    };
    auto load = [&](int64_t i) {
      In x;
      x.slot = a.slots[i];
      x.row = a.grad_map ? a.grad_map[i] : (u32)i;
      x.raw = a.grads[x.row];
      x.nz = make_float2(0.0f, 0.0f);
      if (x.slot != kNoSlot)
        x.nz = a.nz_stash ? reinterpret_cast<const float2*>(a.nz_stash)[i]
                          : *reinterpret_cast<const float2*>(a.table.words + (u64)x.slot * 4 + 2);
      return x;
    };
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    In nx;
    if (i < n) nx = load(i);
    for (; i < n; i += stride) {
      const In x = nx;
      if (i + stride < n) nx = load(i + stride);
      if (a.zero_after) a.grads[x.row] = 0.0f;
      if (a.reset_pos) a.scratch.keys[a.reset_pos[i]] = kEmptyKey;
      if (x.slot == kNoSlot) continue;
      float2 nz = x.nz;
      const float w = ftrl_weight(nz.y, nz.x, fp);
      const float g = norm_grad(x.raw, a.slice_rows, 0);
      ftrl_push(nz.x, nz.y, w, g, fp);
      *reinterpret_cast<float2*>(a.table.words + (u64)x.slot * 4 + 2) = nz;
    }
  }
}

// LR-FTRL, 16-byte slots, CSR gradients (ApplyArgs::csr_*, one launch for
// every slice of the step): a key's entries are its slices' normalised sums in
// slice order -- the reference's per-slice pushes of only the keys a slice
// touched (lr_worker.cc:162-175) -- applied as a chain on (n, z) held in
// registers (sqrt(n) carried), the slot written once.  The first entries of
// the next keys are loaded before this key's chain.
constexpr int kCsrChunk = 8;  // CSR entries a lane loads at once
// Chains longer than this run in a second launch over the deferred keys
constexpr u32 kCsrShortChain = 16;

// Wave-private deferral lists (ApplyArgs::csr_long): wave w of a launch of W
// waves owns [W + w * R, W + (w + 1) * R) (R = the keys one wave visits, kpi
// per iteration of the grid-stride loop) and writes its count to [w]; the
// second launch has the same grid and takes its own wave's list -- no global
// counter (a single one serialised ~10^4 atomics per step at one L2 channel)
struct CsrDefer {
  u32* list = nullptr;
  u32 gw = 0, waves = 0;
  u64 R = 0;
  __device__ __forceinline__ CsrDefer(u32* l, int64_t n_max, int64_t stride, int kpi) : list(l) {
    gw = blockIdx.x * (blockDim.x / kWave) + threadIdx.x / kWave;
    waves = gridDim.x * (blockDim.x / kWave);
    R = (u64)kpi * (u64)((n_max + stride - 1) / stride);
  }
  __device__ __forceinline__ u32* region() const { return list + waves + (u64)gw * R; }
};
// After the first pass the counts are scanned into offsets (waves + 1) and
// the regions gathered into one dense list, so the second pass packs 64 long
// chains per wave (a wave-private list holds ~2 of them: lanes idle)
struct CsrDense {
  const u32* offs;
  const u32* list;
  __device__ __forceinline__ CsrDense(const u32* l, const CsrDefer& d)
      : offs(l + d.waves + (u64)d.waves * d.R), list(offs + d.waves + 1) {}
};

// one wave per source region: its deferred keys to their dense positions
__global__ void __launch_bounds__(kBlock) k_csr_gather(u32* __restrict__ l, int64_t n_max,
                                                       int64_t stride, int kpi, u32 waves) {
  const u32 w = blockIdx.x * (kBlock / kWave) + threadIdx.x / kWave;
  if (w >= waves) return;
  const u64 R = (u64)kpi * (u64)((n_max + stride - 1) / stride);
  const u32* offs = l + waves + (u64)waves * R;
  u32* dense = const_cast<u32*>(offs) + waves + 1;
  const u32* src = l + waves + (u64)w * R;
  const u32 c = l[w], o = offs[w];
  for (u32 k = lane_id(); k < c; k += kWave) dense[o + k] = src[k];
}

// kLong: the second launch (entries of the deferred list), else the first
template <bool kLong>
__global__ void __launch_bounds__(kBlock) k_apply_lr16_csr(ApplyArgs a) {
  if (!kLong) XF_APPLY_SNAPSHOT(a);
  const int64_t stride0 = (int64_t)gridDim.x * blockDim.x;
  const CsrDefer df(a.csr_long, a.n_max, stride0, kWave);
  __shared__ u32 s_def[kBlock / kWave];
  const int wib = threadIdx.x / kWave, lane = lane_id();
  if (!kLong && lane == 0) s_def[wib] = 0u;
  // (pass 2: the dense list of every wave's deferred keys, csr_dense)
  const CsrDense dn(a.csr_long, df);
  const int64_t n = kLong ? (int64_t)dn.offs[df.waves] : dev_count(a.n_dev, a.n_host, a.n_max);
  const u32* __restrict__ lst = dn.list;
  const int64_t stride = stride0;
  const FtrlParams fp = a.opt.ftrl;
  const u64* __restrict__ ent = static_cast<const u64*>(a.csr_ent);
  struct In {
    u32 key, slot, off, cnt;
    u64 e0;
    float2 nz;
  };
  auto load = [&](int64_t j) {
    In x;
    const int64_t i = kLong ? (int64_t)lst[j] : j;
    x.key = (u32)i;
    x.slot = a.slots[i];
    x.off = a.csr_off[i];
    x.cnt = a.csr_cnt[i];
    x.e0 = x.cnt ? ent[x.off] : 0ull;
    x.nz = make_float2(0.0f, 0.0f);
    if (x.slot != kNoSlot && x.cnt && (kLong || !a.csr_long || x.cnt <= kCsrShortChain))
      x.nz = a.nz_stash ? reinterpret_cast<const float2*>(a.nz_stash)[i]
                        : *reinterpret_cast<const float2*>(a.table.words + (u64)x.slot * 4 + 2);
    return x;
  };
  // (pass 2: few keys -- the hot ones -- each a long latency-bound chain:
  // consecutive keys go to consecutive workgroups, so they spread over every
  // CU and several waves share each SIMD, instead of packing 64 per wave
  // onto the first few CUs)
  int64_t i = kLong ? (int64_t)threadIdx.x * gridDim.x + blockIdx.x
                    : (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  In nx;
  if (i < n) nx = load(i);
  for (; i < n; i += stride) {
    const In x = nx;
    if (i + stride < n) nx = load(i + stride);
    if (!kLong && a.csr_long && x.slot != kNoSlot && x.cnt > kCsrShortChain) {
      df.region()[atomicAdd(&s_def[wib], 1u)] = x.key;  // (LDS counter of this wave)
      continue;
    }
    if (x.slot == kNoSlot || !x.cnt) continue;
    float2 nz = x.nz;
    float sn = sqrtf(nz.x);
    auto push = [&](u64 e) {
      const float w = ftrl_weight_sn(nz.y, sn, fp);
      ftrl_push_sn(nz.x, nz.y, sn, w, __uint_as_float((u32)(e >> 32)), fp);
    };
    push(x.e0);
    // the chain's values (the entries' high words) C at a time, all C loads
    // in flight together: indices past the chain are clamped to its last
    // entry, not predicated -- a predicated load is a branch around it and
    // the compiler then waits on each one before the next
    const u32* __restrict__ hv = reinterpret_cast<const u32*>(ent) + 1;
    const u32 last = x.off + x.cnt - 1;
    auto chain = [&](auto cc) {
      constexpr int C = decltype(cc)::value;
      for (u32 j = 1; j < x.cnt; j += C) {
        float e[C];
#pragma unroll
        for (int q = 0; q < C; ++q) e[q] = __uint_as_float(hv[2 * (u64)min(x.off + j + q, last)]);
#pragma unroll
        for (int q = 0; q < C; ++q)
          if (j + q < x.cnt) {
            const float w = ftrl_weight_sn(nz.y, sn, fp);
            ftrl_push_sn(nz.x, nz.y, sn, w, e[q], fp);
          }
      }
    };
    if (!kLong) chain(std::integral_constant<int, 4>());
    else chain(std::integral_constant<int, kCsrChunk>());
    *reinterpret_cast<float2*>(a.table.words + (u64)x.slot * 4 + 2) = nz;
  }
  // (every lane has left the loop: lane 0, the wave's last, saw every defer)
  if (!kLong && a.csr_long && lane == 0) a.csr_long[df.gw] = s_def[wib];
}

__global__ void __launch_bounds__(kBlock) k_apply_generic(ApplyArgs a) {
  XF_APPLY_SNAPSHOT(a);
  int64_t n = dev_count(a.n_dev, a.n_host, a.n_max);
  const TableView& t = a.table;
  const TableLayout& L = t.L;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const int S = a.S, ps = a.pstride, P = a.P;
  const u32 all = (S >= 32) ? 0xFFFFFFFFu : ((1u << S) - 1u);
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    u32 slot = a.slots[i];
    u32 row = a.grad_map ? a.grad_map[i] : (u32)i;
    float* g = a.grads + (size_t)row * S * ps;
    u32 m = a.masks ? a.masks[row] : all;
    if (slot != kNoSlot) {
      u32* sp = t.words + (u64)slot * L.stride;
      u64 key = *reinterpret_cast<u64*>(sp);
      if (a.sum_slices) {
        for (int p = 0; p < P; ++p) {
          float acc = 0.0f;
          for (int s = 0; s < S; ++s)
            if (m & (1u << s)) acc += norm_grad(g[s * ps + p], a.slice_rows, s);
          slot_push(sp, key, p, acc, L, a.opt);
        }
        if (L.has_flag) sp[L.flag_word] = 1u;
      } else {
        for (int s = 0; s < S; ++s) {
          if (!(m & (1u << s))) continue;
          for (int p = 0; p < P; ++p)
            slot_push(sp, key, p, norm_grad(g[s * ps + p], a.slice_rows, s), L, a.opt);
          if (L.has_flag) sp[L.flag_word] = 1u;
        }
      }
    }
    if (a.zero_after) {
      for (int j = 0; j < S * ps; ++j) g[j] = 0.0f;
      if (a.masks_rw) a.masks_rw[row] = 0u;
    }
    if (a.reset_pos) a.scratch.keys[a.reset_pos[i]] = kEmptyKey;
  }
}

// ---- one-launch multi-source apply (ApplyArgs::grp) ------------------------
__device__ __forceinline__ int group_src(const SrcGroups& g, int64_t i) {
  int s = 0;
  while (s + 1 < g.nsrc && i >= g.offs[s + 1]) ++s;
  return s;
}

// Entry i leads its key when no earlier source sent the key this step; then
// row = the key's (slot, source) registrations and src0 = i's source.
__device__ __forceinline__ bool group_leader(const SrcGroups& g, int64_t i, const u64*& row,
                                             int& src0) {
  const u32 so = g.opos[i];
  if (so == kNoSlot) return false;  // owner scratch overflow (flagged by k_owner_group)
  row = g.oidx + (u64)so * (u64)g.nsrc;
  src0 = group_src(g, i);
  for (int s = 0; s < src0; ++s)
    if ((u32)(row[s] >> 32) == g.epoch) return false;
  return true;
}

// Registration of every received entry under (owner-scratch slot of its key,
// source).  The owner scratch persists across steps (hot keys keep their
// slot); stale registrations carry older epochs.
__global__ void __launch_bounds__(kBlock) k_owner_group(OwnerGroupArgs a) {
  const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (i >= a.n) return;
  const u64 key = sanitize_key(a.keys[i]);
  const u64 mask = a.ocap - 1;
  u64 s = fmix64(key) & mask;
  u32 slot = kNoSlot;
  for (u64 c = 0; c < a.ocap; ++c) {
    const u64 cur = a.okeys[s];
    if (cur == key) {
      slot = (u32)s;
      break;
    }
    if (cur == kEmptyKey) {
      const u64 prev = atomicCAS(reinterpret_cast<unsigned long long*>(&a.okeys[s]),
                                 (unsigned long long)kEmptyKey, (unsigned long long)key);
      if (prev == kEmptyKey || prev == key) {
        slot = (u32)s;
        break;
      }
    }
    s = (s + 1) & mask;
  }
  a.opos[i] = slot;
  if (slot == kNoSlot) {
    *a.overflow = 1u;
    return;
  }
  a.oidx[(u64)slot * (u64)a.g.nsrc + (u64)group_src(a.g, i)] = ((u64)a.g.epoch << 32) | (u32)i;
}

void launch_owner_group(const OwnerGroupArgs& a, hipStream_t st) {
  if (a.n <= 0) return;
  if (a.g.nsrc < 1 || a.g.nsrc > kMaxGroupSources) throw std::runtime_error("owner_group: nsrc");
  if (a.ocap == 0 || (a.ocap & (a.ocap - 1))) throw std::runtime_error("owner_group: ocap");
  hipLaunchKernelGGL(k_owner_group, dim3((unsigned)((a.n + kBlock - 1) / kBlock)), dim3(kBlock),
                     0, st, a);
  XF_HIP_CHECK(hipGetLastError());
}

// LR-FTRL, one slice, 16-byte slots, all sources in one launch: the leader
// entry of a key takes (n, z) from its pull stash (or the table), pushes each
// source's gradient in source order and writes the slot once.
__global__ void __launch_bounds__(kBlock) k_apply_lr16_multi(ApplyArgs a) {
  XF_APPLY_SNAPSHOT(a);
  const int64_t n = dev_count(a.n_dev, a.n_host, a.n_max);
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const FtrlParams fp = a.opt.ftrl;
  const SrcGroups& g = a.grp;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const u64* row;
    int src0;
    if (!group_leader(g, i, row, src0)) continue;
    const u32 slot = a.slots[i];
    if (slot == kNoSlot) continue;
    float2* st = reinterpret_cast<float2*>(a.table.words + (u64)slot * 4 + 2);
    float2 nz = a.nz_stash ? reinterpret_cast<const float2*>(a.nz_stash)[i] : *st;
    float sn = sqrtf(nz.x);
    for (int s = src0; s < g.nsrc; ++s) {
      const u64 v = row[s];
      if ((u32)(v >> 32) != g.epoch) continue;
      const float gr = a.grads[(u32)v];
      const float w = ftrl_weight_sn(nz.y, sn, fp);
      ftrl_push_sn(nz.x, nz.y, sn, w, gr, fp);
    }
    *st = nz;
  }
}

// Multi-parameter apply on packed lane groups (packed_lane: P lanes per key,
// lane p owns parameter p's optimizer state), so a wave touches a few
// contiguous slots instead of 64 scattered ones.  Every lane reads the
// "pushed" flag before lane 0 of the group writes it (one group never
// straddles a wave: program order); latent params use their lazy init value
// until the key's first push.  With a.grp (several sources) the group of a
// key's leader entry applies the (source, slice) contributions in that
// order; other entries skip.
// (7 waves per SIMD: <= 72 VGPRs without spills -- 77 at the default gave 6;
// 8 waves spills: FM-8 +1.7 % / -1 %, profiles/r2_s3_fm_pull_apply_pipeline.txt)
// kSl: a step of several slices (S > 1), whose keys take chains of pushes
template <bool kSl>
__global__ void __launch_bounds__(kBlock, 7) k_apply_group(ApplyArgs a) {
  XF_APPLY_SNAPSHOT(a);
  const int64_t n = dev_count(a.n_dev, a.n_host, a.n_max);
  const TableLayout& L = a.table.L;
  const int S = a.S, ps = a.pstride, gs = a.gstride ? a.gstride : ps;
  const u32 all = (S >= 32) ? 0xFFFFFFFFu : ((1u << S) - 1u);
  const PackedLane pl = packed_lane(L.P);
  const int p = pl.p;
  const bool multi = a.grp.oidx != nullptr;
  const bool ftrl = L.opt == kFTRL;
  int64_t i = pl.on ? pl.first : n;
  // (row words loaded an iteration ahead: another entry's slot -- keys are
  // unique per launch, and of a key's entries only the leader writes)
  RowPipe pipe;
  pipe.stride = pl.stride;
  pipe.n = n;
  if (ftrl && a.nz_stash) {  // (the pull's (n, z): the row is only written)
    pipe.stash = reinterpret_cast<const float2*>(a.nz_stash);
    pipe.keys = a.keys;
  }
  pipe.start(a.slots, a.table.words, i, p, L);
  // one source, one slice: the key's gradient row joins the pipeline too
  // (row index two iterations ahead, the lane's value(s) one ahead)
  const bool gpipe = !kSl && !multi && S == 1 && !a.masks && !a.sum_slices;
  auto grad_row = [&](int64_t k) -> u32 { return a.grad_map ? a.grad_map[k] : (u32)k; };
  auto grad_val = [&](u32 r) -> float2 {
    const float* g = a.grads + (size_t)r * gs;
    return a.fm_compact ? *reinterpret_cast<const float2*>(g) : make_float2(g[p], 0.0f);
  };
  u32 gr_cur = 0, gr_nx = 0;
  float2 gv_nx = make_float2(0.0f, 0.0f);
  if (gpipe && i < n) {
    gr_cur = grad_row(i);
    if (i + pl.stride < n) gr_nx = grad_row(i + pl.stride);
    gv_nx = grad_val(gr_cur);
  }
  for (; i < n; i += pl.stride) {
    RowPre rp;
    const u32 slot = pipe.next(a.slots, a.table.words, i, p, L, rp);
    float2 gv = make_float2(0.0f, 0.0f);
    u32 grow_i = 0;
    if (gpipe) {
      gv = gv_nx;
      grow_i = gr_cur;
      gr_cur = gr_nx;
      if (i + pl.stride < n) gv_nx = grad_val(gr_cur);
      if (i + 2 * pl.stride < n) gr_nx = grad_row(i + 2 * pl.stride);
    }
    const u64* grow = nullptr;
    int src0 = 0, nsrc = 1;
    if (multi) {
      if (!group_leader(a.grp, i, grow, src0)) continue;  // uniform over the key's lanes
      nsrc = a.grp.nsrc;
    }
    XF_DASSERT(slot == kNoSlot || slot < a.table.cap);
    if (slot != kNoSlot) {
      u32* sp = a.table.words + (u64)slot * L.stride;
      const u64 key = rp.key;
      bool pushed = rp.flag != 0u;
      float n0 = rp.s0, z0 = rp.s1;  // FTRL (n, z); SGD w
      // current weight; w_next caches it between pushes and is recomputed
      // only when another push follows (the closed form is the bulk of this
      // kernel's instructions: one push per key -- S = 1 -- evaluates it once)
      float w_next = state_weight(key, pushed, n0, z0, p, L, a.opt);
      bool stale = false;
      // (several slices: sqrtf(n) carried through the key's pushes)
      float sn = kSl && ftrl ? sqrtf(n0) : 0.0f;
      auto push = [&](float gv) {
        if constexpr (kSl) {
          if (stale) w_next = ftrl ? ftrl_weight_sn(z0, sn, a.opt.ftrl) : n0;
          if (ftrl) ftrl_push_sn(n0, z0, sn, w_next, gv, a.opt.ftrl);
          else n0 = w_next - a.opt.sgd.lr * gv;
        } else {
          if (stale) w_next = state_weight(key, true, n0, z0, p, L, a.opt);
          if (ftrl) ftrl_push(n0, z0, w_next, gv, a.opt.ftrl);
          else n0 = w_next - a.opt.sgd.lr * gv;
        }
        pushed = true;
        stale = true;
      };
      // compact reference-math FM rows (B, C): expand with the pre-step
      // (pulled) weight, the float recipe k_red_sum<2> uses for full rows
      const float w_pre = a.fm_compact ? (a.pulled ? a.pulled[(size_t)i * ps + p] : w_next) : 0.0f;
      u32 any = 0;
      if (gpipe) {
        any = 1u;
        const float raw = !a.fm_compact ? gv.x
                          : (p == 0 ? (float)a.fm_D * gv.x : gv.y - w_pre * gv.x);
        push(norm_grad(raw, a.slice_rows, 0));
        nsrc = 0;  // (the per-source loop below is skipped)
      }
      for (int sc = src0; sc < nsrc; ++sc) {
        u32 e = (u32)i;
        if (multi) {
          const u64 v = grow[sc];
          if ((u32)(v >> 32) != a.grp.epoch) continue;
          e = (u32)v;
        }
        const u32 row = a.grad_map ? a.grad_map[e] : e;
        const float* g = a.grads + (size_t)row * S * gs;
        const u32 m = a.masks ? a.masks[row] : all;
        if (a.masks_clear && p == 0) const_cast<u32*>(a.masks)[row] = 0u;
        any |= m;
        auto raw_of = [&](int s) -> float {
          if (!a.fm_compact) return g[s * gs + p];
          const float Bv = g[s * gs], Cv = g[s * gs + 1];
          return p == 0 ? (float)a.fm_D * Bv : Cv - w_pre * Bv;
        };
        if (a.sum_slices) {
          float acc = 0.0f;
          for (int s = 0; s < S; ++s)
            if (m & (1u << s)) acc += norm_grad(raw_of(s), a.slice_rows, s);
          if (m) push(acc);
        } else {
          for (int s = 0; s < S; ++s)
            if (m & (1u << s)) push(norm_grad(raw_of(s), a.slice_rows, s));
        }
      }
      if (ftrl) *reinterpret_cast<float2*>(sp + 2 + 2 * p) = make_float2(n0, z0);
      else sp[2 + p] = __float_as_uint(n0);
      if (L.has_flag && p == 0 && any) sp[L.flag_word] = 1u;
    }
    if (!multi && a.zero_after) {
      const u32 row = gpipe ? grow_i : (a.grad_map ? a.grad_map[i] : (u32)i);
      float* g = a.grads + (size_t)row * S * gs;
      const int w = a.fm_compact ? 2 : ps;
      for (int s = 0; s < S; ++s)
        for (int c = p; c < w; c += L.P) g[s * gs + c] = 0.0f;
      if (p == 0 && a.masks_rw) a.masks_rw[row] = 0u;
    }
  }
}

// CSR apply of compact reference-FM rows on packed lane groups (P lanes per
// key, lane p owns param p): the key's entries (slice, B, C), normalised by
// the reduction, expand with its pre-step weight (g_w = D*B, g_v = C - v*B,
// fm_worker.cc:126-157) and push in slice order.  The key's lanes load its
// entries cooperatively -- lane p holds entry c*P + p of chunk c, each push
// takes (B, C) from lane q % P by ds_bpermute -- so a chain of cnt entries
// costs ceil(cnt / P) loads, the next chunk in flight while one is consumed,
// instead of cnt dependent loads per lane.  Two-stage pipeline over the
// grid-stride loop: slot and (off, cnt) two iterations ahead, the row words
// and the first chunk one ahead.  kLong: the second launch, over the dense
// list of the deferred long chains.
// kRows (standard FM, ApplyArgs::csr_ew): full-row entries (slice, g_0 ..
// g_{P-1}) -- lane p reads its own component, kCsrRowChunk entries at a time
// (clamped, all in flight), the key's lanes together one entry's row.
constexpr int kCsrRowChunk = 4;
template <bool kLong, bool kRows = false>
__global__ void __launch_bounds__(kBlock) k_apply_group_csr(ApplyArgs a) {
  if (!kLong) XF_APPLY_SNAPSHOT(a);
  const TableLayout& L = a.table.L;
  const int ps = a.pstride;
  const PackedLane pl = packed_lane(L.P);
  const CsrDefer cdf(a.csr_long, a.n_max, pl.stride, pl.K);
  const CsrDense dn(a.csr_long, cdf);
  __shared__ u32 s_def[kBlock / kWave];
  const int wib = threadIdx.x / kWave;
  if (!kLong && a.csr_long && lane_id() == 0) s_def[wib] = 0u;
  const int64_t n = kLong ? (int64_t)dn.offs[cdf.waves] : dev_count(a.n_dev, a.n_host, a.n_max);
  const int p = pl.p;
  const u32 P = (u32)L.P;
  const int gbase = lane_id() - p;  // the key group's first lane
  const bool ftrl = L.opt == kFTRL;
  // (B, C) of entry e: words 3e + 1, 3e + 2 of the uint3 entries
  const float* __restrict__ ebc = static_cast<const float*>(a.csr_ent) + 1;
  const float2* stash = ftrl ? reinterpret_cast<const float2*>(a.nz_stash) : nullptr;
  // the lane's entry of the chunk at c0 (past the chain: clamped to its last
  // entry, read but never used -- no branch around the load)
  auto chunk = [&](u32 off, u32 cnt, u32 c0) {
    const float* q = ebc + 3 * (u64)(off + min(c0 + (u32)p, cnt - 1u));
    return make_float2(q[0], q[1]);
  };
  struct A {  // stage A: independent loads
    u32 i, slot, off, cnt;
  };
  // (kRows) the lane's component of entry e
  const float* __restrict__ eg = static_cast<const float*>(a.csr_ent) + 1 + p;
  const u32 ew = (u32)a.csr_ew;
  auto rows_chunk = [&](u32 off, u32 cnt, u32 q0, float (&e)[kCsrRowChunk]) {
#pragma unroll
    for (int k = 0; k < kCsrRowChunk; ++k) e[k] = eg[(u64)(off + min(q0 + (u32)k, cnt - 1u)) * ew];
  };
  struct B {  // stage B: the row words and the first chunk
    RowPre r;
    float2 c0;
    float r0[kCsrRowChunk];
  };
  auto stage_a = [&](int64_t j) {
    A x;
    x.i = kLong ? dn.list[j] : (u32)j;
    x.slot = a.slots[x.i];
    x.off = a.csr_off[x.i];
    x.cnt = a.csr_cnt[x.i];
    return x;
  };
  auto stage_b = [&](const A& x) {
    B y;
    y.r = stash ? row_stash(stash, a.keys, x.i, p, L.P) : row_pre(a.table.words, x.slot, p, L);
    if constexpr (kRows) {
      if (x.cnt) rows_chunk(x.off, x.cnt, 0u, y.r0);
    } else {
      y.c0 = x.cnt ? chunk(x.off, x.cnt, 0u) : make_float2(0.0f, 0.0f);
    }
    return y;
  };
  // (kLong: packed like pass 1 -- spreading the long chains one key group
  // per wave, as k_apply_lr16_csr does, measured 10 % slower at S = 256)
  int64_t j = pl.on ? pl.first : n;
  const int64_t st = pl.stride;
  A a0, a1;
  B b0;
  if (j < n) a0 = stage_a(j);
  if (j + st < n) a1 = stage_a(j + st);
  if (j < n) b0 = stage_b(a0);
  for (; j < n; j += st) {
    const A x = a0;
    const B y = b0;
    a0 = a1;
    if (j + st < n) b0 = stage_b(a0);
    if (j + 2 * st < n) a1 = stage_a(j + 2 * st);
    if (x.slot == kNoSlot || !x.cnt) continue;
    if (!kLong && a.csr_long && x.cnt > kCsrShortChain) {  // (uniform over the key's lanes)
      if (p == 0) cdf.region()[atomicAdd(&s_def[wib], 1u)] = x.i;
      continue;
    }
    float n0 = y.r.s0, z0 = y.r.s1;
    const float w0 = state_weight(y.r.key, y.r.flag != 0u, n0, z0, p, L, a.opt);
    float w_next = w0, sn = ftrl ? sqrtf(n0) : 0.0f;
    bool stale = false;
    auto push = [&](float g) {
      if (stale) w_next = ftrl ? ftrl_weight_sn(z0, sn, a.opt.ftrl) : n0;
      if (ftrl) ftrl_push_sn(n0, z0, sn, w_next, g, a.opt.ftrl);
      else n0 = w_next - a.opt.sgd.lr * g;
      stale = true;
    };
    if constexpr (kRows) {
      float e[kCsrRowChunk];
#pragma unroll
      for (int k = 0; k < kCsrRowChunk; ++k) e[k] = y.r0[k];
      for (u32 q0 = 0; q0 < x.cnt; q0 += kCsrRowChunk) {
        float nx[kCsrRowChunk];
        if (q0 + kCsrRowChunk < x.cnt) rows_chunk(x.off, x.cnt, q0 + kCsrRowChunk, nx);
#pragma unroll
        for (int k = 0; k < kCsrRowChunk; ++k)
          if (q0 + k < x.cnt) push(e[k]);
#pragma unroll
        for (int k = 0; k < kCsrRowChunk; ++k) e[k] = nx[k];
      }
      u32* sp = a.table.words + (u64)x.slot * L.stride;
      if (ftrl) *reinterpret_cast<float2*>(sp + 2 + 2 * p) = make_float2(n0, z0);
      else sp[2 + p] = __float_as_uint(n0);
      if (L.has_flag && p == 0) sp[L.flag_word] = 1u;
      continue;
    }
    const float w_pre = a.pulled ? a.pulled[(size_t)x.i * ps + p] : w0;
    float2 cur = y.c0;
    float2 nxt = x.cnt > P ? chunk(x.off, x.cnt, P) : make_float2(0.0f, 0.0f);
    u32 r = 0;  // q % P
    for (u32 q = 0; q < x.cnt; ++q) {
      if (r == P) {  // (uniform over the key's lanes)
        r = 0;
        cur = nxt;
        if (q + P < x.cnt) nxt = chunk(x.off, x.cnt, q + P);
      }
      const int src = (gbase + (int)r) << 2;
      const float Bv = __int_as_float(__builtin_amdgcn_ds_bpermute(src, __float_as_int(cur.x)));
      const float Cv = __int_as_float(__builtin_amdgcn_ds_bpermute(src, __float_as_int(cur.y)));
      ++r;
      push(p == 0 ? (float)a.fm_D * Bv : Cv - w_pre * Bv);
    }
    u32* sp = a.table.words + (u64)x.slot * L.stride;
    if (ftrl) *reinterpret_cast<float2*>(sp + 2 + 2 * p) = make_float2(n0, z0);
    else sp[2 + p] = __float_as_uint(n0);
    if (L.has_flag && p == 0) sp[L.flag_word] = 1u;
  }
  // (lane 0 -- key group 0, the wave's first key of every iteration -- is the
  // last to leave the loop)
  if (!kLong && a.csr_long && lane_id() == 0) a.csr_long[cdf.gw] = s_def[wib];
}

void launch_table_apply(const ApplyArgs& a, hipStream_t st) {
  if (a.n_max <= 0) return;
  const TableLayout& L = a.table.L;
  int grid = grid_for(a.n_dev ? a.n_max : a.n_host);
  const int64_t nm = a.n_dev ? a.n_max : a.n_host;
  const bool lr16_slot = L.stride == 4 && L.P == 1 && L.opt == kFTRL && !L.has_flag &&
                         a.pstride == 1;
  const bool lr16 = lr16_slot && a.S == 1 && !a.masks;
  // S > 1 on unique-order sums and slice bits (Engine::train_step's fused LR step)
  const bool lr16_slices = lr16_slot && a.S > 1 && a.masks && !a.masks_rw && !a.grad_map &&
                           !a.zero_after && !a.reset_pos && !a.sum_slices && !a.slice_rows &&
                           !a.grp.oidx;
  if (a.nz_stash && !a.keys && !a.grp.oidx && L.P > 1)
    throw std::runtime_error("table_apply: a stash needs the entries' keys");
  if (a.csr_cnt) {
    if (a.zero_after || a.reset_pos || a.sum_slices || a.grp.oidx || a.grad_map || a.slice_rows)
      throw std::runtime_error("CSR apply: bad arguments (entries come normalised)");
    // deferral lists (CsrDefer, CsrDense): [counts W][regions W x R][offsets
    // W + 1][dense list <= n][scan tiles]
    const int g2 = lr16_slot ? grid : packed_grid(nm, L.P);
    const int64_t waves = (int64_t)g2 * (kBlock / kWave);
    const int per = lr16_slot ? kWave : kWave / L.P;
    const int64_t stride = waves * per;
    const int64_t R = per * ((nm + stride - 1) / stride);
    u32* offs = a.csr_long + waves + waves * R;
    u32* tiles = offs + waves + 1 + nm;
    if (a.csr_long && (tiles - a.csr_long) + waves / 4096 + 8 > a.csr_long_cap)
      throw std::runtime_error("CSR apply: deferral list too small");
    auto dense = [&] {
      launch_scan_u32(a.csr_long, offs, nullptr, waves, tiles, st);
      hipLaunchKernelGGL(k_csr_gather, dim3((unsigned)((waves + 3) / 4)), dim3(kBlock), 0, st,
                         a.csr_long, nm, stride, per, (u32)waves);
    };
    if (lr16_slot) {
      hipLaunchKernelGGL(k_apply_lr16_csr<false>, dim3(grid), dim3(kBlock), 0, st, a);
      if (a.csr_long) {
        dense();
        hipLaunchKernelGGL(k_apply_lr16_csr<true>, dim3(grid), dim3(kBlock), 0, st, a);
      }
    } else if (a.fm_compact && L.P <= kWave && !a.csr_ew) {
      hipLaunchKernelGGL(k_apply_group_csr<false>, dim3(g2), dim3(kBlock), 0, st, a);
      if (a.csr_long) {
        dense();
        hipLaunchKernelGGL(k_apply_group_csr<true>, dim3(g2), dim3(kBlock), 0, st, a);
      }
    } else if (a.csr_ew >= csr_row_words(L.P) && !a.fm_compact && L.P <= kWave) {
      hipLaunchKernelGGL((k_apply_group_csr<false, true>), dim3(g2), dim3(kBlock), 0, st, a);
      if (a.csr_long) {
        dense();
        hipLaunchKernelGGL((k_apply_group_csr<true, true>), dim3(g2), dim3(kBlock), 0, st, a);
      }
    } else {
      throw std::runtime_error("CSR apply: LR-FTRL 16-byte slots, compact reference-FM rows or full rows");
    }
  } else if (a.grp.oidx) {
    if (a.zero_after || a.reset_pos) throw std::runtime_error("multi-source apply: bad arguments");
    if (lr16) hipLaunchKernelGGL(k_apply_lr16_multi, dim3(grid), dim3(kBlock), 0, st, a);
    else if (a.S > 1)
      hipLaunchKernelGGL(k_apply_group<true>, dim3(packed_grid(nm, L.P)), dim3(kBlock), 0, st, a);
    else hipLaunchKernelGGL(k_apply_group<false>, dim3(packed_grid(nm, L.P)), dim3(kBlock), 0, st, a);
  } else if (lr16) {
    hipLaunchKernelGGL(k_apply_lr16<false>, dim3(grid), dim3(kBlock), 0, st, a);
  } else if (lr16_slices) {
    hipLaunchKernelGGL(k_apply_lr16<true>, dim3(grid), dim3(kBlock), 0, st, a);
  } else if ((a.pstride >= 2 || (L.P == 1 && a.nz_stash)) && L.P <= kWave && !a.reset_pos) {
    // (LR with several slices and the pull's stash: one lane per key, packed)
    if (a.S > 1)
      hipLaunchKernelGGL(k_apply_group<true>, dim3(packed_grid(nm, L.P)), dim3(kBlock), 0, st, a);
    else hipLaunchKernelGGL(k_apply_group<false>, dim3(packed_grid(nm, L.P)), dim3(kBlock), 0, st, a);
  } else {
    hipLaunchKernelGGL(k_apply_generic, dim3(grid), dim3(kBlock), 0, st, a);
  }
  XF_HIP_CHECK(hipGetLastError());
}

// ---------------------------------------------------------------------------
// CSR exchange helpers (the multi-rank step of several slices): exclusive
// scan of per-key entry counts, dense packing of the entries in send order,
// per-owner entry totals.
// ---------------------------------------------------------------------------
constexpr int kScanItems = 16;                     // u32 per lane
constexpr int kScanTile = kBlock * kScanItems;     // 4096 per workgroup

// 1: per-tile sums
__global__ void __launch_bounds__(kBlock) k_scan_tiles(const u32* __restrict__ in,
                                                       const int64_t* __restrict__ n_dev,
                                                       int64_t n_host, u32* __restrict__ tiles) {
  const int64_t n = n_dev ? *n_dev : n_host;
  const int64_t t0 = (int64_t)blockIdx.x * kScanTile;
  if (t0 >= n) return;
  u32 v = 0;
#pragma unroll
  for (int q = 0; q < kScanItems; ++q) {
    const int64_t i = t0 + (int64_t)threadIdx.x * kScanItems + q;
    if (i < n) v += in[i];
  }
  u32 tot;
  (void)block_exclusive_scan<kBlock>(v, &tot);
  if (threadIdx.x == 0) tiles[blockIdx.x] = tot;
}

// 2: exclusive scan of the tile sums (one workgroup), total into tiles[nt]
__global__ void __launch_bounds__(kScanBlock) k_scan_top(u32* __restrict__ tiles,
                                                         const int64_t* __restrict__ n_dev,
                                                         int64_t n_host) {
  const int64_t n = n_dev ? *n_dev : n_host;
  const int nt = (int)((n + kScanTile - 1) / kScanTile);
  u32 carry = 0;
  for (int c0 = 0; c0 < nt; c0 += kScanBlock) {
    const int i = c0 + (int)threadIdx.x;
    const u32 v = i < nt ? tiles[i] : 0u;
    u32 t;
    const u32 ex = block_exclusive_scan<kScanBlock>(v, &t);
    if (i < nt) tiles[i] = carry + ex;
    carry += t;
  }
  if (threadIdx.x == 0) tiles[nt] = carry;
}

// 3: out[i] = exclusive prefix, out[n] = total
__global__ void __launch_bounds__(kBlock) k_scan_write(const u32* __restrict__ in,
                                                       const int64_t* __restrict__ n_dev,
                                                       int64_t n_host, const u32* __restrict__ tiles,
                                                       u32* __restrict__ out) {
  const int64_t n = n_dev ? *n_dev : n_host;
  const int64_t t0 = (int64_t)blockIdx.x * kScanTile;
  if (t0 > n) return;
  const int nt = (int)((n + kScanTile - 1) / kScanTile);
  if (t0 == n) {  // (n a multiple of the tile: the total has no tile of its own)
    if (threadIdx.x == 0) out[n] = tiles[nt];
    return;
  }
  u32 loc[kScanItems], v = 0;
#pragma unroll
  for (int q = 0; q < kScanItems; ++q) {
    const int64_t i = t0 + (int64_t)threadIdx.x * kScanItems + q;
    loc[q] = i < n ? in[i] : 0u;
    v += loc[q];
  }
  u32 tot;
  u32 ex = tiles[blockIdx.x] + block_exclusive_scan<kBlock>(v, &tot);
#pragma unroll
  for (int q = 0; q < kScanItems; ++q) {
    const int64_t i = t0 + (int64_t)threadIdx.x * kScanItems + q;
    if (i < n) out[i] = ex;
    ex += loc[q];
  }
  if (blockIdx.x == (unsigned)(nt - 1) && threadIdx.x == kBlock - 1) out[n] = ex;
}

// small arrays (<= kScanBlock x kScanItems, e.g. the CSR applies' per-wave
// deferral counts): the whole scan in one launch of one workgroup
constexpr int64_t kScanOneMax = (int64_t)kScanBlock * kScanItems;
__global__ void __launch_bounds__(kScanBlock) k_scan_one(const u32* __restrict__ in,
                                                         const int64_t* __restrict__ n_dev,
                                                         int64_t n_max, u32* __restrict__ out) {
  int64_t n = n_dev ? *n_dev : n_max;
  if (n > n_max) n = n_max;
  u32 loc[kScanItems], v = 0;
#pragma unroll
  for (int q = 0; q < kScanItems; ++q) {
    const int64_t i = (int64_t)threadIdx.x * kScanItems + q;
    loc[q] = i < n ? in[i] : 0u;
    v += loc[q];
  }
  u32 tot;
  u32 ex = block_exclusive_scan<kScanBlock>(v, &tot);
#pragma unroll
  for (int q = 0; q < kScanItems; ++q) {
    const int64_t i = (int64_t)threadIdx.x * kScanItems + q;
    if (i < n) out[i] = ex;
    ex += loc[q];
  }
  if (threadIdx.x == 0) out[n] = tot;
}

static bool scan_one_enabled() {
  static const bool on = [] {
    const char* e = std::getenv("XFLOW_SCAN_ONE");
    return !(e && e[0] == '0');
  }();
  return on;
}

void launch_scan_u32(const u32* in, u32* out, const int64_t* n_dev, int64_t n_max, u32* tiles,
                     hipStream_t st) {
  if (n_max <= kScanOneMax && scan_one_enabled()) {
    hipLaunchKernelGGL(k_scan_one, dim3(1), dim3(kScanBlock), 0, st, in, n_dev, n_max, out);
    XF_HIP_CHECK(hipGetLastError());
    return;
  }
  const int g = (int)((n_max + kScanTile - 1) / kScanTile) + 1;
  hipLaunchKernelGGL(k_scan_tiles, dim3(g), dim3(kBlock), 0, st, in, n_dev, n_max, tiles);
  hipLaunchKernelGGL(k_scan_top, dim3(1), dim3(kScanBlock), 0, st, tiles, n_dev, n_max);
  hipLaunchKernelGGL(k_scan_write, dim3(g), dim3(kBlock), 0, st, in, n_dev, n_max, tiles, out);
  XF_HIP_CHECK(hipGetLastError());
}

// entries of key i from the producer layout (off, cnt) to doff[i] (dense)
template <typename E>
__global__ void __launch_bounds__(kBlock) k_csr_pack(const u32* __restrict__ off,
                                                     const u32* __restrict__ cnt,
                                                     const E* __restrict__ src,
                                                     const u32* __restrict__ doff,
                                                     const int64_t* __restrict__ n_dev,
                                                     int64_t n_host, E* __restrict__ dst) {
  const int64_t n = n_dev ? *n_dev : n_host;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const u32 c = cnt[i], o = off[i], d = doff[i];
    for (u32 j = 0; j < c; ++j) dst[d + j] = src[o + j];
  }
}

// full-row entries (standard FM: m 16-byte words each)
__global__ void __launch_bounds__(kBlock) k_csr_pack_u4(const u32* __restrict__ off,
                                                        const u32* __restrict__ cnt,
                                                        const uint4* __restrict__ src,
                                                        const u32* __restrict__ doff,
                                                        const int64_t* __restrict__ n_dev,
                                                        int64_t n_host, int m,
                                                        uint4* __restrict__ dst) {
  const int64_t n = n_dev ? *n_dev : n_host;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const u32 c = cnt[i], o = off[i], d = doff[i];
    for (u32 j = 0; j < c * (u32)m; ++j) dst[(u64)d * m + j] = src[(u64)o * m + j];
  }
}

// per-owner entry totals: owner r's keys are the send-order range of the
// (decoded) key counts before it
__global__ void k_csr_totals(const int64_t* __restrict__ counts, int world, int encoded,
                             const u32* __restrict__ doff, int64_t* __restrict__ totals) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  int64_t o = 0;
  for (int r = 0; r < world; ++r) {
    int64_t c = counts[r];
    if (encoded) c = (c & ((1ll << kCountBits) - 1)) - 1;
    c = c > 0 ? c : 0;
    totals[r] = (int64_t)doff[o + c] - (int64_t)doff[o];
    o += c;
  }
}

void launch_csr_pack(const u32* off, const u32* cnt, const void* src, const u32* doff,
                     const int64_t* n_dev, int64_t n_max, void* dst, int entry_bytes,
                     hipStream_t st) {
  const int g = grid_for(n_max);
  if (entry_bytes == 8)
    hipLaunchKernelGGL(k_csr_pack<u64>, dim3(g), dim3(kBlock), 0, st, off, cnt,
                       static_cast<const u64*>(src), doff, n_dev, n_max, static_cast<u64*>(dst));
  else if (entry_bytes == 12)
    hipLaunchKernelGGL(k_csr_pack<uint3>, dim3(g), dim3(kBlock), 0, st, off, cnt,
                       static_cast<const uint3*>(src), doff, n_dev, n_max, static_cast<uint3*>(dst));
  else if (entry_bytes > 0 && entry_bytes % 16 == 0)
    hipLaunchKernelGGL(k_csr_pack_u4, dim3(g), dim3(kBlock), 0, st, off, cnt,
                       static_cast<const uint4*>(src), doff, n_dev, n_max, entry_bytes / 16,
                       static_cast<uint4*>(dst));
  else throw std::runtime_error("csr_pack: entries of 8, 12 or 16k bytes");
  XF_HIP_CHECK(hipGetLastError());
}

void launch_csr_totals(const int64_t* counts, int world, bool encoded, const u32* doff,
                       int64_t* totals, hipStream_t st) {
  hipLaunchKernelGGL(k_csr_totals, dim3(1), dim3(kWave), 0, st, counts, world, encoded ? 1 : 0,
                     doff, totals);
  XF_HIP_CHECK(hipGetLastError());
}

// ---------------------------------------------------------------------------
// worker-side gradient gather (multi-rank path): pos-indexed raw sums ->
// owner-grouped send buffer, normalised per slice, source rows cleared.
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(kBlock) k_gather_grads(GatherGradArgs a) {
  int64_t n = dev_count(a.n_dev, a.n_max, a.n_max);
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const int S = a.S, ps = a.pstride, W = S * ps, wd = a.width ? a.width : ps;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    u32 row = a.map[i];
    float* __restrict__ src = a.grad_rw + (size_t)row * W;
    float* __restrict__ dst = a.out + (size_t)i * S * wd;
    for (int s = 0; s < S; ++s)
      for (int p = 0; p < wd; ++p) {
        dst[s * wd + p] = norm_grad(src[s * ps + p], a.slice_rows, s);
        src[s * ps + p] = 0.0f;
      }
    if (a.tmask_rw) {
      a.out_mask[i] = a.tmask_rw[row];
      a.tmask_rw[row] = 0u;
    }
  }
}

// The same with one thread per 16-byte unit (width and pstride multiples of
// 4): every unit's load is independent -- the row-per-thread loop above
// serialises a load -> store round trip per float (the stores may alias the
// next loads for the compiler), 225 us per MVM-10 rank-step in the emulated
// 8-GPU step.
__global__ void __launch_bounds__(kBlock) k_gather_grads4(GatherGradArgs a) {
  const int64_t n = dev_count(a.n_dev, a.n_max, a.n_max);
  const u32 S = (u32)a.S, ps4 = (u32)a.pstride / 4, wd4 = (u32)(a.width ? a.width : a.pstride) / 4;
  const u32 per = S * wd4;  // units per entry
  const u32 units = (u32)n * per;  // (< 2^32: checked by the launcher)
  const u32 stride = gridDim.x * blockDim.x;
  float4* __restrict__ g4 = reinterpret_cast<float4*>(a.grad_rw);
  float4* __restrict__ o4 = reinterpret_cast<float4*>(a.out);
  for (u32 u = blockIdx.x * blockDim.x + threadIdx.x; u < units; u += stride) {
    const u32 i = u / per;
    const u32 r = u - i * per, s = r / wd4, q = r - s * wd4;
    const u32 row = a.map[i];
    float4* sp = g4 + (u64)row * S * ps4 + (u64)s * ps4 + q;
    const float4 v = *sp;
    o4[u] = make_float4(norm_grad(v.x, a.slice_rows, (int)s), norm_grad(v.y, a.slice_rows, (int)s),
                        norm_grad(v.z, a.slice_rows, (int)s), norm_grad(v.w, a.slice_rows, (int)s));
    *sp = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    if (r == 0 && a.tmask_rw) {
      a.out_mask[i] = a.tmask_rw[row];
      a.tmask_rw[row] = 0u;
    }
  }
}

void launch_gather_grads(const GatherGradArgs& a, hipStream_t st) {
  if (a.n_max <= 0) return;
  const int wd = a.width ? a.width : a.pstride;
  const bool vec = a.pstride % 4 == 0 && wd % 4 == 0 &&
                   (double)a.n_max * a.S * (wd / 4) < 4294967295.0 &&
                   (reinterpret_cast<uintptr_t>(a.grad_rw) & 15) == 0 &&
                   (reinterpret_cast<uintptr_t>(a.out) & 15) == 0;
  if (vec) {
    const int64_t units = a.n_max * (int64_t)a.S * (wd / 4);
    hipLaunchKernelGGL(k_gather_grads4, dim3(grid_for(units)), dim3(kBlock), 0, st, a);
  } else {
    hipLaunchKernelGGL(k_gather_grads, dim3(grid_for(a.n_max)), dim3(kBlock), 0, st, a);
  }
  XF_HIP_CHECK(hipGetLastError());
}

// ---------------------------------------------------------------------------
// owner bucketing: counts per rank, then a block-aggregated scatter that
// reserves each (block, owner) range with one global atomic.
// ---------------------------------------------------------------------------
constexpr int kBucketItems = 16;                 // items per thread
constexpr int kBucketChunk = kBlock * kBucketItems;
constexpr int kMaxWorld = 256;

__global__ void __launch_bounds__(kBlock) k_bucket_count(const u64* __restrict__ keys,
                                                         const int64_t* n_dev, int64_t n_max,
                                                         int world,
                                                         unsigned long long* __restrict__ counts) {
  __shared__ unsigned int hist[kMaxWorld];
  for (int o = threadIdx.x; o < world; o += blockDim.x) hist[o] = 0;
  __syncthreads();
  int64_t n = dev_count(n_dev, n_max, n_max);
  int64_t base = (int64_t)blockIdx.x * kBucketChunk;
  for (int j = 0; j < kBucketItems; ++j) {
    int64_t i = base + (int64_t)j * kBlock + threadIdx.x;
    if (i < n) atomicAdd(&hist[owner_of(keys[i], (u32)world)], 1u);
  }
  __syncthreads();
  for (int o = threadIdx.x; o < world; o += blockDim.x)
    if (hist[o]) atomicAdd(&counts[o], (unsigned long long)hist[o]);
}

__global__ void __launch_bounds__(kBlock) k_bucket_scatter(
    const u64* __restrict__ keys, const u32* __restrict__ upos, const int64_t* n_dev,
    int64_t n_max, int world, const unsigned long long* __restrict__ counts,
    unsigned long long* __restrict__ cursor, u64* __restrict__ send_keys,
    u32* __restrict__ send_pos) {
  __shared__ unsigned int hist[kMaxWorld];
  __shared__ unsigned long long base_of[kMaxWorld];
  for (int o = threadIdx.x; o < world; o += blockDim.x) hist[o] = 0;
  __syncthreads();
  int64_t n = dev_count(n_dev, n_max, n_max);
  int64_t base = (int64_t)blockIdx.x * kBucketChunk;
  u32 own[kBucketItems];
#pragma unroll
  for (int j = 0; j < kBucketItems; ++j) {
    int64_t i = base + (int64_t)j * kBlock + threadIdx.x;
    own[j] = (i < n) ? owner_of(keys[i], (u32)world) : 0xFFFFFFFFu;
    if (own[j] != 0xFFFFFFFFu) atomicAdd(&hist[own[j]], 1u);
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned long long off = 0;
    for (int o = 0; o < world; ++o) {
      unsigned long long c = counts[o];
      base_of[o] = off + (hist[o] ? atomicAdd(&cursor[o], (unsigned long long)hist[o]) : 0ull);
      off += c;
    }
  }
  __syncthreads();
  for (int o = threadIdx.x; o < world; o += blockDim.x) hist[o] = 0;
  __syncthreads();
#pragma unroll
  for (int j = 0; j < kBucketItems; ++j) {
    if (own[j] == 0xFFFFFFFFu) continue;
    int64_t i = base + (int64_t)j * kBlock + threadIdx.x;
    unsigned int r = atomicAdd(&hist[own[j]], 1u);
    unsigned long long dst = base_of[own[j]] + r;
    send_keys[dst] = keys[i];
    send_pos[dst] = upos[i];
  }
}

__global__ void k_encode_counts(int64_t* __restrict__ counts, int world, int64_t seq) {
  for (int o = threadIdx.x; o < world; o += blockDim.x) counts[o] = encode_count(counts[o], seq);
}

void launch_bucket(const BucketArgs& a, hipStream_t st) {
  if (a.world > kMaxWorld) throw std::runtime_error("bucket: world size > 256 unsupported");
  XF_HIP_CHECK(hipMemsetAsync(a.counts, 0, sizeof(int64_t) * a.world, st));
  XF_HIP_CHECK(hipMemsetAsync(a.scratch, 0, sizeof(int64_t) * a.world, st));
  if (a.n_max <= 0) return;
  int grid = (int)((a.n_max + kBucketChunk - 1) / kBucketChunk);
  hipLaunchKernelGGL(k_bucket_count, dim3(grid), dim3(kBlock), 0, st, a.uniq_keys, a.n_dev,
                     a.n_max, a.world, reinterpret_cast<unsigned long long*>(a.counts));
  hipLaunchKernelGGL(k_bucket_scatter, dim3(grid), dim3(kBlock), 0, st, a.uniq_keys, a.uniq_pos,
                     a.n_dev, a.n_max, a.world,
                     reinterpret_cast<const unsigned long long*>(a.counts),
                     reinterpret_cast<unsigned long long*>(a.scratch), a.send_keys, a.send_pos);
  if (a.seq >= 0)
    hipLaunchKernelGGL(k_encode_counts, dim3(1), dim3(kBlock), 0, st, a.counts, a.world, a.seq);
  XF_HIP_CHECK(hipGetLastError());
}

// ---------------------------------------------------------------------------
// row gather / scatter helpers
// ---------------------------------------------------------------------------
// width a multiple of 4: one thread per 16-byte unit, 32-bit index math (the
// element loop's 64-bit division per float dominated at MVM widths)
__global__ void k_scatter_rows4(const float4* __restrict__ src, float4* __restrict__ dst,
                                const u32* __restrict__ map, const int64_t* n_dev, int64_t n_max,
                                u32 w4, float* __restrict__ zero_out, int zero_width) {
  const int64_t rows = dev_count(n_dev, n_max, n_max);
  const u32 n = (u32)rows * w4;  // (< 2^32: checked by the launcher)
  const u32 stride = gridDim.x * blockDim.x;
  for (u32 e = blockIdx.x * blockDim.x + threadIdx.x; e < n; e += stride) {
    const u32 i = e / w4;
    const u32 c = e - i * w4;
    const u64 r = map ? (u64)map[i] : (u64)i;
    dst[r * w4 + c] = src[e];
  }
  if (zero_out)
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < rows * zero_width;
         i += (int64_t)stride)
      zero_out[i] = 0.0f;
}

__global__ void k_scatter_rows(const float* __restrict__ src, float* __restrict__ dst,
                               const u32* __restrict__ map, const int64_t* n_dev, int64_t n_max,
                               int width, float* __restrict__ zero_out, int zero_width) {
  const int64_t rows = dev_count(n_dev, n_max, n_max), n = rows * width;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < n; e += stride) {
    int64_t i = e / width;
    int c = (int)(e - i * width);
    int64_t r = map ? (int64_t)map[i] : i;
    dst[r * width + c] = src[e];
  }
  if (zero_out)  // the send buffer the reduction fills next (saves a memset launch)
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < rows * zero_width;
         i += stride)
      zero_out[i] = 0.0f;
}

__global__ void k_gather_rows(const float* __restrict__ src, float* __restrict__ dst,
                              const u32* __restrict__ map, const int64_t* n_dev, int64_t n_max,
                              int width, bool zero_src) {
  int64_t n = dev_count(n_dev, n_max, n_max) * width;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < n; e += stride) {
    int64_t i = e / width;
    int c = (int)(e - i * width);
    int64_t r = (int64_t)map[i] * width + c;
    dst[e] = src[r];
    if (zero_src) const_cast<float*>(src)[r] = 0.0f;
  }
}

__global__ void k_gather_u32(const u32* __restrict__ src, u32* __restrict__ dst,
                             const u32* __restrict__ map, const int64_t* n_dev, int64_t n_max,
                             bool zero_src) {
  int64_t n = dev_count(n_dev, n_max, n_max);
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    dst[i] = src[map[i]];
    if (zero_src) const_cast<u32*>(src)[map[i]] = 0u;
  }
}

__global__ void k_scatter_u32(const u32* __restrict__ src, u32* __restrict__ dst,
                              const u32* __restrict__ map, const int64_t* n_dev, int64_t n_max) {
  int64_t n = dev_count(n_dev, n_max, n_max);
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
    dst[map[i]] = src[i];
}

void launch_scatter_rows(const float* src, float* dst, const u32* map, const int64_t* n_dev,
                         int64_t n_max, int width, float* zero_out, int zero_width,
                         hipStream_t st) {
  if (n_max <= 0) return;
  if (width % 4 == 0 && (double)n_max * width < 4294967295.0 &&
      (reinterpret_cast<uintptr_t>(src) & 15) == 0 &&
      (reinterpret_cast<uintptr_t>(dst) & 15) == 0) {
    hipLaunchKernelGGL(k_scatter_rows4, dim3(grid_for(n_max * width / 4)), dim3(kBlock), 0, st,
                       reinterpret_cast<const float4*>(src), reinterpret_cast<float4*>(dst), map,
                       n_dev, n_max, (u32)(width / 4), zero_out, zero_width);
    XF_HIP_CHECK(hipGetLastError());
    return;
  }
  hipLaunchKernelGGL(k_scatter_rows, dim3(grid_for(n_max * width)), dim3(kBlock), 0, st, src, dst,
                     map, n_dev, n_max, width, zero_out, zero_width);
  XF_HIP_CHECK(hipGetLastError());
}

void launch_gather_rows(const float* src, float* dst, const u32* map, const int64_t* n_dev,
                        int64_t n_max, int width, bool zero_src, hipStream_t st) {
  if (n_max <= 0) return;
  hipLaunchKernelGGL(k_gather_rows, dim3(grid_for(n_max * width)), dim3(kBlock), 0, st, src, dst,
                     map, n_dev, n_max, width, zero_src);
  XF_HIP_CHECK(hipGetLastError());
}

void launch_gather_u32(const u32* src, u32* dst, const u32* map, const int64_t* n_dev,
                       int64_t n_max, bool zero_src, hipStream_t st) {
  if (n_max <= 0) return;
  hipLaunchKernelGGL(k_gather_u32, dim3(grid_for(n_max)), dim3(kBlock), 0, st, src, dst, map,
                     n_dev, n_max, zero_src);
  XF_HIP_CHECK(hipGetLastError());
}

void launch_scatter_u32(const u32* src, u32* dst, const u32* map, const int64_t* n_dev,
                        int64_t n_max, hipStream_t st) {
  if (n_max <= 0) return;
  hipLaunchKernelGGL(k_scatter_u32, dim3(grid_for(n_max)), dim3(kBlock), 0, st, src, dst, map,
                     n_dev, n_max);
  XF_HIP_CHECK(hipGetLastError());
}

// ---------------------------------------------------------------------------
// checkpoint export / import
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(kBlock) k_table_export(TableView t, u64* __restrict__ keys_out,
                                                         u32* __restrict__ words_out,
                                                         int64_t max_rows,
                                                         unsigned long long* counter) {
  const int W = t.L.stride - 2;
  const u64 stride = (u64)gridDim.x * blockDim.x;
  for (u64 s = (u64)blockIdx.x * blockDim.x + threadIdx.x; s < t.cap; s += stride) {
    const u32* sp = t.words + s * (u64)t.L.stride;
    u64 key = *reinterpret_cast<const u64*>(sp);
    bool live = key != kEmptyKey;
    unsigned long long idx = wave_append(counter, live);
    if (live && (int64_t)idx < max_rows) {
      keys_out[idx] = key;
      for (int w = 0; w < W; ++w) words_out[idx * W + w] = sp[2 + w];
    }
  }
}

void launch_table_export(const TableView& t, u64* keys_out, u32* words_out, int64_t max_rows,
                         unsigned long long* counter, hipStream_t st) {
  XF_HIP_CHECK(hipMemsetAsync(counter, 0, sizeof(unsigned long long), st));
  hipLaunchKernelGGL(k_table_export, dim3(grid_for((int64_t)t.cap)), dim3(kBlock), 0, st, t,
                     keys_out, words_out, max_rows, counter);
  XF_HIP_CHECK(hipGetLastError());
}

__global__ void __launch_bounds__(kBlock) k_table_import(TableView t, const u64* __restrict__ keys,
                                                         const u32* __restrict__ words,
                                                         int64_t n) {
  const int W = t.L.stride - 2;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  unsigned int claims = 0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    bool claimed = false;
    u32 slot = probe(t, sanitize_key(keys[i]), true, claimed);
    claims += claimed;
    if (slot == kNoSlot) continue;
    u32* sp = t.words + (u64)slot * t.L.stride;
    for (int w = 0; w < W; ++w) sp[2 + w] = words[i * W + w];
  }
  block_count_add<kBlock>(t.size, claims);
}

// Growth by segment splits (TableView geometry, Backend::table_split).  t is
// the geometry after the split: segments [s0, s0 + k) of t.level split into
// their buddies s + 2^level, which are mapped and cleared.  A key moves when
// bit (seg_log2 + level) of its hash is set.
//
// Phase 1 marks the cluster starts of the source segments (an occupied slot
// whose predecessor in the segment is free) in a bitmap, before any slot
// changes: phase 2 rewrites clusters, and a start test racing with those
// writes could see a half-rewritten cluster.  Phase 2: one lane per cluster
// walks it in order (linear probing's backward-shift deletion, for every
// moving key at once).  At walk position d every slot before d is final:
// a moving key is CAS-inserted into the buddy segment (an empty table that
// only other moving keys compete for) with its state words, and slot d is
// freed; a staying key goes to the first free slot from its home on -- a
// slot freed earlier in the walk, or d itself -- and slot d is freed if it
// left.  Slots before d are never freed again, so every chain from a home to
// its key stays occupied.  Clusters are separated by free slots, so lanes
// never touch each other's slots.
__global__ void __launch_bounds__(kBlock) k_table_split_marks(TableView t, u64 s0, u64 k,
                                                              u64* __restrict__ marks) {
  const int g = t.seg_log2;
  const u64 m = (1ull << g) - 1;
  const u64 n = k << g;
  const int W = t.L.stride;
  const u64 stride = (u64)gridDim.x * blockDim.x;
  // (n is a multiple of 64 when g >= 6; the ballot of a partial wave is padded)
  for (u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x; i < ((n + 63) & ~63ull); i += stride) {
    bool start = false;
    if (i < n) {
      const u64 base = (s0 << g) + (i & ~m), c = i & m;
      const u64 kc = *reinterpret_cast<const u64*>(t.words + (base + c) * (u64)W);
      const u64 kp = *reinterpret_cast<const u64*>(t.words + (base + ((c - 1) & m)) * (u64)W);
      start = kc != kEmptyKey && kp == kEmptyKey;
    }
    const unsigned long long b = __ballot(start);
    if ((threadIdx.x & 63) == 0) marks[i >> 6] = b;
  }
}

__global__ void __launch_bounds__(kBlock) k_table_split(TableView t, u64 s0, u64 k,
                                                        const u64* __restrict__ marks) {
  const int g = t.seg_log2;
  const u64 G = 1ull << g, m = G - 1;
  const u64 n = k << g;
  const int W = t.L.stride;
  const u64 move_bit = 1ull << (g + t.level);
  const u64 buddy = (1ull << t.level) << g;  // slot offset of a segment's buddy
  const u64 stride = (u64)gridDim.x * blockDim.x;
  for (u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    if (!((marks[i >> 6] >> (i & 63)) & 1ull)) continue;
    const u64 base = (s0 << g) + (i & ~m), c = i & m;
    auto slot_at = [&](u64 off) { return t.words + (base + ((c + off) & m)) * (u64)W; };
    auto free_slot = [&](u32* sp) {
      sp[0] = 0xFFFFFFFFu;
      sp[1] = 0xFFFFFFFFu;
      for (int w = 2; w < W; ++w) sp[w] = 0u;
    };
    for (u64 d = 0; d < G; ++d) {  // d: walk offset from the cluster start c
      u32* sp = slot_at(d);
      const u64 key = *reinterpret_cast<const u64*>(sp);
      if (key == kEmptyKey) break;
      const u64 h = fmix64(key);
      if (h & move_bit) {
        u64 q = base + buddy + (h & m);
        bool placed = false;
        for (u64 r = 0; r < t.probe_limit; ++r) {
          u32* qp = t.words + q * (u64)W;
          const u64 prev = atomicCAS(reinterpret_cast<unsigned long long*>(qp),
                                     (unsigned long long)kEmptyKey, (unsigned long long)key);
          if (prev == kEmptyKey) {
            for (int w = 2; w < W; ++w) qp[w] = sp[w];
            placed = true;
            break;
          }
          q = table_next(t, q);
        }
        if (!placed) *t.overflow = 1u;
        free_slot(sp);
      } else {
        u64 off = ((h & m) - c) & m;  // home, in [0, d]: the chain from it is unbroken
        while (off < d && *reinterpret_cast<const u64*>(slot_at(off)) != kEmptyKey) ++off;
        if (off != d) {
          u32* dp = slot_at(off);
          for (int w = 0; w < W; ++w) dp[w] = sp[w];
          free_slot(sp);
        }
      }
    }
  }
}

void launch_table_split(const TableView& t, u64 s0, u64 k, u64* marks, hipStream_t st) {
  const int64_t n = (int64_t)(k << t.seg_log2);
  if (n <= 0) return;
  hipLaunchKernelGGL(k_table_split_marks, dim3(grid_for(n, kBlock, 16384)), dim3(kBlock), 0, st,
                     t, s0, k, marks);
  XF_HIP_CHECK(hipGetLastError());
  hipLaunchKernelGGL(k_table_split, dim3(grid_for(n, kBlock, 16384)), dim3(kBlock), 0, st, t, s0,
                     k, (const u64*)marks);
  XF_HIP_CHECK(hipGetLastError());
}

__global__ void __launch_bounds__(kBlock) k_table_prefill(TableView t, int64_t n, u64 seed) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  unsigned int claims = 0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const u64 key = prefill_key(seed, (u64)i);
    bool claimed = false;
    const u32 slot = probe(t, key, true, claimed);
    claims += claimed;
    if (slot != kNoSlot && t.L.has_flag) t.words[(u64)slot * t.L.stride + t.L.flag_word] = 1u;
  }
  block_count_add<kBlock>(t.size, claims);
}

void launch_table_prefill(const TableView& t, int64_t n, u64 seed, hipStream_t st) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_table_prefill, dim3(grid_for(n, kBlock, 16384)), dim3(kBlock), 0, st, t, n,
                     seed);
  XF_HIP_CHECK(hipGetLastError());
}

void launch_table_import(const TableView& t, const u64* keys, const u32* words, int64_t n,
                         hipStream_t st) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_table_import, dim3(grid_for(n)), dim3(kBlock), 0, st, t, keys, words, n);
  XF_HIP_CHECK(hipGetLastError());
}

}  // namespace hip
}  // namespace xflow

namespace xflow {
namespace hip {

// L1 sparsity report: count (key, param) weights that are exactly non-zero.
// A full-table sweep (dwordx4-friendly for 16-B LR slots), one atomic per
// workgroup.
__global__ void __launch_bounds__(kBlock) k_table_nonzero(TableView t, OptSpec o,
                                                          unsigned long long* counter) {
  const TableLayout& L = t.L;
  const u64 stride = (u64)gridDim.x * blockDim.x;
  unsigned int cnt = 0;
  for (u64 s = (u64)blockIdx.x * blockDim.x + threadIdx.x; s < t.cap; s += stride) {
    const u32* sp = t.words + s * (u64)L.stride;
    const u64 key = *reinterpret_cast<const u64*>(sp);
    if (key == kEmptyKey) continue;
    for (int p = 0; p < L.P; ++p) cnt += slot_weight(sp, key, p, L, o) != 0.0f;
  }
  block_count_add<kBlock>(counter, cnt);
}

void launch_table_nonzero(const TableView& t, const OptSpec& o, unsigned long long* counter,
                          hipStream_t st) {
  XF_HIP_CHECK(hipMemsetAsync(counter, 0, sizeof(unsigned long long), st));
  hipLaunchKernelGGL(k_table_nonzero, dim3(grid_for((int64_t)t.cap)), dim3(kBlock), 0, st, t, o,
                     counter);
  XF_HIP_CHECK(hipGetLastError());
}

}  // namespace hip
}  // namespace xflow
