// xflow-amd: device backend interface.
//
// The engine (engine.cpp) is written once against this interface.  Two
// implementations exist: HipBackend (gfx950 kernels, csrc/hip/*.hip) and
// CpuBackend (csrc/cpu/cpu_backend.cpp) which runs the identical per-element
// recipes from common.h/types.h on the host, single threaded and
// deterministic.  The CPU backend exists for the reference "plumbing" config
// (LR+SGD on bundled data without a GPU) and for multi-rank gloo tests; on a
// GPU the HIP backend is the one that runs, and it fails loudly if missing.
//
// Every count argument that can be produced on the device is passed as a
// pointer (`const int64_t* n_dev`) plus an upper bound (`n_max`), so a whole
// single-GPU training step is launched without any host synchronisation.
#pragma once

#include <stddef.h>
#include <stdint.h>

#include <memory>
#include <stdexcept>
#include <string>

#include "xflow/types.h"

namespace xflow {

// Linear-probe chains are bounded: an insert that finds no free slot within
// probe_limit slots of its home flags the table overflow instead of walking a
// (nearly) full table, and a lookup stops at the same distance -- no key is
// ever stored further from its home than an insert may probe.  The engine
// keeps the load below EngineConfig::grow_load by growing the table
// (segment splits, Backend::table_split), so chains stay short and the bound
// is never hit in normal operation.
constexpr u64 kMaxProbe = 1ull << 16;
constexpr int kMaxSegLog2 = 20;  // segment slots (TableView), at most

// Table geometry: linear hashing over equal segments (docs/DESIGN.md §2).
// The slot array is nseg = 2^level + split segments of 2^seg_log2 slots,
// contiguous in one reserved address range.  With h = fmix64(key) and
// b = (h >> seg_log2) mod 2^level -- or mod 2^(level+1) when b < split (that
// segment was split into b and b + 2^level) -- the key's home is slot
// b * 2^seg_log2 + (h mod 2^seg_log2), and its chain wraps inside the
// segment.  A power-of-two table (split = 0) has the home h mod cap, as a
// plain linear-probing table.  Growing adds one segment and splits one: only
// the split segment's keys move (Backend::table_split), the new memory is one
// segment, and the rest of the table is untouched -- growth costs no 2x peak
// and no stop of the world.  The segment index bits (seg_log2 .. 30) stay
// below the owner bits (fmix64 >> 32, parallel/sparse_a2a.py), so a rank's
// shard spreads over all of its segments.
struct TableView {
  u32* words = nullptr;      // slot array
  u64 cap = 0;               // slots in use = nseg << seg_log2
  TableLayout L;
  unsigned long long* size = nullptr;   // device counter: occupied slots
  u32* overflow = nullptr;   // set when an insert finds no slot within probe_limit
  u64 probe_limit = 0;       // min(segment slots, kMaxProbe)
  int seg_log2 = 0;          // slots per segment = 2^seg_log2
  int level = 0;             // 2^level <= nseg < 2^(level+1)
  u64 split = 0;             // segments [0, split) of this level are split
};

XF_HD u64 table_home(const TableView& t, u64 h) {
  const u64 hi = h >> t.seg_log2;
  u64 b = hi & ((1ull << t.level) - 1);
  if (b < t.split) b = hi & ((2ull << t.level) - 1);
  return (b << t.seg_log2) | (h & ((1ull << t.seg_log2) - 1));
}
// the slot after s in its chain (wraps inside the segment)
XF_HD u64 table_next(const TableView& t, u64 s) {
  const u64 m = (1ull << t.seg_log2) - 1;
  return (s & ~m) | ((s + 1) & m);
}

// Worker dedup table.  Persistent across steps: a key keeps its slot, so hot
// keys are never re-inserted (no CAS storms on the skewed head of the key
// distribution).  A slot is "in the current batch" when its stamp equals the
// step's epoch (set by idempotent plain stores); the unique list is recovered
// by scanning stamps.  The table is cleared on the device once `claims` (keys
// inserted since the last clear) exceeds `rebuild_at`.
struct ScratchView {
  u64* keys = nullptr;         // [cap], kEmptyKey when free
  // [cap], epoch of the last batch touching the slot.  One byte (epochs
  // cycle through 1..kStampEpochs, the stamps are cleared at the wrap): the
  // leaders' scattered stamp stores dirty 4x fewer lines and the compaction
  // reads 16 stamps per dwordx4
  unsigned char* stamps = nullptr;
  u64 cap = 0;
  u32 epoch = 1;               // current step (1..kStampEpochs)
  unsigned long long* claims = nullptr;  // device counter of inserted keys
  u64 rebuild_at = 0;          // clear the table before a step once claims > rebuild_at
  // HIP backend: adaptive active capacity, kept on the device (no host sync).
  // ctl[0] = active cap for the next batch (power of two <= cap), ctl[1] = most
  // unique keys seen in one batch, ctl[2] = slots the compaction frees for a
  // rebuild (0: none), ctl[3] = the cap the current batch was deduplicated with,
  // ctl[4] = epoch of the last batch that spilled past the active capacity (a
  // full active table: the insert probes on into [ctl[0], cap) and that
  // batch's compaction and reduction cover the whole allocation).
  // The table is probed modulo ctl[0]; the compaction scan re-sizes it to
  // kScratchHeadroom x the largest batch seen (a table that fits the Infinity
  // Cache instead of one sized for all-distinct batches).  Null: use cap.
  unsigned long long* ctl = nullptr;
  // (with ctl) > 0 when this batch has more occurrences than any before, by
  // this factor: the active capacity grows to kScratchHeadroom x (most unique
  // keys seen) x grow before the insert, so a batch larger than the ones the
  // capacity was fitted to cannot fill the table
  float grow = 0.0f;
  // HIP: owner-partitioned probing for the sharded step.  With parts > 1 the
  // active capacity is split into `parts` equal ranges and a key probes only
  // the range of its owner (owner_of(key, parts)), so the slot-ordered unique
  // list comes out grouped by owner -- the all-to-all send order -- and the
  // per-owner counts are range counts (Backend::partition_counts).
  int parts = 1;
  // HIP, parts == 1: > 0 = the number of hash bits the parameter table's home
  // slot uses (TableView: seg_log2 + level, + 1 while segments are split).
  // The scratch home is then the TOP log2(active cap) of those bits instead
  // of the lowest: the compaction's slot-ordered unique list comes out sorted
  // by table home, so the pull's and the apply's random slot accesses sweep
  // the table in address order -- neighbouring lanes share pages and TLB
  // entries instead of each missing in a 34 GB range.
  int home_bits = 0;
};
constexpr int kMaxParts = 1024;

// Counts of the multi-rank counts exchange (world > 1): one int64 per owner
// carrying the count + 1 (0: the source has no data this step) in the low
// kCountBits bits and the sender's prepare sequence number above them, so a
// rank that skipped an exchange is detected by every peer at the next one.
constexpr int kCountBits = 40;
constexpr int64_t kSeqMask = (1ll << 23) - 1;
XF_HD int64_t encode_count(int64_t count, int64_t seq) {
  return ((seq & kSeqMask) << kCountBits) | (count + 1);
}
constexpr u32 kStampEpochs = 255;
constexpr u64 kScratchHeadroom = 4;      // active cap >= 4 x max unique keys per batch (A/B: 8 and 2 slower)
constexpr u64 kScratchMinCap = 1ull << 16;

struct DedupOut {
  u32* pos = nullptr;          // [nnz] scratch slot of each occurrence
  u64* uniq_keys = nullptr;    // [nnz_max]
  u32* uniq_pos = nullptr;     // [nnz_max]
  int64_t* n_uniq = nullptr;   // device counter
  u32* overflow = nullptr;
  u32* block_counts = nullptr; // [cap/4096 + 1] compaction workspace (HIP backend)
  u32* inv = nullptr;          // optional [cap]: unique-list index of each slot of the batch (HIP)
  int64_t* n_uniq_copy = nullptr;  // optional second destination of the unique count
  unsigned long long* cap_out = nullptr;  // optional: the capacity this batch was deduplicated with
};

// Sparse per-(key, slice) gradient sums in CSR form -- the step's pushes as
// the reference makes them: each Hogwild slice pushes only the keys it
// touched (lr_worker.cc:162-175), so only touched (key, slice) pairs exist.
// Key i (unique / send order) owns entries ent[off[i] .. off[i] + cnt[i]),
// in slice order.  An entry is (slice, value): LR u64 slice | value << 32,
// reference FM u32x3 (slice, B, C).  Dests of the producers are
// key * 2^slog2 + slice (the slice count padded to a power of two), so a
// key's dests never straddle a reduction bucket.
struct CsrOut {
  u32* off = nullptr;            // [unique] first entry of the key
  u32* cnt = nullptr;            // [unique] entries of the key (>= 1 for every key of the batch)
  // entries (FwdArgs: the producers' record regions, free by then; standard
  // FM: a buffer of csr_row_words(P) words per entry, >= the step's records)
  void* ent = nullptr;
  int slog2 = 0;
  const int32_t* rows = nullptr;  // values divided by rows[slice] (null: raw sums)
  int ew = 0, P = 0;              // full-row entries: words per entry, params per key
  // (MVM rows with a repeated field: FwdArgs::mdup, added to their entries
  // after the reduction)
};
// 32-bit words of a full-row CSR entry (slice, g_0 .. g_{P-1}), 16-B padded
constexpr int csr_row_words(int P) { return (1 + P + 3) & ~3; }

// MVM rows with a repeated field (HIP reduction paths: one slice into
// unique-order rows, or CSR entries): their per-occurrence gradients are not
// T / (1 + v) of the key's own v (the field sum is), so they leave records
// (target, c_0 .. c_{D-1}) here and three small passes after the reduction add
// them in fixed point at a per-step scale (the forward's largest |c|): resolve
// the targets (CSR: the (key, slice) entry) and zero their accumulators, sum,
// add each target's sum to its row / entry once -- order-free, so
// deterministic (float atomics were not).  The count and max words are 0
// at a step's start: the passes' last launch resets them.
struct MvmDup {
  float* rec = nullptr;          // [cap][ew]: target (u32 bits), c_0 .. c_{D-1}
  u32* n = nullptr;              // records of this step (device)
  u32* vmax = nullptr;           // max |c| (float bits)
  long long* acc = nullptr;      // [cap][D] fixed-point sums per target
  u32* claim = nullptr;          // [cap] first adder of a target
  int64_t cap = 0;
  int ew = 0;
};

struct FwdArgs {
  BatchView batch;
  MvmDup mdup;
  const u32* pos = nullptr;        // [nnz]
  // dedup slot of overflowed occurrences (the scratch's trash slot, == cap):
  // read as zero weights, never reduced (none: ~0)
  u32 trash_pos = 0xFFFFFFFFu;
  const float* wpull = nullptr;    // [scratch_cap][pstride] (fm_vals: [scratch_cap][4])
  // Reference-math FM on compact value rows: the pull emits (w, Σ_k v_k,
  // Σ_k v_k^2, 0) per key -- all the reference forward and its (B, C)
  // backward need (fm_worker.cc:159-202) -- so a row gathers 16 B per
  // feature instead of the whole (1+D)-float row (PullArgs::fm_vals).
  bool fm_vals = false;
  float* grad = nullptr;           // [scratch_cap][S][pstride] (null: forward only)
  u32* tmask = nullptr;            // [scratch_cap] slice-touch bits (null unless S>1)
  float* pctr = nullptr;           // [rows] optional
  LossStats* stats = nullptr;      // accumulated (device)
  ModelSpec model;
  int S = 1;                       // slices in this batch
  bool agg_ok = false;             // grad indices (pos*S+s)*pstride fit in a u32 (LDS aggregation)
  // HIP LR gradient reduction without global float atomics (null: atomics).
  // Workgroups write their per-column partial sums as (dest, value) pairs,
  // which are partitioned by dest >> kRedShift and summed per bucket in LDS.
  u64* red_pairs = nullptr;        // [nnz] per-workgroup pair regions
  u64* red_sorted = nullptr;       // [nnz] pairs in bucket order
  u32* red_hist = nullptr;         // [red_nb][workgroups] pairs per (bucket, workgroup)
  u32* red_tot = nullptr;          // [red_nb + 1] pairs per bucket, then bucket starts
  u32* red_count = nullptr;        // [workgroups] pairs per workgroup
  int red_nb = 0;                  // buckets allocated (<= the bucket cap)
  // bucket cap of this step's geometry: kRedMaxBuckets (0), or the vector
  // records' vec_red_max_buckets (Engine: standard FM / MVM)
  int red_maxb = 0;
  int64_t red_sorted_words = 0;    // u64 words of red_sorted
  // This step's bucket width is decided on the device: dests = slot*S + s lie
  // below red_bcap[0]*S (the scratch capacity the batch was deduplicated
  // with, adaptive), and the shift is the smallest >= red_shift(NV) giving at
  // most kRedMaxBuckets buckets; a bucket wider than the LDS accumulator is
  // summed by several workgroups (red_nsub: the most that can be needed).
  const unsigned long long* red_bcap = nullptr;
  uint64_t red_cap = 0;            // allocated scratch capacity (upper bound)
  // Unique-index positions (Engine's fused step, Backend::remap_pos): pos
  // holds each occurrence's index in the batch's unique list, wpull is in
  // unique order, dests = unique * S + s lie below red_nuq[0] * S, and the
  // unique-order outputs take dest / S directly (red_inv == null)
  const int64_t* red_nuq = nullptr;
  // optional: the producers add the records they wrote (Engine::count_records)
  unsigned long long* red_records = nullptr;
  // MVM's per-step fixed-point scale: the forward atomically maxes |T| into
  // red_vmax[0] (float bits) and clears red_vmax_next for the next step (two
  // alternating words); the vector reduction scales its int64 sums by it
  u32* red_vmax = nullptr;
  u32* red_vmax_next = nullptr;
  // MVM: set (non-zero) by the forward when a row with a repeated field added
  // its gradients to the rows by atomics; cleared for the next step like
  // red_vmax_next.  With it zero the reduction's epilogue stores its rows
  // without reading them back (they hold the pull's zeros)
  u32* red_dup = nullptr;
  u32* red_dup_next = nullptr;
  int red_nsub = 1;
  // producer workgroups the reduction buffers hold (red_hist rows, red_count);
  // 0: the model's fixed rows per workgroup.  A smaller batch (a slice group
  // of a step of more than 32 slices) may then run narrower workgroups
  int red_groups = 0;
  // S > 1: the reduction also writes each slot's slice-presence bits
  // (red_masks[slot] |= 1 << s for every (key, slice) with an occurrence),
  // replacing one global atomic per occurrence (slice_masks) on hot keys
  u32* red_masks = nullptr;
  // One slice: the bucket sums go straight to a unique-order (= send order in
  // the multi-rank step) buffer through the compaction's slot -> unique map,
  // instead of the slot-indexed grad (no gather, a dense apply read):
  // LR red_out[red_inv[dest]] = sum / red_rows[0]; compact FM
  // red_out[2 red_inv[dest] + {0,1}] = (B, C) (normalised by the apply).
  // red_out must be zeroed by the caller.
  float* red_out = nullptr;
  const u32* red_inv = nullptr;
  const int32_t* red_rows = nullptr;
  // Reference-math FM on the reduction path: keep only (B, C) = (Σ loss,
  // Σ loss*vsum) in the first two floats of each gradient row; the apply
  // expands them with the key's pre-step weights (ApplyArgs::fm_compact).
  bool fm_compact = false;
  // MVM on the reduction path: a dup-free row's occurrence gradient is
  // loss*M_k/(1+v_ik), so records are (dest | row << 32), red_rowv[row] holds
  // T = loss*M ([rows][pstride]) and the sum divides Σ T by (1 + v) per key.
  float* red_rowv = nullptr;
  // CSR outputs (red_csr.cnt != null; LR / reference FM with unique-index
  // positions, S = 2^slog2): one reduction over every slice of the step
  CsrOut red_csr;
  // set to 2 (OR) when a row's prediction is non-finite or out of [0, 1], or
  // a fixed-point input is out of range (a diverged model): the values are
  // clamped before the fixed-point conversion and the capacity monitor
  // raises (Engine::poll_snapshots)
  u32* fx_bad = nullptr;
};
constexpr int kRedShift = 14;      // 16384 gradient destinations per bucket (64 KB of LDS)
constexpr int kRedMaxBuckets = 4096;
// destinations per bucket for NV aggregated values per key (NV x 2^shift x 4 B <= 64 KB)
// (nv >= 3: standard-FM vector records, 1 + D values: 2^shift x nv int64 in
// at most ~114 KB of LDS)
constexpr int red_shift(int nv) {
  return nv == 1 ? kRedShift : (nv == 2 ? kRedShift - 1 : (nv <= 14 ? 10 : (nv <= 28 ? 9 : 8)));
}
// Vector records (standard FM / MVM, produced by k_fm_std_red<D>, NV = 1 + D):
// twice the buckets where the producer's LDS -- its column table of 2 x BLOCK
// slots (tag + NV int64) plus per-bucket counts and cursors -- still fits in
// the CU's 160 KB, so a step of several slices keeps one LDS unit of dests per
// bucket (each extra unit re-reads the bucket's records)
constexpr int fmstd_block(int D) { return D <= 10 ? 512 : (D <= 16 ? 256 : 128); }
constexpr int kSegMaxGroups = 2048;  // producer workgroups of the scatter-free vector form
// LDS of the producer: column-table slots (tag + NV int64 each), the row
// list, per-bucket record cursors
constexpr int64_t fmstd_lds_at(int D, int slots, int maxb) {
  return (int64_t)slots * 8 * (2 + D) + 2 * fmstd_block(D) + (int64_t)maxb * 4 + 1024;
}
// Column-table slots: the largest table of 2, 1.75, 1.5 or 1.25 x BLOCK
// (load <= 0.8 for a column of BLOCK distinct keys) that leaves the CU room
// for two producer workgroups -- the column walk is a chain of barriers and
// LDS round trips, a second workgroup hides them -- else 2 x BLOCK
constexpr int fmstd_slots(int D) {
  for (int q = 8; q >= 5; --q)
    if (fmstd_lds_at(D, fmstd_block(D) * q / 4, kRedMaxBuckets) <= 80 * 1024)
      return fmstd_block(D) * q / 4;
  return 2 * fmstd_block(D);
}
constexpr int64_t fmstd_lds(int D, int maxb) { return fmstd_lds_at(D, fmstd_slots(D), maxb); }
// (only where the workgroups per CU stay the same)
constexpr int vec_red_max_buckets(int D) {
  return fmstd_lds(D, 2 * kRedMaxBuckets) <= 160 * 1024 &&
                 (160 * 1024) / fmstd_lds(D, 2 * kRedMaxBuckets) ==
                     (160 * 1024) / fmstd_lds(D, kRedMaxBuckets)
             ? 2 * kRedMaxBuckets
             : kRedMaxBuckets;
}
// Column-table slots of the int32-accumulator producer (standard FM: a u32
// tag, 1 + D int32 sums and a joined flag per slot): the LDS of the int64
// table buys 2x the slots, i.e. a column load <= 0.33 instead of 0.67 -- the
// insert's linear probe is a chain of dependent LDS round trips, and a wave
// waits for its longest chain
constexpr int fmstd_slots32(int D) {
  for (int q = 16; q >= 5; --q)
    if ((int64_t)(fmstd_block(D) * q / 4) * (4 + 4 * (1 + D) + 1) +
            (int64_t)vec_red_max_buckets(D) * 4 + 2048 <= 80 * 1024)
      return fmstd_block(D) * q / 4;
  return fmstd_slots(D);
}
// 32-bit words of a standard-FM vector record (dest + nv values), 16-B padded
constexpr int vec_rec_words(int nv) { return (1 + nv + 3) & ~3; }
constexpr int kLrGroupRows = 1024;  // rows per LR workgroup on the reduction path
constexpr int kFmGroupRows = 1024;  // rows per reference-FM workgroup on the reduction path (A/B: 512 -1.8 %)
// smallest rows per standard-FM producer workgroup (v_dim > 16; 256 up to
// v_dim 10): sizes the reduction's per-workgroup histogram
constexpr int kFmStdMinGroupRows = 128;
constexpr int kMvmGroupRows = 512;  // rows per MVM forward workgroup on the reduction path (k_mvm2: T rows)

struct PullArgs {
  TableView table;
  OptSpec opt;
  const u64* keys = nullptr;
  const int64_t* n_dev = nullptr;  // count (device) or null => n_host
  int64_t n_host = 0;
  int64_t n_max = 0;
  bool insert = true;
  u32* out_slot = nullptr;         // [n] slot index (UINT32 max when absent)
  float* out_vals = nullptr;       // rows of pstride floats
  const u32* out_map = nullptr;    // row index for entry i (null => i)
  int pstride = 1;
  // LR-FTRL 16-byte slots, fused step: the (n, z) each key was pulled with,
  // in unique order (read back by the apply instead of the table), and a
  // unique-order gradient buffer to zero for the reduction's direct writes.
  float* out_nz = nullptr;         // [n][2] (LR), [n][P][2] (packed pull, FTRL: n = -1 never pushed)
  float* zero_out = nullptr;       // [n][zero_width]
  int zero_width = 1;
  // reference-math FM: out_vals rows are (w, Σ v, Σ v^2, 0) (FwdArgs::fm_vals)
  bool fm_vals = false;
  // optional per-parameter pulled weights [n][pstride] in entry order (the
  // owner keeps them for an apply that runs after other table updates)
  float* out_w = nullptr;
};

// Owner-side grouping of the keys a rank received from several sources in
// one sharded step (HIP): every received entry finds its key's slot in an
// owner scratch table and registers itself under (slot, source).  The apply
// then runs once over all entries: the entry of a key's first source is its
// leader and pushes every source's contributions in source order -- one
// launch per step instead of one per source, and the key's state is read and
// written once (from the pull's stash when nothing touched the table since).
constexpr int kMaxGroupSources = 64;
struct SrcGroups {
  const u32* opos = nullptr;   // [n] owner-scratch slot of each received entry
  const u64* oidx = nullptr;   // [ocap][nsrc]: (epoch << 32) | entry, per (slot, source)
  int nsrc = 0;
  u32 epoch = 0;               // entries of other steps carry other epochs
  int64_t offs[kMaxGroupSources + 1] = {};  // entries of source s: [offs[s], offs[s+1])
};

struct OwnerGroupArgs {
  const u64* keys = nullptr;   // received keys, grouped by source
  int64_t n = 0;
  u64* okeys = nullptr;        // owner scratch keys [ocap] (kEmptyKey when free)
  u64 ocap = 0;                // power of two
  u32* opos = nullptr;         // out [n]
  u64* oidx = nullptr;         // out [ocap][nsrc]
  SrcGroups g;                 // nsrc, epoch, offs
  u32* overflow = nullptr;
};

// libffm text -> CSR batch on the device (Backend::parse_text; HIP:
// kernels_parse.hip, CPU: reader.cpp's parser).  Rules of reader.cpp.
struct TextParseArgs {
  const char* text = nullptr;      // block bytes (backend memory, 16-byte aligned, allocated >= n + 32)
  int64_t n = 0;
  u64* keys = nullptr;             // [max_nnz]
  int32_t* fgid = nullptr;         // [max_nnz]
  int32_t* row_ptr = nullptr;      // [max_rows + 1]
  float* labels = nullptr;         // [max_rows]
  int64_t max_rows = 0, max_nnz = 0;
  int64_t max_lines = 0;           // text_max_lines(n)
  u32* ws = nullptr;               // text_ws_words(n) words of workspace
  int64_t ws_words = 0;
  // rows the caller will use: the first rows - rows % row_mod (the slicing
  // rule, lr_worker.cc:190); counts[6] = their occurrences
  int64_t row_mod = 1;
  // backend [7]: rows, occurrences, shortest / longest row, lines, line
  // overflow, occurrences of the used rows (nothing is written past max_rows
  // / max_nnz: the caller checks)
  long long* counts = nullptr;
};
// lines of n bytes: at most n/2 + 2 ("x\n" per line; a block of mostly empty
// lines overflows the workspace and is flagged)
XF_HD int64_t text_max_lines(int64_t n) { return n / 2 + 2; }
XF_HD int64_t text_ws_words(int64_t n) {
  const int64_t L = text_max_lines(n), nwg = (n + 4095) / 4096;
  return ((nwg + 3) & ~3ll) + ((L + 1 + 3) & ~3ll) + 2 * L + 2 * (L / 1024 + 2);
}

// A step's capacity snapshot (Engine's monitor) in coherent pinned host
// memory, packed into ONE 64-bit word so a single store publishes it whole:
// bits [0, 32) table size (<= 2^31 slots), bit 32/33 the scratch/table
// overflow flags, bit 34 the non-finite-loss flag (FwdArgs::fx_bad), bits
// [35, 64) the snapshot's sequence number.  No fence is needed (a
// system-scope release would write back the L2 every step).
struct HostSnap {
  unsigned long long word;
};
constexpr int kSnapSeqShift = 35;
XF_HD unsigned long long pack_snapshot(unsigned long long size, u32 ovf0, u32 ovf1,
                                              unsigned long long seq) {
  return (seq << kSnapSeqShift) | ((unsigned long long)((ovf0 & 2u) != 0u) << 34) |
         ((unsigned long long)(ovf1 != 0u) << 33) | ((unsigned long long)((ovf0 & 1u) != 0u) << 32) |
         (size & 0xFFFFFFFFull);
}

struct ApplyArgs {
  TableView table;
  // optional: the kernel's first wave writes the capacity snapshot (size,
  // overflow flags -- final once the step's pulls ran) before its work, so a
  // step needs no extra launch or event for the monitor
  HostSnap* snap = nullptr;
  const u32* snap_mon = nullptr;   // device {size u64, overflow[2]}
  unsigned long long snap_seq = 0;
  OptSpec opt;
  const u64* keys = nullptr;       // needed for latent init of un-pushed slots
  const u32* slots = nullptr;
  const int64_t* n_dev = nullptr;
  int64_t n_host = 0;
  int64_t n_max = 0;
  float* grads = nullptr;          // rows of S*pstride floats
  const u32* grad_map = nullptr;   // row index for entry i (null => i)
  const u32* masks = nullptr;      // per-row slice bits (null => all S slices)
  bool masks_clear = false;        // zero each entry's bits once read (unique-order
                                   // bits of a slice group: the next group starts from zero)
  bool zero_after = false;         // clear consumed gradient rows (and masks)
  u32* masks_rw = nullptr;         // masks buffer to clear when zero_after
  int S = 1;
  int pstride = 1;
  int P = 1;
  bool sum_slices = false;         // one push of Σ_s g_s instead of S ordered pushes
  // Raw per-slice loss sums are divided by the slice's row count here, in
  // double like lr_worker.cc:116-118 (null => rows already normalised).
  const int32_t* slice_rows = nullptr;
  // Gradient rows hold (B, C) of reference-math FM (FwdArgs::fm_compact):
  // g_w = D*B, g_v[k] = C - v_k*B with v_k the key's pre-step (pulled) value.
  bool fm_compact = false;
  int fm_D = 0;
  // LR-FTRL 16-byte slots: (n, z) of entry i as pulled this step (PullArgs::
  // out_nz); the slot is then only written.  Valid while no other push to
  // the key intervenes (the fused single-source step).
  const float* nz_stash = nullptr;
  // floats per (row, slice) in grads (0 => pstride; 2 for compact FM rows)
  int gstride = 0;
  // fm_compact with several sources per step: the values this rank's pull
  // served for entry i ([n][pstride], the workers' pre-step weights), since
  // the table already holds the previous sources' updates.  Null: the table.
  const float* pulled = nullptr;
  // Optional fused reset of the worker dedup scratch (single-device path).
  ScratchView scratch;
  const u32* reset_pos = nullptr;
  // CSR gradients (csr_cnt != null, CsrOut): entry i's pushes are its CSR
  // entries in order (the entries carry their slices; grads / masks unused)
  const u32* csr_off = nullptr;
  const u32* csr_cnt = nullptr;
  const void* csr_ent = nullptr;
  // 0: scalar entries (LR u64, reference-FM (slice, B, C)); else the words of
  // a full-row entry (slice, g_0 .. g_{P-1}, pad: standard FM, csr_row_words)
  int csr_ew = 0;
  // (HIP) keys with more than kCsrShortChain entries are deferred to a second
  // launch over the list of them (u32 [n] + a u32 counter): a wave then holds
  // chains of similar length instead of one hot key's slice-long chain and 63
  // idle lanes
  u32* csr_long = nullptr;
  int64_t csr_long_cap = 0;        // u32 words at csr_long
  // Several sources in one launch (grp.oidx != null): n counts all received
  // entries; an entry's gradient row / mask / pulled values / stash are
  // indexed by the entry, and each key is applied by its first source's entry.
  SrcGroups grp;
};

struct GatherGradArgs {           // worker: pos-indexed raw sums -> send order
  const float* grad = nullptr;     // [scratch_cap][S][pstride], cleared after read
  float* grad_rw = nullptr;        // same buffer (for clearing)
  const u32* tmask = nullptr;      // optional slice bits, cleared after read
  u32* tmask_rw = nullptr;
  const u32* map = nullptr;        // send_pos
  const int64_t* n_dev = nullptr;
  int64_t n_max = 0;
  int S = 1;
  int pstride = 1;
  const int32_t* slice_rows = nullptr;  // [S]
  float* out = nullptr;            // [n][S*width] normalised gradients
  u32* out_mask = nullptr;         // [n] (when tmask)
  int width = 0;                   // values per (key, slice) gathered (0 => pstride)
};

struct BucketArgs {                // group unique keys by owning rank
  const u64* uniq_keys = nullptr;
  const u32* uniq_pos = nullptr;
  const int64_t* n_dev = nullptr;
  int64_t n_max = 0;
  int world = 1;
  int64_t* counts = nullptr;       // [world] (device) out
  int64_t seq = -1;                // >= 0: write encode_count(count, seq)
  u64* send_keys = nullptr;        // [n_max] out, grouped by owner
  u32* send_pos = nullptr;         // [n_max] out
  int64_t* scratch = nullptr;      // [2*world] workspace
};

// A packed block of a v3 .xfb shard (xflow_amd/data/binfmt.py, fixed-width
// rows): u8 labels, then one column per field of 1/2/4/8-byte codes -- the
// key itself (direct) or an index into the field's dictionary of u64 keys (a
// device-resident copy of the shard's dictionaries).  Backend::unpack_block
// writes the engine's field-major batch from it: half or less of the
// compact shard's bytes cross the host link, the gathers hit small tables.
constexpr int kMaxPackedFields = 64;
struct UnpackArgs {
  const uint8_t* block = nullptr;          // the block's bytes (backend memory, 16-B aligned)
  int64_t rows = 0;
  int F = 0;
  int width[kMaxPackedFields] = {};        // bytes per code: 1, 2, 4 or 8
  int64_t col_off[kMaxPackedFields] = {};  // byte offset of field f's column in the block
  const u64* dict[kMaxPackedFields] = {};  // null: direct keys
  int32_t fgid_col[kMaxPackedFields] = {}; // the field id of column f
  u64* keys = nullptr;                     // out [F][rows]
  float* labels = nullptr;                 // out [rows] (0 / 1)
  int32_t* fgid = nullptr;                 // out [F][rows], optional
};

struct SynthArgs {                 // synthetic Criteo-shaped batch generator
  u64* keys = nullptr;
  float* labels = nullptr;
  int32_t* fgid = nullptr;         // optional
  int64_t rows = 0;
  int fields = 39;
  const uint64_t* vocab = nullptr;    // [fields] cardinalities (host or device per backend)
  const float* zipf_s = nullptr;      // [fields] exponents
  uint64_t hash_space = 1000000000ull;
  uint64_t seed = 0;
  uint64_t step = 0;
  float planted_scale = 0.3f;
  float planted_bias = -1.2f;
  int64_t col_stride = 0;            // > 0: field-major output (BatchView::col_stride)
};

// Evaluation sums of a prediction set (Backend::eval_metrics): the inputs of
// the reference's calculate_auc print (base.h:84-110).
struct EvalMetrics {
  int64_t n = 0;          // predictions
  int64_t tp = 0;         // positives
  uint64_t area = 0;      // sum over negatives of the positives ranked above (pctr desc, stable)
  double log2_sum = 0;    // sum y*log2(p) + (1-y)*log2(1-p)
  double ln_sum = 0;      // sum of -ln likelihood, p clipped to [1e-7, 1-1e-7]
};

class Backend {
 public:
  virtual ~Backend() = default;
  virtual bool is_gpu() const = 0;
  virtual std::string name() const = 0;

  // memory
  virtual void* alloc(size_t bytes) = 0;
  virtual void free(void* p) = 0;
  // Stream-ordered allocation (HIP: hipMallocAsync / hipFreeAsync on the
  // backend's stream): a buffer freed this way may still be read by work
  // queued before the free, and neither call waits on the host -- buffers
  // that grow in the middle of a step (the sharded step's exchange buffers)
  virtual void* alloc_stream(size_t bytes) { return alloc(bytes); }
  virtual void free_stream(void* p) { free(p); }
  virtual void memset(void* p, int v, size_t bytes) = 0;
  virtual void fill_u64(u64* p, u64 v, size_t n) = 0;
  virtual void copy_h2d(void* dst, const void* src, size_t bytes) = 0;
  virtual void copy_d2h(void* dst, const void* src, size_t bytes) = 0;  // synchronising
  virtual void copy_d2d(void* dst, const void* src, size_t bytes) = 0;
  // queued on the stream, no host wait (checkpoint streaming through pinned
  // staging buffers; the CPU backend copies at once)
  virtual void copy_d2h_async(void* dst, const void* src, size_t bytes) { copy_d2h(dst, src, bytes); }
  virtual void copy_h2d_async(void* dst, const void* src, size_t bytes) { copy_h2d(dst, src, bytes); }
  // page-locked host memory for DMA staging (HIP: non-coherent pinned)
  virtual void* staging_alloc(size_t bytes) { return host_alloc(bytes); }
  virtual void staging_free(void* p) { host_free(p); }
  // <= 256 bytes from the host, queued without a host wait (HIP: the bytes
  // travel as a kernel argument)
  virtual void upload_small(void* dst, const void* src, size_t bytes) = 0;
  // device bytes into mapped pinned host memory, queued without a copy
  // engine or host wait (HIP: a kernel's stores; the host reads them after an
  // event recorded behind it)
  virtual void download_small(void* host_dst, const void* src, size_t bytes) = 0;
  virtual void synchronize() = 0;
  virtual void set_stream(void* stream) = 0;
  virtual void* stream() const = 0;
  // make this backend's device current on the calling thread (a second host
  // thread driving the backend: the async parameter server's server thread)
  virtual void bind_thread() {}
  // Bytes of device memory still free (table growth checks it first).
  virtual size_t free_memory() const { return ~(size_t)0; }
  // Write a capacity snapshot {mon: size u64, overflow[2]} with sequence seq
  // into pinned host memory, queued on the stream (a tiny kernel on HIP; the
  // apply kernels do the same through ApplyArgs::snap when a step has one).
  virtual void snapshot(HostSnap* dst, const u32* mon, unsigned long long seq) = 0;

  // Host-visible step snapshots (Engine's capacity monitor): pinned host
  // memory a kernel can write (download_small), and completion events on the
  // backend's stream.  The CPU backend is synchronous: events are always done.
  virtual void* host_alloc(size_t bytes) = 0;
  virtual void host_free(void* p) = 0;
  virtual void* event_create() { return nullptr; }
  virtual void event_destroy(void* e) { (void)e; }
  virtual void event_record(void* e) { (void)e; }
  virtual bool event_done(void* e) { (void)e; return true; }
  virtual void event_wait(void* e) { (void)e; }
  // wait by polling (no blocking-sync wake-up latency: a host that must
  // enqueue the next device work the moment this event fires -- the CSR
  // exchange's entry totals, the async parameter server's hand-overs)
  void event_spin(void* e) {
    while (!event_done(e)) {
    }
  }

  // Asynchronous double-buffered host -> device staging (the native trainer's
  // input path).  Slot s in {0, 1}: stage_begin(s) waits on the host until
  // slot s's previous copies have left its pinned buffer; stage_pinned
  // returns that pinned buffer (grow-only); stage_copy queues dst <- pinned+off
  // on a copy queue, after the compute work that last read slot s's device
  // buffers (stage_release); stage_commit makes the compute queue wait for the
  // slot's copies.  The CPU backend copies synchronously.
  virtual void stage_begin(int s) { (void)s; }
  virtual void* stage_pinned(int s, size_t bytes) = 0;
  virtual void stage_copy(int s, void* dst, size_t off, size_t bytes) = 0;
  virtual void stage_commit(int s) { (void)s; }
  virtual void stage_release(int s) { (void)s; }

  // kernels
  // Mark every slot free (key words = kEmptyKey) with zero optimizer state.
  virtual void table_clear(const TableView& t) = 0;
  virtual void dedup(const u64* keys, int64_t nnz, ScratchView s, DedupOut o) = 0;
  virtual void scratch_reset(ScratchView s, const u32* pos, const int64_t* n_dev,
                             int64_t n_max) = 0;
  virtual void table_pull(const PullArgs& a) = 0;
  virtual void table_apply(const ApplyArgs& a) = 0;
  virtual void forward_backward(const FwdArgs& a) = 0;
  virtual void slice_masks(const BatchView& b, const u32* pos, u32* tmask) = 0;
  // pos[i] = inv[pos[i]] for i < nnz (scratch slot -> unique-list index; the
  // trash slot's occurrences get `none`): the fused step's unique-index
  // positions (FwdArgs::red_nuq).  HIP only (the compaction writes inv).
  // libffm text -> CSR (see TextParseArgs); counts stay in backend memory
  virtual void parse_text(const TextParseArgs& a) = 0;
  virtual bool remaps_positions() const { return false; }
  virtual void remap_pos(u32* pos, int64_t nnz, const u32* inv, u32 none) {
    (void)pos, (void)nnz, (void)inv, (void)none;
    throw std::runtime_error("remap_pos is not supported by this backend");
  }
  virtual void bucket(const BucketArgs& a) = 0;
  // Owner-partitioned dedup (ScratchView::parts > 1, HIP only): per-owner
  // counts of the unique list from the compaction's chunk offsets.
  virtual bool partitioned_dedup() const { return false; }
  virtual void partition_counts(const ScratchView& s, const u32* chunk_offsets,
                                const int64_t* n_uniq, int64_t* counts, int64_t seq) {
    (void)s, (void)chunk_offsets, (void)n_uniq, (void)counts, (void)seq;
    throw std::runtime_error("partitioned dedup is not supported by this backend");
  }
  // Owner grouping for the one-launch multi-source apply (HIP only).
  virtual bool owner_grouping() const { return false; }
  virtual void owner_group(const OwnerGroupArgs& a) {
    (void)a;
    throw std::runtime_error("owner grouping is not supported by this backend");
  }
  // CSR exchange of the multi-rank step (HIP only): out[i] = sum of in[< i],
  // out[n] = total, n = *n_dev (or n_max); dense packing of key i's entries
  // (entry_bytes each) from src[off[i]..] to dst[doff[i]..]; per-owner entry
  // totals from the step's (encoded) key counts per owner and the dense offsets
  virtual bool csr_exchange() const { return false; }
  virtual void scan_u32(const u32* in, u32* out, const int64_t* n_dev, int64_t n_max) {
    (void)in, (void)out, (void)n_dev, (void)n_max;
    throw std::runtime_error("scan_u32 is not supported by this backend");
  }
  virtual void csr_pack(const u32* off, const u32* cnt, const void* src, const u32* doff,
                        const int64_t* n_dev, int64_t n_max, void* dst, int entry_bytes) {
    (void)off, (void)cnt, (void)src, (void)doff, (void)n_dev, (void)n_max, (void)dst,
        (void)entry_bytes;
    throw std::runtime_error("csr_pack is not supported by this backend");
  }
  virtual void csr_totals(const int64_t* counts, int world, bool encoded, const u32* doff,
                          int64_t* totals) {
    (void)counts, (void)world, (void)encoded, (void)doff, (void)totals;
    throw std::runtime_error("csr_totals is not supported by this backend");
  }
  virtual void gather_grads(const GatherGradArgs& a) = 0;
  // rows of `width` floats: dst[map? map[i] : i] = src[i]   (scatter)
  // (zero_out: also zero zero_out[0..n*zero_width), the direct send buffer)
  virtual void scatter_rows(const float* src, float* dst, const u32* map,
                            const int64_t* n_dev, int64_t n_max, int width,
                            float* zero_out = nullptr, int zero_width = 1) = 0;
  // dst[i] = src[map[i]]; optionally zero the source row   (gather)
  virtual void gather_rows(const float* src, float* dst, const u32* map,
                           const int64_t* n_dev, int64_t n_max, int width,
                           bool zero_src) = 0;
  virtual void gather_u32(const u32* src, u32* dst, const u32* map,
                          const int64_t* n_dev, int64_t n_max, bool zero_src) = 0;
  virtual void scatter_u32(const u32* src, u32* dst, const u32* map,
                           const int64_t* n_dev, int64_t n_max) = 0;
  virtual void synth_batch(const SynthArgs& a) = 0;
  // [rows][F] -> [F][rows] of 4- or 8-byte elements (field-major batches)
  // widen (elem_bytes 4 only): u32 source elements zero-extended to u64 --
  // compact .xfb keys (data/binfmt.py) become the engine's u64 keys in the
  // same pass
  virtual void field_major(const void* src, void* dst, int64_t rows, int F, int elem_bytes,
                           bool widen = false) = 0;
  // packed .xfb block -> field-major keys / labels / fgid (see UnpackArgs)
  virtual void unpack_block(const UnpackArgs& a) = 0;
  // count occupied slots / dump table rows (checkpointing); returns rows written
  virtual int64_t table_export(const TableView& t, u64* keys_out, u32* words_out,
                               int64_t max_rows) = 0;
  // Number of (key, param) weights that are exactly non-zero (L1 sparsity
  // report; lambda1 > 0 makes FTRL weights exactly 0 when |z| <= lambda1).
  virtual int64_t table_nonzero(const TableView& t, const OptSpec& o) = 0;
  virtual void table_import(const TableView& t, const u64* keys, const u32* words,
                            int64_t n) = 0;
  // Insert n synthetic keys (1 << 62 | hash(seed, i) >> 2: disjoint from any
  // key below 2^62, e.g. hashed features) with zero state, marked pushed --
  // keys a long run has accumulated but the current batches do not touch
  // (occupancy-realistic benchmarks).
  virtual void table_prefill(const TableView& t, int64_t n, u64 seed) = 0;
  // Split segments [s0, s0 + k) of level t.level (t.split == s0 + k, i.e. t
  // is the geometry AFTER the split; segments s0 + 2^level .. are mapped and
  // cleared): a key whose home moved to the buddy segment goes there, the keys
  // that stay are re-packed inside their cluster (no tombstones).  Table size
  // is unchanged; slots of the split segments' keys change.
  virtual void table_split(const TableView& t, u64 s0, u64 k) = 0;
  // The slot array's address range: reserve the address space of max_bytes
  // once, commit memory as the table grows.  table_commit(base, bytes) makes
  // [base, base + bytes) usable and returns the (possibly moved) base: with
  // virtual memory management the range stays in place and only the new tail
  // gets memory; without it the backend re-allocates and copies (2x peak).
  // (growable = false: the table never grows -- one plain allocation)
  virtual void* table_reserve(size_t max_bytes, bool growable) = 0;
  virtual void* table_commit(void* base, size_t bytes) = 0;
  virtual void table_release(void* base) = 0;
  // bytes of device memory committed to the table range (>= the bytes asked)
  virtual size_t table_committed() const = 0;
  // true when table_commit extends the range in place (virtual memory); false
  // when it re-allocates: the new size must then fit NEXT to the old table
  virtual bool table_in_place() const { return true; }
  // AUC / logloss sums of n predictions (backend memory; labels 0/1 floats)
  virtual EvalMetrics eval_metrics(const float* pctr, const float* labels, int64_t n) = 0;
};

std::unique_ptr<Backend> make_cpu_backend();
// Defined in csrc/hip/hip_backend.hip; ordinal = HIP device index.
std::unique_ptr<Backend> make_hip_backend(int device);
bool hip_backend_available();

}  // namespace xflow
