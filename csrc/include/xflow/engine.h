// xflow-amd: Engine — one rank's sparse CTR trainer state and step pipeline.
//
// A rank plays both ps-lite roles of the reference at once:
//   worker  (lr_worker.cc / fm_worker.cc / mvm_worker.cc): dedups a batch's
//           keys, forward/backward over its rows, produces per-(key, slice)
//           gradient sums;
//   server  (ftrl.h / sgd.h via server.h): owns a shard of the HBM hash table
//           and answers pulls / applies pushes for the keys it owns.
// Single-rank training fuses both (train_step); multi-rank training drives the
// phase methods from the distributed layer with sparse all-to-alls between
// them (xflow_amd/parallel/sparse_a2a.py).
#pragma once

#include <memory>
#include <string>
#include <vector>

#include "xflow/backend.h"

namespace xflow {

struct EngineConfig {
  ModelSpec model;
  OptSpec opt;
  int table_log2_cap = 20;     // slots = 2^table_log2_cap (<= 2^31)
  int64_t max_rows = 1 << 16;  // per step
  int64_t max_nnz = 1 << 22;   // per step
  // slices per step (any count: a step of more than kSliceGroup slices runs
  // its slices in groups of kSliceGroup over one dedup + pull, see train_step)
  int max_slices = 1;
  bool sum_slices = false;     // apply Σ_s g_s once instead of ordered per-slice pushes
  double scratch_factor = 2.5;  // dedup scratch capacity = pow2 >= factor * max_nnz
  int device = -1;             // -1 => CPU backend, else HIP device ordinal
  // Table capacity management (the reference's store is an unbounded
  // unordered_map, ftrl.h:54-56,84).  Before every inserting pull the engine
  // bounds the table's size from below-lagging device snapshots plus the
  // inserts queued since (each at most the pull's key count), and grows the
  // table by segment splits (TableView, backend.h) on a schedule that keeps
  // the fullest segments' load <= grow_load: with u = the load of a segment
  // not yet split at this level, the first 2^level * (u - grow_start) /
  // (grow_load - grow_start) segments are split.  A split is stream-ordered
  // device work on one segment plus one new segment of memory -- no host
  // sync, no copy of the table -- up to 2^max_log2_cap slots.
  // table_grow = false keeps the capacity fixed: an insert that finds no slot
  // flags the overflow, and the next step start raises within monitor_lag
  // steps of it.
  bool table_grow = true;
  double grow_load = 0.8;
  double grow_start = 0.6;     // (< grow_load; else 3/4 of it)
  int max_log2_cap = 0;        // 0 => 31, and what the device's free memory allows
  // steps the host may run ahead of the device before it waits for a
  // snapshot (bounds both the growth bound's slack and fail-fast latency)
  int monitor_lag = 2;
  // Owner apply of a multi-source sharded step (GPU): 0 = one launch per
  // source in source order (default), 1 = one grouped launch (k_owner_group
  // registration + leader apply).  Per source measured faster for every
  // model in the emulated 8-GPU step (device us per rank-step, LR 617 vs
  // 687, FM-8 846 vs 893, MVM-10 1082 vs 1184:
  // profiles/r3s3_w8_owner_apply_ab.txt).
  int owner_group = 0;
  // Steps of several slices on the GPU for LR-FTRL / reference FM: CSR
  // gradients (one reduction and one apply of the touched (key, slice)
  // pairs, Engine::train_step_csr) -- else slice groups of kSliceGroup
  // (the same pushes, dense per-group buffers; also what a slice count the
  // CSR dests cannot address falls back to)
  bool csr = true;
};

// What the single-rank step's gradient layout depends on (Engine::step_inputs)
struct StepInputs {
  bool gpu = false;        // HIP backend
  bool remaps = false;     // Backend::remaps_positions (unique-index positions)
  bool red_pairs = false;  // the bucket reduction's buffers exist
  bool red_rowv = false;   // ... and its vector records (MVM)
  bool fm_vals = false;    // reference FM on value rows: compact (B, C) gradients
  bool csr = true;         // EngineConfig::csr
  bool sum_slices = false;
  int kind = kLR;  // ModelKind
  int fm_math = kFmReference;  // FmMath
  TableLayout L;
  double scratch_cap = 0.0, max_nnz = 0.0, max_rows = 0.0;
  int pstride = 1, slice_cap = 1;
  int kdim = 1;  // latent width of the kernels (ModelSpec::kernel_dim)
};

// Where a step's gradients land, one per step:
//   kCsr        CSR entries of the touched (key, slice) pairs (S > 1, LR-FTRL 16-byte
//               slots, reference FM, or the full rows of standard FM and MVM): one
//               reduction, one chain apply
//   kUniqueLR   LR-FTRL normalised sums in unique order ([unique][slice] + slice bits)
//   kUniqueFmBC reference-FM normalised (B, C) in unique order
//   kUniqueRows full gradient rows in unique order (standard FM any S, MVM S = 1)
//   kSlotSums   LR-FTRL summed slices, slot-indexed (sum_slices)
//   kSlotRows   slot- or position-indexed rows the apply gathers and zeroes (CPU, fallbacks)
enum class GradPath : int { kCsr = 0, kUniqueLR, kUniqueFmBC, kUniqueRows, kSlotSums, kSlotRows };
const char* grad_path_name(GradPath g);

// The step's layout decisions, made once by plan_step (a pure function of
// StepInputs and S: unit-tested over the whole input space on the CPU) and
// only read by Engine::train_step.  Field meanings at their use there.
struct StepPlan {
  int S = 1, groups = 1, Sf = 1;  // slices, slice groups, slices per group
  int csr_slog2 = -1;             // kCsr: log2 of the padded slice count
  bool csr_rows = false;          // kCsr of full-row entries (standard FM, MVM)
  GradPath grad = GradPath::kSlotRows;
  bool masks = false;     // ordered per-slice pushes read slice bits
  bool upos = false;      // unique-index positions (Backend::remap_pos)
  bool lr16 = false;      // kUniqueLR
  bool lr16s = false;     // kSlotSums
  bool uqm = false;       // slice bits from the reduction
  bool fmu = false;       // kUniqueFmBC
  bool fm_keep_w = false; // the pull keeps per-parameter weights (grouped compact FM)
  bool mvmu = false, fsu = false, rowu = false;  // kUniqueRows (MVM, standard FM, either)
  bool grpst = false;     // the pull stashes (n, z) of multi-parameter FTRL keys
  bool uq = false;        // unique-order slice bits (S > 1 on a unique-order layout)
};
StepPlan plan_step(const StepInputs& in, int S);

class Engine {
 public:
  explicit Engine(const EngineConfig& cfg);
  ~Engine();
  Engine(const Engine&) = delete;
  Engine& operator=(const Engine&) = delete;

  const EngineConfig& config() const { return cfg_; }
  Backend& backend() { return *be_; }
  bool is_gpu() const { return be_->is_gpu(); }
  void set_stream(void* s) { be_->set_stream(s); }
  void synchronize() { be_->synchronize(); }

  // ---- single-rank fused step -------------------------------------------
  // Batch pointers are backend memory (device pointers on the HIP backend).
  void train_step(const BatchView& b);
  // Forward only; pctr (backend memory, may be null) receives predictions.
  // Keys are looked up without insertion.
  void eval_step(const BatchView& b, float* pctr);

  // Push explicit gradients (host arrays) to keys, like the reference's
  // initialisation pushes (lr_worker.cc:180-182, fm_worker.cc:248-252).
  void push_host(const std::vector<u64>& keys, const std::vector<float>& grads);
  // Insert n synthetic keys no batch touches (Backend::table_prefill):
  // occupancy-realistic benchmarks of a long run's table.
  void prefill(int64_t n, uint64_t seed);
  // Backend::download_small on the engine's stream
  void download_small(void* host_dst, const void* src, size_t bytes) {
    be_->download_small(host_dst, src, bytes);
  }
  // Pull current values (host) of keys without inserting them.
  std::vector<float> pull_host(const std::vector<u64>& keys);

  // ---- multi-rank phases --------------------------------------------------
  // Worker phases take a worker buffer set wb (0/1): the dedup positions, send
  // map and counts of a prepared batch live there, so the next batch can be
  // prepared (deduplicated, counts exchanged) while the current one is still
  // in its forward/backward -- the pipelined sharded step.
  // worker: dedup the batch and group its unique keys by owner rank.
  // counts_out: backend int64[world]; send_keys_out: backend u64[>= n_unique].
  // seq (world > 1): the caller's prepare sequence number, carried in the
  // counts (encode_count) so that peers detect a rank that skipped a step.
  void w_prepare(const BatchView& b, int world, int64_t* counts_out, u64* send_keys_out,
                 int wb = 0, int64_t seq = -1);
  // server: probe/insert n received keys, write pulled rows (pstride floats)
  // into out_vals (backend memory), remember slots for s_apply.
  // buf selects one of two server slot buffers (pipelined steps alternate).
  // src_offsets (world+1 entries, optional): the sources' ranges of the
  // received keys; with several sources the GPU backend groups the entries by
  // key here so that s_apply is one launch.
  // keep_weights: also keep the per-parameter pulled weights for the apply
  // (needed when other updates reach the table between this pull and its
  // apply, i.e. the staleness-1 step, with compact FM value rows)
  void s_pull(const u64* recv_keys, int64_t n, float* out_vals, bool insert = true, int buf = 0,
              const std::vector<int64_t>& src_offsets = {}, bool keep_weights = false);
  // worker: forward only from pulled rows (sharded evaluation); pctr may be null.
  void w_forward(const BatchView& b, const float* pulled, int64_t n_send, float* pctr, int wb = 0);
  // worker: place pulled rows (in send order) into the pos-indexed buffer,
  // run forward/backward, then emit normalised gradients in send order.
  // grads_out: [n_send][S*pstride]; masks_out: [n_send] (used when S>1).
  // S_global > kSliceGroup: slice group `group` only (its rows, group_slices
  // slices: grads_out [n_send][group_slices*width]); every group reads the
  // same pulled rows, and the groups' pushes are applied in group order.
  void w_forward_backward(const BatchView& b, const float* pulled, int64_t n_send,
                          float* grads_out, u32* masks_out, int S_global = 0, int wb = 0,
                          int group = 0);
  // ---- the CSR exchange (several slices, GPU: LR-FTRL / reference FM) ----
  // log2 of the padded slice count when a step of S slices runs its gradients
  // as CSR entries (-1: the dense slice-group layout)
  int csr_slog2(int S) const { return plan(S).csr_slog2; }
  // the single-rank step's layout for S slices (plan_step on this engine)
  StepInputs step_inputs() const;
  StepPlan plan(int S) const { return plan_step(step_inputs(), S); }
  // bytes of one CSR entry: LR (slice | value) 8, reference FM (slice, B, C)
  // 12, standard FM a full row (csr_row_words)
  int csr_entry_bytes() const {
    return csr_full_rows() ? 4 * csr_row_words(table_.L.P) : (fm_vals_ ? 12 : 8);
  }
  bool csr_full_rows() const {
    return (cfg_.model.kind == kFM && cfg_.model.fm_math == kFmStandard) ||
           (cfg_.model.kind == kMVM && cfg_.model.kernel_dim() >= 2);
  }
  // worker: forward/backward of every slice of the step at once.  pack:
  // entries packed densely in send order into ent_out (cnt_out: entries per
  // key, u32 [n_send]; totals_out: entries per owner, from the step's owner
  // key counts `counts` (encoded: world > 1)); else they stay in the engine's
  // CSR layout (world 1, read in place by s_apply_csr with null arrays).
  void w_forward_backward_csr(const BatchView& b, const float* pulled, int64_t n_send,
                              int S_global, int wb, bool pack, u32* cnt_out, void* ent_out,
                              const int64_t* counts, int world, bool encoded, int64_t* totals_out);
  // server: apply received CSR gradients source by source: recv_cnt [n] per
  // key, entries of all sources back to back (null recv_cnt: the worker's own
  // entries of this step, world 1)
  void s_apply_csr(const u64* recv_keys, const u32* recv_cnt, const void* recv_ent,
                   const std::vector<int64_t>& src_offsets, int S, int buf = 0);
  // server: apply received gradients source by source (deterministic order).
  // src_offsets has world+1 entries delimiting each source's rows.
  void s_apply(const u64* recv_keys, const float* recv_grads, const u32* recv_masks,
               const std::vector<int64_t>& src_offsets, int S, int buf = 0);
  // worker: release the per-step dedup scratch.
  void w_finish();

  // AUC / logloss sums of n predictions in backend memory (labels 0/1 floats),
  // computed on the device: only the scalars come back (base.h:84-110)
  EvalMetrics eval_metrics(const float* pctr, const float* labels, int64_t n) {
    return be_->eval_metrics(pctr, labels, n);
  }

  // ---- stats / introspection -------------------------------------------
  // which = 0: training forward passes, 1: eval_step passes.
  LossStats read_stats(bool reset, int which = 0);
  int64_t n_unique();            // unique keys of the last prepared batch (syncs)
  int64_t table_size();          // occupied slots (syncs)
  int64_t scratch_capacity();    // active dedup scratch capacity (adaptive on the GPU; syncs)
  uint64_t table_capacity() const { return table_.cap; }
  size_t table_bytes() const { return table_bytes_; }
  bool overflowed();
  // capacity management (EngineConfig::table_grow): growths (split launches)
  // and segments split so far, host waits the monitor needed, and an explicit
  // growth to at least 2^log2_cap slots
  int64_t table_growths() const { return growths_; }
  // steps (fused or worker-side) whose several slices ran on the CSR path
  int64_t csr_steps() const { return csr_steps_; }
  // host copies of the last CSR step's per-key (off, cnt) and its entry words
  // (tests / debugging; syncs)
  void csr_debug(std::vector<u32>& off, std::vector<u32>& cnt, std::vector<u32>& words);
  int64_t table_splits() const { return splits_; }
  // geometry: {segment slots log2, level, split, segments}
  std::vector<int64_t> table_geometry() const {
    return {table_.seg_log2, table_.level, (int64_t)table_.split,
            (int64_t)(table_.cap >> table_.seg_log2)};
  }
  // device bytes committed to the table's range (>= table_bytes())
  size_t table_committed() const;
  // seconds of host time the growth calls took (mapping + launches)
  double grow_seconds() const { return grow_s_; }
  int64_t monitor_waits() const { return monitor_waits_; }
  // host seconds spent blocked on the monitor's run-ahead bound (the device
  // was monitor_lag steps behind): subtracted from the host's issue time
  double monitor_wait_seconds() const { return monitor_wait_s_; }
  // gradient-reduction records written by the producers since the last call
  // (counting on: one atomic per producer workgroup; off: -1).  Syncs.
  void count_records(bool on);
  int64_t take_records();
  void grow_table(int log2_cap);
  // queue a snapshot of (table size, overflow flags) behind the step's
  // work; called at the end of every training step (fused or sharded)
  void end_step();
  // exactly non-zero (key, param) weights of this table shard (L1 sparsity)
  int64_t nonzero_weights() { return be_->table_nonzero(table_, cfg_.opt); }
  int pstride() const { return cfg_.model.pstride(); }
  // floats per pulled value row (pull outputs, the values exchange, the
  // forward's gather): pstride, or 4 for reference-math FM on the GPU
  // reduction path ((w, Σv, Σv^2, 0), FwdArgs::fm_vals)
  int value_width() const { return vstride_; }
  // floats per (key, slice) in the multi-rank gradient exchange: pstride, or
  // 2 for reference-math FM on the GPU reduction path ((B, C) rows, expanded
  // by the owner with the values it served)
  int grad_width() const { return sharded_fm_compact() ? 2 : pstride(); }
  int slices_of(const BatchView& b) const;
  // Hogwild slices beyond kSliceGroup per step (the reference's default is
  // hardware_concurrency threads per block, lr_worker.h:40-41): the step's
  // slices run in groups of kSliceGroup -- one dedup + pull for the whole
  // step (every slice reads the same weights), then per group a
  // forward/backward over the group's rows and an apply of its pushes in
  // slice order, so the pushes of all S slices are applied in global slice
  // order: the same semantics as one S-slice step.  A group of one slice
  // runs as two (masked path; the second slice has no rows).
  static constexpr int kSliceGroup = 32;
  static int slice_groups(int S) { return S <= kSliceGroup ? 1 : (S + kSliceGroup - 1) / kSliceGroup; }
  static int group_slices(int S, int group) {
    if (S <= kSliceGroup) return S;
    const int n = S - group * kSliceGroup;
    return n >= kSliceGroup ? kSliceGroup : (n < 2 ? 2 : n);
  }

  // ---- checkpoint ------------------------------------------------------
  // Host copies of every live slot: keys + (stride-2) state words each.
  void export_table(std::vector<u64>& keys, std::vector<u32>& words);
  void import_table(const std::vector<u64>& keys, const std::vector<u32>& words);
  // The same into / from caller memory of n keys and n * state_words()
  // words (n = table_size() for export), streamed through two pinned
  // staging buffers so the DMA of one chunk overlaps the host copy of the
  // previous one.
  void export_into(u64* keys, u32* words, int64_t n);
  void import_from(const u64* keys, const u32* words, int64_t n);
  int state_words() const { return table_.L.stride - 2; }
  const TableLayout& layout() const { return table_.L; }
  // Binary shard file: header + keys + state words.
  void save(const std::string& path);
  void load(const std::string& path);

  // libffm text block (backend memory, 16-byte aligned) -> CSR arrays in
  // backend memory, on the device (Backend::parse_text).  Returns {rows,
  // occurrences, shortest row, longest row, occurrences of the first rows -
  // rows % row_mod rows}; syncs once (the counts).  Throws when the block
  // holds more rows / occurrences than the arrays (max_rows / max_nnz).
  std::vector<int64_t> parse_text(const char* text, int64_t n, u64* keys, int32_t* fgid,
                                  int32_t* row_ptr, float* labels, int64_t max_rows,
                                  int64_t max_nnz, int64_t row_mod = 1);

  // Synthetic Criteo-shaped batch into engine-owned staging buffers.
  BatchView synth_batch(const SynthArgs& a, int64_t slice_rows);
  // Copy a host CSR batch into engine-owned staging buffers.
  BatchView stage_host_batch(const BatchView& host);
  // Asynchronous, double-buffered variant (the native trainer's input path):
  // the host arrays are copied into a pinned buffer and sent on the
  // backend's copy queue while earlier steps run; the compute queue waits
  // for them.  Call stage_release() after queueing the steps that read the
  // returned batch, before staging the batch after the next one.
  BatchView stage_host_batch_async(const BatchView& host);
  void stage_release();

 private:
  // chunked device<->host transfer through the staging pair (export / save,
  // import / load): sink(host chunk, byte offset, bytes) consumes each chunk
  // while the next one is in flight; fill(host chunk, offset, bytes)
  // produces each chunk while the previous one uploads
  template <typename Sink>
  void d2h_stream(const void* src, size_t bytes, Sink sink);
  template <typename Fill>
  void h2d_stream(void* dst, size_t bytes, Fill fill);
  void table_from_device(const u64* dk, const u32* dw, int64_t n);
  void* stage_io_[2] = {nullptr, nullptr};
  void ensure_server_capacity(int64_t n, int buf = 0);
  // worker buffer sets (see w_prepare): the members pos_, uniq_pos_, inv_,
  // n_uniq_, send_pos_, send_map_, inv_valid_ describe set cur_wb_
  struct WorkerSet {
    u32* pos = nullptr;
    u32* uniq_pos = nullptr;
    u32* inv = nullptr;
    int64_t* n_uniq = nullptr;
    u32* send_pos = nullptr;
    const u32* send_map = nullptr;
    bool inv_valid = false;
    unsigned long long* bcap = nullptr;  // scratch capacity of the set's batch (device)
  };
  WorkerSet wset_[2];
  int cur_wb_ = 0;
  void use_worker_set(int wb);
  // owner grouping for the one-launch multi-source apply (Backend::owner_group)
  u64* own_keys_ = nullptr;      // owner scratch [own_cap_]
  u64 own_cap_ = 0;
  int64_t own_fill_ = 0;         // entries registered since the last clear (upper bound of keys)
  int own_nsrc_ = 0;             // row stride of SrvBuf::own_idx
  u32 own_epoch_ = 0;
  bool group_entries(const u64* recv_keys, int64_t n, int buf,
                     const std::vector<int64_t>& src_offsets);
  // per-slice normalisers, kSliceGroup entries per slice group (group k's
  // local slice s at [k * kSliceGroup + s])
  const int32_t* slice_rows_dev(const BatchView& b, int S);
  // rows of slice group k of a batch of S slices, and the matching dedup
  // positions (a row-range view: same layout, offset pointers)
  BatchView group_view(const BatchView& b, int S, int k, const u32*& pos) const;
  int slice_cap_ = 1;            // slices per group the buffers are sized for
  // parts > 1: owner-partitioned scratch (ScratchView::parts); uniq_keys_out
  // redirects the unique-key list (the sharded step's send buffer)
  void dedup_(const BatchView& b, int parts = 1, u64* uniq_keys_out = nullptr,
              bool want_inv = false, int64_t* n_copy = nullptr);
  const u32* send_map_ = nullptr;  // send order -> scratch slot (send_pos_ or uniq_pos_)
  bool sharded_fm_compact() const {
    return red_pairs_ && cfg_.model.kind == kFM && cfg_.model.fm_math == kFmReference &&
           (double)scratch_.cap * slice_cap_ * pstride() < 4294967295.0;
  }
  bool fm_vals_ = false;
  int vstride_ = 1;
  const float* pulled_weights(int buf, int64_t off) const;

  EngineConfig cfg_;
  std::unique_ptr<Backend> be_;
  TableView table_;
  size_t table_bytes_ = 0;
  ScratchView scratch_;

  // worker buffers (backend memory)
  u32* pos_ = nullptr;          // [max_nnz]
  u64* uniq_keys_ = nullptr;    // [max_nnz]
  u32* uniq_pos_ = nullptr;     // [max_nnz]
  u32* uniq_slot_ = nullptr;    // [max_nnz]
  int64_t* n_uniq_ = nullptr;   // [1]
  u32* block_counts_ = nullptr; // dedup compaction workspace
  u32* mon_ = nullptr;          // [4]: table size (u64), overflow_ (below)
  u32* overflow_ = nullptr;     // [2]: scratch, table (= mon_ + 2)
  float* wpull_ = nullptr;      // [scratch_cap * pstride]
  float* grad_ = nullptr;       // [scratch_cap * slice_cap * pstride]
  u32* tmask_ = nullptr;        // [scratch_cap]
  // HIP LR gradient reduction workspace (FwdArgs::red_*), null when unused
  u64* red_pairs_ = nullptr;
  u64* red_sorted_ = nullptr;
  int64_t red_sorted_words_ = 0;  // u64 words of red_sorted_
  u32* red_hist_ = nullptr;
  u32* red_tot_ = nullptr;
  u32* red_count_ = nullptr;
  float* red_rowv_ = nullptr;    // MVM: per-row loss*M (FwdArgs::red_rowv)
  float* lr_grad_ = nullptr;     // LR-FTRL fused step: unique-order gradients [max_nnz][slice_cap]
  float* lr_nz_ = nullptr;       // LR-FTRL fused step: pulled (n, z) [max_nnz][2]
  int64_t nnz_seen_ = 0;          // most occurrences in one batch (ScratchView::grow)
  u32* lr_mask_ = nullptr;       // LR-FTRL fused step, S > 1: unique-order slice bits [max_nnz]
  float* fm_grad_ = nullptr;     // reference FM fused step: unique-order (B, C) [max_nnz][2]
  float* row_grad_ = nullptr;    // MVM / standard FM fused step (one slice): unique-order rows [max_nnz][pstride]
  float* fm_w_ = nullptr;        // reference FM, grouped step: pulled per-parameter weights [max_nnz][pstride]
  int red_nb_ = 0;
  int red_nsub_ = 1;
  int red_maxb_ = 0;  // FwdArgs::red_maxb
  int red_groups_ = 0;  // FwdArgs::red_groups
  unsigned long long* bcap_ = nullptr;  // current worker set's batch scratch capacity
  u32* inv_ = nullptr;          // [scratch cap] slot -> send index (partitioned dedup, LR)
  bool inv_valid_ = false;      // inv_ describes the batch of the last w_prepare
  void set_reduction(FwdArgs& fa) const;
  // CSR gradients (CsrOut): the single-rank step of several slices, LR-FTRL on
  // 16-byte slots or compact reference-FM rows -- one producer pass, one
  // reduction and one apply for any slice count
  u32* csr_off_ = nullptr;      // [max_nnz]
  u32* csr_cnt_ = nullptr;      // [max_nnz]
  float* csr_vent_ = nullptr;   // standard FM / MVM: full-row entries [max_nnz][csr_row_words(P)]
  // MVM: repeated-field rows' records and fixed-point sums (MvmDup, backend.h)
  float* mdup_rec_ = nullptr;
  long long* mdup_acc_ = nullptr;
  u32* mdup_claim_ = nullptr;
  int64_t mdup_cap_ = 0;
  int mdup_ew_ = 0;
  int64_t csr_steps_ = 0;
  void train_step_csr(const BatchView& b, int S, int slog2);
  u32* csr_doff_ = nullptr;     // [max_nnz + 1] dense offsets (worker pack)
  u32* csr_long_ = nullptr;     // [1 + max keys] the applies' deferred long chains
  int64_t csr_long_cap_ = 0;
  u32* csr_long_list(int64_t n);
  u32* csr_roff_ = nullptr;     // received entries' offsets (server)
  int64_t csr_roff_cap_ = 0;
  // the forward/backward both CSR entry points run: producer pass over every
  // slice with dests unique * 2^slog2 + slice, CSR reduction into csr_*_
  void csr_forward_backward(const BatchView& b, int slog2, const int32_t* srows, bool normalise);
  bool reduction_masks(bool unique_positions) const;
  void ensure_inv();
  LossStats* stats_ = nullptr;  // [1]
  u32* send_pos_ = nullptr;     // [max_nnz]
  int64_t* bucket_ws_ = nullptr;  // [2*256]
  int32_t* slice_rows_ = nullptr;  // [slice_rows_cap_]
  int64_t slice_rows_cap_ = 0;
  int64_t cached_rows_ = -1, cached_slice_rows_ = -1;
  int cached_S_ = -1;
  int64_t last_nsend_ = 0;

  // async staging sets (stage_host_batch_async)
  struct StageSet {
    u64* keys = nullptr;
    int32_t* rowptr = nullptr;
    int32_t* fgid = nullptr;
    float* labels = nullptr;
  };
  StageSet aset_[2];
  int astage_next_ = 0, astage_last_ = -1;
  // staging batch buffers (backend memory)
  u64* st_keys_ = nullptr;
  int32_t* st_rowptr_ = nullptr;
  int32_t* st_fgid_ = nullptr;
  float* st_labels_ = nullptr;

  // Server buffers: a pipelined step with staleness k applies a buffer's
  // pushes after the next k pulls (parallel/async_p2p.py), so k + 1 are live.
 public:
  // (the asynchronous parameter server keeps one per (source, ring slot))
  static constexpr int kSrvBufs = 64;
 private:
  struct SrvBuf {
    u32* slots = nullptr;        // table slot of each received key (s_pull)
    int64_t cap = 0;
    int64_t n = 0;
    const u64* keys = nullptr;   // the received keys (slots re-probed after a table growth)
    // LR-FTRL 16-byte slots: (n, z) as pulled, and whether no apply has
    // touched the table since that pull (then the first source's apply takes
    // its state from here instead of re-reading the table)
    float* nz = nullptr;
    bool nz_fresh = false;
    const float* vals = nullptr;  // s_pull outputs (fm_compact apply)
    float* w = nullptr;           // s_pull(keep_weights) per-param weights
    int64_t w_cap = 0;
    bool w_valid = false;
    u32* own_pos = nullptr;       // owner grouping of the buffer's entries
    int64_t own_pos_cap = 0;
    u64* own_idx = nullptr;
    SrcGroups grp;                // grp.oidx != null: s_pull grouped this buffer
  };
  SrvBuf srv_[kSrvBufs];
  void stale_stashes() {
    for (SrvBuf& b : srv_) b.nz_fresh = false;
  }
  bool lr16_layout() const;

  // capacity monitor (EngineConfig::table_grow): a ring of pinned snapshots
  // (HostSnap: table size, overflow flags, sequence number), one per step,
  // written by the step's apply kernel (or a tiny kernel when the step has
  // none) and polled by the host -- no event, no extra launch; each comes
  // with the cumulative insert bound queued before it
  static constexpr int kSnaps = 64;
  HostSnap* snaps_ = nullptr;       // pinned host [kSnaps]
  int64_t snap_adds_[kSnaps] = {};
  bool snap_carried_ = false;       // an apply since the last inserts carries the next snapshot
  bool snap_ready(int64_t seq) const;
  void close_snapshot();
  void attach_snapshot(ApplyArgs& aa);
  int64_t snap_seq_ = 0;            // snapshots recorded
  int64_t snap_seen_ = 0;           // snapshots consumed (all older ones complete)
  int64_t known_size_ = 0;          // table size at the last consumed snapshot (or sync)
  int64_t known_adds_ = 0;          // cumulative insert bound queued before it
  int64_t queued_adds_ = 0;         // cumulative insert bound queued so far
  int64_t growths_ = 0, splits_ = 0, monitor_waits_ = 0;
  double grow_s_ = 0.0;
  u64 max_segs_ = 0;                // segments of 2^max_log2_cap slots
  double monitor_wait_s_ = 0.0;
  float* grp_nz_ = nullptr;                   // FM / MVM FTRL: the pull's (n, z) stash [unique][P]
  unsigned long long* rec_count_ = nullptr;  // (count_records) device counter
  u32* red_vmax_ = nullptr;                   // MVM: per-step scale words [2], dup words [2]
  u32* text_ws_ = nullptr;                    // parse_text workspace
  int64_t text_ws_words_ = 0;
  long long* text_counts_ = nullptr;          // parse_text counts [7]
  mutable int vmax_parity_ = 0;
  bool rec_on_ = false;
  int log2_cap_ = 0, max_log2_cap_ = 31;
  void poll_snapshots(int64_t wait_upto);
  void guard_inserts(int64_t n);   // before an inserting pull of <= n new keys
  void remap_server_slots();
  // segment count the growth schedule (u0 = grow_start, u1 = grow_load) wants
  u64 segments_for(double keys, double u0, double u1) const;
  // load of the fullest segments at which growth stops pacing itself
  static constexpr double kHardLoad = 0.9;
  void split_to(u64 nseg);              // split segments until there are nseg

  u64* host_keys_dev_ = nullptr;   // push_host / pull_host staging
  float* host_vals_dev_ = nullptr;
  u32* host_slots_dev_ = nullptr;
  int64_t host_cap_ = 0;
};

}  // namespace xflow
