// xflow-amd: Engine implementation (device agnostic; talks to a Backend).
#include <cstdlib>
#include "xflow/engine.h"

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <thread>
#include <fstream>
#include <stdexcept>

namespace xflow {

namespace {

uint64_t next_pow2(uint64_t v) {
  uint64_t p = 1;
  while (p < v) p <<= 1;
  return p;
}

template <typename T>
T* balloc(Backend& be, size_t n) {
  return static_cast<T*>(be.alloc(sizeof(T) * (n ? n : 1)));
}

constexpr char kMagic[8] = {'X', 'F', 'L', 'O', 'W', 'T', 'B', '1'};

// XFLOW_NO_MONITOR=1: no per-step capacity snapshot (A/B of the monitor's
// cost only; growth then relies on exact-size reads, overflow on the
// epoch-end check)
bool monitor_disabled() {
  static const bool off = std::getenv("XFLOW_NO_MONITOR") != nullptr;
  return off;
}

}  // namespace

Engine::Engine(const EngineConfig& cfg) : cfg_(cfg) {
  if (cfg_.table_log2_cap < 4 || cfg_.table_log2_cap > 31)
    throw std::invalid_argument("table_log2_cap must be in [4, 31]");
  if (!(cfg_.grow_load > 0.0 && cfg_.grow_load < 1.0))
    throw std::invalid_argument("grow_load must be in (0, 1)");
  if (cfg_.monitor_lag < 0 || cfg_.monitor_lag >= kSnaps)
    throw std::invalid_argument("monitor_lag must be in [0, 63]");
  if (cfg_.max_slices < 1) throw std::invalid_argument("max_slices must be >= 1");
  // buffers hold one slice group (more slices per step run group by group)
  slice_cap_ = cfg_.max_slices < kSliceGroup ? cfg_.max_slices : kSliceGroup;
  if (cfg_.model.kind != kLR && (cfg_.model.v_dim < 1 || cfg_.model.v_dim > 32))
    throw std::invalid_argument("v_dim must be in [1, 32]");
  be_ = cfg_.device >= 0 ? make_hip_backend(cfg_.device) : make_cpu_backend();
  Backend& be = *be_;
  // the device kernels' latent widths: any other v_dim runs padded (inert
  // padded dims, ModelSpec::pad_dim)
  cfg_.model.pad_dim = 0;
  if (be.is_gpu() && cfg_.model.kind != kLR &&
      device_latent_width(cfg_.model.v_dim) != cfg_.model.v_dim)
    cfg_.model.pad_dim = device_latent_width(cfg_.model.v_dim);

  // persistent table
  table_.L = TableLayout::make(cfg_.model, cfg_.opt);
  log2_cap_ = cfg_.table_log2_cap;
  max_log2_cap_ = cfg_.max_log2_cap > 0 ? (cfg_.max_log2_cap < 31 ? cfg_.max_log2_cap : 31) : 31;
  if (max_log2_cap_ < log2_cap_) max_log2_cap_ = log2_cap_;
  if (!(cfg_.grow_start > 0.0 && cfg_.grow_start < cfg_.grow_load))
    cfg_.grow_start = 0.75 * cfg_.grow_load;
  // geometry (backend.h TableView): segments of at most 2^kMaxSegLog2 (2^20) slots
  table_.seg_log2 = log2_cap_ < kMaxSegLog2 ? log2_cap_ : kMaxSegLog2;
  table_.level = log2_cap_ - table_.seg_log2;
  table_.split = 0;
  table_.cap = 1ull << log2_cap_;
  const u64 seg = 1ull << table_.seg_log2;
  table_.probe_limit = seg < kMaxProbe ? seg : kMaxProbe;
  max_segs_ = cfg_.table_grow ? (1ull << max_log2_cap_) >> table_.seg_log2 : table_.cap >> table_.seg_log2;
  table_bytes_ = (size_t)table_.cap * table_.L.stride * sizeof(u32);
  {
    void* base = be.table_reserve((size_t)(max_segs_ << table_.seg_log2) * table_.L.stride * sizeof(u32),
                                  max_segs_ > (table_.cap >> table_.seg_log2));
    table_.words = static_cast<u32*>(be.table_commit(base, table_bytes_));
  }
  // one 16-byte block {size, overflow[2]}: a step's snapshot is one copy
  mon_ = balloc<u32>(be, 4);
  table_.size = reinterpret_cast<unsigned long long*>(mon_);
  overflow_ = mon_ + 2;
  table_.overflow = overflow_ + 1;
  be.memset(mon_, 0, 4 * sizeof(u32));
  be.table_clear(table_);
  snaps_ = static_cast<HostSnap*>(be.host_alloc(sizeof(HostSnap) * kSnaps));
  std::memset(snaps_, 0, sizeof(HostSnap) * kSnaps);

  // per-step dedup scratch
  const int64_t nnz = cfg_.max_nnz;
  scratch_.cap = next_pow2((uint64_t)((double)nnz * cfg_.scratch_factor) + 1);
  if (scratch_.cap > (1ull << 31)) throw std::invalid_argument("max_nnz too large");
  scratch_.keys = balloc<u64>(be, scratch_.cap);
  be.fill_u64(scratch_.keys, kEmptyKey, scratch_.cap);
  scratch_.stamps = balloc<unsigned char>(be, scratch_.cap);
  be.memset(scratch_.stamps, 0, scratch_.cap);
  scratch_.claims = balloc<unsigned long long>(be, 1);
  be.memset(scratch_.claims, 0, sizeof(unsigned long long));
  // Rebuild once half full: one more step adds at most max_nnz <= cap/factor
  // keys, so the load factor stays below 0.5 + 1/factor.
  scratch_.rebuild_at = scratch_.cap / 2;
  scratch_.epoch = 0;
  if (be.is_gpu()) {
    // adaptive active capacity (ScratchView::ctl): starts at the allocation
    scratch_.ctl = balloc<unsigned long long>(be, 5);
    unsigned long long c0[5] = {scratch_.cap, 0ull, 0ull, 0ull, 0ull};
    be.copy_h2d(scratch_.ctl, c0, sizeof(c0));
  }
  block_counts_ = balloc<u32>(be, scratch_.cap / 4096 + 1);

  const int ps = cfg_.model.pstride();
  pos_ = balloc<u32>(be, nnz);
  uniq_keys_ = balloc<u64>(be, nnz);
  uniq_pos_ = balloc<u32>(be, nnz);
  uniq_slot_ = balloc<u32>(be, nnz);
  send_pos_ = balloc<u32>(be, nnz);
  n_uniq_ = balloc<int64_t>(be, 1);
  be.memset(n_uniq_, 0, sizeof(int64_t));
  wset_[0].pos = pos_;
  wset_[0].uniq_pos = uniq_pos_;
  wset_[0].n_uniq = n_uniq_;
  wset_[0].send_pos = send_pos_;
  bcap_ = balloc<unsigned long long>(be, 1);
  be.memset(bcap_, 0, sizeof(unsigned long long));
  wset_[0].bcap = bcap_;
  // slot-indexed buffers carry one extra row: the trash slot (index cap) that
  // a dedup probe overflow sends its occurrences to (flagged, never applied)
  const uint64_t rows1 = scratch_.cap + 1;
  grad_ = balloc<float>(be, rows1 * slice_cap_ * ps);
  be.memset(grad_, 0, sizeof(float) * rows1 * slice_cap_ * ps);
  tmask_ = balloc<u32>(be, rows1);
  be.memset(tmask_, 0, sizeof(u32) * rows1);
  // atomic-free gradient reduction (FwdArgs::red_*): LR (1 value per key) and
  // reference-math FM (2 values per key, 16-byte records)
  const bool fm_ref = cfg_.model.kind == kFM && cfg_.model.fm_math == kFmReference;
  // standard FM: vector records (dest, 1 + D sums) per (key, slice, column)
  // and workgroup (k_fm_std_red), at most one per occurrence
  const bool fm_std = cfg_.model.kind == kFM && cfg_.model.fm_math == kFmStandard;
  const bool mvm = cfg_.model.kind == kMVM;
  if (be.is_gpu() && (cfg_.model.kind == kLR || fm_ref || fm_std || mvm)) {
    // values per record: 1 (LR), 2 (reference FM), the vector records of
    // standard FM (1 + D) and MVM (D: per-row T = loss*M sums)
    const bool vec = fm_std || mvm;
    const int kd = cfg_.model.kernel_dim();
    const int nv = fm_ref ? 2 : (fm_std ? 1 + kd : (mvm ? kd : 1));
    const int shift = red_shift(nv);
    // u64 words per record slot: nv for LR / reference FM, the vector record otherwise
    const int recw = vec ? vec_rec_words(nv) / 2 : nv;
    const int group_rows = fm_ref ? kFmGroupRows : (vec ? kFmStdMinGroupRows : kLrGroupRows);
    // (the trash slot's occurrences are never reduced: FwdArgs::trash_pos)
    // Buckets of 2^shift dests at the allocated capacity; beyond
    // kRedMaxBuckets the device widens the buckets (FwdArgs::red_bcap) and
    // sums a wide bucket with red_nsub workgroups -- only when the adaptive
    // scratch has grown that far (bench shape: S = 8 at 2^23 active slots
    // stays at 4096 buckets of 2^14).
    const uint64_t dests = scratch_.cap * (uint64_t)slice_cap_;
    // vector records: the producer's larger bucket cap where its LDS allows
    // (vec_red_max_buckets) and the batch fits the scatter-free form
    const int vd = nv - 1;  // k_fm_std_red<vd>: NV = 1 + vd
    const int maxb = vec && (cfg_.max_rows + fmstd_block(vd) - 1) / fmstd_block(vd) <= kSegMaxGroups
                         ? vec_red_max_buckets(vd)
                         : kRedMaxBuckets;
    red_maxb_ = vec ? maxb : 0;
    int nb = (int)((dests + (1ull << shift) - 1) >> shift);
    int nsub = 1;
    while ((uint64_t)nb > (uint64_t)maxb * nsub) nsub <<= 1;
    if (nsub > 1) nb = maxb;
    red_nsub_ = nsub;
    if (nb <= maxb && dests < (1ull << 32)) {
      const int64_t groups = (cfg_.max_rows + group_rows - 1) / group_rows;
      red_nb_ = nb;
      red_pairs_ = balloc<u64>(be, (size_t)nnz * recw);
      red_sorted_ = balloc<u64>(be, (size_t)nnz * recw);
      red_sorted_words_ = (int64_t)nnz * recw;
      red_hist_ = balloc<u32>(be, (size_t)nb * groups);
      red_tot_ = balloc<u32>(be, 2 * (size_t)nb + 2);
      red_count_ = balloc<u32>(be, groups);
      red_groups_ = (int)groups;
      // MVM: T = loss*M per row; standard FM: (loss, loss*vs) per row (k_fm_std_fwd)
      if (mvm || fm_std) red_rowv_ = balloc<float>(be, (size_t)cfg_.max_rows * ps);
      if (mvm) {
        // (vmax, dup flag, dup |c| max, dup record count: two alternating words each)
        red_vmax_ = balloc<u32>(be, 8);
        be.memset(red_vmax_, 0, 8 * sizeof(u32));
        // repeated-field rows' records and fixed-point sums (MvmDup, backend.h)
        const int D = cfg_.model.kernel_dim();
        mdup_ew_ = csr_row_words(D);
        mdup_rec_ = balloc<float>(be, (size_t)nnz * mdup_ew_);
        mdup_acc_ = balloc<long long>(be, (size_t)nnz * D);
        mdup_claim_ = balloc<u32>(be, (size_t)nnz);
        mdup_cap_ = nnz;
      }
    }
  }
  // reference-math FM with the GPU reduction: compact (w, Σv, Σv^2, 0) value rows
  fm_vals_ = red_pairs_ && fm_ref;
  vstride_ = fm_vals_ ? 4 : ps;
  wpull_ = balloc<float>(be, rows1 * vstride_);
  be.memset(wpull_ + scratch_.cap * vstride_, 0, sizeof(float) * vstride_);
  stats_ = balloc<LossStats>(be, 2);
  be.memset(stats_, 0, 2 * sizeof(LossStats));
  bucket_ws_ = balloc<int64_t>(be, 512);
  slice_rows_cap_ = kSliceGroup;
  slice_rows_ = balloc<int32_t>(be, slice_rows_cap_);

  st_keys_ = balloc<u64>(be, nnz);
  st_fgid_ = balloc<int32_t>(be, nnz);
  st_rowptr_ = balloc<int32_t>(be, cfg_.max_rows + 1);
  st_labels_ = balloc<float>(be, cfg_.max_rows);
  be.synchronize();
}

Engine::~Engine() {
  Backend& be = *be_;
  be.synchronize();
  use_worker_set(cur_wb_);  // (records the current set)
  be.table_release(table_.words);
  be.free_stream(csr_roff_);
  be.free_stream(csr_long_);
  void* ptrs[] = {mon_, scratch_.keys, scratch_.stamps,
                  scratch_.claims, block_counts_, uniq_keys_, uniq_slot_, wpull_, grad_, tmask_,
                  stats_, bucket_ws_, slice_rows_, st_keys_, st_fgid_, st_rowptr_, st_labels_,
                  host_keys_dev_, host_vals_dev_,
                  host_slots_dev_, scratch_.ctl, red_pairs_, red_sorted_, red_hist_,
                  red_tot_, red_count_, red_rowv_, lr_grad_, lr_nz_, grp_nz_, own_keys_, fm_grad_,
                  row_grad_,
                  lr_mask_, fm_w_, rec_count_, red_vmax_, text_ws_, text_counts_, csr_off_, csr_vent_,
                  csr_cnt_, csr_doff_, mdup_rec_, mdup_acc_, mdup_claim_};
  for (void* p : ptrs) be.free(p);
  for (void* p : stage_io_) be.staging_free(p);
  for (SrvBuf& b : srv_) {
    void* bp[] = {b.slots, b.nz, b.w, b.own_pos, b.own_idx};
    for (void* p : bp) be.free(p);
  }
  be.host_free(snaps_);
  for (StageSet& a : aset_) {
    void* ap[] = {a.keys, a.rowptr, a.fgid, a.labels};
    for (void* p : ap) be.free(p);
  }
  for (WorkerSet& w : wset_) {
    void* wp[] = {w.pos, w.uniq_pos, w.inv, w.n_uniq, w.send_pos, w.bcap};
    for (void* p : wp) be.free(p);
  }
}

void Engine::use_worker_set(int wb) {
  if (wb < 0 || wb > 1) throw std::invalid_argument("worker buffer set must be 0 or 1");
  WorkerSet& c = wset_[cur_wb_];
  c.pos = pos_;
  c.uniq_pos = uniq_pos_;
  c.inv = inv_;
  c.n_uniq = n_uniq_;
  c.send_pos = send_pos_;
  c.send_map = send_map_;
  c.inv_valid = inv_valid_;
  c.bcap = bcap_;
  WorkerSet& w = wset_[wb];
  if (!w.pos) {  // second set: allocated on first use (pipelined sharded step)
    const int64_t nnz = cfg_.max_nnz;
    w.pos = balloc<u32>(*be_, nnz);
    w.uniq_pos = balloc<u32>(*be_, nnz);
    w.send_pos = balloc<u32>(*be_, nnz);
    w.n_uniq = balloc<int64_t>(*be_, 1);
    be_->memset(w.n_uniq, 0, sizeof(int64_t));
    w.bcap = balloc<unsigned long long>(*be_, 1);
    be_->memset(w.bcap, 0, sizeof(unsigned long long));
  }
  pos_ = w.pos;
  uniq_pos_ = w.uniq_pos;
  inv_ = w.inv;
  n_uniq_ = w.n_uniq;
  send_pos_ = w.send_pos;
  send_map_ = w.send_map;
  inv_valid_ = w.inv_valid;
  bcap_ = w.bcap;
  cur_wb_ = wb;
}

// The GPU reduction path sees every (key, slice) that occurs (a record per
// column-table entry, or per occurrence), so it can write the slice bits:
// every model on its bucket-reduction path.
bool Engine::reduction_masks(bool unique_positions) const {
  // (dest * pstride in 32 bits: dests = unique index x slices with unique-
  // index positions, at most max_nnz keys -- else scratch slot x slices)
  const double keys = unique_positions ? (double)cfg_.max_nnz : (double)scratch_.cap;
  if (!red_pairs_ || keys * slice_cap_ * pstride() >= 4294967295.0) return false;
  return cfg_.model.kind == kLR || cfg_.model.kind == kFM ||
         (cfg_.model.kind == kMVM && red_rowv_ != nullptr);
}

std::vector<int64_t> Engine::parse_text(const char* text, int64_t n, u64* keys, int32_t* fgid,
                                        int32_t* row_ptr, float* labels, int64_t max_rows,
                                        int64_t max_nnz, int64_t row_mod) {
  const int64_t need = text_ws_words(n);
  if (need > text_ws_words_) {
    be_->synchronize();
    be_->free(text_ws_);
    text_ws_words_ = need + need / 4;
    text_ws_ = balloc<u32>(*be_, (size_t)text_ws_words_);
  }
  if (!text_counts_) text_counts_ = balloc<long long>(*be_, 8);
  TextParseArgs a;
  a.text = text;
  a.n = n;
  a.keys = keys;
  a.fgid = fgid;
  a.row_ptr = row_ptr;
  a.labels = labels;
  a.max_rows = max_rows;
  a.max_nnz = max_nnz;
  a.max_lines = text_max_lines(n);
  a.ws = text_ws_;
  a.ws_words = text_ws_words_;
  a.row_mod = row_mod;
  a.counts = text_counts_;
  be_->parse_text(a);
  long long c[7];
  be_->copy_d2h(c, text_counts_, sizeof(c));
  if (c[5]) throw std::runtime_error("parse_text: more lines than n/2 + 2 (a block of empty lines?)");
  if (c[0] > max_rows || c[1] > max_nnz)
    throw std::runtime_error("parse_text: the block holds more rows / features than the arrays");
  return {c[0], c[1], c[0] > 0 ? c[2] : 0, c[3], c[6]};
}

void Engine::count_records(bool on) {
  if (on && !rec_count_) {
    rec_count_ = balloc<unsigned long long>(*be_, 1);
    be_->memset(rec_count_, 0, sizeof(unsigned long long));
  }
  rec_on_ = on;
}

int64_t Engine::take_records() {
  if (!rec_count_) return -1;
  unsigned long long n = 0;
  be_->copy_d2h(&n, rec_count_, sizeof(n));
  be_->memset(rec_count_, 0, sizeof(n));
  return (int64_t)n;
}

void Engine::set_reduction(FwdArgs& fa) const {
  fa.trash_pos = (u32)scratch_.cap;
  if (!red_pairs_) return;
  if (rec_on_) fa.red_records = rec_count_;
  if (red_vmax_) {  // (MVM: two alternating words, see FwdArgs::red_vmax)
    fa.red_vmax = red_vmax_ + vmax_parity_;
    fa.red_vmax_next = red_vmax_ + (vmax_parity_ ^ 1);
    fa.red_dup = red_vmax_ + 2 + vmax_parity_;
    fa.red_dup_next = red_vmax_ + 2 + (vmax_parity_ ^ 1);
    if (mdup_rec_) {
      fa.mdup.rec = mdup_rec_;
      fa.mdup.vmax = red_vmax_ + 4;
      fa.mdup.n = red_vmax_ + 6;
      fa.mdup.acc = mdup_acc_;
      fa.mdup.claim = mdup_claim_;
      fa.mdup.cap = mdup_cap_;
      fa.mdup.ew = mdup_ew_;
    }
    vmax_parity_ ^= 1;
  }
  fa.red_bcap = bcap_;
  fa.red_cap = scratch_.cap;
  fa.red_nsub = red_nsub_;
  fa.red_pairs = red_pairs_;
  fa.red_sorted = red_sorted_;
  fa.red_sorted_words = red_sorted_words_;
  fa.red_hist = red_hist_;
  fa.red_tot = red_tot_;
  fa.red_count = red_count_;
  fa.red_groups = red_groups_;
  fa.red_nb = red_nb_;
  fa.red_maxb = red_maxb_;
  fa.red_rowv = red_rowv_;
}

int Engine::slices_of(const BatchView& b) const {
  if (b.slice_rows <= 0 || b.rows <= 0) return 1;
  return (int)((b.rows + b.slice_rows - 1) / b.slice_rows);
}

const int32_t* Engine::slice_rows_dev(const BatchView& b, int S) {
  if (b.rows == cached_rows_ && b.slice_rows == cached_slice_rows_ && S == cached_S_)
    return slice_rows_;
  const int ng = slice_groups(S);
  if ((int64_t)ng * kSliceGroup > slice_rows_cap_) {
    be_->synchronize();  // (the old normalisers may still be read)
    be_->free(slice_rows_);
    slice_rows_cap_ = (int64_t)ng * kSliceGroup;
    slice_rows_ = balloc<int32_t>(*be_, slice_rows_cap_);
  }
  const int64_t sr = b.slice_rows > 0 ? b.slice_rows : b.rows;
  for (int g = 0; g < ng; ++g) {
    int32_t h[kSliceGroup];
    const int n = ng == 1 ? S : kSliceGroup;
    for (int l = 0; l < n; ++l) {
      const int64_t s = (int64_t)g * kSliceGroup + l;
      int64_t rem = s < S ? b.rows - s * sr : 0;
      rem = rem < 0 ? 0 : rem;
      // an empty slice has no gradient rows; 1 keeps 0/rows finite
      h[l] = (int32_t)(rem < sr ? (rem > 0 ? rem : 1) : sr);
    }
    // (no host wait)
    be_->upload_small(slice_rows_ + (int64_t)g * kSliceGroup, h, sizeof(int32_t) * n);
  }
  cached_S_ = S;
  cached_rows_ = b.rows;
  cached_slice_rows_ = b.slice_rows;
  return slice_rows_;
}

BatchView Engine::group_view(const BatchView& b, int S, int k, const u32*& pos) const {
  if (slice_groups(S) == 1) return b;
  const int64_t sr = b.slice_rows > 0 ? b.slice_rows : b.rows;
  int64_t r0 = (int64_t)k * kSliceGroup * sr;
  r0 = r0 < b.rows ? r0 : b.rows;
  int64_t n = (int64_t)kSliceGroup * sr;
  n = n < b.rows - r0 ? n : b.rows - r0;
  BatchView g = b;
  g.rows = n;
  if (b.row_ptr) {  // CSR: occurrence indices stay absolute
    g.row_ptr = b.row_ptr + r0;
    g.labels = b.labels + r0;
    return g;  // (g.nnz: the whole batch's, an upper bound; no kernel reads it)
  }
  // fixed width: row-major (r, j) at r*npr + j, field-major at j*col_stride + r
  const int64_t off = b.col_stride > 0 ? r0 : r0 * b.nnz_per_row;
  g.keys = b.keys + off;
  if (b.fgid) g.fgid = b.fgid + off;
  g.labels = b.labels + r0;
  g.nnz = n * b.nnz_per_row;
  pos += off;
  return g;
}

void Engine::ensure_inv() {
  if (inv_) return;
  // + the trash slot's entry (and padding to a 16-slot compaction group): no
  // unique index, so reductions skip it
  inv_ = balloc<u32>(*be_, scratch_.cap + 16);
  be_->memset(inv_ + scratch_.cap, 0xFF, 16 * sizeof(u32));
}

void Engine::dedup_(const BatchView& b, int parts, u64* uniq_keys_out, bool want_inv,
                    int64_t* n_copy) {
  if (b.nnz > cfg_.max_nnz) throw std::invalid_argument("batch nnz exceeds max_nnz");
  if (b.rows > cfg_.max_rows) throw std::invalid_argument("batch rows exceed max_rows");
  if (b.col_stride > 0 && (b.row_ptr || b.col_stride < b.rows || b.nnz != b.rows * b.nnz_per_row))
    throw std::invalid_argument("field-major batch needs fixed nnz_per_row and col_stride >= rows");
  // table-ordered unique lists (ScratchView::home_bits) on the one-owner GPU path
  const int hb = be_->is_gpu() && parts == 1
                     ? table_.seg_log2 + table_.level + (table_.split > 0 ? 1 : 0)
                     : 0;
  if (parts != scratch_.parts || hb != scratch_.home_bits) {
    // slots depend on the partitioning / home bits: start from an empty scratch table
    be_->fill_u64(scratch_.keys, kEmptyKey, scratch_.cap);
    be_->memset(scratch_.claims, 0, sizeof(unsigned long long));
    scratch_.parts = parts;
    scratch_.home_bits = hb;
  }
  // (n_uniq is written, not accumulated, by both backends' dedup)
  if (++scratch_.epoch > kStampEpochs) {
    // byte stamps wrap: clear them (0 marks never-stamped slots) and the
    // spill mark, which holds an epoch of the previous cycle
    scratch_.epoch = 1;
    be_->memset(scratch_.stamps, 0, scratch_.cap);
    if (scratch_.ctl) {
      const unsigned long long z = 0ull;
      be_->upload_small(scratch_.ctl + 4, &z, sizeof(z));
    }
  }
  scratch_.grow = 0.0f;
  if (scratch_.ctl && nnz_seen_ > 0 && b.nnz > nnz_seen_)
    scratch_.grow = (float)((double)b.nnz / (double)nnz_seen_);
  if (b.nnz > nnz_seen_) nnz_seen_ = b.nnz;
  DedupOut o;
  o.pos = pos_;
  o.uniq_keys = uniq_keys_out ? uniq_keys_out : uniq_keys_;
  o.uniq_pos = uniq_pos_;
  o.n_uniq = n_uniq_;
  o.overflow = overflow_;
  o.block_counts = block_counts_;
  o.inv = want_inv ? inv_ : nullptr;
  o.n_uniq_copy = n_copy;
  o.cap_out = bcap_;
  be_->dedup(b.keys, b.nnz, scratch_, o);
}


// log2 of the padded slice count when a step of S slices takes the CSR path
const char* grad_path_name(GradPath g) {
  switch (g) {
    case GradPath::kCsr: return "csr";
    case GradPath::kUniqueLR: return "unique_lr";
    case GradPath::kUniqueFmBC: return "unique_fm_bc";
    case GradPath::kUniqueRows: return "unique_rows";
    case GradPath::kSlotSums: return "slot_sums";
    case GradPath::kSlotRows: return "slot_rows";
  }
  return "?";
}

StepInputs Engine::step_inputs() const {
  StepInputs in;
  in.gpu = be_->is_gpu();
  in.remaps = be_->remaps_positions();
  in.red_pairs = red_pairs_ != nullptr;
  in.red_rowv = red_rowv_ != nullptr;
  in.fm_vals = fm_vals_;
  in.csr = cfg_.csr;
  in.sum_slices = cfg_.sum_slices;
  in.kind = cfg_.model.kind;
  in.fm_math = cfg_.model.fm_math;
  in.L = table_.L;
  in.scratch_cap = (double)scratch_.cap;
  in.max_nnz = (double)cfg_.max_nnz;
  in.max_rows = (double)cfg_.max_rows;
  in.pstride = pstride();
  in.slice_cap = slice_cap_;
  in.kdim = cfg_.model.kernel_dim();
  return in;
}

StepPlan plan_step(const StepInputs& in, int S) {
  constexpr double k32 = 4294967295.0;  // (32-bit dest * width bounds)
  StepPlan p;
  p.S = S;
  const TableLayout& L = in.L;
  const bool lr16_slot = in.kind == kLR && L.stride == 4 && L.P == 1 && L.opt == kFTRL &&
                         !L.has_flag;
  // CSR: several ordered slices of LR-FTRL 16-byte slots or reference FM, on
  // unique-index positions; dests = unique * 2^sl + slice inside one bucket
  // and in 32 bits
  // standard FM / MVM: full-row entries from the vector records' scatter-
  // free form (k_red_csr_vec; MVM's vector is its D-wide T, NV = D)
  const bool fm_std = in.kind == kFM && in.fm_math == kFmStandard;
  const bool mvm = in.kind == kMVM && in.kdim >= 2;
  const int vnv = fm_std ? 1 + in.kdim : in.kdim;  // (vector records' NV)
  const bool std_ok = (fm_std || mvm) && in.gpu && in.red_rowv &&
                      std::ceil(in.max_rows / fmstd_block(vnv - 1)) <= kSegMaxGroups;
  // below these slice counts the slice-group layouts win (same-box A/B at the
  // bench batch, profiles/r5_ab.txt #27: LR S = 4 499.8 vs 533.7, standard FM
  // S = 4 266.2 vs 270.4, MVM S = 2 182.9 vs 273.1; reference FM ties at S = 2)
  const int csr_min = (in.kind == kLR || fm_std) ? 8 : 4;
  if (in.csr && S >= csr_min && !in.sum_slices && in.red_pairs && in.remaps &&
      (lr16_slot || in.fm_vals || std_ok)) {
    int sl = 0;
    while ((1 << sl) < S) ++sl;
    const int nv = in.fm_vals ? 2 : (std_ok ? vnv : 1);
    if (sl <= red_shift(nv) && in.max_nnz * (double)(1 << sl) < k32) {
      p.csr_slog2 = sl;
      p.csr_rows = std_ok;
      p.grad = GradPath::kCsr;
      return p;
    }
  }
  p.groups = Engine::slice_groups(S);
  // (slice groups always run the masked multi-slice paths: every group has >= 2 slices)
  p.Sf = p.groups > 1 ? Engine::kSliceGroup : S;
  p.masks = p.Sf > 1 && !in.sum_slices;
  // LR-FTRL on 16-byte slots, bucket reduction: the reduction writes
  // normalised gradients in unique order (through the compaction's slot ->
  // unique index map; S > 1: [unique][slice] plus the slice bits) and the
  // apply takes (n, z) from the pull, so it reads nothing at random and
  // writes the slot once
  const bool lr16_ok = in.gpu && lr16_slot && in.red_pairs && in.scratch_cap < k32;
  // unique-index positions: pulled rows, gradient destinations and every
  // gradient / mask buffer in unique order -- the reductions span the unique
  // keys (S x that with S slices), not the 4x-headroom scratch slots.  The
  // remap pass costs ~40 us per 10.2 M occurrences; same-box A/B
  // (profiles/r4_unique_positions_ab.txt): a win with several slices (FM-8
  // std S = 8 143 -> 222 M samples/s, FM-8 S = 8 +1.9 %, LR S = 8 +0.8 %),
  // for standard FM (+10.5 %) and MVM (live +13 %, degenerate +2.3 %), a loss
  // for one-slice LR (-5.1 %) and reference FM (-1.4 %)
  p.upos = in.remaps && in.red_pairs &&
           (p.Sf > 1 || in.kind == kMVM || (in.kind == kFM && in.fm_math == kFmStandard));
  // slice bits from the reduction (dest * pstride in 32 bits)
  const double key_bound = p.upos ? in.max_nnz : in.scratch_cap;
  const bool red_masks = in.red_pairs && key_bound * in.slice_cap * in.pstride < k32 &&
                         (in.kind == kLR || in.kind == kFM || (in.kind == kMVM && in.red_rowv));
  p.lr16 = lr16_ok && (p.Sf == 1 || (p.masks && red_masks));
  // summed slices: slot-indexed sums (packed apply), still the (n, z) stash
  p.lr16s = lr16_ok && p.Sf > 1 && !p.lr16;
  // several slices on the reduction path: unique-order [unique][slice]
  // gradients plus the slice bits the reduction writes; the pull clears the
  // bits, the apply reads only the present slices
  p.uqm = p.masks && red_masks;
  // reference FM: the normalised (B, C) sums land in unique order
  p.fmu = in.fm_vals && (p.Sf == 1 || p.uqm);
  // compact reference-FM rows of a grouped step: the (B, C) of later groups
  // expand with the PULLED weights, not the table's (updated by the earlier
  // groups), so the pull keeps the per-parameter weights
  p.fm_keep_w = in.fm_vals && p.groups > 1;
  // MVM (one slice) and standard-math FM (any slices) on their reduction
  // paths: the per-key gradient rows land in unique order too (a dense apply
  // read instead of slot-indexed rows the apply had to zero after reading)
  const bool rows_ok = in.gpu && in.red_pairs && key_bound * in.pstride * in.slice_cap < k32;
  p.mvmu = rows_ok && p.Sf == 1 && in.kind == kMVM && in.red_rowv;
  p.fsu = rows_ok && (p.Sf == 1 || p.uqm) && in.kind == kFM && in.fm_math == kFmStandard;
  p.rowu = p.mvmu || p.fsu;
  // FTRL with several params per key on the packed apply: the pull stashes
  // every key's (n, z) in unique order for the first group's apply
  p.grpst = in.gpu && L.opt == kFTRL && L.P > 1;
  // the unique-order outputs of a multi-slice step and their slice bits
  p.uq = p.Sf > 1 && (p.lr16 || p.fmu || p.fsu);
  p.grad = p.lr16 ? GradPath::kUniqueLR
           : p.fmu ? GradPath::kUniqueFmBC
           : p.rowu ? GradPath::kUniqueRows
           : p.lr16s ? GradPath::kSlotSums
           : GradPath::kSlotRows;
  return p;
}

// Several slices, one pass: dedup -> pull (stash) -> one producer pass over
// every slice with dests unique * 2^slog2 + slice -> the CSR reduction (only
// the touched (key, slice) pairs) -> one apply whose per-key chains push the
// slices in order.  Replaces the slice groups' per-group sums and applies.
void Engine::train_step_csr(const BatchView& b, int S, int slog2) {
  const int32_t* srows = slice_rows_dev(b, S);
  const bool fm = fm_vals_;
  // standard FM / MVM: full-row entries (k_red_csr_vec), applied by the packed CSR apply
  const bool rows = csr_full_rows();
  ensure_inv();
  if (!csr_off_) {
    csr_off_ = balloc<u32>(*be_, (size_t)cfg_.max_nnz);
    csr_cnt_ = balloc<u32>(*be_, (size_t)cfg_.max_nnz);
  }
  const int ew = rows ? csr_row_words(table_.L.P) : 0;
  float* stash;
  if (fm || rows) {
    if (!grp_nz_) grp_nz_ = balloc<float>(*be_, 2 * (size_t)cfg_.max_nnz * table_.L.P);
    stash = grp_nz_;
  } else {
    if (!lr_nz_) lr_nz_ = balloc<float>(*be_, 2 * (size_t)cfg_.max_nnz);
    stash = lr_nz_;
  }
  dedup_(b, 1, nullptr, true);
  inv_valid_ = false;
  be_->remap_pos(pos_, b.nnz, inv_, (u32)scratch_.cap);
  guard_inserts(b.nnz);

  PullArgs pa;
  pa.table = table_;
  pa.opt = cfg_.opt;
  pa.keys = uniq_keys_;
  pa.n_dev = n_uniq_;
  pa.n_max = b.nnz;
  pa.insert = true;
  pa.out_slot = uniq_slot_;
  pa.out_vals = wpull_;
  pa.pstride = pstride();
  pa.fm_vals = fm;
  pa.out_nz = stash;
  be_->table_pull(pa);

  // (entries normalised by the reduction; reference FM: B and C before the
  // expansion, as the slice-group path and the multi-rank send buffer do)
  csr_forward_backward(b, slog2, srows, true);

  ApplyArgs aa;
  aa.table = table_;
  aa.opt = cfg_.opt;
  aa.keys = uniq_keys_;
  aa.slots = uniq_slot_;
  aa.n_dev = n_uniq_;
  aa.n_max = b.nnz;
  aa.S = S;
  aa.pstride = pstride();
  aa.P = cfg_.model.P();
  aa.fm_compact = fm;
  aa.fm_D = cfg_.model.v_dim;
  aa.nz_stash = stash;
  aa.csr_off = csr_off_;
  aa.csr_cnt = csr_cnt_;
  aa.csr_ent = rows ? static_cast<const void*>(csr_vent_) : red_pairs_;
  aa.csr_ew = ew;
  // (a chain has at most S entries: with S <= 16 nothing is ever deferred)
  aa.csr_long = S > 16 ? csr_long_list(b.nnz) : nullptr;
  aa.csr_long_cap = csr_long_cap_;
  attach_snapshot(aa);
  be_->table_apply(aa);
  end_step();
}

void Engine::csr_forward_backward(const BatchView& b, int slog2, const int32_t* srows,
                                  bool normalise) {
  if (!csr_off_) {
    csr_off_ = balloc<u32>(*be_, (size_t)cfg_.max_nnz);
    csr_cnt_ = balloc<u32>(*be_, (size_t)cfg_.max_nnz);
  }
  FwdArgs fa;
  fa.batch = b;
  fa.pos = pos_;
  fa.wpull = wpull_;
  fa.grad = grad_;
  fa.stats = stats_;
  fa.model = cfg_.model;
  fa.S = 1 << slog2;
  fa.agg_ok = true;  // (dests below max_nnz * 2^slog2 < 2^32: csr_slog2)
  fa.fx_bad = overflow_;
  set_reduction(fa);
  fa.red_nuq = n_uniq_;
  fa.fm_compact = fm_vals_;
  fa.fm_vals = fm_vals_;
  fa.red_csr.off = csr_off_;
  fa.red_csr.cnt = csr_cnt_;
  fa.red_csr.ent = red_pairs_;
  fa.red_csr.slog2 = slog2;
  fa.red_csr.rows = normalise ? srows : nullptr;
  if (csr_full_rows()) {  // full-row entries
    const int ew = csr_row_words(table_.L.P);
    if (!csr_vent_) csr_vent_ = balloc<float>(*be_, (size_t)cfg_.max_nnz * ew);
    fa.red_csr.ent = csr_vent_;
    fa.red_csr.P = table_.L.P;
    fa.red_csr.ew = ew;
  }
  be_->forward_backward(fa);
  ++csr_steps_;
}

u32* Engine::csr_long_list(int64_t n) {
  if (!be_->is_gpu()) return nullptr;
  // (wave-private lists: n plus a grid-stride iteration of every wave's keys,
  // <= 8192 x 4 waves x 64, and the per-wave counts)
  // (+ the dense list of n, the offsets and the scan tiles)
  const int64_t need = 2 * n + (int64_t)(2u << 20) + 4 * 65536;
  if (need > csr_long_cap_) {
    be_->free_stream(csr_long_);
    csr_long_cap_ = need + n / 4;
    csr_long_ = static_cast<u32*>(be_->alloc_stream(sizeof(u32) * (size_t)csr_long_cap_));
  }
  return csr_long_;
}

void Engine::w_forward_backward_csr(const BatchView& b, const float* pulled, int64_t n_send,
                                    int S_global, int wb, bool pack, u32* cnt_out, void* ent_out,
                                    const int64_t* counts, int world, bool encoded,
                                    int64_t* totals_out) {
  use_worker_set(wb);
  const int St = S_global > 0 ? S_global : slices_of(b);
  const int sl = csr_slog2(St);
  if (sl < 0 || St < slices_of(b) || St > cfg_.max_slices)
    throw std::invalid_argument("w_forward_backward_csr: S_global off the CSR path");
  // (a rank out of data -- a batch of 0 rows -- still takes part: no keys,
  // zero entries per owner)
  if (b.nnz > 0 && !inv_valid_)
    throw std::logic_error("w_forward_backward_csr: needs the partitioned dedup's inv");
  // unique-index (= send-order) positions, and the pulled rows (send order)
  // as the forward's value rows; the trash slot's row stays zero
  be_->remap_pos(pos_, b.nnz, inv_, (u32)scratch_.cap);
  be_->scatter_rows(pulled, wpull_, nullptr, nullptr, n_send, vstride_);
  // (rows per slice: the worker normalises, the owner does not know them)
  csr_forward_backward(b, sl, slice_rows_dev(b, St), true);
  last_nsend_ = n_send;
  if (!pack) return;
  if (!csr_doff_) csr_doff_ = balloc<u32>(*be_, (size_t)cfg_.max_nnz + 1);
  be_->scan_u32(csr_cnt_, csr_doff_, n_uniq_, cfg_.max_nnz);
  be_->csr_pack(csr_off_, csr_cnt_, csr_full_rows() ? static_cast<const void*>(csr_vent_) : red_pairs_,
                csr_doff_, n_uniq_, cfg_.max_nnz, ent_out, csr_entry_bytes());
  be_->copy_d2d(cnt_out, csr_cnt_, sizeof(u32) * (size_t)n_send);
  be_->csr_totals(counts, world, encoded, csr_doff_, totals_out);
}

void Engine::s_apply_csr(const u64* recv_keys, const u32* recv_cnt, const void* recv_ent,
                         const std::vector<int64_t>& src_offsets, int S, int buf) {
  if (buf < 0 || buf >= kSrvBufs) throw std::invalid_argument("server buffer must be in [0, kSrvBufs)");
  SrvBuf& sb = srv_[buf];
  sb.keys = nullptr;  // applied: no slot remap needed after a growth
  bool stash = sb.nz_fresh;
  stale_stashes();
  const u32* off = csr_off_;
  const u32* cnt = csr_cnt_;
  const void* ent = csr_full_rows() ? static_cast<const void*>(csr_vent_) : red_pairs_;
  const int64_t n = src_offsets.empty() ? 0 : src_offsets.back();
  if (n > sb.n) throw std::invalid_argument("s_apply_csr: offsets beyond pull");
  if (recv_cnt) {  // received entries: offsets by a scan of the counts
    if (n + 1 > csr_roff_cap_) {
      be_->free_stream(csr_roff_);
      csr_roff_cap_ = n + n / 4 + 1024;
      csr_roff_ = static_cast<u32*>(be_->alloc_stream(sizeof(u32) * (size_t)csr_roff_cap_));
    }
    be_->scan_u32(recv_cnt, csr_roff_, nullptr, n);
    off = csr_roff_;
    cnt = recv_cnt;
    ent = recv_ent;
  }
  size_t first_src = 0;
  while (first_src + 1 < src_offsets.size() && src_offsets[first_src + 1] <= src_offsets[first_src])
    ++first_src;
  for (size_t src = 0; src + 1 < src_offsets.size(); ++src) {
    const int64_t o = src_offsets[src], c = src_offsets[src + 1] - o;
    if (c <= 0) continue;
    ApplyArgs aa;
    aa.table = table_;
    aa.opt = cfg_.opt;
    aa.keys = recv_keys + o;
    aa.slots = sb.slots + o;
    aa.n_host = c;
    aa.n_max = c;
    aa.S = S;
    aa.pstride = pstride();
    aa.P = cfg_.model.P();
    aa.fm_compact = fm_vals_;
    aa.fm_D = cfg_.model.v_dim;
    aa.csr_ew = csr_full_rows() ? csr_row_words(table_.L.P) : 0;
    if (fm_vals_) {
      aa.pulled = pulled_weights(buf, o);
      if (!aa.pulled && src > first_src)
        throw std::logic_error("s_apply_csr: compact FM rows of several sources need s_pull's weights");
    }
    // (entries normalised by the workers; entry indices are global)
    aa.csr_off = off + o;
    aa.csr_cnt = cnt + o;
    aa.csr_ent = ent;
    aa.csr_long = S > 16 ? csr_long_list(c) : nullptr;
    aa.csr_long_cap = csr_long_cap_;
    if (stash) aa.nz_stash = sb.nz ? sb.nz + 2 * o : nullptr;
    stash = false;
    attach_snapshot(aa);
    be_->table_apply(aa);
  }
}

void Engine::csr_debug(std::vector<u32>& off, std::vector<u32>& cnt, std::vector<u32>& words) {
  off.clear();
  cnt.clear();
  words.clear();
  if (!csr_off_) return;
  const int64_t n = n_unique();
  off.resize((size_t)n);
  cnt.resize((size_t)n);
  be_->copy_d2h(off.data(), csr_off_, sizeof(u32) * (size_t)n);
  be_->copy_d2h(cnt.data(), csr_cnt_, sizeof(u32) * (size_t)n);
  u64 end = 0;
  for (int64_t i = 0; i < n; ++i) end = std::max<u64>(end, (u64)off[i] + cnt[i]);
  const bool rows = csr_vent_ && cfg_.model.kind == kFM && cfg_.model.fm_math == kFmStandard;
  const int w = rows ? csr_row_words(table_.L.P) : csr_entry_bytes() / 4;
  words.resize((size_t)end * w);
  if (end) be_->copy_d2h(words.data(), rows ? static_cast<const void*>(csr_vent_) : red_pairs_,
                         sizeof(u32) * (size_t)end * w);
}

void Engine::train_step(const BatchView& b) {
  stale_stashes();  // the table changes: server stashes are stale
  use_worker_set(0);
  const int S = slices_of(b);
  if (S > cfg_.max_slices) throw std::invalid_argument("batch has more slices than max_slices");
  if (cfg_.sum_slices && slice_groups(S) > 1)
    throw std::invalid_argument("sum_slices: at most 32 slices per step (ordered pushes: any count)");
  // every layout decision, made once (plan_step)
  const StepPlan P = plan(S);
  if (P.grad == GradPath::kCsr) {
    train_step_csr(b, S, P.csr_slog2);
    return;
  }
  const int ng = P.groups;
  const int ps = pstride();
  const bool masks = P.masks;
  const int32_t* srows = slice_rows_dev(b, S);
  const bool lr16 = P.lr16, lr16s = P.lr16s, uqm = P.uqm, fmu = P.fmu, fm_keep_w = P.fm_keep_w;
  const bool rowu = P.rowu, fsu = P.fsu, grpst = P.grpst, uq = P.uq, upos = P.upos;
  // (dest * ps in 32 bits over unique indices or scratch slots, see plan_step)
  const double key_bound = upos ? (double)cfg_.max_nnz : (double)scratch_.cap;
  if (lr16s && !lr_nz_) lr_nz_ = balloc<float>(*be_, 2 * (size_t)cfg_.max_nnz);
  if (lr16) {
    ensure_inv();
    if (!lr_grad_) lr_grad_ = balloc<float>(*be_, (size_t)cfg_.max_nnz * slice_cap_);
    if (!lr_nz_) lr_nz_ = balloc<float>(*be_, 2 * (size_t)cfg_.max_nnz);
  }
  if (fmu) {
    ensure_inv();
    if (!fm_grad_) fm_grad_ = balloc<float>(*be_, 2 * (size_t)cfg_.max_nnz * slice_cap_);
  }
  if (fm_keep_w && !fm_w_) fm_w_ = balloc<float>(*be_, (size_t)cfg_.max_nnz * ps);
  if (rowu) {
    ensure_inv();
    const int rs = fsu ? slice_cap_ : 1;
    if (!row_grad_) row_grad_ = balloc<float>(*be_, (size_t)cfg_.max_nnz * ps * rs);
  }
  if (grpst && !grp_nz_) grp_nz_ = balloc<float>(*be_, 2 * (size_t)cfg_.max_nnz * table_.L.P);
  if (uq && !lr_mask_) lr_mask_ = balloc<u32>(*be_, (size_t)cfg_.max_nnz);
  if (upos) ensure_inv();
  dedup_(b, 1, nullptr, upos || lr16 || fmu || rowu);
  inv_valid_ = false;  // (the sharded step's send order is not this one)
  if (upos) be_->remap_pos(pos_, b.nnz, inv_, (u32)scratch_.cap);
  guard_inserts(b.nnz);  // (<= nnz new keys; may grow the table first)

  PullArgs pa;
  pa.table = table_;
  pa.opt = cfg_.opt;
  pa.keys = uniq_keys_;
  pa.n_dev = n_uniq_;
  pa.n_max = b.nnz;
  pa.insert = true;
  pa.out_slot = uniq_slot_;
  pa.out_vals = wpull_;
  pa.out_map = upos ? nullptr : uniq_pos_;
  pa.pstride = ps;
  pa.fm_vals = fm_vals_;
  if (fm_keep_w) pa.out_w = fm_w_;
  if (lr16) {
    pa.out_nz = lr_nz_;
    pa.zero_out = lr_grad_;
  }
  if (lr16s) pa.out_nz = lr_nz_;
  if (grpst) pa.out_nz = grp_nz_;
  if (fmu) {
    pa.zero_out = fm_grad_;
    pa.zero_width = 2;
  }
  // (one-slice standard FM: every unique key's row is written by the
  // reduction -- each occurrence leaves a record, k_fm_std_red -- so the
  // pull need not zero them)
  if (rowu && !(fsu && P.Sf == 1)) {
    pa.zero_out = row_grad_;
    pa.zero_width = ps;
  }
  if (uq) {  // S > 1: only a key's present slices are read, so only its bits need clearing
    pa.zero_out = reinterpret_cast<float*>(lr_mask_);
    pa.zero_width = 1;
  }
  be_->table_pull(pa);

  for (int k = 0; k < ng; ++k) {
    const u32* posk = pos_;
    const BatchView bk = group_view(b, S, k, posk);
    const int Sg = group_slices(S, k);
    const int32_t* srk = srows + (int64_t)k * kSliceGroup;
    // a later group's unique-order slice bits start from zero again: the
    // pull cleared them for the first group, each group's apply clears the
    // bits it read (ApplyArgs::masks_clear); a later group's apply reads the
    // table, which the earlier groups updated, instead of the pull's stash
    const bool stash = k == 0;

    FwdArgs fa;
    fa.batch = bk;
    fa.pos = posk;
    fa.wpull = wpull_;
    fa.grad = grad_;
    fa.stats = stats_;
    fa.model = cfg_.model;
    fa.S = Sg;
    fa.agg_ok = key_bound * Sg * ps < 4294967295.0;  // (32-bit dest * ps, see rows_ok)
    fa.fx_bad = overflow_;
    set_reduction(fa);
    if (upos) fa.red_nuq = n_uniq_;
    // slice bits from the reduction (unique order with the outputs, else
    // slot-indexed), else per occurrence
    if (uq) fa.red_masks = lr_mask_;
    else if (uqm) fa.red_masks = tmask_;
    else if (masks) be_->slice_masks(bk, posk, tmask_);
    // reference-math FM on the GPU reduction path: (B, C) rows, expanded by the apply
    fa.fm_compact = fa.red_pairs && fa.agg_ok && cfg_.model.kind == kFM &&
                    cfg_.model.fm_math == kFmReference;
    fa.fm_vals = fm_vals_;
    if (fm_vals_ && !fa.fm_compact) throw std::logic_error("train_step: compact FM rows need the reduction");
    // (unique-index positions: the outputs' rows are the dests' own)
    const u32* oinv = upos ? nullptr : inv_;
    if (lr16) {
      fa.red_out = lr_grad_;
      fa.red_inv = oinv;
      fa.red_rows = srk;
    }
    if (fmu) {  // (B, C) normalised before the expansion: 2 divisions a key, not P
      fa.red_out = fm_grad_;
      fa.red_inv = oinv;
      fa.red_rows = srk;
    }
    if (rowu) {
      fa.red_out = row_grad_;
      fa.red_inv = oinv;
    }
    be_->forward_backward(fa);

    ApplyArgs aa;
    aa.table = table_;
    aa.opt = cfg_.opt;
    aa.keys = uniq_keys_;
    aa.slots = uniq_slot_;
    aa.n_dev = n_uniq_;
    aa.n_max = b.nnz;
    aa.grads = grad_;
    aa.grad_map = upos ? nullptr : uniq_pos_;  // (slot- or unique-indexed rows)
    aa.masks = masks ? tmask_ : nullptr;
    aa.masks_rw = masks ? tmask_ : nullptr;
    aa.zero_after = true;
    aa.S = Sg;
    aa.pstride = ps;
    aa.P = cfg_.model.P();
    aa.sum_slices = cfg_.sum_slices;
    aa.slice_rows = srk;
    aa.fm_compact = fa.fm_compact;
    aa.fm_D = cfg_.model.v_dim;
    if (fm_keep_w) aa.pulled = fm_w_;
    if (lr16) {  // unique-order, already normalised, zeroed by the next pull
      aa.grads = lr_grad_;
      aa.grad_map = nullptr;
      aa.zero_after = false;
      aa.slice_rows = nullptr;
      aa.nz_stash = stash ? lr_nz_ : nullptr;
    }
    if (lr16s && stash) aa.nz_stash = lr_nz_;  // (unique order, as the apply's entries)
    if (grpst && stash) aa.nz_stash = grp_nz_;
    if (fmu) {  // unique-order normalised (B, C), zeroed by the next pull
      aa.grads = fm_grad_;
      aa.grad_map = nullptr;
      aa.zero_after = false;
      aa.slice_rows = nullptr;
      aa.gstride = 2;
    }
    if (rowu) {  // unique-order rows, zeroed by the next pull
      aa.grads = row_grad_;
      aa.grad_map = nullptr;
      aa.zero_after = false;
      aa.gstride = ps;
    }
    if (uq) {  // present slices by the unique-order bits (cleared by the next pull)
      aa.masks = lr_mask_;
      aa.masks_rw = nullptr;
      aa.masks_clear = k + 1 < ng;  // (for the next group's reduction)
    }
    attach_snapshot(aa);
    be_->table_apply(aa);
  }
  end_step();
}

void Engine::eval_step(const BatchView& b, float* pctr) {
  use_worker_set(0);
  dedup_(b);
  PullArgs pa;
  pa.table = table_;
  pa.opt = cfg_.opt;
  pa.keys = uniq_keys_;
  pa.n_dev = n_uniq_;
  pa.n_max = b.nnz;
  pa.insert = false;
  pa.out_slot = uniq_slot_;
  pa.out_vals = wpull_;
  pa.out_map = uniq_pos_;
  pa.pstride = pstride();
  pa.fm_vals = fm_vals_;
  be_->table_pull(pa);

  FwdArgs fa;
  fa.batch = b;
  fa.pos = pos_;
  fa.wpull = wpull_;
  fa.grad = nullptr;
  fa.pctr = pctr;
  fa.stats = stats_ + 1;
  fa.model = cfg_.model;
  fa.S = 1;
  fa.fm_vals = fm_vals_;
  be_->forward_backward(fa);
}

void Engine::push_host(const std::vector<u64>& keys, const std::vector<float>& grads) {
  stale_stashes();  // the table changes: server stashes are stale
  const int64_t n = (int64_t)keys.size();
  const int P = cfg_.model.P();
  if ((int64_t)grads.size() != n * P) throw std::invalid_argument("push_host: grads != keys*P");
  if (n == 0) return;
  guard_inserts(n);
  if (n > host_cap_) {
    be_->synchronize();
    be_->free(host_keys_dev_);
    be_->free(host_vals_dev_);
    be_->free(host_slots_dev_);
    host_cap_ = n;
    host_keys_dev_ = balloc<u64>(*be_, n);
    host_vals_dev_ = balloc<float>(*be_, n * P);
    host_slots_dev_ = balloc<u32>(*be_, n);
  }
  be_->copy_h2d(host_keys_dev_, keys.data(), sizeof(u64) * n);
  be_->copy_h2d(host_vals_dev_, grads.data(), sizeof(float) * n * P);
  PullArgs pa;
  pa.table = table_;
  pa.opt = cfg_.opt;
  pa.keys = host_keys_dev_;
  pa.n_host = n;
  pa.n_max = n;
  pa.insert = true;
  pa.out_slot = host_slots_dev_;
  be_->table_pull(pa);
  // Pushes of one call are applied one key at a time in order; duplicate keys
  // inside one call are applied sequentially by separate launches.
  ApplyArgs aa;
  aa.table = table_;
  aa.opt = cfg_.opt;
  aa.keys = host_keys_dev_;
  aa.S = 1;
  aa.pstride = P;
  aa.P = P;
  for (int64_t i = 0; i < n; ++i) {
    aa.slots = host_slots_dev_ + i;
    aa.grads = host_vals_dev_ + i * P;
    aa.n_host = 1;
    aa.n_max = 1;
    be_->table_apply(aa);
  }
  be_->synchronize();
}

void Engine::prefill(int64_t n, uint64_t seed) {
  if (n > 0) guard_inserts(n);  // (may grow the table first)
  if (n < 0 || (uint64_t)n > table_.cap - table_.cap / 16)
    throw std::invalid_argument("prefill: at most 15/16 of the table's slots");
  stale_stashes();
  be_->table_prefill(table_, n, seed);
  be_->synchronize();
  (void)table_size();  // (re-bases the capacity monitor)
}

std::vector<float> Engine::pull_host(const std::vector<u64>& keys) {
  const int64_t n = (int64_t)keys.size();
  const int P = cfg_.model.P();
  std::vector<float> out((size_t)n * P);
  if (n == 0) return out;
  if (n > host_cap_) {
    be_->synchronize();
    be_->free(host_keys_dev_);
    be_->free(host_vals_dev_);
    be_->free(host_slots_dev_);
    host_cap_ = n;
    host_keys_dev_ = balloc<u64>(*be_, n);
    host_vals_dev_ = balloc<float>(*be_, n * P);
    host_slots_dev_ = balloc<u32>(*be_, n);
  }
  be_->copy_h2d(host_keys_dev_, keys.data(), sizeof(u64) * n);
  PullArgs pa;
  pa.table = table_;
  pa.opt = cfg_.opt;
  pa.keys = host_keys_dev_;
  pa.n_host = n;
  pa.n_max = n;
  pa.insert = false;
  pa.out_slot = host_slots_dev_;
  pa.out_vals = host_vals_dev_;
  pa.pstride = P;
  be_->table_pull(pa);
  be_->copy_d2h(out.data(), host_vals_dev_, sizeof(float) * n * P);
  return out;
}

// ---------------------------------------------------------------------------
// multi-rank phases
// ---------------------------------------------------------------------------
void Engine::w_prepare(const BatchView& b, int world, int64_t* counts_out, u64* send_keys_out,
                       int wb, int64_t seq) {
  if (world <= 1) seq = -1;  // (no exchange to check)
  use_worker_set(wb);
  if (slices_of(b) > cfg_.max_slices)
    throw std::invalid_argument("batch has more slices than max_slices");
  if (b.nnz == 0) {
    // nothing to send; a batch without rows (a rank out of data) sends -1
    // counts, which tell the receivers "no data from this source" (the loop
    // ends when every source says so, ShardedEngine.train_step)
    const int64_t c = b.rows == 0 ? -1 : 0;
    be_->fill_u64(reinterpret_cast<u64*>(counts_out), (u64)(seq >= 0 ? encode_count(c, seq) : c),
                  (size_t)(world > 0 ? world : 1));
    be_->memset(n_uniq_, 0, sizeof(int64_t));
    inv_valid_ = false;
    send_map_ = uniq_pos_;
    return;
  }
  if (world >= 1 && world <= kMaxParts && be_->partitioned_dedup()) {
    // owner-partitioned scratch: the slot-ordered unique list is the send
    // order already; counts are range counts (one range at world 1).  inv_
    // (slot -> send index) lets the LR backward write the send buffer directly.
    if (red_pairs_ && (cfg_.model.kind == kLR || fm_vals_ || csr_full_rows())) ensure_inv();
    dedup_(b, world, send_keys_out, true, world == 1 ? counts_out : nullptr);
    inv_valid_ = inv_ != nullptr;
    if (world > 1) be_->partition_counts(scratch_, block_counts_, n_uniq_, counts_out, seq);
    send_map_ = uniq_pos_;
    return;
  }
  dedup_(b);
  inv_valid_ = false;
  BucketArgs ba;
  ba.uniq_keys = uniq_keys_;
  ba.uniq_pos = uniq_pos_;
  ba.n_dev = n_uniq_;
  ba.n_max = b.nnz;
  ba.world = world;
  ba.counts = counts_out;
  ba.send_keys = send_keys_out;
  ba.send_pos = send_pos_;
  ba.scratch = bucket_ws_;
  ba.seq = seq;
  be_->bucket(ba);
  send_map_ = send_pos_;
  // (slice masks are built in w_forward_backward with the step's global S)
}

void Engine::ensure_server_capacity(int64_t n, int buf) {
  if (buf < 0 || buf >= kSrvBufs) throw std::invalid_argument("server buffer must be in [0, kSrvBufs)");
  SrvBuf& sb = srv_[buf];
  if (n <= sb.cap) return;
  be_->synchronize();
  be_->free(sb.slots);
  be_->free(sb.nz);
  sb.nz = nullptr;
  sb.cap = n + n / 4 + 1024;
  sb.slots = balloc<u32>(*be_, sb.cap);
  if (lr16_layout()) sb.nz = balloc<float>(*be_, 2 * (size_t)sb.cap);
}

bool Engine::lr16_layout() const {
  const TableLayout& L = table_.L;
  return be_->is_gpu() && L.stride == 4 && L.P == 1 && L.opt == kFTRL && !L.has_flag;
}

void Engine::w_forward(const BatchView& b, const float* pulled, int64_t n_send, float* pctr,
                       int wb) {
  use_worker_set(wb);
  be_->scatter_rows(pulled, wpull_, send_map_, nullptr, n_send, vstride_);
  FwdArgs fa;
  fa.batch = b;
  fa.pos = pos_;
  fa.wpull = wpull_;
  fa.grad = nullptr;
  fa.pctr = pctr;
  fa.stats = stats_ + 1;
  fa.model = cfg_.model;
  fa.S = 1;
  fa.fm_vals = fm_vals_;
  be_->forward_backward(fa);
}

void Engine::s_pull(const u64* recv_keys, int64_t n, float* out_vals, bool insert, int buf,
                    const std::vector<int64_t>& src_offsets, bool keep_weights) {
  ensure_server_capacity(n, buf);
  SrvBuf& sb = srv_[buf];
  sb.n = n;
  sb.vals = out_vals;
  sb.w_valid = false;
  sb.grp = SrcGroups();
  // (kept until the buffer's s_apply: a table growth re-probes its slots)
  sb.keys = insert && n > 0 ? recv_keys : nullptr;
  if (n == 0) return;
  if (insert) {
    guard_inserts(n);
    group_entries(recv_keys, n, buf, src_offsets);
  }
  PullArgs pa;
  pa.table = table_;
  pa.opt = cfg_.opt;
  pa.keys = recv_keys;
  pa.n_host = n;
  pa.n_max = n;
  pa.insert = insert;
  pa.out_slot = sb.slots;
  pa.out_vals = out_vals;
  pa.pstride = pstride();
  pa.fm_vals = fm_vals_;
  // Compact FM value rows carry no per-parameter weights: an apply that runs
  // after other table updates (the staleness-k step), or source by source
  // because the owner grouping was skipped (world > kMaxGroupSources, or the
  // other buffers' registrations were dropped on an owner-scratch resize),
  // needs the weights the workers' gradients refer to.
  const int nsrc = (int)src_offsets.size() - 1;
  int active = 0;
  for (int s2 = 0; s2 < nsrc; ++s2) active += src_offsets[s2 + 1] > src_offsets[s2];
  if (fm_vals_ && insert && (keep_weights || (!sb.grp.oidx && active > 1))) {
    if (sb.w_cap < n) {
      be_->synchronize();
      be_->free(sb.w);
      sb.w_cap = n + n / 4 + 1024;
      sb.w = balloc<float>(*be_, (size_t)sb.w_cap * pstride());
    }
    pa.out_w = sb.w;
    sb.w_valid = true;
  }
  pa.out_nz = sb.nz;
  sb.nz_fresh = sb.nz != nullptr;
  be_->table_pull(pa);
}

// Owner grouping of the received entries (several sources with keys this
// step, GPU backend): one registration per (key, source) in an owner scratch
// table, so that s_apply runs once over all sources.  The scratch keeps keys
// across steps and is cleared once the entries registered since the last
// clear (an upper bound of its keys) could exceed half of it; it is sized to
// 4x the step's entries, so the load stays below 0.75.
bool Engine::group_entries(const u64* recv_keys, int64_t n, int buf,
                           const std::vector<int64_t>& offs) {
  // (EngineConfig::owner_group: grouping is opt-in)
  const int nsrc = (int)offs.size() - 1;
  if (cfg_.owner_group != 1) return false;
  if (!be_->owner_grouping() || nsrc < 2 || nsrc > kMaxGroupSources) return false;
  if (offs.front() != 0 || offs.back() != n) throw std::invalid_argument("s_pull: source offsets");
  int active = 0;
  for (int s = 0; s < nsrc; ++s) {
    if (offs[s + 1] < offs[s]) throw std::invalid_argument("s_pull: source offsets");
    active += offs[s + 1] > offs[s];
  }
  if (active < 2) return false;  // one source: the per-source apply is one launch already
  const u64 want = next_pow2((uint64_t)n * 4);
  if (want > (1ull << 32)) throw std::invalid_argument("s_pull: too many received keys to group");
  if (want > own_cap_ || nsrc != own_nsrc_) {
    // (re)size: the other buffer's registrations are dropped with the arrays
    // (its apply then runs source by source)
    be_->synchronize();
    const u64 cap = want > own_cap_ ? want : own_cap_;
    be_->free(own_keys_);
    for (SrvBuf& b : srv_) {
      be_->free(b.own_idx);
      b.own_idx = nullptr;
      b.grp = SrcGroups();
    }
    own_cap_ = cap;
    own_nsrc_ = nsrc;
    own_keys_ = balloc<u64>(*be_, cap);
    be_->fill_u64(own_keys_, kEmptyKey, cap);
    own_fill_ = 0;
  }
  SrvBuf& sb = srv_[buf];
  if (!sb.own_idx) {
    sb.own_idx = balloc<u64>(*be_, own_cap_ * (u64)own_nsrc_);
    be_->memset(sb.own_idx, 0, sizeof(u64) * own_cap_ * own_nsrc_);  // epoch 0: never valid
  }
  if (n > sb.own_pos_cap) {
    be_->synchronize();
    be_->free(sb.own_pos);
    sb.own_pos_cap = n + n / 4 + 1024;
    sb.own_pos = balloc<u32>(*be_, sb.own_pos_cap);
  }
  if (own_fill_ + n > (int64_t)(own_cap_ / 2)) {
    be_->fill_u64(own_keys_, kEmptyKey, own_cap_);
    own_fill_ = 0;
  }
  own_fill_ += n;
  if (++own_epoch_ == 0) own_epoch_ = 1;
  OwnerGroupArgs ga;
  ga.keys = recv_keys;
  ga.n = n;
  ga.okeys = own_keys_;
  ga.ocap = own_cap_;
  ga.opos = sb.own_pos;
  ga.oidx = sb.own_idx;
  ga.g.nsrc = nsrc;
  ga.g.epoch = own_epoch_;
  for (int s = 0; s <= nsrc; ++s) ga.g.offs[s] = offs[s];
  ga.overflow = overflow_;
  be_->owner_group(ga);
  sb.grp = ga.g;
  sb.grp.opos = sb.own_pos;
  sb.grp.oidx = sb.own_idx;
  return true;
}

void Engine::w_forward_backward(const BatchView& b, const float* pulled, int64_t n_send,
                                float* grads_out, u32* masks_out, int S_global, int wb,
                                int group) {
  use_worker_set(wb);
  // All ranks of a step must agree on the gradient row width (S*pstride):
  // S_global (>= this batch's slices) lets a rank with a short or empty batch
  // emit the same layout; its extra slices carry no rows and no mask bits.
  const int St = S_global > 0 ? S_global : slices_of(b);
  if (St < slices_of(b) || St > cfg_.max_slices)
    throw std::invalid_argument("w_forward_backward: S_global out of range");
  const int ng = slice_groups(St);
  if (group < 0 || group >= ng) throw std::invalid_argument("w_forward_backward: slice group");
  if (ng > 1 && cfg_.sum_slices)
    throw std::invalid_argument("sum_slices: at most 32 slices per step (ordered pushes: any count)");
  // slice group `group` of the step: its rows, its slices (>= 2 when grouped)
  const u32* posk = pos_;
  const BatchView bk = group_view(b, St, group, posk);
  const int S = group_slices(St, group);
  const int ps = pstride();
  const bool masks = S > 1 && !cfg_.sum_slices;
  const int32_t* srows = slice_rows_dev(b, St) + (int64_t)group * kSliceGroup;
  const bool direct = inv_valid_ && red_pairs_ && S == 1 &&
                      (cfg_.model.kind == kLR || fm_vals_) &&
                      (double)scratch_.cap * S * ps < 4294967295.0;
  // the direct path's send buffer is zeroed by the scatter; the pulled rows
  // are placed once per step (every group reads the same ones)
  if (group == 0)
    be_->scatter_rows(pulled, wpull_, send_map_, nullptr, n_send, vstride_,
                      direct ? grads_out : nullptr, grad_width());
  FwdArgs fa;
  fa.batch = bk;
  fa.pos = posk;
  fa.wpull = wpull_;
  fa.grad = grad_;
  fa.stats = stats_;
  fa.model = cfg_.model;
  fa.S = S;
  fa.agg_ok = (double)scratch_.cap * S * pstride() < 4294967295.0;
  fa.fx_bad = overflow_;
  set_reduction(fa);
  if (masks && reduction_masks(false)) fa.red_masks = tmask_;
  else if (masks) be_->slice_masks(bk, posk, tmask_);
  fa.fm_compact = sharded_fm_compact() && fa.agg_ok;
  fa.fm_vals = fm_vals_;
  if (sharded_fm_compact() && !fa.fm_compact)
    throw std::logic_error("w_forward_backward: compact FM rows need the reduction path");
  if (direct) {
    if (!fa.red_pairs || !fa.agg_ok) throw std::logic_error("direct send path without reduction");
    // the bucket reduction writes the normalised send buffer (no gather)
    fa.red_out = grads_out;
    fa.red_inv = inv_;
    fa.red_rows = srows;
    be_->forward_backward(fa);
    last_nsend_ = n_send;
    return;
  }
  be_->forward_backward(fa);
  GatherGradArgs ga;
  ga.grad = grad_;
  ga.grad_rw = grad_;
  ga.tmask = masks ? tmask_ : nullptr;
  ga.tmask_rw = masks ? tmask_ : nullptr;
  ga.map = send_map_;
  ga.n_max = n_send;
  ga.S = S;
  ga.pstride = ps;
  ga.slice_rows = srows;
  ga.width = grad_width();
  ga.out = grads_out;
  ga.out_mask = masks ? masks_out : nullptr;
  be_->gather_grads(ga);
  last_nsend_ = n_send;
}

void Engine::s_apply(const u64* recv_keys, const float* recv_grads, const u32* recv_masks,
                     const std::vector<int64_t>& src_offsets, int S, int buf) {
  if (buf < 0 || buf >= kSrvBufs) throw std::invalid_argument("server buffer must be in [0, kSrvBufs)");
  SrvBuf& sb = srv_[buf];
  sb.keys = nullptr;  // applied: no slot remap needed after a growth
  const int ps = pstride();
  const int gw = grad_width();
  // the first source applied sees the state its pull saw; a key sent by
  // several sources is updated by the earlier ones, so later sources re-read
  // (the grouped apply pushes every source of a key at once: its stash stays valid)
  bool stash = sb.nz_fresh;
  stale_stashes();
  ApplyArgs base;
  base.table = table_;
  base.opt = cfg_.opt;
  base.gstride = gw;
  if (sharded_fm_compact()) {
    base.fm_compact = true;
    base.fm_D = cfg_.model.v_dim;
  }
  base.zero_after = false;
  base.S = S;
  base.pstride = ps;
  base.P = cfg_.model.P();
  base.sum_slices = cfg_.sum_slices;
  base.slice_rows = nullptr;
  const SrcGroups& g = sb.grp;
  bool same = g.oidx && (int)src_offsets.size() == g.nsrc + 1;
  for (int s = 0; same && s <= g.nsrc; ++s) same = src_offsets[s] == g.offs[s];
  // (other offsets, e.g. one source at a time for a grouped-slice step: per source below)
  if (same) {
    const int64_t n = g.offs[g.nsrc];
    if (n > sb.n) throw std::invalid_argument("s_apply: offsets beyond pull");
    ApplyArgs aa = base;
    aa.keys = recv_keys;
    aa.slots = sb.slots;
    aa.n_host = n;
    aa.n_max = n;
    aa.grads = const_cast<float*>(recv_grads);
    if (aa.fm_compact) aa.pulled = pulled_weights(buf, 0);
    aa.masks = recv_masks;
    if (stash) aa.nz_stash = sb.nz;
    aa.grp = g;
    attach_snapshot(aa);
    be_->table_apply(aa);
    return;
  }
  size_t first_src = 0;
  while (first_src + 1 < src_offsets.size() && src_offsets[first_src + 1] <= src_offsets[first_src])
    ++first_src;
  for (size_t src = 0; src + 1 < src_offsets.size(); ++src) {
    int64_t off = src_offsets[src];
    int64_t cnt = src_offsets[src + 1] - off;
    if (cnt <= 0) continue;
    if (src_offsets[src + 1] > sb.n) throw std::invalid_argument("s_apply: offsets beyond pull");
    ApplyArgs aa = base;
    aa.keys = recv_keys + off;
    aa.slots = sb.slots + off;
    aa.n_host = cnt;
    aa.n_max = cnt;
    aa.grads = const_cast<float*>(recv_grads) + off * (int64_t)S * gw;
    if (aa.fm_compact) {
      aa.pulled = pulled_weights(buf, off);
      // compact value rows carry no per-parameter weights: a later source
      // would expand its (B, C) with weights the earlier sources updated
      if (!aa.pulled && src > first_src)
        throw std::logic_error("s_apply: compact FM rows of several sources need the grouped "
                               "apply or s_pull(keep_weights)");
    }
    aa.masks = recv_masks ? recv_masks + off : nullptr;
    if (stash) aa.nz_stash = sb.nz + 2 * off;
    stash = false;
    attach_snapshot(aa);
    be_->table_apply(aa);
  }
}

// Per-parameter pre-step weights of buffer entries from `off` for the compact
// FM apply: full pulled rows, or the owner's kept weights, or none (the apply
// then takes the slot's current weights -- valid while no other update ran).
const float* Engine::pulled_weights(int buf, int64_t off) const {
  const SrvBuf& sb = srv_[buf];
  if (!fm_vals_) return sb.vals + off * (int64_t)pstride();
  if (sb.w_valid) return sb.w + off * (int64_t)pstride();
  return nullptr;
}

// The dedup scratch is epoch-stamped and persistent: nothing to release; the
// step's capacity snapshot is queued here.
void Engine::w_finish() { end_step(); }

// ---------------------------------------------------------------------------
// table capacity management
// ---------------------------------------------------------------------------

// Consume the recorded snapshots in order (each event completes after the
// older ones: one stream); wait_upto >= 0 waits for snapshots up to that
// sequence number.  A snapshot with an overflow flag raises: keys were
// dropped (table: no slot within the probe bound; dedup or owner scratch:
// full), so the run is invalid -- fail within monitor_lag steps, not at
// epoch end.
bool Engine::snap_ready(int64_t seq) const {
  const volatile unsigned long long* p = &snaps_[seq % kSnaps].word;
  const unsigned long long want = (unsigned long long)seq & ((1ull << (64 - kSnapSeqShift)) - 1);
  return (*p >> kSnapSeqShift) == want;
}

// The next snapshot rides on this apply launch (its first wave stores it):
// valid as long as no insert is queued between it and end_step.
void Engine::attach_snapshot(ApplyArgs& aa) {
  if (!be_->is_gpu() || monitor_disabled() || aa.n_max <= 0) return;
  const int64_t seq = snap_seq_ + 1;
  if (seq - 1 - snap_seen_ >= kSnaps) poll_snapshots(seq - kSnaps);  // (ring slot reuse)
  aa.snap = &snaps_[seq % kSnaps];
  aa.snap_mon = mon_;
  aa.snap_seq = (unsigned long long)seq;
  snap_carried_ = true;
}

void Engine::poll_snapshots(int64_t wait_upto) {
  while (snap_seen_ < snap_seq_) {
    const int64_t seq = snap_seen_ + 1;  // (sequence numbers start at 1)
    const int i = (int)(seq % kSnaps);
    if (!snap_ready(seq)) {
      if (seq > wait_upto) break;
      ++monitor_waits_;
      const auto t0 = std::chrono::steady_clock::now();
      for (int spin = 0; !snap_ready(seq); ++spin) {
        if (spin > 64) std::this_thread::sleep_for(std::chrono::microseconds(20));
        else std::this_thread::yield();
      }
      monitor_wait_s_ += std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    }
    const unsigned long long w = *reinterpret_cast<volatile unsigned long long*>(&snaps_[i].word);
    const int64_t size = (int64_t)(w & 0xFFFFFFFFull);
    const bool ovf0 = (w >> 32) & 1ull, ovf1 = (w >> 33) & 1ull, bad = (w >> 34) & 1ull;
    known_size_ = size;
    known_adds_ = snap_adds_[i];
    ++snap_seen_;
    if (bad && !ovf0 && !ovf1)
      throw std::runtime_error(
          "xflow: non-finite or out-of-range prediction / gradient sum (the model diverged); "
          "the step's values were clamped");
    if (ovf0 || ovf1) {
      char msg[320];
      std::snprintf(msg, sizeof(msg),
                    "xflow: %s overflow -- keys were dropped (table: %lld keys in %llu slots%s); "
                    "raise the capacity (table_log2_cap / max_log2_cap, max_nnz)",
                    ovf1 ? "parameter table" : "dedup/owner scratch", (long long)size,
                    (unsigned long long)table_.cap, cfg_.table_grow ? "" : ", growth disabled");
      throw std::runtime_error(msg);
    }
  }
}

// Close the next snapshot: it is the one an apply of this step carries, or
// a tiny kernel writes it now; its insert bound is everything queued so far.
void Engine::close_snapshot() {
  const int64_t seq = snap_seq_ + 1;
  if (!snap_carried_) {
    if (seq - 1 - snap_seen_ >= kSnaps) poll_snapshots(seq - kSnaps);  // (ring slot reuse)
    be_->snapshot(&snaps_[seq % kSnaps], mon_, (unsigned long long)seq);
  }
  snap_carried_ = false;
  snap_adds_[seq % kSnaps] = queued_adds_;
  snap_seq_ = seq;
}

void Engine::end_step() {
  if (monitor_disabled()) return;
  close_snapshot();
  // bounded run-ahead: the snapshot monitor_lag steps back must be in
  poll_snapshots(snap_seq_ - cfg_.monitor_lag);
}

// Before an inserting pull of n keys (at most n new): grow the table so that
// the growth schedule (EngineConfig::grow_start / grow_load) holds for an
// upper bound of its size -- the last snapshot's size plus every insert bound
// queued since.  No host sync: a split is queued device work (split_to).
void Engine::guard_inserts(int64_t n) {
  if (n <= 0) return;
  // an apply outside a step (e.g. a staleness-k flush) carried a snapshot:
  // close it before these inserts, which it does not include
  if (snap_carried_) close_snapshot();
  poll_snapshots(-1);
  if (cfg_.table_grow) {
    const double bound = (double)(known_size_ + (queued_adds_ - known_adds_) + n);
    const u64 N = table_.cap >> table_.seg_log2;
    const u64 want = segments_for(bound, cfg_.grow_start, cfg_.grow_load);
    if (want > N) {
      // paced: twice what the schedule asks for this call's n keys (and at
      // least ~64 MB of segments), so a schedule that fell behind catches up
      // over several calls instead of one burst -- unless the fullest
      // segments would pass kHardLoad
      const size_t seg_bytes = ((size_t)1 << table_.seg_log2) * table_.L.stride * sizeof(u32);
      const u64 before = segments_for(bound - (double)n, cfg_.grow_start, cfg_.grow_load);
      u64 pace = 2 * (want - (before < want ? before : want)) + 1;
      const u64 floor_pace = seg_bytes >= (64u << 20) ? 1 : (u64)((64u << 20) / seg_bytes);
      if (pace < floor_pace) pace = floor_pace;
      const double hl = cfg_.grow_load > kHardLoad ? cfg_.grow_load : kHardLoad;
      const u64 hard = segments_for(bound, hl, hl);
      u64 target = want < N + pace ? want : N + pace;
      if (hard > target) target = hard;
      split_to(target);
    }
  }
  queued_adds_ += n;
}

// Segments the schedule wants for `keys` keys: at level L with s segments
// split, a segment not yet split holds keys / 2^L (uniform hashing) at load
// u = keys / (2^L * G); the schedule splits 2^L * (u - grow_start) /
// (grow_load - grow_start) of them (all by u = grow_load, when the level is
// complete and u halves).  u0 == u1: the segments that keep every load <= u1
// (whole levels).  Capped at 2^max_log2_cap slots.
u64 Engine::segments_for(double keys, double u0, double u1) const {
  const int g = table_.seg_log2;
  const double G = (double)(1ull << g);
  u64 N = table_.cap >> g;
  while (N < max_segs_) {
    int L = 0;
    while ((2ull << L) <= N) ++L;
    const u64 P = 1ull << L, s = N - P;
    const double u = keys / ((double)P * G);
    if (u <= u0) break;
    u64 want = u >= u1 ? P : (u64)std::ceil((double)P * (u - u0) / (u1 - u0));  // (u0 < u < u1)
    if (want > P) want = P;
    if (want <= s) break;
    N = P + want;
  }
  return N < max_segs_ ? N : max_segs_;
}

// Split segments (level by level, in launches of at most 2^28 slots) until the
// table has nseg segments: commit the new segments' memory at the end of the
// range, clear them, split their source segments (Backend::table_split).
// Slots of the moved keys change: pulled-but-not-applied server buffers are
// looked up again, queued on the stream.
void Engine::split_to(u64 nseg) {
  const auto t0 = std::chrono::steady_clock::now();
  const int g = table_.seg_log2;
  const u64 G = 1ull << g;
  const size_t seg_bytes = (size_t)G * table_.L.stride * sizeof(u32);
  const u64 per_launch = g >= 28 ? 1 : (1ull << (28 - g));
  if (nseg > max_segs_) nseg = max_segs_;
  bool grew = false;
  while ((table_.cap >> g) < nseg) {
    const u64 N = table_.cap >> g, P = 1ull << table_.level, s0 = table_.split;
    u64 k = nseg - N;
    if (k > P - s0) k = P - s0;
    if (k > per_launch) k = per_launch;
    const size_t bytes = (size_t)(N + k) * seg_bytes;
    const size_t have = be_->table_committed();
    if (bytes > have) {
      const size_t fr = be_->free_memory();
      // (a re-allocating backend needs the whole new table next to the old one)
      const size_t need = be_->table_in_place() ? bytes - have : bytes;
      if (fr < need + (size_t)(256u << 20)) {
        if (grew) break;  // (what fits was added; the inserts run at a higher load)
        char msg[256];
        std::snprintf(msg, sizeof(msg),
                      "xflow: table growth to %llu slots needs %.2f GB more, %.2f GB free on the device",
                      (unsigned long long)((N + k) << g), need / 1e9, fr / 1e9);
        throw std::runtime_error(msg);
      }
    }
    table_.words = static_cast<u32*>(be_->table_commit(table_.words, bytes));
    TableView fresh = table_;
    fresh.words = table_.words + (size_t)(N << g) * table_.L.stride;
    fresh.cap = k << g;
    be_->table_clear(fresh);
    table_.cap = (N + k) << g;
    table_.split = s0 + k;
    be_->table_split(table_, s0, k);
    if (table_.split == P) {
      ++table_.level;
      table_.split = 0;
    }
    table_bytes_ = (size_t)table_.cap * table_.L.stride * sizeof(u32);
    splits_ += (int64_t)k;
    grew = true;
  }
  if (grew) {
    ++growths_;
    remap_server_slots();
  }
  grow_s_ += std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
}

size_t Engine::table_committed() const { return be_->table_committed(); }

// Explicit growth to at least 2^lg slots (normally automatic).
void Engine::grow_table(int lg) {
  if (lg > 31) throw std::invalid_argument("grow_table: at most 2^31 slots (32-bit slot indices)");
  if (lg < table_.seg_log2 || (1ull << lg) <= table_.cap) return;
  if (lg > max_log2_cap_) throw std::invalid_argument("grow_table: beyond max_log2_cap");
  poll_snapshots(-1);
  split_to((1ull << lg) >> table_.seg_log2);
}

// Slots of pulled-but-not-yet-applied server buffers point into the old
// table: look their keys up again (all present, no insert).
void Engine::remap_server_slots() {
  for (SrvBuf& sb : srv_) {
    if (!sb.keys || sb.n <= 0) continue;
    PullArgs pa;
    pa.table = table_;
    pa.opt = cfg_.opt;
    pa.keys = sb.keys;
    pa.n_host = sb.n;
    pa.n_max = sb.n;
    pa.insert = false;
    pa.out_slot = sb.slots;
    pa.pstride = pstride();
    be_->table_pull(pa);
  }
}

// ---------------------------------------------------------------------------
LossStats Engine::read_stats(bool reset, int which) {
  if (which < 0 || which > 1) throw std::invalid_argument("read_stats: which must be 0 or 1");
  LossStats h;
  be_->copy_d2h(&h, stats_ + which, sizeof(h));
  if (reset) be_->memset(stats_ + which, 0, sizeof(LossStats));
  return h;
}

int64_t Engine::n_unique() {
  int64_t n = 0;
  be_->copy_d2h(&n, n_uniq_, sizeof(n));
  return n;
}

int64_t Engine::table_size() {
  unsigned long long n = 0;
  be_->copy_d2h(&n, table_.size, sizeof(n));  // (stream-synchronising: every queued insert is in)
  known_size_ = (int64_t)n;
  known_adds_ = queued_adds_;
  return (int64_t)n;
}

int64_t Engine::scratch_capacity() {
  if (!scratch_.ctl) return (int64_t)scratch_.cap;
  unsigned long long c = 0;
  be_->copy_d2h(&c, scratch_.ctl, sizeof(c));
  return (int64_t)c;  // ctl[0]: the capacity the next batch is deduplicated with
}

bool Engine::overflowed() {
  u32 o[2] = {0, 0};
  be_->copy_d2h(o, overflow_, sizeof(o));
  return o[0] || o[1];
}

BatchView Engine::synth_batch(const SynthArgs& a0, int64_t slice_rows) {
  SynthArgs a = a0;
  if (a.rows > cfg_.max_rows || a.rows * a.fields > cfg_.max_nnz)
    throw std::invalid_argument("synth batch exceeds engine capacity");
  if (a.col_stride > 0 && (a.col_stride < a.rows || (!a0.keys && a.col_stride != a.rows)))
    throw std::invalid_argument("synth: col_stride must be >= rows (== rows for staging)");
  // caller-provided outputs (e.g. torch tensors) or the engine's staging buffers
  a.keys = a0.keys ? a0.keys : st_keys_;
  a.labels = a0.labels ? a0.labels : st_labels_;
  if (!a0.fgid) a.fgid = cfg_.model.kind == kMVM ? st_fgid_ : nullptr;
  be_->synth_batch(a);
  BatchView b;
  b.keys = a.keys;
  b.labels = a.labels;
  b.fgid = a.fgid;
  b.rows = a.rows;
  b.nnz = a.rows * a.fields;
  b.nnz_per_row = a.fields;
  b.slice_rows = slice_rows;
  b.col_stride = a.col_stride;
  return b;
}

BatchView Engine::stage_host_batch(const BatchView& h) {
  if (h.rows > cfg_.max_rows || h.nnz > cfg_.max_nnz)
    throw std::invalid_argument("host batch exceeds engine capacity");
  BatchView b = h;
  be_->copy_h2d(st_keys_, h.keys, sizeof(u64) * h.nnz);
  b.keys = st_keys_;
  if (h.row_ptr) {
    be_->copy_h2d(st_rowptr_, h.row_ptr, sizeof(int32_t) * (h.rows + 1));
    b.row_ptr = st_rowptr_;
  }
  if (h.fgid) {
    be_->copy_h2d(st_fgid_, h.fgid, sizeof(int32_t) * h.nnz);
    b.fgid = st_fgid_;
  }
  be_->copy_h2d(st_labels_, h.labels, sizeof(float) * h.rows);
  b.labels = st_labels_;
  return b;
}

BatchView Engine::stage_host_batch_async(const BatchView& h) {
  if (h.rows > cfg_.max_rows || h.nnz > cfg_.max_nnz)
    throw std::invalid_argument("host batch exceeds engine capacity");
  const int s = astage_next_;
  astage_next_ ^= 1;
  StageSet& d = aset_[s];
  if (!d.keys) {
    d.keys = balloc<u64>(*be_, cfg_.max_nnz);
    d.rowptr = balloc<int32_t>(*be_, cfg_.max_rows + 1);
    d.fgid = balloc<int32_t>(*be_, cfg_.max_nnz);
    d.labels = balloc<float>(*be_, cfg_.max_rows);
  }
  auto up = [](size_t b) { return (b + 255) & ~(size_t)255; };
  const size_t bk = sizeof(u64) * h.nnz, br = h.row_ptr ? sizeof(int32_t) * (h.rows + 1) : 0,
               bf = h.fgid ? sizeof(int32_t) * h.nnz : 0, bl = sizeof(float) * h.rows;
  const size_t ok = 0, orp = up(bk), of = orp + up(br), ol = of + up(bf);
  be_->stage_begin(s);
  char* pin = static_cast<char*>(be_->stage_pinned(s, ol + up(bl)));
  std::memcpy(pin + ok, h.keys, bk);
  if (br) std::memcpy(pin + orp, h.row_ptr, br);
  if (bf) std::memcpy(pin + of, h.fgid, bf);
  std::memcpy(pin + ol, h.labels, bl);
  be_->stage_copy(s, d.keys, ok, bk);
  if (br) be_->stage_copy(s, d.rowptr, orp, br);
  if (bf) be_->stage_copy(s, d.fgid, of, bf);
  be_->stage_copy(s, d.labels, ol, bl);
  be_->stage_commit(s);
  astage_last_ = s;
  BatchView b = h;
  b.keys = d.keys;
  b.row_ptr = h.row_ptr ? d.rowptr : nullptr;
  b.fgid = h.fgid ? d.fgid : nullptr;
  b.labels = d.labels;
  return b;
}

void Engine::stage_release() {
  if (astage_last_ >= 0) be_->stage_release(astage_last_);
}

// ---------------------------------------------------------------------------
// checkpoint
// ---------------------------------------------------------------------------
// Checkpoint transfers stream through two pinned staging buffers: a table of
// 1e9 LR keys is 16 GB of keys + state, and a pageable copy of it (plus the
// zero-fill of the destination) ran at ~2.6 GB/s (profiles/r3s3_table_ops.txt).
constexpr size_t kStageChunk = 64u << 20;

// host memcpy of one staged chunk, split over a few threads (a single thread
// copies well below the DMA rate)
static void par_copy(void* dst, const void* src, size_t bytes) {
  constexpr size_t kPiece = 8u << 20;
  const size_t parts = bytes / kPiece;
  if (parts < 2) {
    std::memcpy(dst, src, bytes);
    return;
  }
  const size_t nt = parts < 8 ? parts : 8, per = (bytes + nt - 1) / nt;
  std::vector<std::thread> th;
  for (size_t t = 1; t < nt; ++t) {
    const size_t o = t * per;
    if (o >= bytes) break;
    const size_t n = bytes - o < per ? bytes - o : per;
    th.emplace_back([=] { std::memcpy((char*)dst + o, (const char*)src + o, n); });
  }
  std::memcpy(dst, src, per < bytes ? per : bytes);
  for (std::thread& x : th) x.join();
}

template <typename Sink>
void Engine::d2h_stream(const void* src, size_t bytes, Sink sink) {
  if (bytes == 0) return;
  for (void*& p : stage_io_)
    if (!p) p = be_->staging_alloc(kStageChunk);
  const char* s = static_cast<const char*>(src);
  int cur = 0;
  be_->copy_d2h_async(stage_io_[0], s, bytes < kStageChunk ? bytes : kStageChunk);
  be_->synchronize();
  for (size_t off = 0; off < bytes;) {
    const size_t len = bytes - off < kStageChunk ? bytes - off : kStageChunk;
    const size_t nxt = off + len;
    if (nxt < bytes)  // the next chunk's DMA runs while the host consumes this one
      be_->copy_d2h_async(stage_io_[cur ^ 1], s + nxt,
                          bytes - nxt < kStageChunk ? bytes - nxt : kStageChunk);
    sink(stage_io_[cur], off, len);
    be_->synchronize();
    off = nxt;
    cur ^= 1;
  }
}

template <typename Fill>
void Engine::h2d_stream(void* dst, size_t bytes, Fill fill) {
  if (bytes == 0) return;
  for (void*& p : stage_io_)
    if (!p) p = be_->staging_alloc(kStageChunk);
  char* d = static_cast<char*>(dst);
  int cur = 0;
  for (size_t off = 0; off < bytes;) {
    const size_t len = bytes - off < kStageChunk ? bytes - off : kStageChunk;
    fill(stage_io_[cur], off, len);  // overlaps the previous chunk's DMA
    be_->synchronize();              // (that DMA read the other buffer)
    be_->copy_h2d_async(d + off, stage_io_[cur], len);
    off += len;
    cur ^= 1;
  }
  be_->synchronize();
}

void Engine::export_into(u64* keys, u32* words, int64_t n) {
  const int W = state_words();
  if (n != table_size()) throw std::invalid_argument("export_into: n must equal table_size()");
  if (n == 0) return;
  u64* dk = balloc<u64>(*be_, n);
  u32* dw = balloc<u32>(*be_, n * W);
  const int64_t got = be_->table_export(table_, dk, dw, n);
  if (got == n) {
    d2h_stream(dk, sizeof(u64) * n, [&](const void* c, size_t o, size_t b) {
      par_copy((char*)keys + o, c, b);
    });
    d2h_stream(dw, sizeof(u32) * n * W, [&](const void* c, size_t o, size_t b) {
      par_copy((char*)words + o, c, b);
    });
  }
  be_->free(dk);
  be_->free(dw);
  if (got != n) throw std::runtime_error("export_table: live slot count mismatch");
}

void Engine::export_table(std::vector<u64>& keys, std::vector<u32>& words) {
  const int64_t n = table_size();
  keys.resize((size_t)n);
  words.resize((size_t)n * state_words());
  export_into(keys.data(), words.data(), n);
}

// device arrays of n (key, state) pairs -> the table
void Engine::table_from_device(const u64* dk, const u32* dw, int64_t n) {
  be_->table_import(table_, dk, dw, n);
  be_->synchronize();
  (void)table_size();  // (re-bases the capacity monitor)
}

void Engine::import_from(const u64* keys, const u32* words, int64_t n) {
  stale_stashes();  // the table changes: server stashes are stale
  const int W = state_words();
  if (n <= 0) return;
  guard_inserts(n);
  u64* dk = balloc<u64>(*be_, n);
  u32* dw = balloc<u32>(*be_, n * W);
  h2d_stream(dk, sizeof(u64) * n, [&](void* c, size_t o, size_t b) {
    par_copy(c, (const char*)keys + o, b);
  });
  h2d_stream(dw, sizeof(u32) * n * W, [&](void* c, size_t o, size_t b) {
    par_copy(c, (const char*)words + o, b);
  });
  table_from_device(dk, dw, n);
  be_->free(dk);
  be_->free(dw);
}

void Engine::import_table(const std::vector<u64>& keys, const std::vector<u32>& words) {
  const int64_t n = (int64_t)keys.size();
  if ((int64_t)words.size() != n * state_words())
    throw std::invalid_argument("import_table: size mismatch");
  import_from(keys.data(), words.data(), n);
}

// Shard file: the device export streams chunk by chunk from the staging
// buffers to the file (no whole-table host copy).
void Engine::save(const std::string& path) {
  const int W = state_words();
  const int64_t n = table_size();
  std::FILE* f = std::fopen(path.c_str(), "wb");
  if (!f) throw std::runtime_error("cannot open " + path);
  bool ok = true;
  int32_t hdr[8] = {1, cfg_.model.kind, cfg_.model.v_dim, table_.L.P,
                    table_.L.p_w, table_.L.opt, table_.L.stride, 0};
  const uint64_t un = (uint64_t)n;
  ok = ok && std::fwrite(kMagic, 1, 8, f) == 8;
  ok = ok && std::fwrite(hdr, sizeof(hdr), 1, f) == 1;
  ok = ok && std::fwrite(&un, sizeof(un), 1, f) == 1;
  if (n > 0 && ok) {
    u64* dk = balloc<u64>(*be_, n);
    u32* dw = balloc<u32>(*be_, n * W);
    const int64_t got = be_->table_export(table_, dk, dw, n);
    if (got == n) {
      auto put = [&](const void* c, size_t, size_t b) {
        ok = ok && std::fwrite(c, 1, b, f) == b;
      };
      d2h_stream(dk, sizeof(u64) * n, put);
      d2h_stream(dw, sizeof(u32) * n * W, put);
    }
    be_->free(dk);
    be_->free(dw);
    if (got != n) {
      std::fclose(f);
      throw std::runtime_error("export_table: live slot count mismatch");
    }
  }
  ok = (std::fclose(f) == 0) && ok;
  if (!ok) throw std::runtime_error("write failed: " + path);
}

void Engine::load(const std::string& path) {
  std::FILE* f = std::fopen(path.c_str(), "rb");
  if (!f) throw std::runtime_error("cannot open " + path);
  char magic[8];
  int32_t hdr[8];
  uint64_t n = 0;
  bool ok = std::fread(magic, 1, 8, f) == 8 && std::fread(hdr, sizeof(hdr), 1, f) == 1 &&
            std::fread(&n, sizeof(n), 1, f) == 1;
  if (!ok || std::memcmp(magic, kMagic, 8) != 0) {
    std::fclose(f);
    throw std::runtime_error("bad checkpoint " + path);
  }
  if (hdr[1] != cfg_.model.kind || hdr[3] != table_.L.P || hdr[5] != table_.L.opt ||
      hdr[6] != table_.L.stride) {
    std::fclose(f);
    throw std::runtime_error("checkpoint layout does not match this model/optimizer");
  }
  const int W = state_words();
  stale_stashes();
  if (n > 0) {
    guard_inserts((int64_t)n);
    u64* dk = balloc<u64>(*be_, n);
    u32* dw = balloc<u32>(*be_, n * W);
    auto get = [&](void* c, size_t, size_t b) { ok = ok && std::fread(c, 1, b, f) == b; };
    h2d_stream(dk, sizeof(u64) * n, get);
    h2d_stream(dw, sizeof(u32) * n * W, get);
    if (ok) table_from_device(dk, dw, (int64_t)n);
    be_->free(dk);
    be_->free(dw);
  }
  std::fclose(f);
  if (!ok) throw std::runtime_error("truncated checkpoint " + path);
}

}  // namespace xflow
