// xflow-amd: model / table / batch descriptors shared by both backends.
#pragma once

#include <stddef.h>
#include <stdint.h>

#include "xflow/common.h"

namespace xflow {

// Model families of the reference (src/model/{lr,fm,mvm}).
enum ModelKind : int { kLR = 0, kFM = 1, kMVM = 2 };
enum OptKind : int { kFTRL = 0, kSGD = 1 };

// FM interaction math.  kFmReference reproduces fm_worker.cc:159-202 /
// :126-157 (y = wx + (Σ_k Σ_f v)^2 - Σ_k Σ_f v^2, w-grad accumulated D times);
// kFmStandard is Rendle's ½Σ_k[(Σ_f v_fk)^2 - Σ_f v_fk^2].
enum FmMath : int { kFmReference = 0, kFmStandard = 1 };

// MVM field-product range.  kMvmCompat multiplies fields [0, max_fgid) like
// mvm_worker.cc:198-203 (the max field's sum is written out of bounds there
// and never multiplied); kMvmFixed multiplies [0, max_fgid].
enum MvmMath : int { kMvmCompat = 0, kMvmFixed = 1 };

// Parameters per hashed key.  LR: [w]; FM: [w, v_0..v_{D-1}]; MVM: [v_0..].
// Params with index >= p_w are latent ("v") params: lazily random-initialised
// (FTRL, ftrl.h:114-120) or constant-initialised (SGD, sgd.h:69) until their
// first push, tracked by one per-slot "pushed" flag.
struct ModelSpec {
  int kind = kLR;
  int v_dim = 10;   // fm_worker.h:92 / mvm_worker.h:92
  int fm_math = kFmReference;
  int mvm_math = kMvmCompat;
  int max_fields = 64;  // MVM per-row field buckets (device LDS budget)
  int fm_mfma = 0;      // standard-math FM forward on the matrix cores (HIP, v_dim <= 8)
  // Latent width the device kernels run at (HIP: the kernels are compiled
  // for v_dim 1, 2, 4, 8, 10, 16 and 32; any other v_dim runs at the next one
  // of those, kernel_dim()).  The padded dims are inert: the table holds and
  // pushes only the P() real params, the pull writes 0 into the padding of
  // every value row, so a padded dim's latent sums, products and gradients
  // are exactly 0 and never reach the table.  0: v_dim.
  int pad_dim = 0;

  XF_HD int P() const { return kind == kLR ? 1 : (kind == kFM ? 1 + v_dim : v_dim); }
  XF_HD int p_w() const { return kind == kMVM ? 0 : 1; }
  XF_HD int kernel_dim() const { return pad_dim > v_dim ? pad_dim : v_dim; }
  // Stride (floats) of one key's row in the pulled-weights / gradient buffers:
  // 1 for LR, otherwise (the kernel width's params) padded to 16 bytes so
  // kernels use dwordx4 accesses.
  XF_HD int pstride() const {
    if (kind == kLR) return 1;
    const int p = kind == kFM ? 1 + kernel_dim() : kernel_dim();
    return p == 1 ? 1 : ((p + 3) & ~3);
  }
};
// latent widths the HIP model kernels are instantiated for: the smallest >= d
XF_HD int device_latent_width(int d) {
  return d <= 2 ? d : (d <= 4 ? 4 : (d <= 8 ? 8 : (d <= 10 ? 10 : (d <= 16 ? 16 : 32))));
}

struct OptSpec {
  int kind = kFTRL;
  FtrlParams ftrl;
  SgdParams sgd;
  float v_init_scale = 1e-2f;  // ftrl.h:117
  uint64_t seed = 0x5eed;
};

// Slot layout of the HBM-resident open-addressing table, in 32-bit words:
//   [0,1]  u64 key (kEmptyKey when free)
//   [2, 2+sp*P)  optimizer state: FTRL (n,z) pairs, SGD w
//   [2+sp*P]     pushed flag (only when the model has latent params)
// padded to a multiple of 4 words (16 B).  LR-FTRL is exactly 16 B/slot.
struct TableLayout {
  int P = 1;
  int p_w = 1;
  int opt = kFTRL;
  int sp = 2;          // state words per param
  int has_flag = 0;
  int flag_word = 0;
  int stride = 4;      // words per slot

  static TableLayout make(const ModelSpec& m, const OptSpec& o) {
    TableLayout t;
    t.P = m.P();
    t.p_w = m.p_w();
    t.opt = o.kind;
    t.sp = (o.kind == kFTRL) ? 2 : 1;
    t.has_flag = (t.P > t.p_w) ? 1 : 0;
    t.flag_word = 2 + t.sp * t.P;
    int words = 2 + t.sp * t.P + t.has_flag;
    t.stride = (words + 3) & ~3;
    return t;
  }
};

// Weight of param p from already-loaded slot words: the pushed flag and the
// param's state (FTRL: s0 = n, s1 = z; SGD: s0 = w).
XF_HD float state_weight(u64 key, bool pushed, float s0, float s1, int p, const TableLayout& L,
                         const OptSpec& o) {
  if (p >= L.p_w && L.has_flag && !pushed) {
    return L.opt == kFTRL ? normal_init(key, (u32)(p - L.p_w), o.seed) * o.v_init_scale
                          : o.sgd.v_init;
  }
  if (L.opt == kFTRL) return ftrl_weight(s1, s0, o.ftrl);
  return s0;
}

// Current weight of param p stored in `slot` (reference pull semantics).
XF_HD float slot_weight(const u32* slot, u64 key, int p, const TableLayout& L,
                        const OptSpec& o) {
  const float* st = reinterpret_cast<const float*>(slot + 2);
  const bool pushed = !L.has_flag || slot[L.flag_word] != 0u;
  return L.opt == kFTRL ? state_weight(key, pushed, st[2 * p], st[2 * p + 1], p, L, o)
                        : state_weight(key, pushed, st[p], 0.0f, p, L, o);
}

// Weight of a key that is not in the table (lookup-only pulls at eval time).
XF_HD float absent_weight(u64 key, int p, const TableLayout& L, const OptSpec& o) {
  if (p >= L.p_w) {
    return L.opt == kFTRL ? normal_init(key, (u32)(p - L.p_w), o.seed) * o.v_init_scale
                          : o.sgd.v_init;
  }
  return 0.0f;
}

// Apply one push of gradient g to param p of `slot` (slot lock-free: callers
// guarantee a single writer per slot per launch).
XF_HD void slot_push(u32* slot, u64 key, int p, float g, const TableLayout& L,
                     const OptSpec& o) {
  float w = slot_weight(slot, key, p, L, o);
  float* st = reinterpret_cast<float*>(slot + 2);
  if (L.opt == kFTRL) {
    ftrl_push(st[2 * p], st[2 * p + 1], w, g, o.ftrl);
  } else {
    st[p] = w - o.sgd.lr * g;
  }
}

// A batch (device or host pointers, depending on the backend).  Three layouts
// of the per-occurrence arrays (keys, fgid, and the engine's dedup positions):
//   CSR          row_ptr != null: row r = [row_ptr[r], row_ptr[r+1])
//   row-major    fixed nnz_per_row, col_stride == 0: (r, j) at r*nnz_per_row + j
//   field-major  fixed nnz_per_row, col_stride > 0: (r, j) at j*col_stride + r
// Field-major is the layout of fixed-width CTR batches on the device: a
// workgroup's rows of one field are contiguous, so per-field passes (dedup
// windows, gradient aggregation) read and write coalesced.
struct BatchView {
  const u64* keys = nullptr;      // [nnz]
  const int32_t* row_ptr = nullptr;  // [rows+1]; null => fixed nnz_per_row
  const int32_t* fgid = nullptr;  // [nnz], MVM only
  const float* labels = nullptr;  // [rows], 0/1
  int64_t rows = 0;
  int64_t nnz = 0;
  int nnz_per_row = 0;            // used when row_ptr == null
  int64_t slice_rows = 0;         // rows per slice (gradient normaliser); 0 => rows
  int64_t col_stride = 0;         // field-major stride (>= rows), 0 => row-major
};

// Occurrences of one row: j-th at base + j*step.
struct RowSpan {
  int64_t base = 0, step = 1;
  int len = 0;
  XF_HD int64_t at(int j) const { return base + (int64_t)j * step; }
};

XF_HD RowSpan row_span(const BatchView& b, int64_t r) {
  RowSpan s;
  if (b.row_ptr) {
    s.base = b.row_ptr[r];
    s.len = (int)(b.row_ptr[r + 1] - b.row_ptr[r]);
  } else if (b.col_stride > 0) {
    s.base = r;
    s.step = b.col_stride;
    s.len = b.nnz_per_row;
  } else {
    s.base = r * b.nnz_per_row;
    s.len = b.nnz_per_row;
  }
  return s;
}

// Loss statistics accumulated by forward passes (device or host memory).
struct LossStats {
  double ln_loss;      // Σ -[y ln p + (1-y) ln(1-p)], p clipped to [1e-7, 1-1e-7]
  double log2_lik;     // Σ  [y log2 p + (1-y) log2(1-p)] (reference print, base.h:97-101)
  double rows;
  double positives;
};

}  // namespace xflow
