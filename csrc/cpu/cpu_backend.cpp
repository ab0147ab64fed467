// xflow-amd: CpuBackend — host implementation of xflow::Backend.
//
// Executes the same per-element recipes (common.h / types.h / synth.h) as the
// gfx950 kernels, single threaded and in a fixed order, so it is
// deterministic.  Used for the reference's CPU "plumbing" configuration, for
// multi-rank gloo tests, and as the numerics oracle of the HIP kernels.
#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <stdexcept>
#include <vector>
#include <sys/mman.h>

#include "xflow/backend.h"
#include "xflow/reader.h"
#include "xflow/synth.h"

namespace xflow {

namespace {

constexpr u32 kNoSlot = 0xFFFFFFFFu;

inline int64_t count_of(const int64_t* n_dev, int64_t n_host, int64_t n_max) {
  int64_t n = n_dev ? *n_dev : n_host;
  return n < n_max ? n : n_max;
}


inline int slice_of(const BatchView& b, int64_t r, int S) {
  if (b.slice_rows <= 0) return 0;
  int64_t s = r / b.slice_rows;
  return (int)(s < S ? s : S - 1);
}

inline float norm_grad(float raw, const int32_t* slice_rows, int s) {
  return slice_rows ? (float)((double)raw / (double)slice_rows[s]) : raw;
}

void add_stats(LossStats* st, float p, float y) {
  if (!st) return;
  float pc = std::fmin(std::fmax(p, 1e-7f), 1.0f - 1e-7f);
  st->ln_loss += (y > 0.5f) ? -(double)std::log(pc) : -(double)std::log(1.0f - pc);
  st->log2_lik += (y > 0.5f) ? (double)std::log2(p) : (double)std::log2(1.0f - p);
  st->rows += 1.0;
  st->positives += (y > 0.5f) ? 1.0 : 0.0;
}

u32 probe(const TableView& t, u64 key, bool insert, bool& claimed) {
  u64 s = table_home(t, fmix64(key));
  for (u64 n = 0; n < t.probe_limit; ++n) {
    u64* kp = reinterpret_cast<u64*>(t.words + s * (u64)t.L.stride);
    if (*kp == key) return (u32)s;
    if (*kp == kEmptyKey) {
      if (!insert) return kNoSlot;
      *kp = key;
      claimed = true;
      return (u32)s;
    }
    s = table_next(t, s);
  }
  if (insert) *t.overflow = 1u;
  return kNoSlot;
}

class CpuBackend final : public Backend {
 public:
  bool is_gpu() const override { return false; }
  std::string name() const override { return "cpu"; }

  void upload_small(void* dst, const void* src, size_t bytes) override {
    if (bytes) std::memcpy(dst, src, bytes);
  }
  void download_small(void* dst, const void* src, size_t bytes) override {
    if (bytes) std::memcpy(dst, src, bytes);
  }
  void* stage_pinned(int s, size_t bytes) override {
    if (stage_buf_[s].size() < bytes) stage_buf_[s].resize(bytes);
    return stage_buf_[s].data();
  }
  void stage_copy(int s, void* dst, size_t off, size_t bytes) override {
    if (bytes) std::memcpy(dst, stage_buf_[s].data() + off, bytes);
  }
  void* alloc(size_t bytes) override {
    void* p = std::aligned_alloc(64, ((bytes ? bytes : 16) + 63) & ~size_t(63));
    if (!p) throw std::bad_alloc();
    return p;
  }
  void free(void* p) override { std::free(p); }
  void memset(void* p, int v, size_t bytes) override { std::memset(p, v, bytes); }
  void fill_u64(u64* p, u64 v, size_t n) override {
    for (size_t i = 0; i < n; ++i) p[i] = v;
  }
  void copy_h2d(void* d, const void* s, size_t b) override { std::memcpy(d, s, b); }
  void copy_d2h(void* d, const void* s, size_t b) override { std::memcpy(d, s, b); }
  void copy_d2d(void* d, const void* s, size_t b) override { std::memmove(d, s, b); }
  void synchronize() override {}
  void set_stream(void*) override {}
  void* stream() const override { return nullptr; }
  void* host_alloc(size_t bytes) override { return alloc(bytes); }
  void snapshot(HostSnap* dst, const u32* mon, unsigned long long seq) override {
    dst->word = pack_snapshot(*reinterpret_cast<const unsigned long long*>(mon), mon[2], mon[3], seq);
  }
  void host_free(void* p) override { std::free(p); }

  void table_clear(const TableView& t) override {
    for (u64 s = 0; s < t.cap; ++s) {
      u32* sp = t.words + s * (u64)t.L.stride;
      sp[0] = 0xFFFFFFFFu;
      sp[1] = 0xFFFFFFFFu;
      for (int w = 2; w < t.L.stride; ++w) sp[w] = 0u;
    }
  }
  // Same persistent, epoch-stamped scratch protocol as the HIP kernels
  // (k_scratch_maybe_clear / k_dedup_insert / k_dedup_compact).
  void dedup(const u64* keys, int64_t nnz, ScratchView s, DedupOut o) override {
    const u64 mask = s.cap - 1;
    if (*s.claims > s.rebuild_at) {
      for (u64 i = 0; i < s.cap; ++i) s.keys[i] = kEmptyKey;
      *s.claims = 0;
    }
    for (int64_t i = 0; i < nnz; ++i) {
      u64 k = sanitize_key(keys[i]);
      u64 p = fmix64(k) & mask;
      u64 n = 0;
      for (; n < s.cap; ++n) {
        if (s.keys[p] == k) break;
        if (s.keys[p] == kEmptyKey) {
          s.keys[p] = k;
          ++*s.claims;
          break;
        }
        p = (p + 1) & mask;
      }
      if (n == s.cap) { *o.overflow = 1u; p = 0; }
      o.pos[i] = (u32)p;
      s.stamps[p] = (unsigned char)s.epoch;
    }
    int64_t u = 0;
    for (u64 p = 0; p < s.cap; ++p) {
      if (s.stamps[p] != (unsigned char)s.epoch) continue;
      o.uniq_keys[u] = s.keys[p];
      o.uniq_pos[u] = (u32)p;
      ++u;
    }
    *o.n_uniq = u;
    if (o.n_uniq_copy) *o.n_uniq_copy = u;
    if (o.cap_out) *o.cap_out = s.cap;
  }

  void scratch_reset(ScratchView s, const u32* pos, const int64_t* n_dev, int64_t n_max) override {
    int64_t n = count_of(n_dev, n_max, n_max);
    for (int64_t i = 0; i < n; ++i) s.keys[pos[i]] = kEmptyKey;
  }

  void table_pull(const PullArgs& a) override {
    int64_t n = count_of(a.n_dev, a.n_host, a.n_max);
    const TableView& t = a.table;
    const TableLayout& L = t.L;
    for (int64_t i = 0; i < n; ++i) {
      u64 key = sanitize_key(a.keys[i]);
      bool claimed = false;
      u32 slot = probe(t, key, a.insert, claimed);
      if (claimed) ++*t.size;
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
  }

  void table_apply(const ApplyArgs& a) override {
    int64_t n = count_of(a.n_dev, a.n_host, a.n_max);
    const TableView& t = a.table;
    const TableLayout& L = t.L;
    const int S = a.S, ps = a.pstride, P = a.P;
    const u32 all = (S >= 32) ? 0xFFFFFFFFu : ((1u << S) - 1u);
    for (int64_t i = 0; i < n; ++i) {
      u32 slot = a.slots[i];
      u32 row = a.grad_map ? a.grad_map[i] : (u32)i;
      float* g = a.grads + (size_t)row * S * ps;
      u32 m = a.masks ? a.masks[row] : all;
      if (a.masks && a.masks_clear) const_cast<u32*>(a.masks)[row] = 0u;
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

  void forward_backward(const FwdArgs& a) override {
    const BatchView& b = a.batch;
    const ModelSpec& m = a.model;
    const int ps = m.pstride();
    const int D = m.v_dim;
    std::vector<float> vs(D > 0 ? D : 1), M(D > 0 ? D : 1);
    std::vector<float> S;
    for (int64_t r = 0; r < b.rows; ++r) {
      const RowSpan rs = row_span(b, r);
      float y = 0.0f;
      float vsum = 0.0f;
      int maxf = 0, G = 0;
      if (m.kind == kLR) {
        for (int64_t j = 0, o = rs.base; j < rs.len; ++j, o += rs.step) y += a.wpull[a.pos[o]];
      } else if (m.kind == kFM) {
        float wx = 0.0f, vp = 0.0f;
        for (int k = 0; k < D; ++k) vs[k] = 0.0f;
        for (int64_t j = 0, o = rs.base; j < rs.len; ++j, o += rs.step) {
          const float* w = a.wpull + (size_t)a.pos[o] * ps;
          wx += w[0];
          for (int k = 0; k < D; ++k) {
            float v = w[1 + k];
            vs[k] += v;
            vp += v * v;
          }
        }
        if (m.fm_math == kFmStandard) {
          float sq = 0.0f;
          for (int k = 0; k < D; ++k) sq += vs[k] * vs[k];
          y = wx + 0.5f * (sq - vp);
        } else {
          for (int k = 0; k < D; ++k) vsum += vs[k];
          y = wx + (vsum * vsum - vp);
        }
      } else {  // MVM
        if (!b.fgid) throw std::runtime_error("MVM needs field ids (fgid)");
        for (int64_t j = 0, o = rs.base; j < rs.len; ++j, o += rs.step) maxf = std::max(maxf, (int)b.fgid[o]);
        G = (m.mvm_math == kMvmCompat) ? maxf : maxf + 1;
        S.assign((size_t)(maxf + 1) * D, 0.0f);
        for (int k = 0; k < D; ++k) {
          for (int64_t j = 0, o = rs.base; j < rs.len; ++j, o += rs.step)
            S[(size_t)b.fgid[o] * D + k] += a.wpull[(size_t)a.pos[o] * ps + k];
          float prod = 1.0f;
          for (int g = 0; g < G; ++g) prod *= S[(size_t)g * D + k];
          M[k] = prod;
          y += prod;
        }
      }
      float p = sigmoid_ref(y);
      float lab = b.labels[r];
      float loss = p - lab;
      if (a.pctr) a.pctr[r] = p;
      add_stats(a.stats, p, lab);
      if (a.fx_bad && !(p >= 0.0f && p <= 1.0f)) *a.fx_bad |= 2u;
      if (!a.grad) continue;
      const int s = slice_of(b, r, a.S);
      for (int64_t j = 0, o = rs.base; j < rs.len; ++j, o += rs.step) {
        float* g = a.grad + ((size_t)a.pos[o] * a.S + s) * ps;
        if (m.kind == kLR) {
          g[0] += loss;
        } else if (m.kind == kFM) {
          const float* w = a.wpull + (size_t)a.pos[o] * ps;
          bool standard = m.fm_math == kFmStandard;
          g[0] += standard ? loss : loss * (float)D;
          for (int k = 0; k < D; ++k)
            g[1 + k] += loss * ((standard ? vs[k] : vsum) - w[1 + k]);
        } else {
          for (int k = 0; k < D; ++k) {
            float sg = S[(size_t)b.fgid[o] * D + k];
            float gr = (sg == 0.0f) ? 0.0f
                                    : (float)((double)loss * ((double)M[k] / (1.0 + (double)sg)));
            g[k] += gr;
          }
        }
      }
    }
  }

  void parse_text(const TextParseArgs& a) override {
    CsrBlock blk;
    parse_libffm(a.text, (size_t)a.n, blk);
    long long* c = a.counts;
    c[0] = blk.rows();
    c[1] = (long long)blk.keys.size();
    c[2] = 0x7FFFFFFFll;
    c[3] = 0;
    c[4] = 0;
    c[5] = 0;
    const int64_t used = c[0] - c[0] % a.row_mod;
    c[6] = blk.row_ptr[used];
    for (int64_t i = 0; i < a.n; ++i) c[4] += a.text[i] == '\n';
    if (a.n > 0 && a.text[a.n - 1] != '\n') ++c[4];
    a.row_ptr[0] = 0;
    if (c[0] > a.max_rows || c[1] > a.max_nnz) return;  // (the caller checks the counts)
    for (int64_t r = 0; r < blk.rows(); ++r) {
      a.labels[r] = blk.labels[r];
      a.row_ptr[r + 1] = blk.row_ptr[r + 1];
      const long long len = blk.row_ptr[r + 1] - blk.row_ptr[r];
      c[2] = std::min<long long>(c[2], len);
      c[3] = std::max<long long>(c[3], len);
    }
    std::copy(blk.keys.begin(), blk.keys.end(), a.keys);
    std::copy(blk.fgid.begin(), blk.fgid.end(), a.fgid);
  }

  void slice_masks(const BatchView& b, const u32* pos, u32* tmask) override {
    int S = b.slice_rows > 0 ? (int)((b.rows + b.slice_rows - 1) / b.slice_rows) : 1;
    for (int64_t r = 0; r < b.rows; ++r) {
      const RowSpan rs = row_span(b, r);
      u32 bit = 1u << slice_of(b, r, S);
      for (int64_t j = 0, o = rs.base; j < rs.len; ++j, o += rs.step) tmask[pos[o]] |= bit;
    }
  }

  void bucket(const BucketArgs& a) override {
    int64_t n = count_of(a.n_dev, a.n_max, a.n_max);
    std::vector<int64_t> cnt(a.world, 0), off(a.world, 0);
    for (int64_t i = 0; i < n; ++i) ++cnt[owner_of(a.uniq_keys[i], (u32)a.world)];
    for (int o = 1; o < a.world; ++o) off[o] = off[o - 1] + cnt[o - 1];
    for (int o = 0; o < a.world; ++o) a.counts[o] = a.seq >= 0 ? encode_count(cnt[o], a.seq) : cnt[o];
    for (int64_t i = 0; i < n; ++i) {
      int o = (int)owner_of(a.uniq_keys[i], (u32)a.world);
      int64_t d = off[o]++;
      a.send_keys[d] = a.uniq_keys[i];
      a.send_pos[d] = a.uniq_pos[i];
    }
  }

  void gather_grads(const GatherGradArgs& a) override {
    int64_t n = count_of(a.n_dev, a.n_max, a.n_max);
    const int W = a.S * a.pstride;
    for (int64_t i = 0; i < n; ++i) {
      u32 row = a.map[i];
      float* src = a.grad_rw + (size_t)row * W;
      float* dst = a.out + (size_t)i * W;
      for (int s = 0; s < a.S; ++s)
        for (int p = 0; p < a.pstride; ++p) {
          dst[s * a.pstride + p] = norm_grad(src[s * a.pstride + p], a.slice_rows, s);
          src[s * a.pstride + p] = 0.0f;
        }
      if (a.tmask_rw) {
        a.out_mask[i] = a.tmask_rw[row];
        a.tmask_rw[row] = 0u;
      }
    }
  }

  void scatter_rows(const float* src, float* dst, const u32* map, const int64_t* n_dev,
                    int64_t n_max, int width, float* zero_out, int zero_width) override {
    int64_t n = count_of(n_dev, n_max, n_max);
    if (zero_out) std::fill(zero_out, zero_out + n * zero_width, 0.0f);
    for (int64_t i = 0; i < n; ++i) {
      int64_t r = map ? map[i] : i;
      std::memcpy(dst + r * width, src + i * width, sizeof(float) * width);
    }
  }
  void gather_rows(const float* src, float* dst, const u32* map, const int64_t* n_dev,
                   int64_t n_max, int width, bool zero_src) override {
    int64_t n = count_of(n_dev, n_max, n_max);
    for (int64_t i = 0; i < n; ++i) {
      float* s = const_cast<float*>(src) + (int64_t)map[i] * width;
      std::memcpy(dst + i * width, s, sizeof(float) * width);
      if (zero_src) std::memset(s, 0, sizeof(float) * width);
    }
  }
  void gather_u32(const u32* src, u32* dst, const u32* map, const int64_t* n_dev, int64_t n_max,
                  bool zero_src) override {
    int64_t n = count_of(n_dev, n_max, n_max);
    for (int64_t i = 0; i < n; ++i) {
      dst[i] = src[map[i]];
      if (zero_src) const_cast<u32*>(src)[map[i]] = 0u;
    }
  }
  void scatter_u32(const u32* src, u32* dst, const u32* map, const int64_t* n_dev,
                   int64_t n_max) override {
    int64_t n = count_of(n_dev, n_max, n_max);
    for (int64_t i = 0; i < n; ++i) dst[map[i]] = src[i];
  }

  void synth_batch(const SynthArgs& a) override {
    if (a.fields > kSynthMaxFields) throw std::runtime_error("synth: at most 64 fields");
    std::vector<SynthField> F(a.fields);
    for (int f = 0; f < a.fields; ++f) F[f] = synth_field(a.vocab[f], (double)a.zipf_s[f], f);
    for (int64_t r = 0; r < a.rows; ++r) {
      const u64 rs = synth_row_seed(a.seed, a.step, r);
      float logit = a.planted_bias;
      for (int f = 0; f < a.fields; ++f) {
        float w;
        const u64 key = synth_sample(rs, f, F[f], a.hash_space, a.planted_scale, w);
        const int64_t o = a.col_stride > 0 ? f * a.col_stride + r : r * a.fields + f;
        a.keys[o] = key;
        if (a.fgid) a.fgid[o] = f;
        logit += w;
      }
      a.labels[r] = synth_label(rs, logit);
    }
  }

  void unpack_block(const UnpackArgs& a) override {
    if (a.F > kMaxPackedFields) throw std::invalid_argument("unpack_block: at most 64 fields");
    for (int f = 0; f < a.F; ++f) {
      const uint8_t* col = a.block + a.col_off[f];
      const int w = a.width[f];
      if (w != 1 && w != 2 && w != 4 && w != 8)
        throw std::invalid_argument("unpack_block: code widths 1/2/4/8");
      for (int64_t r = 0; r < a.rows; ++r) {
        u64 c = 0;
        std::memcpy(&c, col + r * w, (size_t)w);  // (little endian)
        a.keys[(int64_t)f * a.rows + r] = a.dict[f] ? a.dict[f][c] : c;
        if (a.fgid) a.fgid[(int64_t)f * a.rows + r] = a.fgid_col[f];
      }
    }
    for (int64_t r = 0; r < a.rows; ++r) a.labels[r] = (float)a.block[r];
  }
  void field_major(const void* src, void* dst, int64_t rows, int F, int elem_bytes,
                   bool widen) override {
    if (widen) {
      if (elem_bytes != 4) throw std::invalid_argument("field_major: widen needs 4-byte elements");
      const u32* s = static_cast<const u32*>(src);
      u64* d = static_cast<u64*>(dst);
      for (int64_t r = 0; r < rows; ++r)
        for (int f = 0; f < F; ++f) d[(int64_t)f * rows + r] = (u64)s[r * F + f];
      return;
    }
    const char* s = static_cast<const char*>(src);
    char* d = static_cast<char*>(dst);
    for (int64_t r = 0; r < rows; ++r)
      for (int f = 0; f < F; ++f)
        std::memcpy(d + ((int64_t)f * rows + r) * elem_bytes, s + (r * F + f) * elem_bytes,
                    (size_t)elem_bytes);
  }
  int64_t table_export(const TableView& t, u64* keys_out, u32* words_out,
                       int64_t max_rows) override {
    const int W = t.L.stride - 2;
    int64_t n = 0;
    for (u64 s = 0; s < t.cap; ++s) {
      const u32* sp = t.words + s * (u64)t.L.stride;
      u64 key = *reinterpret_cast<const u64*>(sp);
      if (key == kEmptyKey) continue;
      if (n < max_rows) {
        keys_out[n] = key;
        std::memcpy(words_out + n * W, sp + 2, sizeof(u32) * W);
      }
      ++n;
    }
    return n;
  }
  void table_import(const TableView& t, const u64* keys, const u32* words, int64_t n) override {
    const int W = t.L.stride - 2;
    for (int64_t i = 0; i < n; ++i) {
      bool claimed = false;
      u32 slot = probe(t, sanitize_key(keys[i]), true, claimed);
      if (claimed) ++*t.size;
      if (slot == kNoSlot) continue;
      std::memcpy(t.words + (u64)slot * t.L.stride + 2, words + i * W, sizeof(u32) * W);
    }
  }
  void table_prefill(const TableView& t, int64_t n, u64 seed) override {
    for (int64_t i = 0; i < n; ++i) {
      bool claimed = false;
      const u32 slot = probe(t, prefill_key(seed, (u64)i), true, claimed);
      if (claimed) ++*t.size;
      if (slot != kNoSlot && t.L.has_flag) t.words[(u64)slot * t.L.stride + t.L.flag_word] = 1u;
    }
  }
  // The HIP split kernels' algorithm (kernels_table.hip k_table_split_marks /
  // k_table_split), one cluster after the other: cluster starts are marked
  // before any slot changes, then each cluster is walked with backward-shift
  // placement of its staying keys.
  void table_split(const TableView& t, u64 s0, u64 k) override {
    const int W = t.L.stride;
    const int g = t.seg_log2;
    const u64 G = 1ull << g, m = G - 1, n = k << g;
    const u64 move_bit = 1ull << (g + t.level), buddy = (1ull << t.level) << g;
    auto key_at = [&](u64 s) { return *reinterpret_cast<const u64*>(t.words + s * (u64)W); };
    std::vector<u64> starts;
    for (u64 i = 0; i < n; ++i) {
      const u64 base = (s0 << g) + (i & ~m), c = i & m;
      if (key_at(base + c) != kEmptyKey && key_at(base + ((c - 1) & m)) == kEmptyKey)
        starts.push_back(i);
    }
    auto free_slot = [&](u32* sp) {
      sp[0] = sp[1] = 0xFFFFFFFFu;
      for (int w = 2; w < W; ++w) sp[w] = 0u;
    };
    for (u64 i : starts) {
      const u64 base = (s0 << g) + (i & ~m), c = i & m;
      auto at = [&](u64 off) { return base + ((c + off) & m); };
      for (u64 d = 0; d < G; ++d) {
        u32* sp = t.words + at(d) * (u64)W;
        const u64 key = *reinterpret_cast<const u64*>(sp);
        if (key == kEmptyKey) break;
        const u64 h = fmix64(key);
        if (h & move_bit) {
          u64 q = base + buddy + (h & m);
          u64 r = 0;
          for (; r < t.probe_limit && key_at(q) != kEmptyKey; ++r) q = table_next(t, q);
          if (r < t.probe_limit) std::memcpy(t.words + q * (u64)W, sp, sizeof(u32) * W);
          else *t.overflow = 1u;
          free_slot(sp);
        } else {
          u64 off = ((h & m) - c) & m;
          while (off < d && key_at(at(off)) != kEmptyKey) ++off;
          if (off != d) {
            std::memcpy(t.words + at(off) * (u64)W, sp, sizeof(u32) * W);
            free_slot(sp);
          }
        }
      }
    }
  }
  // The table's range: address space reserved with mmap (pages get memory
  // when first touched), so growth never copies; a plain allocation that is
  // re-allocated on growth when the reservation fails.
  void* table_reserve(size_t max_bytes, bool growable) override {
    (void)growable;
    void* p = mmap(nullptr, max_bytes, PROT_READ | PROT_WRITE,
                   MAP_PRIVATE | MAP_ANONYMOUS | MAP_NORESERVE, -1, 0);
    if (p == MAP_FAILED) {
      mm_bytes_ = 0;
      fb_bytes_ = 0;
      return nullptr;
    }
    mm_bytes_ = max_bytes;
    committed_ = 0;
    return p;
  }
  void* table_commit(void* base, size_t bytes) override {
    if (mm_bytes_) {
      if (bytes > mm_bytes_) throw std::runtime_error("xflow: table beyond its reserved range");
      if (bytes > committed_) committed_ = bytes;
      return base;
    }
    if (bytes <= fb_bytes_) return base;
    void* p = alloc(bytes);
    if (base) {
      std::memcpy(p, base, fb_bytes_);
      std::free(base);
    }
    fb_bytes_ = bytes;
    return p;
  }
  void table_release(void* base) override {
    if (mm_bytes_) {
      if (base) munmap(base, mm_bytes_);
      mm_bytes_ = 0;
    } else {
      std::free(base);
    }
    committed_ = fb_bytes_ = 0;
  }
  size_t table_committed() const override { return mm_bytes_ ? committed_ : fb_bytes_; }
  bool table_in_place() const override { return mm_bytes_ != 0; }
  EvalMetrics eval_metrics(const float* pctr, const float* labels, int64_t n) override {
    // same definition as the HIP kernels: stable order by pctr descending
    EvalMetrics m;
    m.n = n;
    std::vector<int64_t> idx((size_t)n);
    for (int64_t i = 0; i < n; ++i) idx[(size_t)i] = i;
    std::stable_sort(idx.begin(), idx.end(),
                     [&](int64_t a, int64_t b) { return pctr[a] > pctr[b]; });
    uint64_t tp = 0;
    for (int64_t i : idx) {
      if (labels[i] > 0.5f) ++tp;
      else m.area += tp;
    }
    m.tp = (int64_t)tp;
    for (int64_t i = 0; i < n; ++i) {
      const float p = pctr[i];
      const int y = labels[i] > 0.5f ? 1 : 0;
      m.log2_sum += (double)((float)y * std::log2(p)) + (1.0 - y) * std::log2(1.0 - (double)p);
      const float pc = std::fmin(std::fmax(p, 1e-7f), 1.0f - 1e-7f);
      m.ln_sum += y ? -std::log((double)pc) : -std::log(1.0 - (double)pc);
    }
    return m;
  }
  int64_t table_nonzero(const TableView& t, const OptSpec& o) override {
    int64_t n = 0;
    for (u64 s = 0; s < t.cap; ++s) {
      const u32* sp = t.words + s * (u64)t.L.stride;
      const u64 key = *reinterpret_cast<const u64*>(sp);
      if (key == kEmptyKey) continue;
      for (int p = 0; p < t.L.P; ++p) n += slot_weight(sp, key, p, t.L, o) != 0.0f;
    }
    return n;
  }

 private:
  std::vector<char> stage_buf_[2];
  size_t mm_bytes_ = 0, committed_ = 0, fb_bytes_ = 0;
};

}  // namespace

std::unique_ptr<Backend> make_cpu_backend() { return std::unique_ptr<Backend>(new CpuBackend()); }

}  // namespace xflow
