// xflow-amd: native training loop (see xflow/trainer.h).
#include "xflow/trainer.h"

#include <cstdlib>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <fstream>
#include <iostream>
#include <sstream>
#include <stdexcept>
#include <thread>

namespace xflow {

EvalResult reference_auc(std::vector<std::pair<int, float>>& v) {
  // base.h:84-110, reproduced operation for operation (float accumulators,
  // std::sort by pctr descending, log2 of float / double mix).
  std::sort(v.begin(), v.end(),
            [](const std::pair<int, float>& a, const std::pair<int, float>& b) {
              return a.second > b.second;
            });
  float area = 0.0f;
  int tp_n = 0;
  float logloss = 0.0f;
  double ln = 0.0;
  for (size_t i = 0; i < v.size(); ++i) {
    int label = v[i].first;
    float pctr = v[i].second;
    if (label == 1) tp_n += 1;
    else area += tp_n;
    logloss += label * std::log2(pctr) + (1.0 - label) * std::log2(1.0 - pctr);
    float pc = std::fmin(std::fmax(pctr, 1e-7f), 1.0f - 1e-7f);
    ln += label ? -std::log((double)pc) : -std::log(1.0 - (double)pc);
  }
  EvalResult r;
  r.n = (int64_t)v.size();
  r.tp = tp_n;
  if (!v.empty()) logloss /= v.size();
  r.logloss_printed = logloss;
  r.ln_logloss = v.empty() ? 0.0 : ln / (double)v.size();
  std::ostringstream os;
  os << "logloss: " << logloss << "\t";
  if (tp_n == 0 || tp_n == (int)v.size()) {
    os << "tp_n = " << tp_n;
    r.auc = std::nan("");
  } else {
    area /= 1.0 * (tp_n * (v.size() - tp_n));
    r.auc = area;
    os << "auc = " << area << "\ttp = " << tp_n << " fp = " << v.size() - tp_n;
  }
  r.line = os.str();
  return r;
}

EvalResult eval_result(const EvalMetrics& m) {
  EvalResult r;
  r.n = m.n;
  r.tp = m.tp;
  float logloss = (float)m.log2_sum;
  if (m.n > 0) logloss /= (float)m.n;  // (base.h:100: float /= size_t)
  r.logloss_printed = logloss;
  r.ln_logloss = m.n > 0 ? m.ln_sum / (double)m.n : 0.0;
  std::ostringstream os;
  os << "logloss: " << logloss << "\t";
  if (m.tp == 0 || m.tp == m.n) {
    os << "tp_n = " << m.tp;
    r.auc = std::nan("");
  } else {
    float area = (float)m.area;
    area /= 1.0 * ((uint64_t)m.tp * (uint64_t)(m.n - m.tp));
    r.auc = area;
    os << "auc = " << area << "\ttp = " << m.tp << " fp = " << m.n - m.tp;
  }
  r.line = os.str();
  return r;
}

Trainer::Trainer(const TrainerConfig& cfg) : cfg_(cfg) {
  // the reference's slice count is std::thread::hardware_concurrency()
  // (lr_worker.h:40-41); XFLOW_HARDWARE_CONCURRENCY stands in for it (tests
  // of many-core hosts on a small one)
  const char* hc = std::getenv("XFLOW_HARDWARE_CONCURRENCY");
  const int hw = hc && std::atoi(hc) > 0 ? std::atoi(hc) : (int)std::thread::hardware_concurrency();
  threads_ = cfg_.threads > 0 ? cfg_.threads : hw;
  if (threads_ < 1) threads_ = 1;
  // (any count: more than Engine::kSliceGroup slices run group by group)
  if (cfg_.test_block_bytes <= 0) cfg_.test_block_bytes = cfg_.model == kLR ? (4 << 20) : (2 << 20);
  EngineConfig ec;
  ec.model = cfg_.model_spec;
  ec.model.kind = cfg_.model;
  ec.opt = cfg_.opt;
  ec.table_log2_cap = cfg_.table_log2_cap;
  int64_t maxb = std::max(cfg_.train_block_bytes, cfg_.test_block_bytes);
  ec.max_rows = maxb / 2 + 16;   // a row needs >= 2 bytes ("0\t")
  ec.max_nnz = maxb / 2 + 16;    // a token needs >= 2 bytes ("a:")
  ec.max_slices = cfg_.serial_slices ? 1 : threads_;
  ec.sum_slices = cfg_.sum_slices;
  ec.device = cfg_.device;
  engine_.reset(new Engine(ec));
  pctr_dev_ = static_cast<float*>(engine_->backend().alloc(sizeof(float) * ec.max_rows));
}

Trainer::~Trainer() {
  if (engine_ && pctr_dev_) {
    engine_->synchronize();
    engine_->backend().free(pctr_dev_);
  }
}

std::ostream& Trainer::out() { return std::cout; }

static std::string shard_path(const std::string& prefix, int rank) {
  char buf[32];
  std::snprintf(buf, sizeof(buf), "-%05d", rank);
  return prefix + buf;
}

void Trainer::train_block(const CsrBlock& blk) {
  const int64_t rows = blk.rows();
  int64_t ts = rows / threads_;
  int64_t used = ts * threads_;
  int64_t slice_rows = ts;
  if (cfg_.keep_remainder) {
    slice_rows = (rows + threads_ - 1) / threads_;
    used = rows;
  }
  if (slice_rows <= 0 || used <= 0) return;  // every slice empty (lr_worker.cc:190-196)
  BatchView h;
  h.keys = blk.keys.data();
  h.row_ptr = blk.row_ptr.data();
  h.fgid = blk.fgid.data();
  h.labels = blk.labels.data();
  h.rows = used;
  h.nnz = blk.row_ptr[used];
  h.slice_rows = slice_rows;
  static const bool sync_staging = std::getenv("XFLOW_SYNC_STAGING") != nullptr;  // (A/B)
  if (!cfg_.serial_slices && !sync_staging) {
    // double-buffered: this block's H2D copies run on the copy queue while
    // the previous block trains; the host returns to parsing right away
    BatchView d = engine_->stage_host_batch_async(h);
    engine_->train_step(d);
    engine_->stage_release();
    return;
  }
  BatchView d = engine_->stage_host_batch(h);
  // serial: one engine step per slice, in slice order
  for (int64_t s0 = 0; s0 < used; s0 += slice_rows) {
    int64_t n = std::min(slice_rows, used - s0);
    BatchView sb = d;
    // re-base the CSR window: stage this slice separately (row_ptr offsets)
    std::vector<int32_t> rp(n + 1);
    int32_t base = blk.row_ptr[s0];
    for (int64_t r = 0; r <= n; ++r) rp[r] = blk.row_ptr[s0 + r] - base;
    BatchView hs;
    hs.keys = blk.keys.data() + base;
    hs.row_ptr = rp.data();
    hs.fgid = blk.fgid.data() + base;
    hs.labels = blk.labels.data() + s0;
    hs.rows = n;
    hs.nnz = rp[n];
    hs.slice_rows = n;
    sb = engine_->stage_host_batch(hs);
    engine_->train_step(sb);
  }
}

void Trainer::train_epochs(int epochs) {
  const std::string path = shard_path(cfg_.train_prefix, cfg_.rank);
  if (cfg_.init_push) {
    // lr_worker.cc:180-182 (key 0), fm_worker.cc:248-252 (key 0, w and v),
    // mvm_worker.cc:276-278 (key 1, v)
    const int P = engine_->config().model.P();
    std::vector<u64> k(1, cfg_.model == kMVM ? 1ull : 0ull);
    std::vector<float> g((size_t)P, 0.0f);
    engine_->push_host(k, g);
  }
  CsrBlock blk;
  for (int epoch = 0; epoch < epochs; ++epoch) {
    PrefetchReader reader(path, (size_t)cfg_.train_block_bytes);
    while (reader.next(blk)) train_block(blk);
    if ((epoch + 1) % 30 == 0 && cfg_.verbose) out() << "epoch : " << epoch << std::endl;
  }
  engine_->synchronize();
}

EvalResult Trainer::predict(int block) {
  char name[64];
  std::snprintf(name, sizeof(name), "pred_%d_%d.txt", cfg_.rank, block);
  std::string fname = cfg_.pred_dir + "/" + name;
  std::ofstream md(fname);
  if (!md.is_open()) out() << "open pred file failure!" << std::endl;
  const std::string path = shard_path(cfg_.test_prefix, cfg_.rank);
  BlockReader reader(path, (size_t)cfg_.test_block_bytes);
  std::vector<std::pair<int, float>> auc;
  std::vector<float> pctr;
  CsrBlock blk;
  while (reader.next(blk)) {
    const int64_t rows = blk.rows();
    int64_t ts = rows / threads_;
    int64_t used = ts * threads_;
    if (cfg_.keep_remainder) used = rows;
    if (used <= 0) continue;
    BatchView h;
    h.keys = blk.keys.data();
    h.row_ptr = blk.row_ptr.data();
    h.fgid = blk.fgid.data();
    h.labels = blk.labels.data();
    h.rows = used;
    h.nnz = blk.row_ptr[used];
    BatchView d = engine_->stage_host_batch(h);
    engine_->eval_step(d, pctr_dev_);
    pctr.resize(used);
    engine_->backend().copy_d2h(pctr.data(), pctr_dev_, sizeof(float) * used);
    for (int64_t r = 0; r < used; ++r) {
      if (cfg_.model == kMVM && cfg_.mvm_predict_compat && ts > 0) {
        // mvm_worker.cc:96 emits v_multi.size() (= v_dim) rows per slice
        int64_t in_slice = r % ts;
        if (in_slice >= std::min<int64_t>(engine_->config().model.v_dim, ts)) continue;
      }
      int label = blk.labels[r] > 0.5f ? 1 : 0;
      auc.emplace_back(label, pctr[r]);
      md << pctr[r] << "\t" << 1 - label << "\t" << label << std::endl;
    }
  }
  md.close();
  EvalResult res = reference_auc(auc);
  if (cfg_.verbose) out() << res.line << std::endl;
  return res;
}

void Trainer::train() {
  if (cfg_.verbose) out() << "my rank is = " << cfg_.rank << std::endl;
  train_epochs(cfg_.epochs);
  if (cfg_.rank == 0) {
    if (cfg_.verbose) out() << (cfg_.model == kLR ? "LR AUC: " : "FM AUC: ") << std::endl;
    predict(0);
  }
  if (cfg_.verbose) out() << "train end......" << std::endl;
}

}  // namespace xflow
