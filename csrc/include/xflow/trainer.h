// xflow-amd: native single-rank training loop over libffm shard files.
//
// Mirrors the reference workers' batch_training / predict / train
// (/root/reference/src/model/lr/lr_worker.cc:73-217 and the FM/MVM twins):
// epochs over `<train_prefix>-%05d` (rank), blocks of `block_bytes`, each
// block split into `threads` slices of rows/threads rows (remainder dropped
// unless keep_remainder), then rank 0 predicts `<test_prefix>-%05d`, writes
// pred_<rank>_0.txt and prints the reference's logloss/AUC line.
//
// The reference's `core_num` Hogwild threads become the slices of one engine
// step (slice_mode "concurrent": all slices read the same weights and push in
// slice order), or one engine step per slice ("serial").
#pragma once

#include <cstdint>
#include <iosfwd>
#include <memory>
#include <string>
#include <vector>

#include "xflow/engine.h"
#include "xflow/reader.h"

namespace xflow {

struct TrainerConfig {
  std::string train_prefix;
  std::string test_prefix;
  int model = kLR;
  int epochs = 60;                 // lr_worker.h:63
  int threads = 0;                 // 0 => std::thread::hardware_concurrency (lr_worker.h:40)
  int64_t train_block_bytes = 2 << 20;   // lr_worker.h:68
  int64_t test_block_bytes = 0;    // 0 => 4 MB for LR, 2 MB for FM/MVM
  bool serial_slices = false;
  bool keep_remainder = false;     // reference drops rows % threads (lr_worker.cc:190)
  bool mvm_predict_compat = false; // reference predicts only 10 rows per MVM slice
  bool init_push = true;           // lr_worker.cc:180-182 / fm_worker.cc:248-252 / mvm :276-278
  int rank = 0;
  std::string pred_dir = ".";
  int device = -1;                 // -1 CPU backend, >=0 HIP device
  int table_log2_cap = 22;
  ModelSpec model_spec;            // v_dim, math modes (kind is taken from `model`)
  OptSpec opt;
  bool sum_slices = false;
  bool verbose = true;
};

struct EvalResult {
  double logloss_printed = 0;  // reference: signed mean log2-likelihood (float accumulation)
  double ln_logloss = 0;       // standard logloss, p clipped to [1e-7, 1-1e-7]
  double auc = 0;
  int64_t tp = 0, n = 0;
  std::string line;            // the exact line printed by calculate_auc
};

// Reference AUC / logloss printer semantics (base.h:84-110) on host data.
EvalResult reference_auc(std::vector<std::pair<int, float>>& label_pctr);
// The same printed line from device-computed sums (Backend::eval_metrics):
// exact integer area, deterministic double log-likelihood sums, rounded to
// the reference's float accumulators once at the end.
EvalResult eval_result(const EvalMetrics& m);

class Trainer {
 public:
  explicit Trainer(const TrainerConfig& cfg);
  ~Trainer();
  void train();                   // full run incl. rank-0 predict (prints like the reference)
  void train_epochs(int epochs);  // training only
  EvalResult predict(int block = 0);
  Engine& engine() { return *engine_; }
  const TrainerConfig& config() const { return cfg_; }
  int threads() const { return threads_; }

 private:
  void train_block(const CsrBlock& blk);
  std::ostream& out();
  TrainerConfig cfg_;
  int threads_ = 1;
  std::unique_ptr<Engine> engine_;
  float* pctr_dev_ = nullptr;
};

}  // namespace xflow
